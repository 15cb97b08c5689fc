"""Sharded sampler index parity with torch.utils.data.DistributedSampler (SURVEY.md §2.3 'Data sharding')."""
import numpy as np
import pytest
import torch
from torch.utils.data.distributed import DistributedSampler

from pgdist.parallel.sampler import ShardSampler


class _DS:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


@pytest.mark.parametrize("n,world", [(50000, 1), (50000, 2), (50000, 8), (10000, 4), (103, 8), (5, 8), (7, 3)])
@pytest.mark.parametrize("shuffle", [True, False])
@pytest.mark.parametrize("drop_last", [False, True])
def test_index_parity(n, world, shuffle, drop_last):
    for epoch in (0, 3):
        for rank in range(world):
            ref = DistributedSampler(_DS(n), num_replicas=world, rank=rank, shuffle=shuffle, drop_last=drop_last)
            ref.set_epoch(epoch)
            mine = ShardSampler(n, world, rank, shuffle=shuffle, drop_last=drop_last)
            mine.set_epoch(epoch)
            want = list(iter(ref))
            assert len(mine) == len(ref)
            assert mine._indices_py(mine.permutation().numpy()).tolist() == want
            assert mine.indices().tolist() == want   # native path (falls back if unbuilt)


def test_native_shard_indices_used():
    pytest.importorskip("pgdist._pgdist_C")
    s = ShardSampler(1000, 4, 1)
    assert s.indices(native=True).tolist() == s._indices_py(s.permutation().numpy()).tolist()


def test_shards_partition_dataset():
    n, world = 50000, 8
    seen = np.concatenate([ShardSampler(n, world, r).indices() for r in range(world)])
    assert np.array_equal(np.sort(seen), np.arange(n))


def test_device_batches_cpu():
    s = ShardSampler(300, 2, 0, shuffle=False)
    bs = list(s.device_batches(64, torch.device("cpu")))
    assert [b.numel() for b in bs] == [64, 64, 22]
    assert torch.equal(torch.cat(bs), torch.arange(0, 300, 2))
