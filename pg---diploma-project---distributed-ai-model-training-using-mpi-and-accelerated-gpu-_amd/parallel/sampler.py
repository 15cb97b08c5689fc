"""Data sharding with ``torch.utils.data.distributed.DistributedSampler`` index math.

Reference: ``DistributedSampler(train, num_replicas=W, rank=r, shuffle=True)``,
``DistributedSampler(test, ..., shuffle=False)`` and ``set_epoch(epoch)``
(``cifar10_mpi_mobilenet_224.py:119-124,165``).  Algorithm: ``randperm(N)`` from
a generator seeded ``seed + epoch`` (or ``arange`` when not shuffling) -> pad by
repeating the head to ``ceil(N/W)*W`` (or truncate when ``drop_last``) ->
``indices[rank::W]``.

The permutation is drawn with torch's CPU generator (bit-identical to the
reference); the padding/striding runs in the native runtime
(``_pgdist_C.shard_indices``) and the result is uploaded once per epoch as a
device int64 tensor that the GPU augmentation kernel gathers from — no
DataLoader worker processes.
"""
import math
from typing import Iterator, Optional

import numpy as np
import torch


class ShardSampler:
    def __init__(self, dataset_len: int, num_replicas: int = 1, rank: int = 0, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False):
        if rank < 0 or rank >= num_replicas:
            raise ValueError(f"invalid rank {rank} for {num_replicas} replicas")
        self.n = dataset_len
        self.num_replicas, self.rank = num_replicas, rank
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0
        if drop_last and self.n % num_replicas != 0:
            self.num_samples = math.ceil((self.n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(self.n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def permutation(self) -> torch.Tensor:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            return torch.randperm(self.n, generator=g)
        return torch.arange(self.n)

    def indices(self, native: Optional[bool] = None) -> np.ndarray:
        perm = self.permutation().numpy().astype(np.int64)
        use_native = native if native is not None else True
        if use_native:
            try:
                from ..ops._lib import lib
                return np.asarray(lib().shard_indices(perm, self.num_replicas, self.rank, self.drop_last))
            except Exception:
                if native:
                    raise
        return self._indices_py(perm)

    def _indices_py(self, perm: np.ndarray) -> np.ndarray:
        idx = list(perm)
        if not self.drop_last:
            pad = self.total_size - len(idx)
            if pad <= len(idx):
                idx += idx[:pad]
            else:
                idx += (idx * math.ceil(pad / len(idx)))[:pad]
        else:
            idx = idx[: self.total_size]
        return np.asarray(idx[self.rank:self.total_size:self.num_replicas], dtype=np.int64)

    def __iter__(self) -> Iterator[int]:
        return iter(self.indices().tolist())

    def __len__(self) -> int:
        return self.num_samples

    def device_batches(self, batch_size: int, device, drop_last: bool = False):
        """Yield int64 device index tensors of ``batch_size`` (last one possibly short)."""
        idx = torch.from_numpy(self.indices()).to(device)
        n = idx.numel()
        end = n - (n % batch_size) if drop_last else n
        for s in range(0, end, batch_size):
            yield idx[s:min(s + batch_size, end)]
