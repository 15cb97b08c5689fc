"""Data-parallel layer on CPU with the gloo backend, world_size 2 (SURVEY.md §4 'Distributed (fake)').

* bucketed all-reduce == all-reduce of the whole gradient
* W ranks on shards == 1 rank on the concatenated batch (BN in eval mode, so the
  per-rank batch statistics of training-mode BN do not enter the comparison)
* the full Trainer (torch backend) runs 2 ranks and keeps replicas identical
"""
import os

import pytest
import torch
import torch.distributed as dist

from mp_util import free_port as _free_port, run_ranks
from pgdist.parallel.ddp import build_buckets


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def test_build_buckets_small_first_bucket():
    ranges = [(f"p{i}", i * 1000, i * 1000 + 1000) for i in range(20)]   # 20 x 4 KB
    b = build_buckets(ranges, cap_bytes=16000, first_cap_bytes=4000)
    assert b[0][2] == ["p0"]
    assert all(len(x[2]) == 4 for x in b[1:-1])
    covered = [n for _, _, names in b for n in names]
    assert covered == [f"p{i}" for i in range(20)]


def _worker_equivalence(rank, world, port, q):
    import pgdist  # noqa: F401
    from pgdist.models import mobilenet_v2
    from pgdist.engine.flat import FlatParams
    from pgdist.parallel.ddp import BucketedGradReducer
    _init(rank, world, port)
    torch.manual_seed(0)
    model = mobilenet_v2(10).eval()
    flat = FlatParams(model, torch.device("cpu"), with_shadow=False)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(8, 3, 32, 32, generator=g)
    y = torch.randint(0, 10, (8,), generator=g)
    # full-batch reference gradient on every rank
    flat.grad.zero_()
    torch.nn.functional.cross_entropy(model(x), y).backward()
    ref = flat.grad.clone()
    # sharded gradient + bucketed all-reduce (small caps -> many buckets)
    flat.grad.zero_()
    sl = slice(rank * 4, rank * 4 + 4)
    torch.nn.functional.cross_entropy(model(x[sl]), y[sl]).backward()
    red = BucketedGradReducer(flat.grad, [(n,) + flat.range_of(n) for n in flat.order],
                              bucket_cap_mb=0.5, first_bucket_mb=0.05)
    red.begin()
    for n in flat.order:            # parameters become ready one by one (backward order)
        red.mark_ready([n])
    red.finish()
    flat.grad.mul_(1.0 / world)
    err = ((flat.grad - ref).norm() / ref.norm()).item()
    q.put(("ok", rank, err, len(red.buckets)))
    dist.destroy_process_group()


def test_sharded_gradient_equals_full_batch():
    world, port = 2, _free_port()
    res = run_ranks(_worker_equivalence, world, (world, port), expect=world, timeout=240)
    for _, rank, err, nb in res:
        assert err < 1e-5, (rank, err)
        assert nb > 3


def _worker_trainer(rank, world, port, tmp, bn_sync, q):
    import pgdist  # noqa: F401
    from pgdist.config import TrainConfig
    from pgdist.engine.trainer import Trainer
    from pgdist.parallel.bootstrap import DistInfo
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    info = DistInfo(rank=rank, world_size=world, local_rank=rank, local_world_size=world, master_port=port)
    cfg = TrainConfig(data="synthetic", synthetic_train_size=48, synthetic_test_size=16, batch_size=8, epochs=1,
                      img_size=32, device="cpu", backend="torch", precision="fp32", augment="none",
                      save_path=os.path.join(tmp, "best_mpi.pth"), log_format="ddp", seed=42, bn_sync=bn_sync)
    tr = Trainer(cfg, info=info)
    tr.fit()
    w = tr.flat.master.clone()
    allw = [torch.zeros_like(w) for _ in range(world)]
    dist.all_gather(allw, w)
    rs = torch.cat([b.float().reshape(-1) for b in tr._bn_buffers()])
    allrs = [torch.zeros_like(rs) for _ in range(world)]
    dist.all_gather(allrs, rs)
    q.put(("ok", rank, max((a - w).abs().max().item() for a in allw), tr.history[-1]["train_images"],
           max((a - rs).abs().max().item() for a in allrs), tr.replicas_ok))
    dist.destroy_process_group()


@pytest.mark.parametrize("bn_sync", ["eval", "broadcast", "none"])
def test_trainer_two_ranks_keeps_replicas_in_sync(tmp_path, bn_sync):
    world, port = 2, _free_port()
    res = run_ranks(_worker_trainer, world, (world, port, str(tmp_path), bn_sync), expect=world, timeout=300)
    for _, rank, diff, n, bn_diff, rep_ok in res:
        assert diff == 0.0
        assert n == 48
        assert rep_ok == (True, bn_sync != "none")   # Trainer.replica_check agrees with the gather
        if bn_sync == "none":       # rank-local running statistics (different shards)
            assert bn_diff > 0.0
        else:                       # rank-0 statistics broadcast (reference DDP broadcast_buffers)
            assert bn_diff == 0.0
    assert (tmp_path / "best_mpi.pth").exists()
    sd = torch.load(tmp_path / "best_mpi.pth", weights_only=True)
    assert not any(k.startswith("module.") for k in sd) and len(sd) == 314


def test_would_launch_predicts_bucket_launches():
    """The executor skips the side-stream join for per-layer ready calls that launch no
    bucket; ``would_launch`` must predict exactly the calls after which ``mark_ready`` launches."""
    import random
    from pgdist.parallel.ddp import BucketedGradReducer
    ranges, o = [], 0
    for i in range(40):
        n = 1000 * (1 + i % 7)
        ranges.append((f"p{i}", o, o + n))
        o += n
    red = BucketedGradReducer(torch.zeros(o), ranges, bucket_cap_mb=0.05, first_bucket_mb=0.01)
    red.world = 2   # pretend data parallel; collectives are recorded instead of issued
    launched = []
    red._launch = lambda bi: launched.append(bi)
    assert len(red.buckets) > 3
    rng = random.Random(0)
    for trial in range(5):
        red.begin()
        launched.clear()
        names = [r[0] for r in ranges][::-1]
        groups = []
        while names:
            k = rng.randint(1, 4)
            groups.append(names[:k])
            names = names[k:]
        for g in groups:
            pred = red.would_launch(g)
            before = len(launched)
            red.mark_ready(g)
            assert pred == (len(launched) > before), (trial, g)
        assert launched == list(range(len(red.buckets)))
