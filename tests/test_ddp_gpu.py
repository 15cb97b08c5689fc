"""Native data-parallel step on the GPU with 2 ranks sharing one MI355X.

RCCL needs one GPU per rank, so on the single-GPU test box the collective
backend is gloo (device tensors staged through the host); the code path under
test — rank-0 broadcast, backward-completion bucketing, overlapped async
all-reduce, 1/world folded into the fused Adam — is the one RCCL drives on a
multi-GPU node (bench.py / train.py with backend nccl).
"""
import os

import pytest
import torch
import torch.distributed as dist

from mp_util import free_port as _free_port, run_ranks as _run_ranks

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, model_name, q):
    os.environ["PGDIST_PLAN"] = "force"   # the replayed (launch-plan) step, as with RCCL
    import pgdist  # noqa: F401
    from pgdist.models import build_model
    from pgdist.engine.native_step import NativeTrainStep
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.manual_seed(100 + rank)            # different init per rank: the broadcast must fix it
    model = build_model(model_name, num_classes=10)
    st = NativeTrainStep(model, 8, dev, img_size=64, lr=1e-3, world_size=world, rank=rank,
                         bucket_mb=0.5 if model_name == "mobilenet_v2" else 8.0, first_bucket_mb=0.1)
    g = torch.Generator(device=dev).manual_seed(7)
    src = torch.randint(0, 256, (64, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
    labels = torch.randint(0, 10, (64,), device=dev, generator=g)
    st.set_data(src, labels)
    for i in range(4):
        st.run(torch.arange(8, device=dev) + 8 * (2 * i + rank))   # different shards per rank
    torch.cuda.synchronize()
    w = st.flat.master.clone()
    allw = [torch.zeros_like(w) for _ in range(world)]
    dist.all_gather(allw, w)
    diff = max((a - w).abs().max().item() for a in allw)
    l, c, n = st.read_metrics()
    q.put(("ok", rank, diff, n, len(st.reducer.buckets), bool(torch.isfinite(w).all())))
    dist.destroy_process_group()


@pytest.mark.parametrize("model_name", ["mobilenet_v2", "resnet50"])
def test_native_ddp_two_ranks_one_gpu(model_name):
    """4 data-parallel steps, launch-plan replay forced (MobileNetV2): replicas stay identical."""
    world, port = 2, _free_port()
    res = _run_ranks(_worker, world, (world, port, model_name), expect=world)
    for _, rank, diff, n, nb, finite in res:
        assert finite
        assert diff == 0.0, f"replicas diverged on rank {rank}: {diff}"
        assert n == 32
        assert nb >= 3


def _grad_worker(rank, world, port, q):
    import pgdist  # noqa: F401
    from pgdist.models import build_model
    from pgdist.engine.native_step import NativeTrainStep
    from pgdist.ops import kernels as K
    K.set_deterministic(True)   # the shard-sum comparison needs bitwise-reproducible BN statistics
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    src = torch.randint(0, 256, (32, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
    labels = torch.randint(0, 10, (32,), device=dev, generator=g)

    def make(world_size, r):
        torch.manual_seed(100)
        st = NativeTrainStep(build_model("mobilenet_v2", num_classes=10), 8, dev, img_size=64, lr=1e-3,
                             world_size=world_size, rank=r, bucket_mb=0.5, first_bucket_mb=0.1)
        st.set_data(src, labels)
        return st

    shard = lambda r: torch.arange(8, device=dev) + 8 * r   # noqa: E731
    st = make(world, rank)
    st.run(shard(rank))
    torch.cuda.synchronize()
    reduced = st.flat.grad.clone()
    if rank == 0:
        # the same first step on each shard alone (same weights, dropout / augmentation seeds)
        singles = []
        for r in range(world):
            s1 = make(1, r)
            s1.run(shard(r))
            torch.cuda.synchronize()
            singles.append(s1.flat.grad.clone())
        expect = singles[0] + singles[1]
        # per bucket: every bucket must hold a nonzero gradient (a zeroed / never-written
        # bucket would otherwise pass a relative check) and match the shard sum
        per = []
        for bi, (b0, b1, names) in enumerate(st.reducer.buckets):
            e, r_ = expect[b0:b1], reduced[b0:b1]
            scale = e.abs().max().item()
            err = (r_ - e).abs().max().item() / (scale + 1e-12)
            per.append((bi, names[0], names[-1], scale, err))
        q.put(("ok", per))
    dist.barrier()
    dist.destroy_process_group()


def test_native_ddp_reduced_gradient_equals_sum_of_shards():
    """After one data-parallel step the flat gradient buffer holds the SUM of the per-shard
    gradients (the 1/world is folded into Adam): checks the bucket launches are ordered after
    every producer of their gradients (main-stream dgrad-side BN grads and side-stream wgrads)."""
    world, port = 2, _free_port()
    (_, per), = _run_ranks(_grad_worker, world, (world, port), expect=1)
    assert len(per) >= 3
    for bi, first, last, scale, err in per:
        assert scale > 0, f"bucket {bi} ({first} .. {last}) has an all-zero gradient"
        assert err < 1e-5, f"bucket {bi} ({first} .. {last}): rel err {err}"


def _lazy_bn_grad_worker(rank, world, port, q):
    """Lazy BN finalize (default mode) under data parallelism: the BN weight / bias gradients
    are written by the side-stream batched finalizes, and every gradient bucket holding them
    must be all-reduced only after those ran.  After one step each rank recomputes its LOCAL
    dgamma / dbeta from the backward accumulators (still intact until the next forward) and
    all-reduces them itself: the reducer's buckets must hold exactly that sum."""
    import pgdist  # noqa: F401
    from pgdist.models import build_model
    from pgdist.engine.native_step import NativeTrainStep
    from pgdist.ops import kernels as K
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(7)
    src = torch.randint(0, 256, (32, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
    labels = torch.randint(0, 10, (32,), device=dev, generator=g)
    torch.manual_seed(100)
    st = NativeTrainStep(build_model("mobilenet_v2", num_classes=10), 8, dev, img_size=64, lr=1e-3,
                         world_size=world, rank=rank, bucket_mb=0.5, first_bucket_mb=0.1)
    assert st.exe.bn_mode == "lazy"
    st.set_data(src, labels)
    st.run(torch.arange(8, device=dev) + 8 * rank)
    torch.cuda.synchronize()
    bns = st.exe.all_bns()
    local = []
    for bn in bns:
        coef = torch.zeros(3, bn.C, device=dev)
        dg, db = torch.zeros(bn.C, device=dev), torch.zeros(bn.C, device=dev)
        K.bn_bwd_finalize(bn.acc_b, bn.rows_b, bn.C, bn.M, bn.mean, bn.rstd, bn.gamma, coef, dg, db)
        local += [dg, db]
    torch.cuda.synchronize()
    mine = torch.cat(local).cpu()
    dist.all_reduce(mine)
    got = torch.cat([st.flat.grad[slice(*st.flat.range_of(n))] for bn in bns for n in bn.param_names]).cpu()
    err = ((got - mine).abs().max() / (mine.abs().max() + 1e-12)).item()
    q.put(("ok", rank, err, mine.abs().max().item()))
    dist.barrier()
    dist.destroy_process_group()


def test_native_ddp_lazy_bn_gradients_reduced_after_side_finalize():
    world, port = 2, _free_port()
    res = _run_ranks(_lazy_bn_grad_worker, world, (world, port), expect=world)
    for _, rank, err, scale in res:
        assert scale > 0
        assert err < 1e-6, f"rank {rank}: BN gradients in the buckets differ from the summed local ones ({err})"
