"""Native data-parallel step on the GPU with 2 ranks sharing one MI355X, and the native
communicator at world size 1.

RCCL refuses two ranks on one GPU, so the 2-rank tests run the default process group on gloo
and the gradient buckets either through c10d (``PGDIST_COMM=c10d``: host-staged gloo
collectives) or through the native communicator's P2P xGMI kernels between the two processes
(``PGDIST_COMM=p2p``: IPC-mapped staging, collectives recorded into the replayed launch plan
— the production data-parallel step minus RCCL).  RCCL itself is exercised at world size 1
with the reducer forced on: every bucket is a recorded ncclAllReduce on the comm stream, and
the weights after 6 replayed steps must be bitwise equal to the plain single-GPU step.
"""
import os

import pytest
import torch
import torch.distributed as dist

from mp_util import free_port as _free_port, run_ranks as _run_ranks

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, model_name, comm, q):
    os.environ["PGDIST_PLAN"] = "force"   # the replayed (launch-plan) step, as with RCCL
    os.environ["PGDIST_COMM"] = comm
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
    native = getattr(st.reducer, "native", False)
    err = st.comm.error() if st.comm is not None else 0
    q.put(("ok", rank, diff, n, len(st.reducer.buckets), bool(torch.isfinite(w).all()), native, err))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("comm", ["c10d", "p2p"])
@pytest.mark.parametrize("model_name", ["mobilenet_v2", "resnet50"])
def test_native_ddp_two_ranks_one_gpu(model_name, comm):
    """4 data-parallel steps, launch-plan replay forced (MobileNetV2): replicas stay identical."""
    world, port = 2, _free_port()
    res = _run_ranks(_worker, world, (world, port, model_name, comm), expect=world)
    for _, rank, diff, n, nb, finite, native, err in res:
        assert native == (comm == "p2p")
        assert err == 0
        assert finite
        assert diff == 0.0, f"replicas diverged on rank {rank}: {diff}"
        assert n == 32
        assert nb >= 3


def _grad_worker(rank, world, port, comm, q):
    os.environ["PGDIST_COMM"] = comm
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


@pytest.mark.parametrize("comm", ["c10d", "p2p"])
def test_native_ddp_reduced_gradient_equals_sum_of_shards(comm):
    """After one data-parallel step the flat gradient buffer holds the SUM of the per-shard
    gradients (the 1/world is folded into Adam): checks the bucket launches are ordered after
    every producer of their gradients (main-stream dgrad-side BN grads and side-stream wgrads)."""
    world, port = 2, _free_port()
    (_, per), = _run_ranks(_grad_worker, world, (world, port, comm), expect=1)
    assert len(per) >= 3
    for bi, first, last, scale, err in per:
        assert scale > 0, f"bucket {bi} ({first} .. {last}) has an all-zero gradient"
        assert err < 1e-5, f"bucket {bi} ({first} .. {last}): rel err {err}"


def _lazy_bn_grad_worker(rank, world, port, comm, q):
    """Lazy BN finalize (default mode) under data parallelism: the BN weight / bias gradients
    are written by the side-stream batched finalizes, and every gradient bucket holding them
    must be all-reduced only after those ran.  After one step each rank recomputes its LOCAL
    dgamma / dbeta from the backward accumulators (still intact until the next forward) and
    all-reduces them itself: the reducer's buckets must hold exactly that sum."""
    os.environ["PGDIST_COMM"] = comm
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


@pytest.mark.parametrize("comm", ["c10d", "p2p"])
def test_native_ddp_lazy_bn_gradients_reduced_after_side_finalize(comm):
    world, port = 2, _free_port()
    res = _run_ranks(_lazy_bn_grad_worker, world, (world, port, comm), expect=world)
    for _, rank, err, scale in res:
        assert scale > 0
        assert err < 1e-6, f"rank {rank}: BN gradients in the buckets differ from the summed local ones ({err})"


@pytest.mark.parametrize("comm,model_name", [("rccl", "mobilenet_v2"), ("p2p", "mobilenet_v2"), ("rccl", "resnet50")])
def test_native_reducer_world1_bitwise_equals_plain_step(dev, comm, model_name):
    """RCCL (or the P2P kernels) at world size 1 with the reducer forced on: buckets, comm
    stream, event ordering and (MobileNetV2) the recorded launch plan replayed for steps 4-6.
    In deterministic mode the weights, BN buffers and metrics after 6 steps are bitwise equal
    to the plain single-GPU step's."""
    from pgdist.models import build_model
    from pgdist.engine.native_step import NativeTrainStep
    from pgdist.ops import kernels as K
    K.set_deterministic(True)
    try:
        g = torch.Generator(device=dev).manual_seed(7)
        src = torch.randint(0, 256, (64, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
        labels = torch.randint(0, 10, (64,), device=dev, generator=g)

        def run(force):
            torch.manual_seed(100)
            st = NativeTrainStep(build_model(model_name, num_classes=10), 8, dev, img_size=64, lr=1e-3,
                                 force_ddp=force, comm=comm if force else None, bucket_mb=0.5,
                                 first_bucket_mb=0.1, use_graph=False)
            st.set_data(src, labels)
            for i in range(6):
                st.run(torch.arange(8, device=dev) + 8 * i)
            torch.cuda.synchronize()
            return st

        plain, ddp = run(False), run(True)
        assert plain.reducer is None
        assert ddp.reducer is not None and ddp.reducer.native and len(ddp.reducer.buckets) >= 3
        assert ddp.comm.error() == 0
        if model_name == "mobilenet_v2":
            assert ddp.use_plan and ddp.plan is not None and len(ddp.plan) > 0
        assert torch.equal(plain.flat.master, ddp.flat.master)
        bn = lambda st: [b for m in st.exe.model.modules() if isinstance(m, torch.nn.BatchNorm2d)   # noqa: E731
                         for b in (m.running_mean, m.running_var)]
        for a, b in zip(bn(plain), bn(ddp)):
            assert torch.equal(a, b)
        assert plain.read_metrics() == ddp.read_metrics()
    finally:
        K.set_deterministic(False)


def _bn_bcast_worker(rank, world, port, det, q):
    os.environ["PGDIST_PLAN"] = "force"   # the replayed step, as with RCCL
    os.environ["PGDIST_COMM"] = "p2p"
    import pgdist  # noqa: F401
    from pgdist.models import build_model
    from pgdist.engine.native_step import NativeTrainStep
    from pgdist.ops import kernels as K
    if det:
        K.set_deterministic(True)   # launch-mode finalize: the join precedes the first finalize
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.manual_seed(100)
    model = build_model("mobilenet_v2", num_classes=10)
    st = NativeTrainStep(model, 8, dev, img_size=64, lr=1e-3, world_size=world, rank=rank,
                         bucket_mb=0.5, first_bucket_mb=0.1, bn_broadcast=True)
    assert st.bn_broadcast
    g = torch.Generator(device=dev).manual_seed(7)
    src = torch.randint(0, 256, (64, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
    st.set_data(src, torch.randint(0, 10, (64,), device=dev, generator=g))
    bns = st.exe.all_bns()
    if rank == 1:   # rank 1's buffers start wrong: only the per-step broadcast can fix them
        with torch.no_grad():
            st.bn_flat.add_(torch.rand_like(st.bn_flat))
            st.bn_nbt.add_(1000)
    for i in range(5):
        if i == 4:
            torch.cuda.synchronize()
            snap = st.bn_flat.cpu().clone()
            nbt0 = st.bn_nbt.cpu().clone()
            dist.broadcast(snap, 0)
            dist.broadcast(nbt0, 0)
        st.run(torch.arange(8, device=dev) + 8 * (2 * i + rank))
    torch.cuda.synchronize()
    assert st.plan is not None or st._plans, "the step must have been replayed from a launch plan"
    # rank r's running mean after the step = (1 - m) * rank 0's buffer before it + m * r's batch mean
    snap_mods = {}
    o = 0
    for m in st.exe.model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            C = m.running_mean.numel()
            snap_mods[id(m)] = (snap[o:o + C], snap[o + C:o + 2 * C])
            o += 2 * C
    worst = 0.0
    for bn in bns:
        rm0, _ = snap_mods[id(bn.module)]
        mom = bn.momentum
        expect = (1.0 - mom) * rm0.to(dev) + mom * bn.mean
        err = ((bn.module.running_mean - expect).abs() / (expect.abs() + 1e-3)).max().item()
        worst = max(worst, err)
    nbt_ok = bool(torch.equal(st.bn_nbt.cpu(), nbt0 + 1))
    q.put(("ok", rank, worst, nbt_ok, st.comm.error()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("det", [False, True])
def test_bn_broadcast_overlapped_with_forward_has_ddp_semantics(det):
    """Per-step BN-buffer broadcast (DDP broadcast_buffers=True, reference :142-145) issued on the
    comm stream and joined only before the forward's first running-statistics update (VERDICT r5
    item 4): rank 1 starts with wrong buffers, and after a replayed step every rank's running mean
    is (1 - momentum) * rank 0's pre-step buffer + momentum * its own batch mean, and its
    num_batches_tracked is rank 0's + 1.  Lazy finalize (one batched update at the end of the
    forward) and deterministic launch mode (a finalize after every producer)."""
    world, port = 2, _free_port()
    res = _run_ranks(_bn_bcast_worker, world, (world, port, det), expect=world)
    for _, rank, worst, nbt_ok, err in res:
        assert err == 0
        assert nbt_ok, f"rank {rank}: num_batches_tracked not rank 0's + 1"
        assert worst < 1e-5, f"rank {rank}: running mean off by {worst}"
