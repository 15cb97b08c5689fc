"""Native communicator on one MI355X (parallel/comm.py, csrc/runtime/comm.cpp,
csrc/kernels/allreduce.hip).

* P2P one-shot / two-shot all-reduce and broadcast with N = 2 / 4 / 8 ranks emulated in one
  process (one launch drives every rank's blocks, each rank with its own staging buffer,
  counters and signal slots): results equal the fp32 sum in rank order and are bitwise
  identical on every rank, over several back-to-back calls (epochs, double-buffered regions).
* The same kernels between 2 PROCESSES sharing the GPU through hipIpc handles exchanged over
  the c10d TCPStore (gloo default group): the real inter-process path.
* A rank that never arrives: the barrier gives up after the timeout, the kernel exits and the
  error word reports it (no hung GPU).
* RCCL at world size 1: the communicator, its stream / join ordering and the fp64 metric
  all-reduce.
"""
import os

import pytest
import torch
import torch.distributed as dist

from mp_util import free_port, run_ranks

pytestmark = pytest.mark.gpu


def _expect(xs, bf16):
    acc = torch.zeros_like(xs[0])
    for x in xs:
        acc = acc + (x.to(torch.bfloat16).float() if bf16 else x)
    return acc.to(torch.bfloat16).float() if bf16 else acc


@pytest.mark.parametrize("world", [2, 4, 8])
@pytest.mark.parametrize("algo", ["oneshot", "twoshot"])
@pytest.mark.parametrize("bf16", [False, True])
def test_p2p_emulated_allreduce(dev, world, algo, bf16):
    from pgdist.parallel.comm import NativeComm
    sizes = [8, 8 * 1001, 393216 + 8, 1 << 20]
    c = NativeComm(0, world, dev, p2p_bytes=max(sizes) * 4, blocks=16, timeout_s=5.0, emulate=True)
    try:
        g = torch.Generator(device=dev).manual_seed(world * 10 + len(algo))
        for rep in range(3):          # back-to-back calls: epochs and both staging regions
            for n in sizes:
                xs = [torch.randn(n, device=dev, generator=g) * (p + 1) for p in range(world)]
                want = _expect(xs, bf16)
                bufs = [x.clone() for x in xs]
                c.allreduce(bufs, algo, bf16)
                c.join()
                torch.cuda.synchronize()
                assert c.error() == 0
                for p in range(world):
                    assert torch.equal(bufs[p], bufs[0]), f"rank {p} differs from rank 0 (n={n})"
                assert torch.equal(bufs[0], want), \
                    f"n={n}: max err {(bufs[0] - want).abs().max().item()}"
    finally:
        c.close()


@pytest.mark.parametrize("world", [2, 8])
def test_p2p_emulated_broadcast(dev, world):
    from pgdist.parallel.comm import NativeComm
    c = NativeComm(0, world, dev, p2p_bytes=1 << 20, blocks=8, timeout_s=5.0, emulate=True)
    try:
        for root in range(world):
            xs = [torch.randn(4096 + 4, device=dev) for _ in range(world)]
            src = xs[root].clone()
            c.broadcast(xs, root, "oneshot")
            c.join()
            torch.cuda.synchronize()
            assert c.error() == 0
            for p in range(world):
                assert torch.equal(xs[p], src)
    finally:
        c.close()


def test_p2p_rejects_oversized_and_misaligned(dev):
    from pgdist.parallel.comm import NativeComm
    c = NativeComm(0, 2, dev, p2p_bytes=4096, blocks=4, emulate=True)
    try:
        with pytest.raises(Exception):
            c.allreduce([torch.zeros(4096, device=dev)] * 2, "oneshot")   # 16 KB > 4 KB region
        with pytest.raises(Exception):
            c.allreduce([torch.zeros(12, device=dev)] * 2, "oneshot")     # n % 8 != 0
        with pytest.raises(Exception):
            c.allreduce([torch.zeros(8, device=dev)], "oneshot")          # one buffer per rank
    finally:
        c.close()


def _ipc_worker(rank, world, port, q):
    import pgdist  # noqa: F401
    from pgdist.parallel.comm import NativeComm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c = NativeComm.for_process_group(dev, use_rccl=False, p2p_bytes=1 << 22, blocks=16, timeout_s=10.0)
    results = []
    for algo in ("oneshot", "twoshot"):
        for bf16 in (False, True):
            for n in (8, 65536 + 8, 1 << 20):
                xs = [torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(1000 * p + n))
                      for p in range(world)]
                want = _expect(xs, bf16)
                t = xs[rank].clone()
                c.allreduce(t, algo, bf16)
                c.join()
                torch.cuda.synchronize()
                results.append((algo, bf16, n, c.error(), torch.equal(t, want),
                                (t - want).abs().max().item()))
    ok = c.validate_p2p()
    dist.barrier()
    c.close()
    q.put(("ok", rank, results, ok))
    dist.destroy_process_group()


def test_p2p_two_processes_one_gpu():
    """Two processes, one GPU: staging mapped through hipIpc handles exchanged over the store."""
    world, port = 2, free_port()
    res = run_ranks(_ipc_worker, world, (world, port), expect=world, timeout=300)
    for _, rank, results, ok in res:
        assert ok, f"rank {rank}: validate_p2p failed"
        for algo, bf16, n, err, eq, maxerr in results:
            assert err == 0, f"rank {rank} {algo} bf16={bf16} n={n}: error word {err}"
            assert eq, f"rank {rank} {algo} bf16={bf16} n={n}: max err {maxerr}"


def _timeout_worker(rank, world, port, q):
    import pgdist  # noqa: F401
    from pgdist.parallel.comm import NativeComm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c = NativeComm.for_process_group(dev, use_rccl=False, p2p_bytes=1 << 16, blocks=2, timeout_s=1.0)
    err = 0
    if rank == 0:   # rank 1 never joins this collective
        t = torch.ones(1024, device=dev)
        c.allreduce(t, "oneshot")
        c.join()
        torch.cuda.synchronize()
        err = c.error()
    dist.barrier()
    c.close()
    q.put(("ok", rank, err))
    dist.destroy_process_group()


def test_p2p_missing_peer_times_out_instead_of_hanging():
    world, port = 2, free_port()
    res = dict((r, e) for _, r, e in run_ranks(_timeout_worker, world, (world, port), expect=world, timeout=200))
    assert res[0] & 1, "the barrier timeout bit must be set on the rank left waiting"
    assert res[1] == 0


def _mixed_worker(rank, world, port, q):
    """one communicator, per-bucket one-shot / two-shot all-reduces of different sizes
    (fp32 and bf16 wire) interleaved with P2P broadcasts, back to back with NO host sync in
    between (the even/odd staging halves and the two-shot region are reused across kernels),
    for several 'steps'; every result checked afterwards."""
    import pgdist  # noqa: F401
    from pgdist.parallel.comm import NativeComm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c = NativeComm.for_process_group(dev, use_rccl=False, p2p_bytes=1 << 22, blocks=16, timeout_s=10.0)
    plan = [("broadcast", 4096 + 4, False), ("oneshot", 424976, False), ("twoshot", 393216 + 8, False),
            ("oneshot", 8, True), ("twoshot", 1 << 20, True), ("broadcast", 136, False), ("twoshot", 65536, False)]
    checks = []
    for stp in range(4):
        for k, (algo, n, bf16) in enumerate(plan):
            xs = [torch.randn(n, device=dev, generator=torch.Generator(device=dev).manual_seed(7919 * stp + 97 * k + p))
                  for p in range(world)]
            t = xs[rank].clone()
            if algo == "broadcast":
                root = (stp + k) % world
                c.broadcast(t, root, "oneshot")
                want = xs[root]
            else:
                c.allreduce(t, algo, bf16)
                want = _expect(xs, bf16)
            checks.append((stp, algo, n, bf16, t, want))
    c.join()
    torch.cuda.synchronize()
    err = c.error()
    bad = [(s_, a, n, bf) for s_, a, n, bf, t, w in checks if not torch.equal(t, w)]
    dist.barrier()
    c.close()
    q.put(("ok", rank, err, bad))
    dist.destroy_process_group()


def test_p2p_mixed_algorithms_interleaved_two_processes():
    world, port = 2, free_port()
    for _, rank, err, bad in run_ranks(_mixed_worker, world, (world, port), expect=world, timeout=300):
        assert err == 0, f"rank {rank}: error word {err}"
        assert not bad, f"rank {rank}: wrong results for {bad}"


def _fault_worker(rank, world, port, mode, q):
    """A data-parallel 'training' sequence (per step: BN-buffer broadcast + 3 gradient buckets of
    different sizes and algorithms) where rank 1 misbehaves at step 2: ``skip`` (issues none of
    that step's collectives) or ``size`` (all-reduces a bucket of the wrong size).  Every rank
    then runs the collective health check, which must raise on EVERY rank (within the timeout,
    no hang), and the poisoned communicator must refuse later collectives."""
    import time
    import pgdist  # noqa: F401
    from pgdist.parallel.comm import CommError, NativeComm
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    c = NativeComm.for_process_group(dev, use_rccl=False, p2p_bytes=1 << 22, blocks=8, timeout_s=3.0)
    bn = torch.zeros(1024, device=dev)
    grads = [torch.ones(n, device=dev) for n in (65536, 262144, 4096)]
    t0 = time.time()
    for stp in range(5):
        if mode == "skip" and rank == 1 and stp == 2:
            continue
        c.broadcast(bn, 0, "oneshot")
        for k, g in enumerate(grads):
            if mode == "size" and rank == 1 and stp == 2 and k == 1:
                c.allreduce(g[:131072], "twoshot")
            else:
                c.allreduce(g, "oneshot" if k != 1 else "twoshot")
    c.join()
    torch.cuda.synchronize()
    raised, msg = False, ""
    try:
        c.check_all()
    except CommError as e:
        raised, msg = True, str(e)
    refused = False
    try:
        c.allreduce(grads[0], "oneshot")
    except Exception:   # noqa: BLE001 - the poisoned communicator refuses
        refused = True
    elapsed = time.time() - t0
    dist.barrier()
    c.close()
    q.put(("ok", rank, raised, msg, refused, elapsed))
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["skip", "size"])
def test_p2p_out_of_step_rank_fails_every_rank(mode):
    world, port = 2, free_port()
    res = run_ranks(_fault_worker, world, (world, port, mode), expect=world, timeout=300)
    for _, rank, raised, msg, refused, elapsed in res:
        assert raised, f"rank {rank}: the health check did not raise ({mode})"
        assert "native communicator failed" in msg
        assert elapsed < 60, f"rank {rank}: detection took {elapsed:.1f} s"
    # every rank's communicator is poisoned: later collectives are refused
    assert all(refused for *_, refused, _ in res)


def test_rccl_world1_collectives_and_join(dev):
    from pgdist.ops._lib import lib
    from pgdist.parallel.comm import NativeComm
    if not lib().rccl_available():
        pytest.fail("RCCL is not loadable in this process")
    c = NativeComm(0, 1, dev, use_rccl=True)
    try:
        assert c.has_rccl
        x = torch.randn(1 << 20, device=dev)
        ref = x.clone()
        # producer on the current stream, collective on the comm stream, consumer after join
        x.mul_(2.0)
        c.allreduce(x, "rccl")
        c.join()
        y = x + 1.0
        m = torch.tensor([1.5, 2.5], dtype=torch.float64, device=dev)
        c.allreduce_f64(m)
        c.broadcast(x, 0, "rccl")
        c.join()
        torch.cuda.synchronize()
        assert c.error() == 0
        assert torch.equal(x, ref * 2.0)
        assert torch.equal(y, ref * 2.0 + 1.0)
        assert m.tolist() == [1.5, 2.5]
        us = c.time_allreduce(x, "rccl", iters=5)
        assert us > 0
    finally:
        c.close()
