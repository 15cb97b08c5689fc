"""Failure handling of the native communicator on the RCCL path.

* a collective that has started on the comm stream but does not complete (a dead peer inside an
  RCCL kernel, emulated by a bounded spin kernel injected between the collective's start marker
  and the collective) makes the watchdog print the stalled collective, abort the RCCL
  communicator and end the process with status 75 -- within the deadline, instead of hanging;
* the same inside a training step: the stall hits the first gradient bucket (RCCL algorithm) of a
  replayed step;
* a poisoned communicator (error word set) makes the fused Adam skip its update, so un-reduced
  gradients never change the weights, and the trainer's per-step poll sees the error.
Each fault runs in its own subprocess (the watchdog ends that process).  Reference: the DDP
gradient all-reduce, cifar10_mpi_mobilenet_224.py:142-145,179; SURVEY.md §5.3.
"""
import os
import subprocess
import sys
import textwrap
import time

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code, timeout=120):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    t0 = time.time()
    r = subprocess.run([sys.executable, "-u", "-c", textwrap.dedent(code)], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=timeout)
    return r, time.time() - t0


def test_watchdog_aborts_a_stalled_rccl_collective():
    r, dt = _run("""
        import sys, time, torch
        sys.path.insert(0, '.')
        import pgdist
        from pgdist.parallel.comm import NativeComm
        dev = torch.device('cuda', 0)
        comm = NativeComm(0, 1, dev, use_rccl=True, watchdog_s=1.0)
        assert comm.has_rccl and abs(comm.watchdog_s - 1.0) < 1e-9
        t = torch.ones(4096, device=dev)
        comm.allreduce(t, 'rccl'); comm.join(); torch.cuda.synchronize()   # healthy call passes
        print('healthy', flush=True)
        comm.inject_stall(8.0)
        comm.allreduce(t, 'rccl'); comm.join()
        t0 = time.time()
        torch.cuda.synchronize()
        print('NOT ABORTED after', time.time() - t0, flush=True)
    """)
    assert "healthy" in r.stdout, r.stderr[-2000:]
    assert r.returncode == 75, (r.returncode, r.stdout[-1000:], r.stderr[-2000:])
    assert "comm watchdog" in r.stderr and "RCCL all-reduce of 4096 floats" in r.stderr
    assert "NOT ABORTED" not in r.stdout
    assert dt < 60


def test_training_step_with_a_stalled_rccl_bucket_exits_nonzero():
    r, dt = _run("""
        import sys, torch
        sys.path.insert(0, '.')
        import pgdist
        from pgdist.engine.native_step import NativeTrainStep
        from pgdist.models import mobilenet_v2
        dev = torch.device('cuda', 0)
        torch.manual_seed(0)
        st = NativeTrainStep(mobilenet_v2(10), 16, dev, img_size=96, force_ddp=True, allreduce_algo='rccl',
                             comm='rccl', use_graph=False)
        src = torch.randint(0, 256, (64, 32, 32, 3), dtype=torch.uint8, device=dev)
        st.set_data(src, torch.randint(0, 10, (64,), device=dev))
        st.comm.set_watchdog(1.5)
        for i in range(4):   # eager warm-up, recorded, replayed
            st.run(torch.arange(16, device=dev))
        torch.cuda.synchronize()
        assert st.comm.error() == 0
        print('steps ok', flush=True)
        st.comm.inject_stall(10.0)   # the first gradient bucket of the next (replayed) step
        st.run(torch.arange(16, device=dev))
        torch.cuda.synchronize()
        print('NOT ABORTED', flush=True)
    """, timeout=240)
    assert "steps ok" in r.stdout, r.stderr[-3000:]
    assert r.returncode == 75, (r.returncode, r.stdout[-1000:], r.stderr[-3000:])
    assert "comm watchdog" in r.stderr and "RCCL all-reduce" in r.stderr
    assert "NOT ABORTED" not in r.stdout


def test_poisoned_communicator_skips_the_optimizer_update():
    import pgdist  # noqa: F401
    from pgdist.engine.native_step import NativeTrainStep
    from pgdist.ops._lib import lib
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    from pgdist.models import mobilenet_v2
    st = NativeTrainStep(mobilenet_v2(10), 16, dev, img_size=96, force_ddp=True, allreduce_algo="rccl",
                         comm="rccl", use_graph=False)
    src = torch.randint(0, 256, (64, 32, 32, 3), dtype=torch.uint8, device=dev)
    st.set_data(src, torch.randint(0, 10, (64,), device=dev))
    for _ in range(3):
        st.run(torch.arange(16, device=dev))
    torch.cuda.synchronize()
    assert st.comm.poll_error() == 0
    before = st.flat.master.clone()
    st.run(torch.arange(16, device=dev))
    torch.cuda.synchronize()
    assert not torch.equal(before, st.flat.master), "a healthy step updates the weights"
    lib().comm_poison(st.comm.id, "test: a peer failed")
    st.comm.poll_error()   # enqueue the copy; the next poll returns it
    torch.cuda.synchronize()
    assert st.comm.poll_error() != 0
    frozen = st.flat.master.clone()
    with pytest.raises(RuntimeError, match="poisoned"):
        st.run(torch.arange(16, device=dev))   # the bucket collectives refuse to launch
    torch.cuda.synchronize()
    assert torch.equal(frozen, st.flat.master), "a poisoned step must not change the weights"
    st.comm.close()


def test_adam_skips_while_the_error_word_is_set():
    import pgdist  # noqa: F401
    from pgdist.ops import kernels as K
    dev = torch.device("cuda", 0)
    n = 4096
    g = torch.Generator(device=dev).manual_seed(3)
    p = torch.randn(n, device=dev, generator=g)
    grad = torch.randn(n, device=dev, generator=g)
    m, v = torch.zeros_like(p), torch.zeros_like(p)
    pb = torch.zeros(n, dtype=torch.bfloat16, device=dev)
    hyper = torch.tensor([1e-3, 1.0], device=dev)
    word = torch.ones(4, dtype=torch.int32, device=dev)
    p0 = p.clone()
    K.adam_flat(p, grad, m, v, pb, hyper, 0.9, 0.999, 1e-8, skip=word.data_ptr())
    torch.cuda.synchronize()
    assert torch.equal(p, p0) and not m.any()
    word.zero_()
    K.adam_flat(p, grad, m, v, pb, hyper, 0.9, 0.999, 1e-8, skip=word.data_ptr())
    torch.cuda.synchronize()
    assert not torch.equal(p, p0) and m.any()


def test_poison_only_watchdog_then_error_and_close():
    """exit_status=0 (poison + abort only): after the stall fires the communicator's
    RCCL handle is gone, so comm_error and close() must neither use the aborted communicator
    nor wait for the stalled comm stream."""
    r, dt = _run("""
        import sys, time, torch
        sys.path.insert(0, '.')
        import pgdist
        from pgdist.engine.native_step import NativeTrainStep
        from pgdist.models import mobilenet_v2
        dev = torch.device('cuda', 0)
        torch.manual_seed(0)
        st = NativeTrainStep(mobilenet_v2(10), 16, dev, img_size=96, force_ddp=True, allreduce_algo='rccl',
                             comm='rccl', use_graph=False)
        src = torch.randint(0, 256, (64, 32, 32, 3), dtype=torch.uint8, device=dev)
        st.set_data(src, torch.randint(0, 10, (64,), device=dev))
        st.comm.set_watchdog(1.0, exit_status=0)
        for i in range(3):
            st.run(torch.arange(16, device=dev))
        torch.cuda.synchronize()
        assert st.comm.error() == 0
        st.comm.inject_stall(4.0)
        st.run(torch.arange(16, device=dev))
        torch.cuda.synchronize()   # the stall kernel ends; the aborted collective does not hang
        err = st.comm.error()
        assert err != 0, err
        assert st.comm.rccl_ranks() == 0, 'the aborted RCCL handle must be dropped'
        print('error', hex(err), st.comm.error_string()[:60], flush=True)
        t0 = time.time()
        st.comm.close()
        print('closed in %.1f s' % (time.time() - t0), flush=True)
    """, timeout=180)
    assert "comm watchdog" in r.stderr, (r.returncode, r.stdout[-1000:], r.stderr[-3000:])
    assert r.returncode == 0, (r.returncode, r.stdout[-1000:], r.stderr[-3000:])
    assert "closed in" in r.stdout
    assert dt < 150
