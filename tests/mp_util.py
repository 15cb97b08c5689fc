"""Multi-process test harness: spawn one process per rank, surface a rank's exception with
its traceback, and never leave a child behind (a rank stuck in a collective would otherwise
hold the CPU / GPU for the rest of the session)."""
import queue
import socket
import traceback

import pytest
import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def guarded(body, rank, q, *args):
    """Run a rank's body; any exception is put on the queue with its traceback (so the test
    reports the real failure instead of a queue timeout)."""
    try:
        body(rank, *args, q)
    except BaseException:
        q.put(("error", rank, traceback.format_exc()))
        raise


def run_ranks(body, world, args, expect, timeout=400):
    """Spawn ``world`` ranks of ``body``, collect ``expect`` results, then make sure every
    child is gone (terminate/kill survivors, e.g. a rank stuck in a collective holding the GPU)
    and exited with status 0."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=guarded, args=(body, r, q) + tuple(args)) for r in range(world)]
    for p in procs:
        p.start()
    res = []
    try:
        while len(res) < expect:
            try:
                item = q.get(timeout=timeout)
            except queue.Empty:
                pytest.fail(f"no result from the ranks within {timeout} s "
                            f"(exit codes {[p.exitcode for p in procs]})")
            if item[0] == "error":
                pytest.fail(f"rank {item[1]} raised:\n{item[2]}")
            res.append(item)
        for p in procs:
            p.join(timeout=120)
    finally:
        for p in procs:
            if p.is_alive():
                p.terminate()
                p.join(timeout=10)
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
    assert [p.exitcode for p in procs] == [0] * world
    return res
