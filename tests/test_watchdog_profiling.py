"""Failure detection (watchdog, heartbeats) and step timing — CPU tests."""
import os
import socket
import threading
import time

import torch
import torch.distributed as dist

import pgdist  # noqa: F401
from pgdist.parallel.watchdog import Watchdog
from pgdist.utils.profiling import StepTimer, trace_range


def test_watchdog_fires_on_stall_and_not_while_kicked():
    fired = []
    wd = Watchdog(0.4, rank=3, world=4, on_timeout=fired.append, poll_s=0.05).start()
    for _ in range(10):          # steady progress: no alarm
        time.sleep(0.05)
        wd.kick(phase="train")
    assert not fired
    time.sleep(1.0)              # stall
    assert fired and "rank 3/4" in fired[0] and "phase 'train'" in fired[0]
    assert wd.fired
    wd.stop()


def test_watchdog_disabled_with_zero_timeout():
    wd = Watchdog(0.0).start()
    assert wd._thread is None
    wd.stop()


def test_heartbeat_stale_ranks_via_store():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    store = dist.TCPStore("127.0.0.1", port, 2, True, wait_for_workers=False)
    w0 = Watchdog(0.3, rank=0, world=2, store=store, on_timeout=lambda m: None)
    w1 = Watchdog(0.3, rank=1, world=2, store=store, on_timeout=lambda m: None)
    w0.kick(), w1.kick()
    assert w0.stale_ranks() == []
    for _ in range(8):           # rank 0 keeps beating, rank 1 is silent
        time.sleep(0.1)
        w0.kick()
        stale = w0.stale_ranks()
    assert stale == [1]


def test_step_timer_cpu():
    t = StepTimer(images_per_step=128, warmup=1, device=torch.device("cpu"))
    for _ in range(4):
        t.start()
        time.sleep(0.01)
        t.stop()
    s = t.summary()
    assert s["steps"] == 3 and 5 < s["mean_ms"] < 100 and s["img_per_s"] > 0
    with trace_range("noop"):    # no GPU: a no-op
        pass
