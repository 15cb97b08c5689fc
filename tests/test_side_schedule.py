"""Side-stream scheduling of the MobileNetV2 executor's backward (engine/executor.py), on the CPU.

The weight gradients are deferred in groups: one side-stream join per group, the group's lazy
BN finalizes first (one batched launch), its split reductions recorded while the group's
weight-gradient launches run and launched together afterwards, and every DDP bucket launch
preceded by a flush.  The executor needs a GPU to be built, so these tests drive its
scheduling methods on a bare instance with the native ops replaced by a recorder: they pin
the ORDER of the enqueued operations, which is what the stream semantics rely on.
"""
import contextlib

import pytest
import torch

import pgdist  # noqa: F401
from pgdist.engine import executor as X


class Rec:
    """Stands in for ops.kernels: records the calls the scheduling code makes."""

    def __init__(self):
        self.log = []

    def stream_wait(self, waiter, signaler):
        self.log.append(("wait", waiter, signaler))

    def wgrad_reduce_defer(self, on):
        self.log.append(("defer", bool(on)))

    def wgrad_reduce_flush(self):
        self.log.append(("flush_reduce",))

    def bn_desc_table(self, descs):
        return ("tab", tuple(descs))

    def bn_finalize_batch(self, tab, n, max_c):
        self.log.append(("fin_batch", n, max_c))

    def bn_rows(self, P):
        return min(int(P), 8)

    def plan_py(self, fn):
        fn()


class FakeStream:
    def __init__(self, rec):
        self.rec = rec

    def wait_stream(self, other):
        self.rec.log.append(("join", other))

    def __repr__(self):
        return "side"


class FakeBN:
    def __init__(self, name, C, rows_b=8):
        self.prefix, self.C, self.rows_b = name, C, rows_b
        self.desc_b = "desc_" + name
        self.acc_b = None
        self.finalized = []

    def finalize_bwd(self, part, P, force=False):
        self.finalized.append((P, force))


@pytest.fixture
def exe(monkeypatch):
    rec = Rec()
    monkeypatch.setattr(X, "K", rec)
    monkeypatch.setattr(torch.cuda, "stream", lambda s: contextlib.nullcontext())
    monkeypatch.setattr(torch.cuda, "current_stream", lambda device=None: "main")
    e = object.__new__(X.MobileNetV2Executor)
    e.side = FakeStream(rec)
    e.device = None
    e.side_batch = 3
    e.batch_reductions = True
    e.lazy_bn = True
    e._side_pending = []
    e._fin_tabs = {}
    e.ws_wgrad = "ws0"
    e.ws_wgrad_pool = ["ws0", "ws1", "ws2"]
    e.on_params_ready = None
    e.ready_probe = None
    e.rec = rec
    return e


def wg(exe, tag):
    """A weight-gradient callable that logs its launch and the workspace it got."""
    return lambda ws: exe.rec.log.append(("wgrad", tag, ws))


def test_group_of_three_one_join(exe):
    a, b, c = FakeBN("a", 16), FakeBN("b", 96), FakeBN("c", 24)
    exe._wgrad(wg(exe, 1), fins=((a, 5),))
    exe._wgrad(wg(exe, 2), fins=((b, 7),))
    assert exe.rec.log == []                      # deferred until the group is full
    exe._wgrad(wg(exe, 3), fins=((c, 3),))
    log = exe.rec.log
    assert log[0][0] == "wait" and log[0][1] is exe.side and log[0][2] == "main"   # ONE join for the group
    assert log[1] == ("fin_batch", 3, 96)         # the group's finalizes, batched, before any wgrad
    assert log[2] == ("defer", True)
    assert [x for x in log if x[0] == "wgrad"] == [("wgrad", 1, "ws0"), ("wgrad", 2, "ws1"), ("wgrad", 3, "ws2")]
    assert log[-2:] == [("defer", False), ("flush_reduce",)]
    assert sum(1 for x in log if x[0] == "wait") == 1
    assert exe._side_pending == []


def test_single_finalize_is_a_plain_launch_and_tables_are_cached(exe):
    a = FakeBN("a", 16)
    exe._wgrad(wg(exe, 1), fins=((a, 5),))
    exe._flush_side()
    assert a.finalized == [(5, True)]
    assert not any(x[0] == "fin_batch" for x in exe.rec.log)
    b, c = FakeBN("b", 32), FakeBN("c", 64)
    for _ in range(2):
        exe._wgrad(wg(exe, 2), fins=((b, 1), (c, 2)))
        exe._flush_side()
    assert len(exe._fin_tabs) == 1                # same BN group -> one cached table


def test_bucket_launch_flushes_pending_work_first(exe):
    ready = []
    exe.on_params_ready = lambda names: ready.append((list(names), len(exe.rec.log)))
    exe.ready_probe = lambda names: names == ["launches"]
    exe._wgrad(wg(exe, 1), fins=((FakeBN("a", 8), 2),))
    exe._ready(["quiet"])                         # no bucket: nothing flushed
    assert not any(x[0] == "wgrad" for x in exe.rec.log)
    exe._ready(["launches"])                      # a bucket launch: the pending group runs first
    (names, at), = [r for r in ready if r[0] == ["launches"]]
    launched = [x for x in exe.rec.log[:at] if x[0] == "wgrad"]
    assert launched == [("wgrad", 1, "ws0")]


def test_no_side_stream_runs_inline(exe):
    exe.side = None
    a = FakeBN("a", 16)
    exe._wgrad(wg(exe, 1), fins=((a, 4),))
    assert a.finalized == [(4, True)]
    assert exe.rec.log == [("wgrad", 1, "ws0")]


def test_launch_mode_skips_side_finalizes(exe):
    exe.lazy_bn = False
    a = FakeBN("a", 16)
    exe._wgrad(wg(exe, 1), fins=((a, 4),))
    exe._flush_side()
    assert a.finalized == []
    assert not any(x[0] == "fin_batch" for x in exe.rec.log)


def test_rows_beyond_the_accumulator_are_rejected(exe):
    a = FakeBN("a", 16, rows_b=2)
    exe._wgrad(wg(exe, 1), fins=((a, 5),))
    with pytest.raises(AssertionError):
        exe._flush_side()
