"""NativeBucketReducer bookkeeping on the CPU (parallel/ddp.py): bucket alignment for the P2P
kernels, the launch order / arguments handed to the communicator and the final join.  The
communicator is a recorder (the real one is exercised on the GPU: tests/test_comm_gpu.py,
tests/test_ddp_gpu.py)."""
import torch

import pgdist  # noqa: F401
from pgdist.parallel.ddp import NativeBucketReducer


class FakeComm:
    def __init__(self, world=2, rccl=True, p2p=True):
        self.world, self.has_rccl, self.has_p2p, self.region = world, rccl, p2p, 1 << 20
        self.log = []
        self.tuned = None
        self.p2p_error = None

    def validate_p2p(self):
        self.log.append(("validate",))
        return self.has_p2p

    def autotune(self, sizes, bf16_wire=False, iters=10, measure=False):
        self.tuned = list(sizes)
        # latency-dominated model: 20 us per call + 1 us per 64 KiB
        self.tuning = {s: {"rccl": 20.0 + s * 4 / 65536, "oneshot": 30.0 + s * 4 / 16384} for s in sizes}
        return {s: ("oneshot" if s * 4 <= 64 * 1024 else "rccl") for s in sizes}

    def allreduce(self, t, algo, bf16, wait=()):
        self.log.append(("ar", t.data_ptr(), t.numel(), algo, bf16))

    def join(self, stream=None):
        self.log.append(("join",))


class _FakeStreamModule:
    class S:
        cuda_stream = 1

    @staticmethod
    def current_stream(dev=None):
        return _FakeStreamModule.S()


def _ranges():
    out, o = [], 0
    for i in range(30):
        n = 100 * (1 + i % 5) + (i % 3)          # not multiples of 8
        out.append((f"p{i}", o, o + n))
        o = (o + n + 63) // 64 * 64              # FlatParams: 64-element aligned starts
    return out, (o + 63) // 64 * 64


def test_buckets_are_64_aligned_and_cover_the_buffer(monkeypatch):
    monkeypatch.setattr(torch.cuda, "current_stream", _FakeStreamModule.current_stream)
    ranges, n = _ranges()
    comm = FakeComm()
    red = NativeBucketReducer(comm, torch.zeros(n), ranges, bucket_cap_mb=0.01, first_bucket_mb=0.002)
    assert ("validate",) in comm.log
    assert len(red.buckets) > 3
    prev = 0
    for s, e, _ in red.buckets:
        assert s == prev and s % 64 == 0 and (e % 64 == 0 or e == n) and (e - s) % 8 == 0
        prev = e
    assert prev == n
    assert comm.tuned == [e - s for s, e, _ in red.buckets]
    assert red.algos == ["oneshot" if (e - s) * 4 <= 64 * 1024 else "rccl" for s, e, _ in red.buckets]


def test_launch_order_slices_and_join(monkeypatch):
    monkeypatch.setattr(torch.cuda, "current_stream", _FakeStreamModule.current_stream)
    ranges, n = _ranges()
    comm = FakeComm()
    g = torch.zeros(n)
    red = NativeBucketReducer(comm, g, ranges, bucket_cap_mb=0.01, first_bucket_mb=0.002, algo="twoshot")
    comm.log.clear()
    red.begin()
    for name, _, _ in reversed(ranges):   # backward completion order is the buffer order reversed here
        red.mark_ready([name])
    red.finish()
    ars = [x for x in comm.log if x[0] == "ar"]
    assert len(ars) == len(red.buckets)
    for (tag, ptr, numel, algo, bf), (s, e, _) in zip(ars, red.buckets):
        assert ptr == g[s:].data_ptr() and numel == e - s and algo == "twoshot" and not bf
    assert comm.log[-1] == ("join",)


def test_world1_reducer_only_runs_when_forced(monkeypatch):
    monkeypatch.setattr(torch.cuda, "current_stream", _FakeStreamModule.current_stream)
    ranges, n = _ranges()
    comm = FakeComm(world=1, p2p=False)
    red = NativeBucketReducer(comm, torch.zeros(n), ranges, algo="rccl")
    assert not red.enabled
    red.finish()
    assert comm.log == []
    red = NativeBucketReducer(comm, torch.zeros(n), ranges, algo="rccl", force=True)
    assert red.enabled
    red.begin()
    red.mark_ready([r[0] for r in ranges])
    red.finish()
    assert [x[0] for x in comm.log] == ["ar"] * len(red.buckets) + ["join"]


def test_bucket_layout_minimises_simulated_exposed_time(monkeypatch):
    """bucket_cap_mb=None: every (cap, last-bucket cap) layout is scored by the simulated exposed
    communication (parallel/ddp.py simulate_buckets) from the measured all-reduce times and the
    gradients' ready times; the cheapest wins and the buckets still tile the buffer."""
    monkeypatch.setattr(torch.cuda, "current_stream", _FakeStreamModule.current_stream)
    big, o = [], 0
    for i in range(30):                                                # ~ 1.7e7 elements (~66 MB)
        n_i = 200000 * (1 + i % 5) + (i % 3)
        big.append((f"p{i}", o, o + n_i))
        o = (o + n_i + 63) // 64 * 64
    n = o
    comm = FakeComm()
    red = NativeBucketReducer(comm, torch.zeros(n), big, bucket_cap_mb=None, first_bucket_mb=1.0)
    assert red.bucket_tuning and len(red.bucket_tuning) >= 8
    key = f"{red.bucket_cap_mb}/{red.last_bucket_mb}"
    assert red.bucket_tuning[key] == min(red.bucket_tuning.values())
    prev = 0
    for s, e, _ in red.buckets:
        assert s == prev and s % 64 == 0
        prev = e
    assert prev == n


def _mnv2_ranges():
    from pgdist.engine.flat import FlatParams
    from pgdist.models import mobilenet_v2
    torch.manual_seed(0)
    model = mobilenet_v2(10)
    flat = FlatParams(model, torch.device("cpu"))
    return model, flat, [(nm,) + flat.range_of(nm) for nm in flat.order]


def test_mobilenet_layout_overlaps_the_backward():
    """with a latency-dominated all-reduce (25 us + 60 GB/s) and a 3 ms backward
    whose gradients become ready as the MobileNetV2 backward visits its layers, the chosen
    layout has >= 3 buckets and a last (exposed) bucket <= 1.5 MiB -- the old objective (sum of
    all bucket times + the last) chose 2 buckets, the second holding ~80 % of the gradient and
    ready only at the very end of the backward."""
    from pgdist.parallel.ddp import (build_buckets, candidate_layouts, choose_layout, estimate_ready_times,
                                     simulate_buckets)
    model, flat, ranges = _mnv2_ranges()
    ready = estimate_ready_times(model, 224, 3000.0)
    assert set(ready) == {nm for nm, _, _ in ranges}
    assert ready["classifier.1.weight"] < ready["features.18.0.weight"] < ready["features.0.0.weight"]
    t_ar = lambda n: 25.0 + n * 4 / 60e3   # noqa: E731  (us)
    cands = candidate_layouts(ranges, 1.0, flat.numel * 4 / 2 ** 20)
    cost, key = choose_layout(cands, ready, 3000.0, t_ar)
    best = cands[key]
    assert len(best) >= 3, (key, [(e - s) * 4 / 2 ** 20 for s, e, _ in best])
    s, e, _ = best[-1]
    assert (e - s) * 4 <= 1.5 * 2 ** 20
    # the old objective's pick (8 MiB cap, no tail bucket) exposes more communication
    old = build_buckets(ranges, 8 << 20, 1 << 20)
    assert len(old) == 2
    assert simulate_buckets(old, ready, 3000.0, t_ar) > cost[key] + 50.0


def test_retune_from_measured_ready_times(monkeypatch):
    """A measured ready-time table replaces the model: retune re-chooses the layout and the
    per-bucket algorithms from it (collective on the real communicator)."""
    monkeypatch.setattr(torch.cuda, "current_stream", _FakeStreamModule.current_stream)
    model, flat, ranges = _mnv2_ranges()
    comm = FakeComm()
    red = NativeBucketReducer(comm, torch.zeros(flat.numel), ranges, bucket_cap_mb=None, first_bucket_mb=1.0)
    # everything final only at the end of a 100 us backward: one big bucket is best
    late = {nm: 100.0 for nm, _, _ in ranges}
    red.retune(late, 100.0)
    assert len(red.buckets) <= 2
    assert len(red.algos) == len(red.buckets)
