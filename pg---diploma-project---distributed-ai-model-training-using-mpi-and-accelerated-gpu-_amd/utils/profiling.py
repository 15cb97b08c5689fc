"""Tracing and step timing.

The reference only measures wall-clock epoch time with ``time.time()``
(``cifar10_serial_mobilenet_224.py:88,132``), including eval and data loading.
Here:

* :func:`trace_range` — named ranges that show up in rocprofv3 traces
  (``torch.cuda.nvtx`` is backed by roctx on ROCm builds); a no-op on CPU or
  when disabled.
* :class:`StepTimer` — per-step device time from HIP events (no host sync per
  step: events are resolved lazily), with warm-up exclusion, mean / p50 / p90
  and images/sec.
"""
import contextlib
import statistics
from typing import List, Optional

import torch


@contextlib.contextmanager
def trace_range(name: str, enabled: bool = True):
    """roctx range around a region (rocprofv3 ``--marker-trace`` shows it)."""
    on = enabled and torch.cuda.is_available()
    if on:
        try:
            torch.cuda.nvtx.range_push(name)
        except Exception:   # roctx not available in this build
            on = False
    try:
        yield
    finally:
        if on:
            torch.cuda.nvtx.range_pop()


class StepTimer:
    """Device-side step timing with HIP events.

    ``start()`` / ``stop()`` bracket one step on the current stream; ``summary()``
    synchronises once and reports statistics over the steps after ``warmup``.
    On CPU it falls back to ``time.perf_counter``.
    """

    def __init__(self, images_per_step: int, warmup: int = 2, device: Optional[torch.device] = None):
        self.images = images_per_step
        self.warmup = warmup
        self.cuda = torch.cuda.is_available() and (device is None or device.type == "cuda")
        self._pairs: List = []
        self._t0 = None

    def start(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._t0 = e
        else:
            import time
            self._t0 = time.perf_counter()

    def stop(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self._pairs.append((self._t0, e))
        else:
            import time
            self._pairs.append((self._t0, time.perf_counter()))

    def times_ms(self) -> List[float]:
        if self.cuda:
            if self._pairs:
                self._pairs[-1][1].synchronize()
            return [a.elapsed_time(b) for a, b in self._pairs]
        return [(b - a) * 1e3 for a, b in self._pairs]

    def summary(self) -> dict:
        t = self.times_ms()[self.warmup:]
        if not t:
            return {"steps": 0}
        ts = sorted(t)
        mean = statistics.fmean(t)
        return {"steps": len(t), "mean_ms": mean, "p50_ms": ts[len(ts) // 2],
                "p90_ms": ts[min(len(ts) - 1, int(0.9 * len(ts)))], "img_per_s": self.images / mean * 1e3}

    def reset(self):
        self._pairs = []
