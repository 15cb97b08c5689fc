"""Host-side cost of enqueuing one replayed training step (no profiler): the step function is
timed from an idle GPU (synchronised before each call) until it returns, i.e. the time the
launch-plan replay spends submitting the step's ~270 operations, against the GPU time of the
step.  Host time close to the GPU time means stretches of the step are submission-bound.

    python scripts/host_cost.py [--model mobilenet_v2] [--batch-size 128] [--steps 20]
"""
import argparse
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pgdist  # noqa: E402,F401


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mobilenet_v2")
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--steps", type=int, default=20)
    a = ap.parse_args()
    from pgdist.engine.bench_step import build_bench_step
    dev = torch.device("cuda", 0)
    step, meta = build_bench_step(a.model, a.batch_size, dev, use_graph=0)
    for _ in range(10):
        step()
    torch.cuda.synchronize()
    host = []
    for _ in range(a.steps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step()
        host.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps):
        step()
    e1.record()
    torch.cuda.synchronize()
    print(f"host enqueue per step: median {statistics.median(host):.3f} ms (min {min(host):.3f}); "
          f"GPU step {e0.elapsed_time(e1) / a.steps:.3f} ms")


if __name__ == "__main__":
    main()
