"""Diagnostic bound on what the side stream costs the MobileNetV2 step (not a benchmark).

    python scripts/side_bound.py --mode base|nowgrad|serial [--steps 20]

base     the bench step (weight gradients on the side stream, overlapped)
nowgrad  weight-gradient launches skipped (INVALID as a training step: the lower bound of a
         step whose side-stream work were free)
serial   no side stream: every weight gradient on the main stream (the no-overlap sum)
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pgdist  # noqa: E402,F401


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="base", choices=("base", "nowgrad", "serial"))
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch-size", type=int, default=128)
    a = ap.parse_args()
    from pgdist.engine.executor import MobileNetV2Executor
    from pgdist.engine.bench_step import build_bench_step
    if a.mode == "nowgrad":
        MobileNetV2Executor._wgrad = lambda self, fn, fins=(): None
    dev = torch.device("cuda", 0)
    step, meta = build_bench_step("mobilenet_v2", a.batch_size, dev, use_graph=0, side_stream=a.mode != "serial")
    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.steps):
        step()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"mode": a.mode, "ms_per_step": round(e0.elapsed_time(e1) / a.steps, 3)}))


if __name__ == "__main__":
    main()
