#!/usr/bin/env python3
"""Per-op roofline of the native training step (MobileNetV2 bs128 224^2 by default).

The step is recorded as a launch plan with the kernel-wrapper launch log on
(ops/kernels.py launch_log_start): every wrapper call gives its op range in the plan, the
bytes of its tensor operands (activations, gradients, weights: the op's compulsory HBM
traffic, workspaces excluded) and its shape arguments.  Each range is then re-run in
isolation (lib().plan_time_ops: device synchronised around N back-to-back repetitions), so
the table gives isolated time, compulsory bytes and achieved TB/s per op, next to the
replayed step's own time (both streams overlapped).

usage: python scripts/roofline.py [--model mobilenet_v2] [--batch 128] [--iters 20] [--out FILE]
"""
import argparse
import os
import sys
import time
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import pgdist  # noqa: E402,F401
from pgdist.engine.native_step import NativeTrainStep  # noqa: E402
from pgdist.ops import kernels as K  # noqa: E402
from pgdist.ops._lib import lib  # noqa: E402

HBM_TBS = 6.3   # achievable HBM bandwidth (float4 copy, MI355X_MICROARCH.md)


def shape_str(d):
    keys = [k for k in ("M", "N", "K", "Kg", "Ng", "B", "H", "W", "C", "stride", "n", "HW", "Ci", "R", "S")
            if k in d]
    return " ".join(f"{k}={d[k]}" for k in keys)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mobilenet_v2")
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--fp8", type=int, default=0)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    st = NativeTrainStep.for_benchmark(a.model, a.batch, dev, use_graph=False, fp8=bool(a.fp8))
    assert st.use_plan, "the roofline needs the launch-plan path"
    for _ in range(2):
        st.bench_step()
    K.launch_log_start()
    st.bench_step()           # third step: recorded into the plan
    log = K.launch_log_stop()
    assert st.plan is not None
    torch.cuda.synchronize()
    for _ in range(5):
        st.bench_step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n = 30
    for _ in range(n):
        st.bench_step()
    torch.cuda.synchronize()
    step_us = (time.perf_counter() - t0) / n * 1e6
    main_stream = torch.cuda.current_stream(dev).cuda_stream
    times = lib().plan_time_ops(st.plan.id, [(e["first"], e["last"]) for e in log], a.iters)
    rows = []
    for e, t in zip(log, times):
        rows.append(dict(op=e["op"], shape=shape_str(e["shape"]), stream="main" if e["stream"] == main_stream else "side",
                         us=t, mb=e["bytes"] / 1e6, tbs=e["bytes"] / (t * 1e-6) / 1e12 if t > 0 else 0.0))
    lines = [f"# {a.model} bs{a.batch}{' fp8' if a.fp8 else ''}: replayed step {step_us:.1f} us "
             f"({a.batch / step_us * 1e6:.0f} img/s); {len(rows)} ops",
             "# isolated = op range re-run alone (N back-to-back, device-synchronised); MB = its operands' bytes "
             "(compulsory traffic, workspaces excluded); floor = MB at 6.3 TB/s",
             f"{'#':>3} {'stream':<5} {'op':<18} {'isolated_us':>11} {'MB':>8} {'TB/s':>6} {'floor_us':>8}  shape"]
    for i, r in enumerate(rows):
        lines.append(f"{i:>3} {r['stream']:<5} {r['op']:<18} {r['us']:>11.1f} {r['mb']:>8.1f} {r['tbs']:>6.2f} "
                     f"{r['mb'] / HBM_TBS:>8.1f}  {r['shape']}")
    fam = defaultdict(lambda: [0, 0.0, 0.0])
    for r in rows:
        f = fam[(r["stream"], r["op"])]
        f[0] += 1
        f[1] += r["us"]
        f[2] += r["mb"]
    lines.append("")
    lines.append(f"{'stream':<5} {'op':<18} {'n':>3} {'isolated_us':>11} {'MB':>9} {'TB/s':>6} {'floor_us':>8} "
                 f"{'excess_us':>9}")
    tot = defaultdict(lambda: [0.0, 0.0])
    for (s, op), (c, us, mb) in sorted(fam.items(), key=lambda kv: -kv[1][1]):
        lines.append(f"{s:<5} {op:<18} {c:>3} {us:>11.1f} {mb:>9.1f} {mb / us if us else 0:>6.2f} "
                     f"{mb / HBM_TBS:>8.1f} {us - mb / HBM_TBS:>9.1f}")
        tot[s][0] += us
        tot[s][1] += mb
    for s, (us, mb) in tot.items():
        lines.append(f"total {s}: isolated {us:.1f} us, {mb:.1f} MB ({mb / us:.2f} TB/s), floor {mb / HBM_TBS:.1f} us")
    out = "\n".join(lines)
    print(out, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(out + "\n")


if __name__ == "__main__":
    main()
