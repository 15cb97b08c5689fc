"""Per-phase wall clock of the 1x1 weight gradient (pw_wgrad_kernel, csrc/kernels/pwconv.hip) on
MobileNetV2 shapes.  It runs on the side stream at 1.3 TB/s (profiles/r5_roofline_mnv2.txt).
Needs a diagnostics build:

    PGDIST_DEFINES=PGDIST_PWT_TRACE python -c "import __graft_entry__ as g; g.build()"
    python scripts/pwg_phases.py [--out FILE]

Per shape: event time of the kernel plus its split reduction (20 launches), then one traced
launch.  Thread 0 of every workgroup stamps: start (0), parameters staged (1), first tile in LDS
(2), k loop done (3), partial stored (4).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import pgdist  # noqa: E402,F401
from pgdist.ops import kernels as K  # noqa: E402

# (label, M, N = conv Cout, K = conv Cin, x prologue)
SHAPES = [
    ("14x14 expand 64->384", 25088, 384, 64, "none"),
    ("14x14 project 384->64", 25088, 64, 384, "relu6"),
    ("14x14 project 576->96", 25088, 96, 576, "relu6"),
    ("7x7 expand 160->960", 6272, 960, 160, "none"),
    ("7x7 project 960->160", 6272, 160, 960, "relu6"),
    ("28x28 expand 32->192", 100352, 192, 32, "none"),
    ("56x56 project 144->24", 401408, 24, 144, "relu6"),
]
PHASES = ["params", "first tile", "k loop", "partial store"]


def q(v, f):
    v = sorted(v)
    return v[min(len(v) - 1, int(f * len(v)))]


def run(label, M, N, Kd, xp, dev, out):
    g = torch.Generator(device="cpu").manual_seed(0)
    r = lambda *s: torch.randn(*s, generator=g).to(dev)  # noqa: E731
    bf = torch.bfloat16
    G, Y, X = r(M, N).to(bf), r(M, N).to(bf), r(M, Kd).to(bf)
    ga, gb, gc = torch.rand(N, device=dev) + 0.5, torch.rand(N, device=dev) - 0.5, torch.rand(N, device=dev) - 0.5
    xs, xt = torch.rand(Kd, device=dev) + 0.5, torch.rand(Kd, device=dev) - 0.5
    ws = torch.zeros(K.pw_wgrad_workspace(M, N, Kd), device=dev)
    grad = torch.empty(N * Kd, device=dev)
    act = K.ACT_BN_RELU6 if xp == "relu6" else K.ACT_NONE

    def launch():
        K.pw_wgrad(G, Y, ga, gb, gc, X, xs, xt, act, ws, grad, M, N, Kd)

    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(20):
        e0.record()
        launch()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    buf = torch.zeros(65536 * 8, dtype=torch.int64, device=dev)
    K.pwg_trace_set(buf)
    launch()
    torch.cuda.synchronize()
    K.pwg_trace_set(None)
    t = buf.view(-1, 8).cpu()
    t = t[t[:, 0] != 0].double() / 100.0
    n = t.shape[0]
    if n == 0:
        print(f"{label}: no trace (build with PGDIST_DEFINES=PGDIST_PWT_TRACE)", file=out)
        return
    t0 = t[:, 0].min()
    span = (t[:, 4].max() - t0).item()
    starts = (t[:, 0] - t0).tolist()
    mb = (2 * M * N + M * Kd) * 2 / 1e6
    print(f"{label}: M={M} N={N} K={Kd}  event (+reduce) p50 {q(ts, .5):.1f} us  workgroups {n}  "
          f"kernel span {span:.1f} us ({mb / span:.2f} TB/s of operands)  start spread p50/max "
          f"{q(starts, .5):.1f}/{max(starts):.1f} us", file=out)
    life = (t[:, 4] - t[:, 0]).tolist()
    print(f"    workgroup lifetime p50/p90 {q(life, .5):.2f}/{q(life, .9):.2f} us", file=out)
    for i, ph in enumerate(PHASES):
        d = (t[:, i + 1] - t[:, i]).tolist()
        print(f"    {ph:14s} p50 {q(d, .5):6.2f}  p90 {q(d, .9):6.2f} us", file=out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = open(a.out, "w") if a.out else sys.stdout
    for s in SHAPES:
        run(*s, dev, out)
        out.flush()


if __name__ == "__main__":
    main()
