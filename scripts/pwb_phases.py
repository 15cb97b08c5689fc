"""Per-phase wall clock of the fused large-M pointwise backward (pw_bwd_fused_kernel,
csrc/kernels/pwbwd.hip) on the MobileNetV2 112x112 / 56x56 / 28x28 shapes.  Needs a
diagnostics build:

    PGDIST_DEFINES=PGDIST_PWT_TRACE python -c "import __graft_entry__ as g; g.build()"
    python scripts/pwb_phases.py [--out FILE]

Per shape: event time (20 launches), then one traced launch in which thread 0 of every
workgroup sums the 100 MHz wall clock per phase over its tiles: prologue, staging (includes
the wait for the prefetched tile), MFMAs, C tile, epilogue stores, tail.  Printed: the median
over workgroups of each phase sum, and per tile.
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import pgdist  # noqa: E402,F401
from pgdist.ops import kernels as K  # noqa: E402

# (label, M, Kg = conv Cout, Ng = conv Cin, epilogue)
SHAPES = [
    ("features.2 expand 112x112 16->96", 1605632, 96, 16, "lin"),
    ("features.1 project 112x112 32->16", 1605632, 16, 32, "relu6"),
    ("features.3 expand 56x56 24->144", 401408, 144, 24, "lin"),
    ("features.3 project 56x56 144->24", 401408, 24, 144, "relu6"),
    ("features.2 project 56x56 96->24", 401408, 24, 96, "relu6"),
    ("features.5 expand 28x28 32->192", 100352, 192, 32, "lin"),
    ("features.5 project 28x28 192->32", 100352, 32, 192, "relu6"),
]
PHASES = ["prologue", "staging", "MFMAs", "C tile", "epilogue", "tail"]


def q(v, f):
    v = sorted(v)
    return v[min(len(v) - 1, int(f * len(v)))]


def run(label, M, Kg, Ng, epi, dev, out):
    g = torch.Generator(device="cpu").manual_seed(0)
    r = lambda *s: torch.randn(*s, generator=g).to(dev)  # noqa: E731
    bf = torch.bfloat16
    G, Y = r(M, Kg).to(bf), r(M, Kg).to(bf)
    ca, cb, cc = torch.rand(Kg, device=dev) + 0.5, torch.rand(Kg, device=dev) - 0.5, torch.rand(Kg, device=dev) - 0.5
    WT = (r(Ng, Kg) / math.sqrt(Kg)).to(bf)
    o = torch.empty(M, Ng, dtype=bf, device=dev)
    Yt = r(M, Ng).to(bf)
    P = K.pw_bwd_num_partials(M, Kg, Ng)
    part = torch.zeros(K.bn_rows(P) * 2 * Ng, device=dev)
    wpart = torch.zeros(K.pw_bwd_wgrad_workspace(M, Kg, Ng), device=dev)
    kw = {}
    if epi == "lin":
        E = K.EPI_BWD_LIN
        kw = dict(X=r(M, Ng).to(bf))
    else:
        E = K.EPI_BWD_RELU6
        kw = dict(es=torch.rand(Ng, device=dev) + 0.5, et=torch.rand(Ng, device=dev) - 0.5)

    def launch():
        K.pw_bwd(E, G, Y, ca, cb, cc, WT, o, Yt, part, wpart, None, M, Kg, Ng, **kw)

    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(20):
        part.zero_()
        e0.record()
        launch()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    buf = torch.zeros(65536 * 8, dtype=torch.int64, device=dev)
    K.pwb_trace_set(buf)
    part.zero_()
    launch()
    torch.cuda.synchronize()
    K.pwb_trace_set(None)
    t = buf.view(-1, 8).cpu()
    t = t[t[:, 6] != 0].double()
    n = t.shape[0]
    if n == 0:
        print(f"{label}: no trace (build with PGDIST_DEFINES=PGDIST_PWT_TRACE)", file=out)
        return
    tiles = t[:, 6]
    print(f"{label}: M={M} Kg={Kg} Ng={Ng}  event p50 {q(ts, .5):.1f} us  workgroups {n}  "
          f"tiles/wg {q(tiles.tolist(), .5):.0f}", file=out)
    tot = t[:, :6].sum(1) / 100.0
    print(f"    traced lifetime p50 {q(tot.tolist(), .5):.1f} us", file=out)
    for i, ph in enumerate(PHASES):
        d = (t[:, i] / 100.0).tolist()
        per = (t[:, i] / 100.0 / tiles).tolist()
        print(f"    {ph:10s} sum p50 {q(d, .5):7.2f} us   per tile p50 {q(per, .5):6.3f} us", file=out)


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
