"""Per-phase wall clock of the small-M pointwise GEMM (pw_tile, csrc/kernels/pwtile.hip) on the
MobileNetV2 14x14 / 7x7 shapes with the largest excess over their byte floor
(profiles/r5_roofline_mnv2.txt).  Needs a diagnostics build:

    PGDIST_DEFINES=PGDIST_PWT_TRACE python -c "import __graft_entry__ as g; g.build()"
    python scripts/pwt_phases.py [--out FILE]

Per shape: event time of the op (30 back-to-back launches), then one traced launch; thread 0 of
every workgroup stamps the 100 MHz wall clock at kernel start (0), prologue parameters staged
(1), first operand tile in LDS (2), k loop done (3), C tile stored (4), BN partials added (5),
end (6).  Printed: workgroups, launch span, start spread, and the median / p90 of each phase.
"""
import argparse
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import pgdist  # noqa: E402,F401
from pgdist.ops import kernels as K  # noqa: E402

# (label, M, N, K, pro, epi)
SHAPES = [
    ("final-conv dgrad 7x7 1280->320", 6272, 320, 1280, "bwd", "lin"),
    ("project fwd 7x7 960->160", 6272, 160, 960, "relu6", "fwd"),
    ("project fwd 14x14 576->96", 25088, 96, 576, "relu6", "fwd"),
    ("expand fwd 14x14 96->576", 25088, 576, 96, "bnres", "fwd"),
    ("expand dgrad 14x14 576->96", 25088, 96, 576, "bwd", "lin"),
    ("project dgrad 7x7 160->960", 6272, 960, 160, "bwd", "relu6"),
    ("expand fwd 7x7 160->960", 6272, 960, 160, "bnres", "fwd"),
]

PHASES = ["params", "first tile", "k loop", "C tile + stores", "BN partials", "fin tail"]


def q(v, f):
    v = sorted(v)
    return v[min(len(v) - 1, int(f * len(v)))]


def run(label, M, N, Kd, pro, epi, dev, out):
    g = torch.Generator(device="cpu").manual_seed(0)
    r = lambda *s: torch.randn(*s, generator=g).to(dev)  # noqa: E731
    bf = torch.bfloat16
    A = r(M, Kd).to(bf)
    W = (r(N, Kd) / math.sqrt(Kd)).to(bf)
    o = torch.empty(M, N, dtype=bf, device=dev)
    P = K.pw_num_partials(M, N, Kd)
    part = torch.zeros(K.bn_part_floats(P, N) if hasattr(K, "bn_part_floats") else P * 2 * N, device=dev)
    pa, pb, pc = (torch.rand(Kd, device=dev) + 0.5, torch.rand(Kd, device=dev) - 0.5, torch.rand(Kd, device=dev) - 0.5)
    kw = {}
    if pro == "bwd":
        kw = dict(A2=r(M, Kd).to(bf), pa=pa, pb=pb, pc=pc, Yt=r(M, N).to(bf))
        if epi == "relu6":
            kw.update(es=torch.rand(N, device=dev) + 0.5, et=torch.rand(N, device=dev) - 0.5)
        P_ = K.PRO_BNBWD
        E_ = K.EPI_BWD_LIN if epi == "lin" else K.EPI_BWD_RELU6
    elif pro == "relu6":
        kw = dict(pa=pa, pb=pb)
        P_, E_ = K.ACT_BN_RELU6, K.EPI_FWD
    else:   # bnres: BN (+ residual) prologue of a pending block output
        kw = dict(pa=pa, pb=pb, A2=r(M, Kd).to(bf))
        P_, E_ = K.PRO_BNRES, K.EPI_FWD

    def launch():
        part.zero_()
        K.pw_gemm(P_, E_, A, W, o, part, M, N, Kd, **kw)

    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    # time the GEMM alone: the zeroing of the partials is a separate (tiny) memset
    ts = []
    for _ in range(30):
        part.zero_()
        e0.record()
        K.pw_gemm(P_, E_, A, W, o, part, M, N, Kd, **kw)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    buf = torch.zeros(65536 * 8, dtype=torch.int64, device=dev)
    K.pwt_trace_set(buf)
    launch()
    torch.cuda.synchronize()
    K.pwt_trace_set(None)
    t = buf.view(-1, 8).cpu()
    t = t[t[:, 0] != 0].double() / 100.0   # 100 MHz -> us
    n = t.shape[0]
    if n == 0:
        print(f"{label}: no trace (build with PGDIST_DEFINES=PGDIST_PWT_TRACE)", file=out)
        return
    t0 = t[:, 0].min()
    span = (t[:, 6].max() - t0).item()
    starts = (t[:, 0] - t0).tolist()
    print(f"{label}: M={M} N={N} K={Kd}  event {q(ts, 0.5):.1f} us  workgroups {n}  traced span {span:.1f} us  "
          f"start spread p50/p90/max {q(starts, .5):.1f}/{q(starts, .9):.1f}/{max(starts):.1f} us", file=out)
    life = (t[:, 6] - t[:, 0]).tolist()
    print(f"    workgroup lifetime p50/p90 {q(life, .5):.2f}/{q(life, .9):.2f} us", file=out)
    for i, ph in enumerate(PHASES):
        d = (t[:, i + 1] - t[:, i]).tolist()
        print(f"    {ph:16s} p50 {q(d, .5):6.2f}  p90 {q(d, .9):6.2f} us", file=out)


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
