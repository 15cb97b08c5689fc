#!/usr/bin/env python3
"""Per-layer achieved bandwidth of the native MobileNetV2 step from a rocprofv3
kernel trace (``--kernel-trace --output-format csv``).

Kernels of one family are dispatched in a fixed layer order by the executor, so
the k-th ``dw_fwd`` dispatch of a step is block k's depthwise conv, etc.  The
minimum HBM bytes of each op are computed from the layer shapes and divided by
the measured duration.

usage: analyze_trace.py run_kernel_trace.csv [batch] [img]
"""
import csv
import sys
from collections import defaultdict

SETTING = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 2),
           (6, 320, 1, 1)]


def blocks(B, S):
    H = (S - 1) // 2 + 1
    cin = 32
    out = []
    for t, c, n, s in SETTING:
        for i in range(n):
            st = s if i == 0 else 1
            hid = cin * t
            Ho = (H - 1) // st + 1
            out.append(dict(t=t, cin=cin, cout=c, hid=hid, s=st, H=H, Ho=Ho, Min=B * H * H, Mout=B * Ho * Ho))
            cin, H = c, Ho
    return out, H


def main(path, B=128, S=224):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # take the last occurrence window: the last stem_fwd dispatch starts the last step
    starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("stem_fwd")]
    step = rows[starts[-2]:starts[-1]] if len(starts) >= 2 else rows
    bl, Hf = blocks(B, S)
    by = defaultdict(list)
    for r in step:
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        fam = name.split("<")[0]
        by[fam].append((name, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    tot = sum(d for v in by.values() for _, d in v)
    print(f"step kernel time {tot / 1e3:.3f} ms ({len(step)} dispatches)")
    # depthwise
    for fam, order, byt in (
            ("dw_fwd_kernel", bl, lambda b: (b["Min"] + b["Mout"]) * b["hid"] * 2),
            ("dw_dgrad_kernel", bl[::-1], lambda b: (2 * b["Mout"] + 2 * b["Min"]) * b["hid"] * 2),
            ("dw_wgrad_kernel", bl[::-1], lambda b: (2 * b["Mout"] + b["Min"]) * b["hid"] * 2)):
        ds = by.get(fam, [])
        print(f"\n{fam}: {sum(d for _, d in ds):.1f} us total")
        for (nm, d), b in zip(ds, order):
            gb = byt(b) / 1e9
            print(f"  C={b['hid']:4d} H={b['H']:3d} s={b['s']}  {d:7.1f} us  {gb * 1e3:7.1f} MB  {gb / d * 1e6 / 1e3:6.2f} TB/s")
    # pointwise: forward (expand, project per block, then final 1x1), backward in reverse
    fwd, bwd = [], []
    for b in bl:
        if b["t"] != 1:
            fwd.append(("exp", b["Min"], b["cin"], b["hid"]))
        fwd.append(("prj", b["Mout"], b["hid"], b["cout"]))
    Mf = B * Hf * Hf
    fwd.append(("last", Mf, bl[-1]["cout"], 1280))
    bwd = fwd[::-1]
    # forward + dgrad GEMMs in dispatch order (row-stream kernel for large M, tiled for small M)
    pw = [(r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3) for r in step
          if r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0] in ("pw_gemm_kernel", "pw_tile_kernel")]
    fused = [d for n, d in by.get("pw_bwd_fused_kernel", [])]
    wg = by.get("pw_wgrad_kernel", [])
    n = len(fwd)
    print(f"\npw layers (M, K->N): fwd / dgrad / wgrad  us @ TB/s")
    tf = td = tw = 0.0
    # the large-M backward layers are fused (dgrad + wgrad in one kernel): they are missing from
    # the dgrad/wgrad lists, so map dgrad/wgrad dispatches onto the unfused layers only
    unfused = [i for i, (kind, M, K, N) in enumerate(fwd) if M < 65536 or kind == "last"]
    nf = len(fwd) - len(unfused) if fused else 0
    dg = {}
    wg_ = {}
    if fused:
        for k, i in enumerate(sorted(unfused, reverse=True)):
            if len(fwd) + k < len(pw):
                dg[i] = pw[len(fwd) + k][1]
            if k < len(wg):
                wg_[i] = wg[k][1]
    for i, (kind, M, K, N) in enumerate(fwd):
        j = n - 1 - i
        bf = M * (K + N) * 2
        bd = M * (2 * N + 2 * K) * 2      # G, Y in; out (+ Yt / residual) -- approx
        bw = M * (2 * N + K) * 2
        f_ = pw[i][1] if i < len(pw) else 0
        if fused:
            d_, w_ = dg.get(i, 0.0), wg_.get(i, 0.0)
        else:
            d_ = pw[n + j][1] if n + j < len(pw) else 0
            w_ = wg[j][1] if j < len(wg) else 0
        tf, td, tw = tf + f_, td + d_, tw + w_
        print(f"  {kind:4s} M={M:8d} {K:4d}->{N:4d}  fwd {f_:6.1f} {bf / f_ / 1e6 if f_ else 0:5.2f}  "
              f"dgrad {d_:6.1f} {bd / d_ / 1e6 if d_ else 0:5.2f}  wgrad {w_:6.1f} {bw / w_ / 1e6 if w_ else 0:5.2f}")
    print(f"  totals: fwd {tf:.0f} us  dgrad {td:.0f} us  wgrad {tw:.0f} us (+ stem wgrad {wg[-1][1] if wg else 0:.0f})")
    for fam in ("pw_bwd_fused_kernel", "pw_gemm_kernel", "pw_wgrad_kernel", "colsum_kernel", "bn_fwd_finalize_kernel", "split_reduce_kernel"):
        ds = by.get(fam, [])
        print(f"\n{fam}: {len(ds)} dispatches {sum(d for _, d in ds):.1f} us total; per dispatch: " +
              " ".join(f"{d:.0f}" for _, d in ds[:80]))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], int(a[1]) if len(a) > 1 else 128, int(a[2]) if len(a) > 2 else 224)
