#!/usr/bin/env python3
"""Per-conv MFMA throughput of the native ResNet-50 step from a rocprofv3 kernel trace
(``--kernel-trace --output-format csv``).

The executor dispatches each kernel family in a fixed layer order (forward: stem, then
conv1/conv2/conv3/[projection] per bottleneck; dgrad: per bottleneck in reverse
conv3/[projection]/conv2/conv1; wgrad on the side stream in the same order + stem), so
the k-th dispatch of a family is identified with its layer and its useful FLOPs
(2*M*N*K) divided by the measured duration.

usage: analyze_resnet_trace.py run_kernel_trace.csv [batch] [img]
"""
import csv
import sys
from collections import defaultdict


def convs(B, S):
    """(name, cin, cout, k, stride, H_in) in forward order"""
    out = [("stem", 3, 64, 7, 2, S)]
    H = ((S + 6 - 7) // 2 + 1 - 1) // 2 + 1
    cin = 64
    for li, (planes, n, s) in enumerate(((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))):
        for bi in range(n):
            st = s if bi == 0 else 1
            Ho = (H - 1) // st + 1
            pre = f"l{li + 1}.{bi}"
            blk = [(pre + ".c1", cin, planes, 1, 1, H), (pre + ".c2", planes, planes, 3, st, H),
                   (pre + ".c3", planes, planes * 4, 1, 1, Ho)]
            if bi == 0:
                blk.append((pre + ".cd", cin, planes * 4, 1, st, H))
            out.append(blk)
            cin, H = planes * 4, Ho
    return out


def flops(c, B):
    name, cin, cout, k, st, H = c
    pad = k // 2
    Ho = (H + 2 * pad - k) // st + 1
    return 2.0 * B * Ho * Ho * cout * k * k * (4 if cin == 3 else cin)


def main(path, B=128, S=224):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].startswith("image_prep")]
    step = rows[starts[-2]:starts[-1]] if len(starts) >= 2 else rows
    t0 = int(step[0]["Start_Timestamp"])
    t1 = max(int(r["End_Timestamp"]) for r in step)
    fams = defaultdict(list)
    for r in step:
        nm = r["Kernel_Name"].replace("void ", "")
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        if nm.startswith("conv_igemm_kernel<0"):
            fams["fwd"].append((nm, d))
        elif nm.startswith("conv_igemm_kernel<1"):
            fams["dgrad"].append((nm, d))
        elif nm.startswith("conv_wgrad_kernel"):
            fams["wgrad"].append((nm, d))
        else:
            fams[nm.split("<")[0].split("(")[0]].append((nm, d))
    tot = sum(d for v in fams.values() for _, d in v)
    print(f"step wall (first..last kernel) {(t1 - t0) / 1e6:.3f} ms, kernel time {tot / 1e3:.3f} ms, "
          f"{len(step)} dispatches")
    for f, v in sorted(fams.items(), key=lambda kv: -sum(d for _, d in kv[1])):
        print(f"  {f:40s} {sum(d for _, d in v) / 1e3:8.3f} ms  x{len(v)}")
    cl = convs(B, S)
    fwd_order = [cl[0]] + [c for blk in cl[1:] for c in blk]
    bwd_order = []
    for blk in reversed(cl[1:]):
        b = [blk[2]] + ([blk[3]] if len(blk) > 3 else []) + [blk[1], blk[0]]
        bwd_order += b
    wg_order = bwd_order + [cl[0]]
    total_fl, total_t = 0.0, 0.0
    for fam, order in (("fwd", fwd_order), ("dgrad", bwd_order), ("wgrad", wg_order)):
        ds = fams.get(fam, [])
        fl = sum(flops(c, B) for c in order[:len(ds)])
        t = sum(d for _, d in ds)
        total_fl += fl
        total_t += t
        print(f"\n{fam}: {t / 1e3:.3f} ms, {fl / 1e9:.0f} GFLOP -> {fl / (t * 1e-6) / 1e12:.0f} TFLOP/s")
        for (nm, d), c in zip(ds, order):
            tile = nm.split("<")[1].split(">")[0] if "<" in nm else ""
            print(f"  {c[0]:10s} cin={c[1]:4d} cout={c[2]:4d} k={c[3]} s={c[4]} H={c[5]:3d}  {d:8.1f} us "
                  f"{flops(c, B) / (d * 1e-6) / 1e12:6.0f} TF  <{tile}>")
    print(f"\nall convs: {total_t / 1e3:.3f} ms, {total_fl / 1e12:.2f} TFLOP -> "
          f"{total_fl / (total_t * 1e-6) / 1e12:.0f} TFLOP/s")


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:]))
