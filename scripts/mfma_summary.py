#!/usr/bin/env python3
"""Per-kernel-family MFMA summary of one rocprofv3 --pmc run (scripts/gpu_pmc_mfma.sh).

usage: mfma_summary.py <rocprofv3 output dir> <steps in the run> [title]

Counters: SQ_INSTS_VALU_MFMA_MOPS_BF16 / _F8 (units of 512 FLOP), SQ_VALU_MFMA_BUSY_CYCLES
(SIMD-cycles the matrix core was busy, summed over the 1024 SIMDs), GRBM_GUI_ACTIVE (GPU
cycles summed over the 8 XCDs).  Peak: 2.5 PFLOP/s dense for bf16 and for the non-scaled fp8
MFMA (same cycles per instruction as bf16 on gfx950).
"""
import csv
import glob
import re
import sys
from collections import defaultdict

PEAK = 2.5e15


def fam(name):
    return re.sub(r"\(.*", "", name).replace("void ", "").split("<")[0]


def main(d, steps, title=""):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    disp = {}
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"])
        e = disp.setdefault(k, {"name": fam(r["Kernel_Name"]), "t": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                "c": defaultdict(float)})
        e["c"][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = defaultdict(lambda: defaultdict(float))
    for e in disp.values():
        a = agg[e["name"]]
        a["calls"] += 1
        a["t"] += e["t"]
        for c, v in e["c"].items():
            a[c] += v
    tot = defaultdict(float)
    for a in agg.values():
        for c, v in a.items():
            tot[c] += v
    gfl = lambda a: 512 * (a["SQ_INSTS_VALU_MFMA_MOPS_BF16"] + a["SQ_INSTS_VALU_MFMA_MOPS_F8"]) / 1e9  # noqa: E731
    print(f"== {title} (rocprofv3 --pmc, {steps} steps in the run; per-step figures)")
    print(f"total MFMA work {gfl(tot) / steps:.1f} GFLOP/step (bf16 {512 * tot['SQ_INSTS_VALU_MFMA_MOPS_BF16'] / 1e9 / steps:.1f}, "
          f"fp8 {512 * tot['SQ_INSTS_VALU_MFMA_MOPS_F8'] / 1e9 / steps:.1f}); kernel time {tot['t'] / 1e6 / steps:.2f} ms/step "
          f"(counter run); MFMA-kernel share of peak over the whole step "
          f"{100 * gfl(tot) * 1e9 / (tot['t'] * 1e-9) / PEAK:.1f}%")
    print(f"{'kernel':34s} {'calls':>6s} {'ms/step':>8s} {'GFLOP/st':>9s} {'f8 %':>5s} {'TF/s':>7s} {'% peak':>7s} {'MFMA busy %':>11s}")
    for n, a in sorted(agg.items(), key=lambda x: -gfl(x[1])):
        g = gfl(a)
        if g <= 0:
            continue
        t = a["t"] * 1e-9
        busy = a["SQ_VALU_MFMA_BUSY_CYCLES"] / max(a["GRBM_GUI_ACTIVE"] / 8 * 1024, 1)
        f8 = 100 * a["SQ_INSTS_VALU_MFMA_MOPS_F8"] / max(a["SQ_INSTS_VALU_MFMA_MOPS_F8"] + a["SQ_INSTS_VALU_MFMA_MOPS_BF16"], 1)
        print(f"{n[:34]:34s} {a['calls'] / steps:6.0f} {a['t'] / 1e6 / steps:8.3f} {g / steps:9.1f} {f8:5.0f} "
              f"{g * 1e9 / t / 1e12:7.1f} {100 * g * 1e9 / t / PEAK:7.1f} {100 * busy:11.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), sys.argv[3] if len(sys.argv) > 3 else "")
