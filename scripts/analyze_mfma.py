#!/usr/bin/env python3
"""MFMA activity per kernel family from a rocprofv3 --pmc pass of
SQ_INSTS_VALU_MFMA_MOPS_{BF16,F8}, SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE.

usage: analyze_mfma.py run_counter_collection.csv [n_steps]
MFMA FLOPs = MOPS x 512 (matches the analytic ResNet-50 count: 3.15 TFLOP per bs128 step);
"% peak" is against the 2.5 PFLOP/s dense bf16 figure.
Kernel durations come from the counter run (serialised dispatches), so TF/s is per kernel,
not per step.
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    disp = defaultdict(dict)
    meta = {}
    for r in csv.DictReader(open(path)):
        d = r["Dispatch_Id"]
        disp[d][r["Counter_Name"]] = float(r["Counter_Value"])
        meta[d] = (r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0],
                   int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    fam = defaultdict(lambda: defaultdict(float))
    for d, c in disp.items():
        name, dur = meta[d]
        f = fam[name]
        f["n"] += 1
        f["ns"] += dur
        f["flop"] += 512.0 * (c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) + c.get("SQ_INSTS_VALU_MFMA_MOPS_F8", 0))
        f["busy"] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0)
        f["gui"] += c.get("GRBM_GUI_ACTIVE", 0)
    tot_flop = sum(f["flop"] for f in fam.values())
    tot_ns = sum(f["ns"] for f in fam.values())
    print(f"total MFMA work {tot_flop / steps / 1e9:.1f} GFLOP/step over {steps} steps; "
          f"kernel time {tot_ns / steps / 1e6:.2f} ms/step (counter run)")
    print(f"{'kernel':34s} {'calls':>6s} {'ms/step':>8s} {'GFLOP/st':>9s} {'TF/s':>7s} {'% peak':>7s}")
    for name, f in sorted(fam.items(), key=lambda kv: -kv[1]["flop"]):
        if f["flop"] <= 0:
            continue
        tfs = f["flop"] / max(1.0, f["ns"]) / 1e3
        print(f"{name[:34]:34s} {int(f['n']):6d} {f['ns'] / steps / 1e6:8.3f} {f['flop'] / steps / 1e9:9.1f} "
              f"{tfs:7.1f} {100.0 * tfs / 2500.0:7.1f}")


if __name__ == "__main__":
    main()
