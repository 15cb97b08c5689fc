#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes per kernel family (last step of a run).

usage: analyze_pmc.py gpurun_out/pmc
Prints per kernel family: time, HBM bytes (FETCH_SIZE x2 calibration for wide
streaming reads on gfx950, WRITE_SIZE), achieved TB/s, L2 hit rate, VALU/VMEM
activity and wait fractions.
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def load(path):
    rows = list(csv.DictReader(open(path)))
    per = defaultdict(dict)   # dispatch -> counter -> value
    meta = {}
    for r in rows:
        d = int(r["Dispatch_Id"])
        per[d][r["Counter_Name"]] = per[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        meta[d] = (r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return per, meta


def fam(name):
    return name.split("(")[0].replace("void ", "").split("<")[0]


def main(d):
    agg = defaultdict(lambda: defaultdict(float))
    for p in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        per, meta = load(p)
        ds = sorted(meta)
        # second half of dispatches ~ the last step
        ds = ds[len(ds) // 2:]
        for k in ds:
            f = fam(meta[k][0])
            for c, v in per[k].items():
                agg[f][c] += v
            agg[f]["_t_" + os.path.basename(os.path.dirname(p))] += meta[k][1]
    print(f"{'kernel':28s} {'t_us':>8s} {'rdMB':>8s} {'wrMB':>8s} {'TB/s':>6s} {'L2hit':>6s} {'VALU%':>6s} {'VMEM%':>6s} {'waitI%':>6s} {'wait%':>6s}")
    for f, c in sorted(agg.items(), key=lambda x: -x[1].get("_t_p1", 0)):
        t = c.get("_t_p1", 0) / 1e3
        rd = 2 * c.get("FETCH_SIZE", 0) * 1024 / 1e6
        wr = c.get("WRITE_SIZE", 0) * 1024 / 1e6
        bw = (rd + wr) / 1e6 / (t / 1e6) if t else 0
        hit = c.get("TCC_HIT_sum", 0) / max(1, c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0))
        wc = c.get("SQ_WAVE_CYCLES", 0) or 1
        print(f"{f[:28]:28s} {t:8.1f} {rd:8.1f} {wr:8.1f} {bw:6.2f} {hit:6.2f} "
              f"{100 * c.get('SQ_ACTIVE_INST_VALU', 0) / wc:6.1f} {100 * c.get('SQ_ACTIVE_INST_VMEM', 0) / wc:6.1f} "
              f"{100 * c.get('SQ_WAIT_INST_ANY', 0) / wc:6.1f} {100 * c.get('SQ_WAIT_ANY', 0) / wc:6.1f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
