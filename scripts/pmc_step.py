#!/usr/bin/env python3
"""Per-dispatch PMC summary of one training step from scripts/gpu_pmc.sh passes.

usage: pmc_step.py gpurun_out/pmc [--top N]

Each pass (p1..p4) is a separate run of the same bench; dispatches of the last complete step
(between the last two Adam kernels) are aligned across passes by position.  Per dispatch:
duration, HBM-side bytes (FETCH_SIZE + WRITE_SIZE, KB counters), achieved bandwidth, L2 hit
rate, VALU issue utilisation (SQ_INSTS_VALU x 4 cycles over 1024 SIMDs at 2.4 GHz) and
VMEM instruction counts.
"""
import csv
import os
import re
import sys
from collections import OrderedDict, defaultdict


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"^void ", "", n)
    return n[:44]


def load(path):
    disp = OrderedDict()
    for r in csv.DictReader(open(path)):
        d = disp.setdefault(int(r["Dispatch_Id"]), {"name": short(r["Kernel_Name"]), "grid": int(r["Grid_Size"]),
                                                    "t": (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    seq = [disp[k] for k in sorted(disp)]
    idx = [i for i, d in enumerate(seq) if "adam" in d["name"]]
    return seq[idx[-2] + 1: idx[-1] + 1] if len(idx) >= 2 else seq


def main(root, top):
    passes = [load(os.path.join(root, p, "run_counter_collection.csv"))
              for p in sorted(os.listdir(root)) if os.path.isdir(os.path.join(root, p))]
    n = min(len(p) for p in passes)
    rows = []
    for i in range(n):
        d = {}
        for p in passes:
            d.update({k: v for k, v in p[i].items() if k not in d})
        dur = (d["t"][1] - d["t"][0]) / 1e3   # us
        mb = (d.get("FETCH_SIZE", 0) + d.get("WRITE_SIZE", 0)) / 1024
        hit = d.get("TCC_HIT_sum", 0) / max(d.get("TCC_HIT_sum", 0) + d.get("TCC_MISS_sum", 0), 1)
        valu = d.get("SQ_INSTS_VALU", 0) * 4 / max(dur * 2400 * 1024, 1)
        rows.append((d["name"], d["grid"], dur, d.get("FETCH_SIZE", 0) / 1024, d.get("WRITE_SIZE", 0) / 1024,
                     mb / max(dur, 1e-9) * 1e-6 * 1e6 / 1e6, hit, valu, d.get("SQ_INSTS_VMEM_RD", 0),
                     d.get("SQ_INSTS_LDS", 0)))
    fam = defaultdict(lambda: [0, 0.0, 0.0])
    for r in rows:
        fam[r[0]][0] += 1
        fam[r[0]][1] += r[2]
        fam[r[0]][2] += r[3] + r[4]
    print(f"{'family':44s} {'n':>3s} {'us':>8s} {'MB':>8s} {'TB/s':>6s}")
    for k, (c, us, mb) in sorted(fam.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{k:44s} {c:3d} {us:8.1f} {mb:8.1f} {mb / us:6.2f}")
    print(f"\n{'kernel':44s} {'grid':>8s} {'us':>7s} {'rdMB':>7s} {'wrMB':>7s} {'TB/s':>5s} {'L2hit':>5s} {'valu':>5s}")
    for r in sorted(rows, key=lambda r: -r[2])[:top]:
        print(f"{r[0]:44s} {r[1]:8d} {r[2]:7.1f} {r[3]:7.1f} {r[4]:7.1f} {(r[3] + r[4]) / r[2]:5.2f} "
              f"{r[6]:5.2f} {r[7]:5.2f}")


if __name__ == "__main__":
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 40
    main(sys.argv[1], top)
