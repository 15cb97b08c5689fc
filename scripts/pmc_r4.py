#!/usr/bin/env python3
"""Per-dispatch PMC table of one MobileNetV2 training step (scripts/gpu_r4_pmc.sh passes).

usage: pmc_r4.py <dir with p1..p3>

Dispatches of the last complete step (between the last two Adam kernels) are aligned across
passes by position.  Columns: duration, waves, wave-cycle split (parked at s_waitcnt / barrier =
SQ_WAIT_ANY, issue-stalled = SQ_WAIT_INST_ANY, issuing = SQ_ACTIVE_INST_ANY; quad-cycle
counters, shares of SQ_WAVE_CYCLES), VALU instructions per wave, HBM bytes (FETCH_SIZE doubled:
gfx950 tallies 128-B requests at 64 B, MI355X_MICROARCH.md) and the L2 hit rate.
"""
import csv
import glob
import os
import re
import sys
from collections import OrderedDict, defaultdict


def short(name):
    n = re.sub(r"\(.*", "", name)
    return re.sub(r"^void ", "", n)[:46]


def load(path):
    disp = OrderedDict()
    for r in csv.DictReader(open(path)):
        d = disp.setdefault(int(r["Dispatch_Id"]), {"name": short(r["Kernel_Name"]),
                                                    "t": (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    seq = [disp[k] for k in sorted(disp)]
    idx = [i for i, d in enumerate(seq) if "adam" in d["name"]]
    return seq[idx[-2] + 1: idx[-1] + 1] if len(idx) >= 2 else seq


def main(root):
    passes = []
    for p in sorted(glob.glob(os.path.join(root, "p*"))):
        if os.path.isdir(p):
            f = glob.glob(os.path.join(p, "**", "*counter_collection.csv"), recursive=True)
            if f:
                passes.append(load(f[0]))
    n = min(len(p) for p in passes)
    rows = []
    for i in range(n):
        d = {}
        for p in passes:
            for k, v in p[i].items():
                d.setdefault(k, v)
        dur = (d["t"][1] - d["t"][0]) / 1e3
        wc = max(d.get("SQ_WAVE_CYCLES", 0.0), 1.0)
        waves = max(d.get("SQ_WAVES", 0.0), 1.0)
        mb = (2 * d.get("FETCH_SIZE", 0.0) + d.get("WRITE_SIZE", 0.0)) / 1024
        hit = d.get("TCC_HIT_sum", 0.0) / max(d.get("TCC_HIT_sum", 0.0) + d.get("TCC_MISS_sum", 0.0), 1.0)
        rows.append(dict(name=d["name"], us=dur, waves=waves, wait=d.get("SQ_WAIT_ANY", 0) / wc,
                         stall=d.get("SQ_WAIT_INST_ANY", 0) / wc, act=d.get("SQ_ACTIVE_INST_ANY", 0) / wc,
                         valu=d.get("SQ_INSTS_VALU", 0) / waves, lds=d.get("SQ_INSTS_LDS", 0) / waves, mb=mb, hit=hit))
    fam = defaultdict(lambda: defaultdict(float))
    for r in rows:
        f = fam[r["name"]]
        f["n"] += 1
        for k in ("us", "mb"):
            f[k] += r[k]
        for k in ("wait", "stall", "act"):
            f[k] += r[k] * r["us"]
    print(f"{'family':46s} {'n':>3s} {'us':>7s} {'MB':>7s} {'TB/s':>5s} {'wait':>5s} {'stall':>5s} {'act':>5s}")
    for k, f in sorted(fam.items(), key=lambda x: -x[1]["us"]):
        print(f"{k:46s} {int(f['n']):3d} {f['us']:7.1f} {f['mb']:7.1f} {f['mb'] / max(f['us'], 1e-9):5.2f} "
              f"{f['wait'] / f['us']:5.2f} {f['stall'] / f['us']:5.2f} {f['act'] / f['us']:5.2f}")
    print(f"\n{'#':>3s} {'kernel':46s} {'us':>6s} {'waves':>6s} {'MB':>6s} {'TB/s':>5s} {'wait':>5s} {'stall':>5s} "
          f"{'act':>5s} {'valu/w':>6s} {'lds/w':>5s} {'L2hit':>5s}")
    for i, r in enumerate(rows):
        print(f"{i:3d} {r['name']:46s} {r['us']:6.1f} {int(r['waves']):6d} {r['mb']:6.1f} {r['mb'] / max(r['us'], 1e-9):5.2f} "
              f"{r['wait']:5.2f} {r['stall']:5.2f} {r['act']:5.2f} {r['valu']:6.0f} {r['lds']:5.0f} {r['hit']:5.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
