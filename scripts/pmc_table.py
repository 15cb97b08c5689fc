#!/usr/bin/env python3
"""Pivot rocprofv3 counter_collection.csv files: one row per dispatch (kernel, grid), counters
as columns (several passes of the same program are joined by dispatch order per kernel).
usage: pmc_table.py dir1 [dir2 ...] [--filter substr]"""
import csv
import glob
import re
import sys
from collections import OrderedDict, defaultdict


def load(d):
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    disp = OrderedDict()
    for r in csv.DictReader(open(f)):
        k = int(r["Dispatch_Id"])
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace(", ", "_")
        e = disp.setdefault(k, {"name": name, "grid": r.get("Grid_Size", ""), "c": defaultdict(float)})
        e["c"][r["Counter_Name"]] += float(r["Counter_Value"])
    return list(disp.values())


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    flt = sys.argv[sys.argv.index("--filter") + 1] if "--filter" in sys.argv else ""
    if flt in args:
        args.remove(flt)
    runs = [load(d) for d in args]
    base = runs[0]
    for other in runs[1:]:
        byname = defaultdict(list)
        for e in other:
            byname[e["name"]].append(e)
        seen = defaultdict(int)
        for e in base:
            L = byname[e["name"]]
            i = seen[e["name"]]
            seen[e["name"]] += 1
            if i < len(L):
                e["c"].update(L[i]["c"])
    cols = sorted({c for e in base for c in e["c"]})
    print("kernel," + "grid," + ",".join(cols))
    for e in base:
        if flt and flt not in e["name"]:
            continue
        print(e["name"][:40] + "," + str(e["grid"]) + "," + ",".join(f"{e['c'].get(c, 0):.4g}" for c in cols))


if __name__ == "__main__":
    main()
