#!/usr/bin/env python3
"""Per-op comparison of several roofline tables (scripts/roofline.py outputs) of the same step
recorded under different configurations: for every op of a chosen family, the isolated time under
each configuration and the best one.

usage: roofline_compare.py FAMILY cfg0.txt cfg1.txt ... [--names a,b,...]
"""
import re
import sys


def load(path):
    rows = {}
    for line in open(path):
        m = re.match(r"\s*(\d+)\s+(main|side)\s+(\S+)\s+([\d.]+)\s+([\d.]+)\s+([\d.]+)\s+([\d.]+)\s*(.*)$", line)
        if m:
            rows[int(m.group(1))] = (m.group(3), float(m.group(4)), m.group(8).strip())
    return rows


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    names = None
    for a in sys.argv[1:]:
        if a.startswith("--names="):
            names = a.split("=", 1)[1].split(",")
    fam, paths = args[0], args[1:]
    names = names or [f"cfg{i}" for i in range(len(paths))]
    tabs = [load(p) for p in paths]
    tot = [0.0] * len(paths)
    best_tot = 0.0
    for idx in sorted(tabs[0]):
        op, _, shape = tabs[0][idx]
        if op != fam or any(idx not in t or t[idx][0] != op for t in tabs):
            continue
        ts = [t[idx][1] for t in tabs]
        b = min(range(len(ts)), key=lambda i: ts[i])
        for i, v in enumerate(ts):
            tot[i] += v
        best_tot += ts[b]
        print(f"{idx:4d} {shape:40s} " + " ".join(f"{n}:{v:7.1f}" for n, v in zip(names, ts)) + f"  best={names[b]}")
    print("totals: " + " ".join(f"{n}:{v:.1f}" for n, v in zip(names, tot)) + f"  per-op best: {best_tot:.1f}")


if __name__ == "__main__":
    main()
