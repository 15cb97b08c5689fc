#!/usr/bin/env python3
"""Per-stream timeline of one training step from a rocprofv3 kernel trace.

usage: timeline.py run_kernel_trace.csv [step_marker_substring] [--list]

Steps are delimited by the kernel whose name contains the marker (default: the Adam
kernel).  For the last complete step it prints, per stream, busy time, idle gaps and the
longest gaps, and the per-family time on each stream; with --list every dispatch.
"""
import csv
import re
import sys
from collections import defaultdict


def short(name):
    n = re.sub(r"\(.*", "", name)
    n = re.sub(r"^void ", "", n)
    return n[:60]


def main(path, marker="adam", listing=False):
    rows = list(csv.DictReader(open(path)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], short(r["Kernel_Name"]))
          for r in rows]
    ks.sort()
    idx = [i for i, k in enumerate(ks) if marker in k[3]]
    if len(idx) < 2:
        print("not enough steps")
        return
    a, b = idx[-2] + 1, idx[-1] + 1
    step = ks[a:b]
    t0, t1 = step[0][0], max(k[1] for k in step)
    print(f"step span {(t1 - t0) / 1e3:.1f} us, {len(step)} dispatches")
    by = defaultdict(list)
    for k in step:
        by[k[2]].append(k)
    for s, L in sorted(by.items()):
        busy = sum(e - b_ for b_, e, *_ in L)
        gaps = []
        for p, q in zip(L, L[1:]):
            gaps.append((q[0] - p[1], p[3], q[3]))
        idle = sum(max(g[0], 0) for g in gaps)
        print(f"\nstream {s}: {len(L)} kernels, busy {busy / 1e3:.1f} us, gaps {idle / 1e3:.1f} us "
              f"(mean {idle / max(len(gaps), 1) / 1e3:.2f} us)")
        fam = defaultdict(lambda: [0, 0])
        for b_, e, _, n in L:
            fam[n][0] += 1
            fam[n][1] += e - b_
        for n, (c, t) in sorted(fam.items(), key=lambda x: -x[1][1]):
            print(f"   {t / 1e3:8.1f} us  {c:4d}x  {n}")
        print("   longest gaps:")
        for g in sorted(gaps, key=lambda x: -x[0])[:8]:
            print(f"   {g[0] / 1e3:8.1f} us  after {g[1]}  before {g[2]}")
    if listing:
        for b_, e, s, n in step:
            print(f"{(b_ - t0) / 1e3:9.1f} {(e - b_) / 1e3:8.1f}  s{s}  {n}")


if __name__ == "__main__":
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    main(args[0], args[1] if len(args) > 1 else "adam", "--list" in sys.argv)
