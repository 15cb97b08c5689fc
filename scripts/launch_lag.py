#!/usr/bin/env python3
"""Host submission vs GPU start of every kernel of the last training step, from a rocprofv3
``--kernel-trace --hip-trace`` run (scripts/gpu_hiptrace.sh): for each dispatch, the idle gap
on its stream before it and how long after its launch API call returned it started.  A large
gap with a small lag means the GPU was waiting on something else (slots, a dependency); a gap
with the launch call arriving late means the host was behind.

usage: launch_lag.py <dir with run_kernel_trace.csv and run_hip_api_trace.csv> [min_gap_us]
"""
import csv
import glob
import os
import re
import sys


def main(d, min_gap=5.0):
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)[0]
    at = glob.glob(os.path.join(d, "**", "*hip_api_trace.csv"), recursive=True)[0]
    api = {}
    for r in csv.DictReader(open(at)):
        api[r["Correlation_Id"]] = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"])
    ks = []
    for r in csv.DictReader(open(kt)):
        name = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "")[:48]
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Stream_Id"], name, r["Correlation_Id"]))
    ks.sort()
    idx = [i for i, k in enumerate(ks) if "adam" in k[3]]
    step = ks[idx[-2] + 1:idx[-1] + 1]
    t0 = step[0][0]
    last_end = {}
    for s, e, st, name, cid in step:
        gap = (s - last_end[st]) / 1e3 if st in last_end else 0.0
        last_end[st] = e
        a = api.get(cid)
        lag = (s - a[1]) / 1e3 if a else float("nan")
        if gap >= min_gap:
            print(f"{(s - t0) / 1e3:8.1f} us  stream {st}  gap {gap:6.1f}  start-after-API {lag:7.1f}  {name}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 5.0)
