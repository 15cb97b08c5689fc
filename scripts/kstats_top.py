"""Top kernels of a rocprofv3 ``--stats`` kernel_stats.csv (total time, calls, share).

    python scripts/kstats_top.py gpurun_out/r3c/prof_mb/.../run_kernel_stats.csv [N]
"""
import csv
import re
import sys


def short(name):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"^void ", "", name)
    return re.sub(r"\((?:[^()]|\([^()]*\))*\)$", "", name)


def main(path, n=25):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {path}: {len(rows)} kernels, {tot / 1e6:.2f} ms total GPU kernel time")
    print(f"{'total_ms':>9} {'calls':>6} {'avg_us':>8} {'share':>6}  kernel")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:n]:
        t = float(r["TotalDurationNs"])
        print(f"{t / 1e6:9.3f} {int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:8.1f} {100 * t / tot:5.1f}%  {short(r['Name'])}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
