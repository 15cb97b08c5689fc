#!/usr/bin/env python3
"""All-reduce latency vs bucket size on one MI355X: the P2P one-shot / two-shot kernels with
N = 2 / 4 / 8 ranks emulated in one launch (every rank's staging in this GPU's HBM: measures
the kernels' barrier + copy-in + reduce cost, not xGMI), and RCCL at world size 1.

Usage: python scripts/comm_bench.py [--out profiles/r3_comm_microbench.txt]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import pgdist  # noqa: E402,F401
from pgdist.parallel.comm import NativeComm  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sizes_kib = [64, 256, 1024, 1536, 4096, 9216, 16384]
    lines = ["# all-reduce latency (us per call, back to back on the comm stream), fp32 elements",
             "# P2P rows: N ranks emulated on ONE GPU (all staging local; no xGMI traffic)",
             f"{'path':<22}" + "".join(f"{s:>10}KiB" for s in sizes_kib)]
    c1 = NativeComm(0, 1, dev, use_rccl=True)
    x = torch.zeros(max(sizes_kib) * 256, device=dev)
    row = [c1.time_allreduce(x[:s * 256], "rccl", iters=a.iters) for s in sizes_kib]
    lines.append(f"{'rccl world=1':<22}" + "".join(f"{v:>13.1f}" for v in row))
    c1.close()
    for world in (2, 4, 8):
        for blocks in (16, 32):
            c = NativeComm(0, world, dev, p2p_bytes=max(sizes_kib) * 1024, blocks=blocks, emulate=True,
                           timeout_s=10.0)
            bufs = [torch.zeros(max(sizes_kib) * 256, device=dev) for _ in range(world)]
            for algo in ("oneshot", "twoshot"):
                for bf in (False, True):
                    row = [c.time_allreduce([b[:s * 256] for b in bufs], algo, bf, iters=a.iters)
                           for s in sizes_kib]
                    name = f"{algo} N={world} G={blocks}{' bf16' if bf else ''}"
                    lines.append(f"{name:<22}" + "".join(f"{v:>13.1f}" for v in row))
            c.check()
            c.close()
    out = "\n".join(lines)
    print(out, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(out + "\n")


if __name__ == "__main__":
    main()
