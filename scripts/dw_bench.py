#!/usr/bin/env python3
"""Isolated timing of the depthwise 3x3 kernels on every MobileNetV2 layer shape (bs 128).

usage: python scripts/dw_bench.py [--reps N] [--kinds fwd,dgrad,dgradw,wgrad] [--csv out.csv]

Times each kernel with HIP events (median of N launches, warm caches between layers are
flushed by a 512 MiB write) and reports achieved bandwidth against the compulsory bytes:
fwd  x -> y;  dgrad  (g, y, yprev) -> gout;  dgradw the same plus the fused weight-gradient
partials;  wgrad  (g, y, yprev) -> partials.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import pgdist  # noqa: E402,F401
from pgdist.ops import kernels as K  # noqa: E402

SHAPES = [  # (C, H, stride, count in the network)
    (32, 112, 1, 1), (96, 112, 2, 1), (144, 56, 1, 1), (144, 56, 2, 1), (192, 28, 1, 2), (192, 28, 2, 1),
    (384, 14, 1, 4), (576, 14, 1, 2), (576, 14, 2, 1), (960, 7, 1, 3),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--kinds", default="fwd,dgrad,dgradw,wgrad")
    ap.add_argument("--csv", default="")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B = a.batch
    flush = torch.empty(512 * 2 ** 20 // 4, dtype=torch.float32, device=dev)
    kinds = a.kinds.split(",")
    rows = []
    tot = {k: 0.0 for k in kinds}
    for C, H, s, cnt in SHAPES:
        Ho = (H - 1) // s + 1
        g = torch.Generator(device=dev).manual_seed(0)
        bf = dict(dtype=torch.bfloat16, device=dev)
        x = torch.randn(B * H * H, C, generator=g, device=dev).to(torch.bfloat16)
        yo = torch.randn(B * Ho * Ho, C, generator=g, device=dev).to(torch.bfloat16)
        go = torch.randn(B * Ho * Ho, C, generator=g, device=dev).to(torch.bfloat16)
        w = (torch.randn(9 * C, generator=g, device=dev) * 0.3).to(torch.bfloat16)
        sc = torch.rand(C, generator=g, device=dev) + 0.5
        sh = torch.rand(C, generator=g, device=dev) - 0.5
        coef = torch.randn(3 * C, generator=g, device=dev) * 0.1
        out_y = torch.empty(B * Ho * Ho, C, **bf)
        gout = torch.empty(B * H * H, C, **bf)
        Pf = K.dw_num_partials("fwd", B, H, H, C, s)
        Pd = K.dw_num_partials("dgrad", B, H, H, C, s)
        part = torch.zeros(max(K.bn_part_floats(Pf, C), K.bn_part_floats(Pd, C)) + 1024, device=dev)
        wpart = torch.zeros(K.dw_dgrad_wgrad_workspace(B, H, H, C, s) + 1024, device=dev)
        wws = torch.zeros(K.dw_wgrad_workspace(B, H, H, C, s) + 1024, device=dev)
        grad = torch.zeros(9 * C, device=dev)
        in_b, out_b = B * H * H * C * 2, B * Ho * Ho * C * 2
        fns = {
            "fwd": (lambda: K.dw_fwd(x, sc, sh, K.ACT_BN_RELU6, w, out_y, part, B, H, H, C, s), in_b + out_b),
            "dgrad": (lambda: K.dw_dgrad(go, yo, coef, w, x, sc, sh, gout, part, B, H, H, C, s),
                      2 * out_b + 2 * in_b),
            "dgradw": (lambda: K.dw_dgrad(go, yo, coef, w, x, sc, sh, gout, part, B, H, H, C, s, wpart=wpart),
                       2 * out_b + 2 * in_b),
            "wgrad": (lambda: K.dw_wgrad(go, yo, coef, x, sc, sh, wws, grad, B, H, H, C, s), 2 * out_b + in_b),
        }
        line = f"C={C:4d} H={H:3d} s={s}"
        for k in kinds:
            fn, nbytes = fns[k]
            fn()
            ts = []
            for _ in range(a.reps):
                flush.fill_(1.0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3)
            ts.sort()
            us = ts[len(ts) // 2]
            tot[k] += us * cnt
            line += f"  {k} {us:7.1f} us {nbytes / us / 1e6:5.2f} TB/s"
            rows.append((C, H, s, k, us, nbytes / us / 1e6))
        print(line, flush=True)
    print("network totals (x layer count): " + "  ".join(f"{k} {v:.0f} us" for k, v in tot.items()))
    if a.csv:
        with open(a.csv, "w") as f:
            f.write("C,H,stride,kind,us,TBps\n")
            for r in rows:
                f.write(",".join(str(v) for v in r) + "\n")


if __name__ == "__main__":
    main()
