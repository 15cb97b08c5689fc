#!/usr/bin/env python3
"""Isolated timing of the dense implicit-GEMM conv kernels on every ResNet-50 layer shape (bs 128).

usage: python scripts/conv_bench.py [--reps N] [--kinds fwd,fwdbn,dgrad,wgrad] [--only l3]

Each kernel is timed with HIP events (median of N launches; the caches are flushed by a 512 MiB
write between launches) and reported as TFLOP/s of the layer's GEMM work (2*M*N*K):
  fwd    y = conv(x, w)                      (no prologue: the block-input convs)
  fwdbn  y = conv(relu(bn(x)), w)            (BN+ReLU prologue: every other forward conv)
  dgrad  dx = conv^T(bn_bwd(G, Y), w) * mask (CE_BWD_RELU epilogue)
  wgrad  dW = sum_m bn_bwd(G, Y) (x) im2col(relu(bn(x)))  (split-M + reduction)
  dgradm / wgradm / wgradma: the same on a materialised dy (wgradma: materialised x as well)
  mata / matb: the bn_mat passes that materialise relu(bn(x)) / bn_bwd(G, Y)
The network totals weight every shape by its count in ResNet-50.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import pgdist  # noqa: E402,F401
from pgdist.ops import kernels as K  # noqa: E402

# (name, Ci, N, H, R, stride, count)
SHAPES = [
    ("l1.c1a", 64, 64, 56, 1, 1, 1), ("l1.c1", 256, 64, 56, 1, 1, 2), ("l1.c2", 64, 64, 56, 3, 1, 3),
    ("l1.c3", 64, 256, 56, 1, 1, 4),
    ("l2.c1a", 256, 128, 56, 1, 1, 1), ("l2.c2a", 128, 128, 56, 3, 2, 1), ("l2.cd", 256, 512, 56, 1, 2, 1),
    ("l2.c1", 512, 128, 28, 1, 1, 3), ("l2.c2", 128, 128, 28, 3, 1, 3), ("l2.c3", 128, 512, 28, 1, 1, 4),
    ("l3.c1a", 512, 256, 28, 1, 1, 1), ("l3.c2a", 256, 256, 28, 3, 2, 1), ("l3.cd", 512, 1024, 28, 1, 2, 1),
    ("l3.c1", 1024, 256, 14, 1, 1, 5), ("l3.c2", 256, 256, 14, 3, 1, 5), ("l3.c3", 256, 1024, 14, 1, 1, 6),
    ("l4.c1a", 1024, 512, 14, 1, 1, 1), ("l4.c2a", 512, 512, 14, 3, 2, 1), ("l4.cd", 1024, 2048, 14, 1, 2, 1),
    ("l4.c1", 2048, 512, 7, 1, 1, 2), ("l4.c2", 512, 512, 7, 3, 1, 2), ("l4.c3", 512, 2048, 7, 1, 1, 3),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--kinds", default="fwd,fwdbn,dgrad,wgrad")
    ap.add_argument("--only", default="")
    ap.add_argument("--glds", default="", help="comma list of staging modes for 'fwd' (0, 2, 3): fwd0, fwd2, ...")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B = a.batch
    flush = torch.empty(512 * 2 ** 20 // 4, dtype=torch.float32, device=dev)
    kinds = a.kinds.split(",")
    if a.glds and "fwd" in kinds:
        i = kinds.index("fwd")
        kinds[i:i + 1] = [f"fwd{m}" for m in a.glds.split(",")]
    tot_us = {k: 0.0 for k in kinds}
    tot_fl = {k: 0.0 for k in kinds}
    for name, Ci, N, H, R, s, cnt in SHAPES:
        if a.only and not name.startswith(a.only):
            continue
        pad = R // 2
        Ho, Wo = K.conv_out_hw(H, H, R, R, s, pad)
        M, Kd = B * Ho * Wo, R * R * Ci
        flops = 2.0 * M * N * Kd
        g = torch.Generator(device=dev).manual_seed(0)

        def rnd(n, scale=1.0):
            return (torch.randn(n, generator=g, device=dev) * scale).to(torch.bfloat16)

        x = rnd(B * H * H * Ci)
        w = rnd(N * Kd, 0.05)
        wt = rnd(N * Kd, 0.05)
        y = torch.empty(B * Ho * Wo * N, dtype=torch.bfloat16, device=dev)
        G, Y = rnd(B * Ho * Wo * N), rnd(B * Ho * Wo * N)
        dx = torch.empty(B * H * H * Ci, dtype=torch.bfloat16, device=dev)
        pa = torch.rand(Ci, generator=g, device=dev) + 0.5
        pb = torch.rand(Ci, generator=g, device=dev) - 0.5
        ga, gb, gc = (torch.randn(N, generator=g, device=dev) * 0.1 for _ in range(3))
        Pf = K.conv_fwd_num_partials(B, Ho, Wo, N, Kd, Ci)
        part = torch.zeros(Pf * 2 * N + 1024, device=dev)
        fns = {
            "fwd": lambda: K.conv_fwd(K.CP_NONE, x, w, y, part, B, H, H, Ci, N, R, R, s, pad),
            "fwdbn": lambda: K.conv_fwd(K.CP_BN_RELU, x, w, y, part, B, H, H, Ci, N, R, R, s, pad, pa=pa, pb=pb),
        }
        if R <= 3 and H % s == 0:
            Pd = K.conv_dgrad_num_partials(B, H, H, Ci, N, R, R, s)
            partd = torch.zeros(Pd * 2 * Ci + 1024, device=dev)
            fns["dgrad"] = lambda: K.conv_dgrad(K.CE_BWD_RELU, G, Y, ga, gb, gc, wt, dx, partd, B, H, H, Ci, N, R, R,
                                                s, pad, Yt=x, es=pa, et=pb)
        ws = torch.zeros(K.conv_wgrad_workspace(B, H, H, Ci, N, R, R, s, pad) + 1024, device=dev)
        grad = torch.zeros(N * Kd, device=dev)
        fns["wgrad"] = lambda: K.conv_wgrad(G, Y, ga, gb, gc, x, ws, grad, B, H, H, Ci, N, R, R, s, pad,
                                            xpro=K.CP_BN_RELU, xs=pa, xt=pb)
        dym = rnd(B * Ho * Wo * N)
        act = torch.empty(B * H * H * Ci, dtype=torch.bfloat16, device=dev)
        fns["mata"] = lambda: K.bn_mat(K.BN_MAT_ACT, x.view(-1, Ci), pa, pb, act.view(-1, Ci))
        fns["matb"] = lambda: K.bn_mat(K.BN_MAT_BWD, Y.view(-1, N), ga, gb, dym.view(-1, N), G=G.view(-1, N), c=gc)
        if "dgrad" in fns:
            fns["dgradm"] = lambda: K.conv_dgrad(K.CE_BWD_RELU, dym, None, None, None, None, wt, dx, partd, B, H, H, Ci,
                                                 N, R, R, s, pad, Yt=x, es=pa, et=pb)
        fns["wgradm"] = lambda: K.conv_wgrad(dym, None, None, None, None, x, ws, grad, B, H, H, Ci, N, R, R, s, pad,
                                             xpro=K.CP_BN_RELU, xs=pa, xt=pb)
        fns["wgradma"] = lambda: K.conv_wgrad(dym, None, None, None, None, x, ws, grad, B, H, H, Ci, N, R, R, s, pad)
        for m in (a.glds.split(",") if a.glds else []):
            fns[f"fwd{m}"] = (lambda m=int(m): (K.conv_set_glds(m), fns["fwd"]()))
        line = f"{name:7s} Ci={Ci:4d} N={N:4d} H={H:3d} {R}x{R} s{s} x{cnt}"
        for k in kinds:
            if k not in fns:
                line += f"  {k:5s}    --   "
                continue
            fn = fns[k]
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
            tot_us[k] += us * cnt
            tot_fl[k] += flops * cnt
            line += f"  {k} {us:7.1f} us {flops / us / 1e6:4.0f} TF"
        print(line, flush=True)
    print("network totals (x layer count): " + "  ".join(
        f"{k} {tot_us[k]:.0f} us {tot_fl[k] / max(tot_us[k], 1e-9) / 1e6:.0f} TF" for k in kinds))


if __name__ == "__main__":
    main()
