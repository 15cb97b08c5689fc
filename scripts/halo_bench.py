"""Isolated timing of the ResNet-50 stride-1 3x3 forward convs (bs128): halo-tile kernel vs the
implicit-GEMM (LDS-DMA) kernel, with the dense bf16 MFMA utilisation they reach."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import pgdist  # noqa: F401
from pgdist.ops import kernels as K


def timeit(fn, iters=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


dev = torch.device("cuda", 0)
for B, H, C in [(128, 56, 64), (128, 28, 128), (128, 14, 256), (128, 7, 512)]:
    x = torch.randn(B, H, H, C, device=dev).to(torch.bfloat16)
    w = (torch.randn(C, 3, 3, C, device=dev) * (9 * C) ** -0.5).to(torch.bfloat16)
    y = torch.empty(B, H, H, C, dtype=torch.bfloat16, device=dev)
    P = K.conv_fwd_num_partials(B, H, H, C, 9 * C, C)
    part = torch.zeros(P, 2, C, device=dev)
    res = {}
    for halo in (1, 0):
        K.conv_set_halo(halo)
        res[halo] = timeit(lambda: K.conv_fwd(K.CP_NONE, x, w, y, part, B, H, H, C, C, 3, 3, 1, 1))
    K.conv_set_halo(1)
    fl = 2.0 * B * H * H * C * C * 9
    print(f"B={B} H={H} C={C}: halo {res[1]:6.1f} us ({fl / res[1] / 1e6 / 2500 * 100:4.1f} % of 2.5 PF)  "
          f"igemm {res[0]:6.1f} us ({fl / res[0] / 1e6 / 2500 * 100:4.1f} %)", flush=True)
