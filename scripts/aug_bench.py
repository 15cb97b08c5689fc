"""Isolated augmentation timing (bs128, 224x224, train): N back-to-back K.augment calls, for
`rocprofv3 --kernel-trace --stats` (params / render split) or plain wall time."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/scripts/", 1)[0])
from pgdist.ops import kernels as K  # noqa: E402


def main(n=50, B=128, S=224):
    dev = torch.device("cuda", 0)
    src = torch.randint(0, 256, (50000, 32, 32, 3), dtype=torch.uint8, device=dev)
    labels = torch.randint(0, 10, (50000,), device=dev)
    idx = torch.randint(0, 50000, (B,), device=dev)
    out = torch.empty(B, S, S, 4, dtype=torch.bfloat16, device=dev)
    lab = torch.empty(B, dtype=torch.int64, device=dev)
    prm = torch.empty(B, K.AUG_NPARAMS, device=dev)
    hyper = torch.tensor([0.0, 1.0], device=dev)
    for _ in range(5):
        K.augment(src, idx, labels, out, lab, prm, train=True, seed=1, hyper=hyper)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        K.augment(src, idx, labels, out, lab, prm, train=True, seed=1, hyper=hyper)
    torch.cuda.synchronize()
    print(f"augment bs{B} {S}x{S}: {(time.perf_counter() - t) / n * 1e6:.1f} us/call")


if __name__ == "__main__":
    main()
