"""Per-phase timing of the fused inverted-residual block kernels (csrc/kernels/irblock.hip).

Every fused launch of one training step (forward and backward) runs alone (synchronised before
and after) with the kernels' phase trace on: thread 0 of each workgroup stamps the 100 MHz wall
clock at the phase boundaries.  Per launch it prints the median / max over workgroups of each
phase and, for the two grid barriers, the arrival spread (first to last workgroup reaching it)
and the release latency (last arrival to first departure).

    python scripts/ir_phases.py [--batch-size 128] [--img-size 224] [--out FILE]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import pgdist  # noqa: E402,F401
from pgdist.ops import kernels as K  # noqa: E402

FWD = ("P0 input", "P1 expand", "h1 store", "bar1", "P2 bn", "P2 relu6", "P2 dw", "dd atomics", "bar2",
       "P3 bn", "P3 reload", "P3 project")
BWD = ("B0 pc+h2", "B0 dy", "B1 proj-dgrad", "bar1", "B2 coef", "B2 dh2", "B2 dw-dgrad", "de atomics",
       "bar2", "B3 coef", "B3 dh1", "B3 exp-dgrad")


def summarize(tag, ts, names):
    t = ts.double() / 100.0     # us
    t = t - t[:, 0].min()
    lines = [f"{tag}: {t.shape[0]} workgroups, total {t[:, 12].max().item():.1f} us"]
    for k, nm in enumerate(names):
        d = t[:, k + 1] - t[:, k]
        lines.append(f"    {nm:14s} median {d.median().item():7.2f}  max {d.max().item():7.2f} us")
    for a, nm in ((3, "bar1"), (8, "bar2")):
        spread = (t[:, a].max() - t[:, a].min()).item()
        release = (t[:, a + 1].min() - t[:, a].max()).item()
        lines.append(f"    {nm}: arrival spread {spread:.2f} us, release latency {release:.2f} us")
    return "\n".join(lines)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--img-size", type=int, default=224)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from pgdist.models import mobilenet_v2
    from pgdist.engine.executor import MobileNetV2Executor
    MobileNetV2Executor.IR_FUSE = "1"
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    exe = MobileNetV2Executor(mobilenet_v2(10), a.batch_size, a.img_size, dev)
    exe.img.normal_()
    exe.labels.random_(0, 10)
    out = []
    state = {"on": False}

    def wrap(fn, names, grid_fn):
        def run(*args):
            if not state["on"]:
                return fn(*args)
            B, H, cin, ch, cout = args[-5:]
            n = grid_fn(B, H, cin, ch, cout)
            buf = torch.zeros(n * 16, dtype=torch.int64, device=dev)
            torch.cuda.synchronize()
            K.ir_trace_set(buf)
            fn(*args)
            torch.cuda.synchronize()
            K.ir_trace_set(None)
            out.append(summarize(f"{fn.__name__} H={H} {cin}->{ch}->{cout}", buf.view(n, 16).cpu(), names))
        return run

    K.ir_fwd = wrap(K.ir_fwd, FWD, K.ir_fwd_grid)
    K.ir_bwd = wrap(K.ir_bwd, BWD, K.ir_bwd_grid)
    for i in range(3):
        state["on"] = i == 2
        exe.forward(train=True)
        exe.backward()
        torch.cuda.synchronize()
    assert exe.ir_error() == 0
    text = "\n".join(out)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
