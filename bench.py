#!/usr/bin/env python3
"""Headline benchmark: images/sec (whole node), MobileNetV2 / CIFAR-10 224x224,
bs=128 per GPU, synthetic data, random-init weights, bf16 compute.

Contract (see BASELINE.json / task spec):
  python bench.py --gpus N --steps K --warmup W
For N>1 it is launched by ``torch.distributed.run`` with one rank per GPU
(RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from the env).  W untimed warm-up steps,
then EXACTLY K timed steps bracketed by barrier + synchronize on both sides;
the MAX elapsed over ranks is used; rank 0 prints one JSON line.

A timed step is a full training step of the flagship path: GPU augmentation of
a device-resident synthetic uint8 32x32 CIFAR-shaped batch to 224x224 (the
reference's Resize->RandomResizedCrop->Flip->ColorJitter->Rotation->Normalize
chain, fused on the GPU), forward, cross-entropy, backward, DDP gradient
all-reduce over RCCL (N>1), fused Adam update.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import pgdist  # noqa: E402,F401
from pgdist.parallel.bootstrap import init_distributed, cleanup  # noqa: E402

# Reference throughput (BASELINE.md "Derived throughput"): 1xV100 93.5 img/s,
# 2xV100 DDP 191.6 img/s.  4/8 GPUs were not measured by the reference; we
# compare against the reference's 2-GPU per-GPU rate x N (linear extrapolation).
REF_IMG_S = {1: 93.5, 2: 191.6}


def ref_for(n: int) -> float:
    return REF_IMG_S.get(n, 191.6 / 2 * n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--model", default="mobilenet_v2")
    ap.add_argument("--backend", default="auto", help="hip (native kernels) | torch (MIOpen/PyTorch ops)")
    ap.add_argument("--graph", type=int, default=0,
                    help="capture the step in a hipGraph (1) or launch eagerly (0, default: measured faster "
                         "with the weight-gradient side stream, whose branches the graph replay serialises)")
    ap.add_argument("--side-stream", type=int, default=1, help="weight gradients on a second HIP stream")
    ap.add_argument("--img-size", type=int, default=224)
    ap.add_argument("--fp8", type=int, default=0,
                    help="BASELINE config 5: forward 1x1 convs on e4m3 MFMA (use with --batch-size 512)")
    args = ap.parse_args()

    # PGDIST_DIST_BACKEND=gloo: rehearse the multi-rank bench with several ranks on one GPU
    # (RCCL needs one GPU per rank); the default picks RCCL ("nccl") on GPUs
    info, device, backend = init_distributed(backend=os.environ.get("PGDIST_DIST_BACKEND", "auto"))
    world = info.world_size
    if world != args.gpus and info.rank == 0:
        print(f"[bench] warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)

    from pgdist.engine.bench_step import build_bench_step
    step_fn, meta = build_bench_step(args.model, args.batch_size, device, backend=args.backend,
                                     img_size=args.img_size, use_graph=args.graph, side_stream=bool(args.side_stream),
                                     fp8=bool(args.fp8), world_size=world, rank=info.rank)

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier(device_ids=[device.index] if device.type == "cuda" else None)
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    for _ in range(args.warmup):
        step_fn()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step_fn()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ms_per_step = elapsed / args.steps * 1e3
    imgs_per_s = args.batch_size * world * args.steps / elapsed
    # the BASELINE.json metric is MobileNetV2 bs128/GPU bf16; other configs report their own metric
    headline = args.model == "mobilenet_v2" and args.batch_size == 128 and not args.fp8
    if info.rank == 0:
        out = {
            "metric": ("images/sec (whole node) MobileNetV2/CIFAR-10 224² bs128 at 1/2/4/8 MI355X; val acc"
                       if headline else
                       f"images/sec (whole node) {args.model} 224² synthetic {'fp8 ' if args.fp8 else ''}"
                       f"bs{args.batch_size}/GPU"),
            "value": round(imgs_per_s, 2),
            "unit": "images/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(imgs_per_s / ref_for(world), 3) if headline else None,
            "dtype": "fp8-e4m3 fwd GEMMs / bf16" if args.fp8 else "bf16",
            "data": ("synthetic (device-resident uint8 32x32x3 CIFAR-shaped images, GPU-augmented to 224x224; "
                     "random-init weights)" if args.model == "mobilenet_v2" else
                     "synthetic (device-resident uint8 224x224x3 ImageNet-shaped images, GPU flip + normalise; "
                     "random-init weights, 1000 classes)"),
            "config": {"model": args.model, "global_batch": args.batch_size * world,
                       "per_gpu_batch": args.batch_size, "seq_len": None, "img_size": args.img_size,
                       "parallelism": f"dp{world}", "backend": meta.get("backend"),
                       "hip_graph": meta.get("graph"), "side_stream": meta.get("side_stream"),
                       "fp8": bool(args.fp8), "allreduce": meta.get("allreduce")},
        }
        print(json.dumps(out), flush=True)
    cleanup()


if __name__ == "__main__":
    main()
