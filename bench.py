#!/usr/bin/env python3
"""Headline benchmark: images/sec (whole node), MobileNetV2 / CIFAR-10 224x224,
bs=128 per GPU, synthetic data, random-init weights, bf16 compute.

Contract (see BASELINE.json / task spec):
  python bench.py --gpus N --steps K --warmup W
For N>1 it is launched by ``torch.distributed.run`` with one rank per GPU
(RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* from the env).  Without any launcher, ``--gpus N > 1``
starts that launcher itself (127.0.0.1 rendezvous, N fresh rank processes; this process never
touches the GPU and exits with the launcher's status), so a launcher-less multi-GPU call can
not silently measure one rank.  A rank count that differs from ``--gpus`` is an error.
W untimed warm-up steps, then EXACTLY K timed steps bracketed by barrier + synchronize on both
sides; the MAX elapsed over ranks is used; rank 0 prints one JSON line.

A timed step is a full training step of the flagship path: GPU augmentation of
a device-resident synthetic uint8 32x32 CIFAR-shaped batch to 224x224 (the
reference's Resize->RandomResizedCrop->Flip->ColorJitter->Rotation->Normalize
chain, fused on the GPU), forward, cross-entropy, backward, DDP gradient
all-reduce (N>1: native communicator, RCCL / P2P xGMI buckets), fused Adam update.
For N>1 the step also broadcasts rank 0's BatchNorm buffers before the forward, as the
reference's DDP does (``broadcast_buffers=True``, cifar10_mpi_mobilenet_224.py:142-145).

After the timed region an N>1 run checks the communicator on every rank (peer timeouts,
out-of-step peers, RCCL errors) and that parameters and Adam state are bitwise identical
across ranks; the JSON carries ``comm_error``, ``replicas_identical`` and ``rccl_ranks`` and
the process exits non-zero if either check fails.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Reference throughput (BASELINE.md "Derived throughput"): 1xV100 93.5 img/s,
# 2xV100 DDP 191.6 img/s.  4/8 GPUs were not measured by the reference; we
# compare against the reference's 2-GPU per-GPU rate x N (linear extrapolation).
REF_IMG_S = {1: 93.5, 2: 191.6}
METRIC = "images/sec (whole node) MobileNetV2/CIFAR-10 224² bs128 at 1/2/4/8 MI355X; val acc"


def ref_for(n: int) -> float:
    return REF_IMG_S.get(n, 191.6 / 2 * n)


def parse_args(argv=None):
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
                    help="BASELINE config 5: 1x1 convs on e4m3 MFMA (use with --batch-size 512)")
    ap.add_argument("--bn-broadcast", type=int, default=-1,
                    help="broadcast rank 0's BN buffers before every forward (reference DDP "
                         "broadcast_buffers=True); -1 (default): on when N > 1")
    return ap.parse_args(argv)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _launcher_env() -> bool:
    """True if some launcher (torchrun, mpirun, PMI, srun) already defines the rank layout."""
    from pgdist.parallel.bootstrap import discover   # env only: no GPU, no process group
    return discover().world_size > 1 or "WORLD_SIZE" in os.environ


def self_launch(args) -> int:
    """Run this script under torch.distributed.run with --gpus ranks (parent stays off the GPU)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.abspath(__file__)] + sys.argv[1:]
    print(f"[bench] no launcher for --gpus {args.gpus}: starting {args.gpus} rank processes", file=sys.stderr,
          flush=True)
    return subprocess.call(cmd, cwd=ROOT)


def main():
    args = parse_args()
    import pgdist  # noqa: F401  (package alias; imports no GPU code)
    if args.gpus > 1 and not _launcher_env():
        sys.exit(self_launch(args))

    import torch
    import torch.distributed as dist
    from pgdist.parallel.bootstrap import init_distributed, cleanup

    # PGDIST_DIST_BACKEND=gloo: rehearse the multi-rank bench with several ranks on one GPU
    # (RCCL needs one GPU per rank); the default picks RCCL ("nccl") on GPUs
    info, device, backend = init_distributed(backend=os.environ.get("PGDIST_DIST_BACKEND", "auto"))
    world = info.world_size
    if world != args.gpus:
        print(f"[bench] error: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks",
              file=sys.stderr, flush=True)
        cleanup()
        sys.exit(2)
    bn_broadcast = (world > 1) if args.bn_broadcast < 0 else bool(args.bn_broadcast)

    from pgdist.engine.bench_step import build_bench_step
    step_fn, meta = build_bench_step(args.model, args.batch_size, device, backend=args.backend,
                                     img_size=args.img_size, use_graph=args.graph, side_stream=bool(args.side_stream),
                                     fp8=bool(args.fp8), world_size=world, rank=info.rank,
                                     bn_broadcast=bn_broadcast)
    step = meta.pop("_step", None)

    # fault injection for the failure-detection tests: rank PGDIST_FAULT_RANK skips timed step
    # PGDIST_FAULT_SKIP_STEP (its collectives never happen), which must fail the run on every rank
    skip_step = int(os.environ.get("PGDIST_FAULT_SKIP_STEP", "-1"))
    if int(os.environ.get("PGDIST_FAULT_RANK", "-1")) != info.rank:
        skip_step = -1

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier(device_ids=[device.index] if device.type == "cuda" and backend == "nccl" else None)
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    for _ in range(args.warmup):
        step_fn()
    sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        if i != skip_step:
            step_fn()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- data-parallel health (N > 1), outside the timed region, on every rank
    health = {}
    healthy = True
    if world > 1:
        from pgdist.parallel.ddp import all_reduce_scalars, replicas_identical
        comm = getattr(step, "comm", None)
        err, why = 0, ""
        if comm is not None:
            err = comm.error()
            why = comm.error_string()
        red_dev = device if backend == "nccl" else torch.device("cpu")
        worst = int(all_reduce_scalars([float(err)], red_dev, op=dist.ReduceOp.MAX)[0])
        flat = getattr(step, "flat", None)
        tensors = [flat.master, flat.exp_avg, flat.exp_avg_sq] if flat is not None else \
            [p for p in meta.get("_params", [])]
        same = bool(replicas_identical(tensors, red_dev)[0]) if tensors else None
        ranks = comm.rccl_ranks() if comm is not None else (world if backend == "nccl" else 0)
        health = {"comm_error": worst, "replicas_identical": same, "rccl_ranks": ranks}
        healthy = worst == 0 and same is not False
        if not healthy:
            print(f"[bench] rank {info.rank}: data-parallel run FAILED: communicator error 0x{worst:x} "
                  f"(this rank: 0x{err:x} {why}), replicas identical: {same}", file=sys.stderr, flush=True)
    meta.pop("_params", None)

    ms_per_step = elapsed / args.steps * 1e3
    imgs_per_s = args.batch_size * world * args.steps / elapsed
    # the BASELINE.json metric is MobileNetV2 bs128/GPU bf16; other configs report their own metric
    headline = args.model == "mobilenet_v2" and args.batch_size == 128 and not args.fp8
    if info.rank == 0:
        out = {
            "metric": (METRIC if headline else
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
            "dtype": "fp8-e4m3 forward 1x1 GEMMs (K>=64) / bf16" if args.fp8 else "bf16",
            "data": ("synthetic (device-resident uint8 32x32x3 CIFAR-shaped images, GPU-augmented to 224x224; "
                     "random-init weights)" if args.model == "mobilenet_v2" else
                     "synthetic (device-resident uint8 224x224x3 ImageNet-shaped images, GPU flip + normalise; "
                     "random-init weights, 1000 classes)"),
            "config": {"model": args.model, "global_batch": args.batch_size * world,
                       "per_gpu_batch": args.batch_size, "seq_len": None, "img_size": args.img_size,
                       "parallelism": f"dp{world}", "backend": meta.get("backend"),
                       "hip_graph": meta.get("graph"), "side_stream": meta.get("side_stream"),
                       "fp8": bool(args.fp8), "bn_broadcast": bn_broadcast and world > 1,
                       "dist_backend": backend if world > 1 else None,
                       "allreduce": meta["allreduce"]() if callable(meta.get("allreduce")) else meta.get("allreduce")},
        }
        out.update(health)
        if world > 1 and device.type == "cuda" and info.local_world_size > torch.cuda.device_count():
            out["rehearsal_on_one_gpu"] = True   # ranks share a GPU: not an N-GPU measurement
        print(json.dumps(out), flush=True)
    cleanup()
    if not healthy:
        sys.exit(3)


if __name__ == "__main__":
    main()
