"""Benchmark step builders used by ``bench.py``.

``hip`` backend: the native static-plan executor (HIP kernels, fused Adam,
bucketed RCCL all-reduce, optional hipGraph capture).
``torch`` backend: the PyTorch/MIOpen path (channels_last bf16 autocast +
``torch.nn.parallel.DistributedDataParallel`` + fused torch Adam) — kept as the
measured baseline the native path has to beat.
"""
import torch
import torch.nn.functional as F

from ..models import build_model
from ..data.synthetic import synthetic_cifar


def _resolve_backend(backend: str, device: torch.device) -> str:
    if backend == "auto":
        return "hip" if device.type == "cuda" else "torch"
    return backend


def allreduce_meta(step) -> dict:
    """Gradient all-reduce layout of a native step: buckets, algorithms, the bucket objective's
    table (simulated exposed microseconds per candidate "cap/last-cap" layout) and the measured
    all-reduce times."""
    red = step.reducer
    out = {
        "comm": "native" if getattr(red, "native", False) else "c10d",
        "buckets_kib": [round((e - s) * 4 / 1024, 1) for s, e, _ in red.buckets],
        "algos": list(getattr(red, "algos", ["c10d"] * len(red.buckets))),
        "launch_plan": bool(step.use_plan),
        "bucket_cap_mb": getattr(red, "bucket_cap_mb", None),
        "last_bucket_mb": getattr(red, "last_bucket_mb", None),
        "ready_times": "measured" if getattr(step, "bucket_ready_us", None) else "modelled",
    }
    if getattr(red, "bucket_tuning", None):
        out["bucket_cost_us"] = red.bucket_tuning
    tuning = getattr(step.comm, "tuning", None) if step.comm is not None else None
    if tuning:   # the chosen buckets' sizes (every candidate size was timed)
        sizes = {e - s for s, e, _ in red.buckets}
        out["tuned_us"] = {str(k): {a: round(v, 1) for a, v in d.items()} for k, d in tuning.items() if k in sizes}
    ready = getattr(step, "bucket_ready_us", None)
    if ready:
        out["bucket_ready_us"] = [round(max(ready.get(n, 0.0) for n in names), 1) for _, _, names in red.buckets]
    return out


def build_bench_step(model_name: str, batch_size: int, device: torch.device, backend: str = "auto",
                     img_size: int = 224, use_graph: bool = True, world_size: int = 1, rank: int = 0,
                     side_stream: bool = True, fp8: bool = False, bn_broadcast: bool = False):
    backend = _resolve_backend(backend, device)
    if backend == "hip":
        from .native_step import NativeTrainStep
        # use_graph: 0 eager, 1 whole step in one hipGraph, 2 forward in a hipGraph + eager backward
        step = NativeTrainStep.for_benchmark(model_name, batch_size, device, img_size=img_size,
                                             use_graph=int(use_graph) == 1, world_size=world_size, rank=rank,
                                             side_stream=side_stream, fp8=fp8, graph_forward=int(use_graph) == 2,
                                             bn_broadcast=bn_broadcast)
        graph = "forward" if step.graph_forward else step.graph_enabled
        meta = {"backend": "hip", "graph": graph, "side_stream": side_stream, "fp8": fp8, "_step": step}
        if step.reducer is not None:
            # read when the JSON line is written: the bucket layout is re-chosen from the ready times
            # measured on the second warm-up step (NativeTrainStep._retune_buckets)
            meta["allreduce"] = lambda step=step: allreduce_meta(step)
        return step.bench_step, meta
    if fp8:
        raise NotImplementedError("fp8 runs on the native (hip) backend")
    return _torch_bench_step(model_name, batch_size, device, img_size, world_size, rank, bn_broadcast)


def _torch_bench_step(model_name, batch_size, device, img_size, world_size, rank, bn_broadcast=False):
    torch.manual_seed(42 + rank)
    n_data = 4096
    imgs_np, labels_np = synthetic_cifar(n_data, seed=rank)
    imgs = torch.from_numpy(imgs_np).to(device)            # [N,32,32,3] uint8, device resident
    labels_all = torch.from_numpy(labels_np).to(device)
    mean = torch.tensor([0.485, 0.456, 0.406], device=device).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225], device=device).view(1, 3, 1, 1)

    model = build_model(model_name, num_classes=10 if model_name == "mobilenet_v2" else 1000).to(device)
    if device.type == "cuda":
        model = model.to(memory_format=torch.channels_last)
    ddp = model
    if world_size > 1:
        ddp = torch.nn.parallel.DistributedDataParallel(
            model, device_ids=[device.index] if device.type == "cuda" else None, broadcast_buffers=bn_broadcast)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4, fused=device.type == "cuda")
    crit = torch.nn.CrossEntropyLoss()
    amp_dtype = torch.bfloat16
    state = {"i": 0}
    n_cls = 10 if model_name == "mobilenet_v2" else 1000

    def step():
        i = state["i"]
        state["i"] += 1
        idx = torch.randint(0, n_data, (batch_size,), device=device)
        x = imgs.index_select(0, idx).permute(0, 3, 1, 2).float().div_(255.0)
        x = F.interpolate(x, size=(img_size, img_size), mode="bilinear", align_corners=False)
        flip = (torch.rand(batch_size, 1, 1, 1, device=device) < 0.5)
        x = torch.where(flip, x.flip(3), x)
        x = ((x - mean) / std).contiguous(memory_format=torch.channels_last)
        y = labels_all.index_select(0, idx) % n_cls
        opt.zero_grad(set_to_none=True)
        with torch.autocast(device_type=device.type, dtype=amp_dtype, enabled=device.type == "cuda"):
            out = ddp(x)
            loss = crit(out.float(), y)
        loss.backward()
        opt.step()
        return loss

    return step, {"backend": "torch", "graph": False, "_params": list(model.parameters())}
