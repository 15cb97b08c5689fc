"""Checkpointing: reference-compatible best-model export + full-state resume.

Reference: in-memory ``deepcopy(state_dict)`` whenever
test accuracy improves, one ``torch.save`` at the end —
``best_mobilenetv2_cifar10_224.pth`` (serial / 1 GPU) or
``best_mobilenetv2_cifar10_224_mpi.pth`` (DDP rank 0, no ``module.`` prefix);
plain torchvision-keyed fp32 NCHW ``state_dict``, weights only, so a crash loses
the run.

pgdist keeps that exact file format and adds resumable checkpoints
(``ckpt_epoch{N}.pt``): model, flat Adam moments + step, LR schedule state,
epoch, sampler epoch, RNG states, world size and config.  Everything is
written from rank 0 atomically (tmp + rename) and read by all ranks with
``weights_only=True``.
"""
import copy
import os
from typing import Any, Dict, Optional

import torch


def snapshot_state_dict(model: torch.nn.Module) -> Dict[str, torch.Tensor]:
    """CPU copy of the torchvision-keyed state dict (the reference's deepcopy, without holding GPU memory)."""
    sd = model.state_dict()
    return {k: v.detach().to("cpu", copy=True) for k, v in sd.items()}


def save_best(state: Dict[str, torch.Tensor], path: str):
    _atomic_save(state, path)


def load_model_weights(model: torch.nn.Module, path: str, map_location="cpu", strict: bool = True):
    sd = torch.load(path, map_location=map_location, weights_only=True)
    if any(k.startswith("module.") for k in sd):
        sd = {k[len("module."):]: v for k, v in sd.items()}
    model.load_state_dict(sd, strict=strict)
    return model


def _atomic_save(obj: Any, path: str):
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_full(path: str, *, model: torch.nn.Module, epoch: int, step: int, lr: float,
              exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor, flat_order=None, best_acc: float = 0.0,
              best_state: Optional[Dict[str, torch.Tensor]] = None, world_size: int = 1,
              config: Optional[dict] = None, scheduler_state: Optional[dict] = None):
    obj = {
        "format": "pgdist-full-v1",
        "model": snapshot_state_dict(model),
        "epoch": int(epoch),
        "step": int(step),
        "lr": float(lr),
        "exp_avg": exp_avg.detach().cpu(),
        "exp_avg_sq": exp_avg_sq.detach().cpu(),
        "flat_order": list(flat_order) if flat_order is not None else None,
        "best_acc": float(best_acc),
        "best_state": best_state,
        "world_size": int(world_size),
        "config": config or {},
        "scheduler": scheduler_state or {},
        "rng_cpu": torch.get_rng_state(),
    }
    _atomic_save(obj, path)


def load_full(path: str) -> dict:
    obj = torch.load(path, map_location="cpu", weights_only=True)
    if obj.get("format") != "pgdist-full-v1":
        raise ValueError(f"{path} is not a pgdist full checkpoint")
    return obj


def latest_checkpoint(ckpt_dir: str) -> Optional[str]:
    if not ckpt_dir or not os.path.isdir(ckpt_dir):
        return None
    cands = [f for f in os.listdir(ckpt_dir) if f.startswith("ckpt_epoch") and f.endswith(".pt")]
    if not cands:
        return None
    cands.sort(key=lambda f: int(f[len("ckpt_epoch"):-3]))
    return os.path.join(ckpt_dir, cands[-1])
