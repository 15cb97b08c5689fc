"""Single dataclass configuration with CLI overrides and the reference's presets.

The reference hard-codes every hyper-parameter as a module constant and keeps
one copy of the script per mode:

* serial CPU  — ``cifar10_serial_mobilenet_224.py`` (device=cpu :19, bs=64 :59)
* single GPU  — ``cifar10_128batch.py`` (device=cuda :19, bs=128 :59)
* MPI + DDP   — ``cifar10_mpi_mobilenet_224.py`` (bs=128/rank :117, seed 42 :58)

Here those are presets of one :class:`TrainConfig`.
"""
import argparse
import dataclasses
import typing
from dataclasses import dataclass, field
from typing import Optional, Tuple


@dataclass
class TrainConfig:
    # model
    model: str = "mobilenet_v2"
    num_classes: int = 10
    pretrained: Optional[str] = None          # path to a torchvision-format state_dict
    img_size: int = 224                       # IMG_SIZE (:28)
    # optimisation (reference :75-77)
    batch_size: int = 128                     # per process
    epochs: int = 20
    lr: float = 1e-4
    betas: Tuple[float, float] = (0.9, 0.999)
    eps: float = 1e-8
    weight_decay: float = 0.0
    step_size: int = 10                       # StepLR
    gamma: float = 0.1
    scale_lr: bool = False                    # linear LR scaling with world size (off = reference)
    # data
    data: str = "cifar10"                     # cifar10 | synthetic | synthetic-hard
    data_root: str = "./data"
    synthetic_train_size: int = 50000
    synthetic_test_size: int = 10000
    synthetic_signal: Optional[float] = None  # synthetic-hard: class-template strength (None: generator default)
    augment: str = "gpu"                      # gpu (fused HIP kernel) | torch (reference-semantics torch ops) | none
    num_workers: int = 2
    # execution
    device: str = "auto"                      # auto | cpu | cuda
    backend: str = "auto"                     # auto (hip on GPU, torch on CPU) | hip | torch
    precision: str = "bf16"                   # bf16 | fp32 (torch backend only) | fp8 (hip: e4m3 forward 1x1 GEMMs)
    seed: Optional[int] = 42
    graph: bool = False                       # hipGraph capture of the step (hip backend; eager + side stream measured faster)
    deterministic: bool = False
    # distributed
    dist_backend: str = "auto"                # auto (nccl on GPU = RCCL, gloo on CPU)
    bucket_mb: Optional[float] = None         # gradient all-reduce bucket cap (MiB); None: ~total/6
    first_bucket_mb: float = 1.0
    grad_reduce_dtype: str = "fp32"           # fp32 | bf16
    bn_sync: str = "eval"                     # broadcast (every step, reference DDP default) | eval (before eval/save) | none
    global_accuracy: bool = True              # also all-reduce correct/total (reference reports rank-local)
    # checkpoint / logging
    save_path: Optional[str] = None           # best-model .pth (defaults per mode)
    ckpt_dir: Optional[str] = None            # full-state resume checkpoints
    resume: Optional[str] = None
    log_format: str = "serial"                # serial | ddp (reference line formats)
    max_steps_per_epoch: Optional[int] = None
    eval_every: int = 1
    profile: bool = False                     # roctx ranges + per-step HIP-event timing summary per epoch
    watchdog_s: float = 0.0                   # >0: abort a rank that makes no progress for this long (s)
    #                                           (the native communicator's collective watchdog is separate:
    #                                           on for every multi-rank run, PGDIST_COMM_TIMEOUT)
    dist_timeout_s: float = 1800.0            # collective timeout (init_process_group)

    def replace(self, **kw) -> "TrainConfig":
        return dataclasses.replace(self, **kw)


PRESETS = {
    # cifar10_serial_mobilenet_224.py
    "serial": dict(device="cpu", batch_size=64, backend="torch", precision="fp32", augment="torch",
                   save_path="best_mobilenetv2_cifar10_224.pth", log_format="serial", seed=None),
    # cifar10_128batch.py
    "gpu128": dict(device="cuda", batch_size=128, save_path="best_mobilenetv2_cifar10_224.pth",
                   log_format="serial", seed=None),
    # cifar10_mpi_mobilenet_224.py
    # (bn_sync="broadcast": the reference DDP's broadcast_buffers=True, rank 0's BN running statistics
    #  sent before every training forward; --bn-sync eval is the faster option: sync before eval/save)
    "mpi": dict(batch_size=128, save_path="best_mobilenetv2_cifar10_224_mpi.pth", log_format="ddp", seed=42,
                bn_sync="broadcast", watchdog_s=1800.0),
    # BASELINE.json config 5: MobileNetV2 fp8 (e4m3 forward GEMMs), bs 512 per GPU, DDP
    "mpi_fp8": dict(batch_size=512, precision="fp8", backend="hip",
                    save_path="best_mobilenetv2_cifar10_224_mpi_fp8.pth", log_format="ddp", seed=42,
                    watchdog_s=1800.0),
}


def preset(name: str, **overrides) -> TrainConfig:
    cfg = TrainConfig(**PRESETS[name])
    return cfg.replace(**overrides) if overrides else cfg


def add_cli_args(p: argparse.ArgumentParser) -> argparse.ArgumentParser:
    for f in dataclasses.fields(TrainConfig):
        name = "--" + f.name.replace("_", "-")
        if f.type in (bool, "bool"):
            p.add_argument(name, dest=f.name, type=_str2bool, default=None)
        elif f.name == "betas":
            p.add_argument(name, dest=f.name, type=float, nargs=2, default=None)
        else:
            t = f.type
            args = [a for a in typing.get_args(t) if a is not type(None)]   # Optional[X] -> X
            if len(args) == 1:
                t = args[0]
            typ = {"int": int, "float": float, "Optional[int]": int,
                   "Optional[float]": float}.get(str(t), None)
            if typ is None:
                typ = int if t is int else float if t is float else str
            p.add_argument(name, dest=f.name, type=typ, default=None)
    return p


def _str2bool(s: str) -> bool:
    return str(s).lower() in ("1", "true", "yes", "on")


def config_from_args(args: argparse.Namespace, base: Optional[TrainConfig] = None) -> TrainConfig:
    base = base or TrainConfig()
    kw = {f.name: getattr(args, f.name) for f in dataclasses.fields(TrainConfig)
          if getattr(args, f.name, None) is not None}
    if "betas" in kw:
        kw["betas"] = tuple(kw["betas"])
    return base.replace(**kw)
