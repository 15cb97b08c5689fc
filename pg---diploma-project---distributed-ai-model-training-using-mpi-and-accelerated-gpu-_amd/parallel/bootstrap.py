"""Process bootstrap / rank discovery and ``torch.distributed`` initialisation.

Reference (``cifar10_mpi_mobilenet_224.py:24-48``): rank/size come from
``mpi4py.MPI.COMM_WORLD``, then ``MASTER_ADDR=localhost`` / ``MASTER_PORT=29500``
are written into the environment and ``init_process_group("nccl"|"gloo")`` is
called; the device is ``cuda:{rank % device_count}``.  That hard-codes a single
node (SURVEY.md §2.3 "Spatial / multi-node").

Here discovery is layered and multi-node correct:

1. torchrun / explicit env: ``RANK``, ``WORLD_SIZE``, ``LOCAL_RANK``
2. Open MPI (``mpirun``): ``OMPI_COMM_WORLD_RANK/SIZE/LOCAL_RANK`` — read from
   the environment, so mpi4py is optional (it is not installed here); MPICH/PMI
   ``PMI_RANK/PMI_SIZE`` likewise
3. SLURM (``srun``): ``SLURM_PROCID``, ``SLURM_NTASKS``, ``SLURM_LOCALID``;
   ``MASTER_ADDR`` = first host of ``SLURM_JOB_NODELIST``
4. mpi4py, if importable and nothing above matched
5. single process

The collective backend is ``nccl`` on GPU, which on ROCm *is* RCCL (xGMI
peer-to-peer inside an MI355X node), and ``gloo`` on CPU.
"""
import datetime
import os
import re
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistInfo:
    rank: int = 0
    world_size: int = 1
    local_rank: int = 0
    local_world_size: int = 1
    master_addr: str = "127.0.0.1"
    master_port: int = 29500
    source: str = "single"

    @property
    def is_distributed(self) -> bool:
        return self.world_size > 1

    @property
    def is_main(self) -> bool:
        return self.rank == 0


def _first_slurm_host(nodelist: str) -> str:
    """Expand the first host of a SLURM nodelist such as ``gpu[008-011,020],cn1``."""
    m = re.match(r"^([^,\[]+)(\[([^\]]+)\])?", nodelist)
    if not m:
        return nodelist
    prefix, _, ranges = m.groups()
    if not ranges:
        return prefix
    first = ranges.split(",")[0].split("-")[0]
    return prefix + first


def discover(env: Optional[dict] = None) -> DistInfo:
    env = os.environ if env is None else env
    port = int(env.get("MASTER_PORT", 29500))
    addr = env.get("MASTER_ADDR")
    if "RANK" in env and "WORLD_SIZE" in env:
        ws = int(env["WORLD_SIZE"])
        return DistInfo(int(env["RANK"]), ws, int(env.get("LOCAL_RANK", 0)),
                        int(env.get("LOCAL_WORLD_SIZE", ws)), addr or "127.0.0.1", port, "env")
    if "OMPI_COMM_WORLD_RANK" in env:
        ws = int(env["OMPI_COMM_WORLD_SIZE"])
        return DistInfo(int(env["OMPI_COMM_WORLD_RANK"]), ws,
                        int(env.get("OMPI_COMM_WORLD_LOCAL_RANK", 0)),
                        int(env.get("OMPI_COMM_WORLD_LOCAL_SIZE", ws)), addr or "127.0.0.1", port, "openmpi")
    if "PMI_RANK" in env and "PMI_SIZE" in env:
        ws = int(env["PMI_SIZE"])
        lr = int(env.get("MPI_LOCALRANKID", env.get("PMI_LOCAL_RANK", 0)))
        return DistInfo(int(env["PMI_RANK"]), ws, lr, int(env.get("MPI_LOCALNRANKS", ws)),
                        addr or "127.0.0.1", port, "pmi")
    if "SLURM_PROCID" in env and "SLURM_NTASKS" in env and int(env["SLURM_NTASKS"]) > 1:
        ws = int(env["SLURM_NTASKS"])
        nodelist = env.get("SLURM_JOB_NODELIST", env.get("SLURM_NODELIST", "127.0.0.1"))
        per_node = str(env.get("SLURM_NTASKS_PER_NODE", ws)).split("(")[0].split(",")[0]
        return DistInfo(int(env["SLURM_PROCID"]), ws, int(env.get("SLURM_LOCALID", 0)),
                        int(per_node), addr or _first_slurm_host(nodelist), port, "slurm")
    try:  # mpi4py (reference path) — only if launched under an MPI runtime
        from mpi4py import MPI  # noqa: F401
        comm = MPI.COMM_WORLD
        if comm.Get_size() > 1:
            local = comm.Split_type(MPI.COMM_TYPE_SHARED)
            return DistInfo(comm.Get_rank(), comm.Get_size(), local.Get_rank(), local.Get_size(),
                            addr or "127.0.0.1", port, "mpi4py")
    except Exception:
        pass
    return DistInfo()


def init_distributed(backend: str = "auto", device: str = "auto",
                     timeout_s: float = 600.0, info: Optional[DistInfo] = None):
    """Initialise the process group; returns ``(info, device, backend)``.

    Device binding uses ``LOCAL_RANK`` (not ``rank % device_count`` as in the
    reference, which assumed block rank placement)."""
    info = info or discover()
    use_cuda = torch.cuda.is_available() if device == "auto" else device.startswith("cuda")
    if use_cuda:
        n = torch.cuda.device_count()
        local = info.local_rank % max(n, 1)
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    if backend == "auto":
        backend = "nccl" if use_cuda else "gloo"
    if info.is_distributed and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", info.master_addr)
        os.environ.setdefault("MASTER_PORT", str(info.master_port))
        kw = {}
        if backend == "nccl":
            kw["device_id"] = dev
        dist.init_process_group(backend=backend, init_method="env://", rank=info.rank,
                                world_size=info.world_size,
                                timeout=datetime.timedelta(seconds=timeout_s), **kw)
    return info, dev, backend


def cleanup():
    """Reference ``cleanup()`` (:47-48)."""
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def barrier(device: Optional[torch.device] = None):
    if dist.is_available() and dist.is_initialized():
        if device is not None and device.type == "cuda" and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()
