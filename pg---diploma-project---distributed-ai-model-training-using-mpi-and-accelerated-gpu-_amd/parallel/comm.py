"""Native data-parallel communicator: RCCL and peer-to-peer xGMI collectives driven from C++
(``csrc/runtime/comm.cpp``, ``csrc/kernels/allreduce.hip``) on a dedicated HIP stream.

Reference: the NCCL collectives behind ``DistributedDataParallel`` and the explicit metric
all-reduces (``cifar10_mpi_mobilenet_224.py:34-35,142-145,187-196,215-224``; SURVEY.md §2.4,
§2.7 N4-N8).  There they are issued by c10d's Python-visible work objects; here every
collective of a training step is a native launch-plan op (the replayed step contains no
Python), ordered after its producer streams by events and joined back by the consumer.

Bootstrap: the RCCL unique id and the P2P staging buffers' IPC handles travel through the
c10d TCPStore of the default process group (whatever its backend: the gloo default group of
a one-GPU multi-process rehearsal can bootstrap a P2P-only communicator).

Algorithms (``CommAlgo``): ``rccl`` (ncclAllReduce), ``oneshot`` and ``twoshot`` (P2P
kernels reading all peers over xGMI at once).  :meth:`NativeComm.autotune` times every
available algorithm on the real buckets at start-up, takes the MAX over ranks (so every rank
picks the same one) and validates the P2P result against an exact integer pattern first
(a P2P path that times out or miscomputes is dropped on every rank).
"""
import itertools
import os
from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist

from ..ops._lib import lib

ALGOS = {"rccl": 0, "oneshot": 1, "twoshot": 2}
ALGO_NAMES = {v: k for k, v in ALGOS.items()}
_SEQ = itertools.count()


class CommError(RuntimeError):
    """A native collective failed (peer timeout, out-of-step peer, RCCL error)."""


def _stream_handle(s) -> int:
    return s.cuda_stream if hasattr(s, "cuda_stream") else int(s)


def _ptrs(ts) -> List[int]:
    ts = ts if isinstance(ts, (list, tuple)) else [ts]
    for t in ts:
        if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
            raise TypeError("native collectives take contiguous fp32 device tensors")
    return [t.data_ptr() for t in ts]


def host_allreduce(t: torch.Tensor, op=None) -> torch.Tensor:
    """All-reduce of a small host tensor over the default process group (through the device
    when the group is RCCL's)."""
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return t
    op = op or dist.ReduceOp.SUM
    if dist.get_backend() == "nccl":
        d = t.to(torch.device("cuda", torch.cuda.current_device()))
        dist.all_reduce(d, op=op)
        return d.cpu()
    dist.all_reduce(t, op=op)
    return t


def default_store():
    if not (dist.is_available() and dist.is_initialized()):
        return None
    from torch.distributed.distributed_c10d import _get_default_store
    return _get_default_store()


class NativeComm:
    """One communicator of ``world`` ranks (this process is ``rank``) on ``device``.

    ``use_rccl``: create an RCCL communicator (ids through ``store``).  ``p2p_bytes`` > 0:
    allocate an uncached staging buffer of that region size and map every peer's (all ranks
    must be on this node).  ``nlocal == world`` builds the single-process emulation of
    ``world`` ranks on one GPU (P2P only)."""

    # process exit status when the watchdog finds a stalled collective (EX_TEMPFAIL)
    STALL_EXIT = 75

    def __init__(self, rank: int, world: int, device: torch.device, store=None, use_rccl: bool = True,
                 p2p_bytes: int = 0, blocks: Optional[int] = None, timeout_s: Optional[float] = None,
                 emulate: bool = False, tag: Optional[str] = None, watchdog_s: Optional[float] = None):
        self.rank, self.world, self.device = rank, world, device
        self.emulated = emulate
        self.nlocal = world if emulate else 1
        blocks = blocks or int(os.environ.get("PGDIST_P2P_BLOCKS", "32"))
        # PGDIST_COMM_TIMEOUT (s): a P2P barrier gives up after it; the watchdog aborts an RCCL
        # collective that has not completed that long after it started (P2P ones: twice that)
        timeout_s = timeout_s or float(os.environ.get("PGDIST_COMM_TIMEOUT", "60"))
        region = (int(p2p_bytes) + 255) // 256 * 256
        tag = tag or f"pgdist/comm/{next(_SEQ)}"
        uid = b""
        if use_rccl and not emulate:
            if world > 1:
                if store is None:
                    raise RuntimeError("NativeComm: a store is needed to exchange the RCCL unique id")
                if rank == 0:
                    uid = lib().comm_unique_id()
                    store.set(tag + "/nccl_id", uid)
                else:
                    uid = store.get(tag + "/nccl_id")
            else:
                uid = lib().comm_unique_id()
        self.has_rccl = bool(uid)
        self.id = lib().comm_create(0 if emulate else rank, world, device.index or 0, uid, region, blocks,
                                    self.nlocal, float(timeout_s))
        self.region = region
        self.blocks = blocks
        self.timeout_s = float(timeout_s)
        self.has_p2p = False
        self.p2p_error = None
        if region > 0:
            if emulate or world == 1:
                self.has_p2p = True
            else:
                if store is None:
                    raise RuntimeError("NativeComm: a store is needed to exchange the P2P IPC handles")
                try:
                    h = lib().comm_p2p_handle(self.id)
                except Exception as e:   # noqa: BLE001 - this rank publishes an empty handle
                    h, self.p2p_error = b"", repr(e)
                store.set(f"{tag}/ipc/{rank}", h)
                handles = [store.get(f"{tag}/ipc/{r}") for r in range(world)]
                if self.p2p_error is None and all(handles):
                    try:
                        lib().comm_p2p_open(self.id, handles)
                        self.has_p2p = True
                    except Exception as e:   # noqa: BLE001 - agreed on in validate_p2p
                        self.p2p_error = repr(e)
                elif self.p2p_error is None:
                    self.p2p_error = "a peer could not export its staging buffer"
        self.stream = torch.cuda.ExternalStream(lib().comm_stream(self.id), device=device)
        # the comm watchdog: on by default for a real multi-rank job (a dead peer inside an RCCL
        # collective would otherwise hang every rank), off for world 1 / the one-process emulation
        if watchdog_s is None:
            watchdog_s = self.timeout_s if (world > 1 and not emulate) else 0.0
        self.set_watchdog(watchdog_s)
        self._err_host = torch.zeros(1, dtype=torch.int32).pin_memory() if device.type == "cuda" else None
        self._err_polled = False

    # ------------------------------------------------------------------ factory
    @classmethod
    def for_process_group(cls, device: torch.device, use_rccl: bool = True, p2p_bytes: int = 0, **kw):
        """Communicator over the default process group's ranks (store = its TCPStore)."""
        world = dist.get_world_size() if dist.is_initialized() else 1
        rank = dist.get_rank() if dist.is_initialized() else 0
        return cls(rank, world, device, store=default_store(), use_rccl=use_rccl, p2p_bytes=p2p_bytes, **kw)

    # ------------------------------------------------------------------ collectives
    def allreduce(self, bufs, algo="rccl", bf16_wire: bool = False, wait: Sequence = ()):
        """In-place fp32 sum of ``bufs`` (one tensor; one per emulated rank) over the ranks, on the
        comm stream after every stream in ``wait`` (default: the current stream)."""
        a = ALGOS[algo] if isinstance(algo, str) else int(algo)
        ptrs = _ptrs(bufs)
        n = (bufs[0] if isinstance(bufs, (list, tuple)) else bufs).numel()
        ws = [_stream_handle(s) for s in (wait or [torch.cuda.current_stream(self.device)])]
        lib().comm_allreduce(self.id, ptrs, n, a, bool(bf16_wire), ws)

    def broadcast(self, bufs, root: int = 0, algo="rccl", wait: Sequence = ()):
        a = ALGOS[algo] if isinstance(algo, str) else int(algo)
        if a == ALGOS["twoshot"]:
            a = ALGOS["oneshot"]   # the P2P broadcast has one form
        ptrs = _ptrs(bufs)
        n = (bufs[0] if isinstance(bufs, (list, tuple)) else bufs).numel()
        ws = [_stream_handle(s) for s in (wait or [torch.cuda.current_stream(self.device)])]
        lib().comm_broadcast(self.id, ptrs, n, int(root), a, ws)

    def allreduce_f64(self, t: torch.Tensor, op: str = "sum", wait: Sequence = ()):
        assert t.is_cuda and t.dtype == torch.float64 and t.is_contiguous()
        ws = [_stream_handle(s) for s in (wait or [torch.cuda.current_stream(self.device)])]
        lib().comm_allreduce_f64(self.id, t.data_ptr(), t.numel(), 0 if op == "sum" else 2, ws)

    def join(self, stream=None):
        """``stream`` (default: current) waits for every collective issued so far."""
        s = stream or torch.cuda.current_stream(self.device)
        lib().comm_join(self.id, _stream_handle(s))

    def time_allreduce(self, bufs, algo, bf16_wire=False, iters=20) -> float:
        """Microseconds per all-reduce of ``bufs`` back to back on the comm stream (collective:
        every rank must call it with the same arguments)."""
        a = ALGOS[algo] if isinstance(algo, str) else int(algo)
        n = (bufs[0] if isinstance(bufs, (list, tuple)) else bufs).numel()
        return lib().comm_time_allreduce(self.id, _ptrs(bufs), n, a, bool(bf16_wire), int(iters))

    def error(self) -> int:
        """0, or this rank's error code: P2P error-word bits (1 peer timeout, 2 peer out of step,
        4 poisoned) | RCCL async error << 8 | 1 << 16 for a synchronous RCCL failure.  Nonzero
        poisons the communicator: every later collective raises (synchronises the comm stream)."""
        return lib().comm_error(self.id)

    def error_string(self) -> str:
        return lib().comm_error_string(self.id)

    def check(self):
        """Raise if THIS rank's communicator failed (local check, no collective)."""
        e = self.error()
        if e:
            raise CommError(f"native communicator error 0x{e:x} on rank {self.rank}: {self.error_string()}")

    def check_all(self, group=None) -> int:
        """Collective health check (every rank must call it): this rank's error code is
        all-reduced (MAX) over the default process group, so a failure on ANY rank raises
        :class:`CommError` on EVERY rank — no rank is left waiting in a later collective for a
        peer that aborted.  Returns 0 when every rank is healthy."""
        e = self.error()
        if self.world > 1 and not self.emulated and dist.is_available() and dist.is_initialized():
            t = host_allreduce(torch.tensor([float(e), float(self.rank if e else -1)], dtype=torch.float64),
                               dist.ReduceOp.MAX)
            worst, who = int(t[0].item()), int(t[1].item())
        else:
            worst, who = e, self.rank
        if worst:
            mine = f"; this rank: {self.error_string() or 'healthy'}"
            if not e:   # a peer failed: this rank's communicator is unusable too
                lib().comm_poison(self.id, f"rank {who} failed with error 0x{worst:x}")
            raise CommError(f"native communicator failed (error 0x{worst:x}, reported by rank {who}){mine}")
        return 0

    # ------------------------------------------------------------------ failure detection
    def set_watchdog(self, seconds: float, exit_status: Optional[int] = None):
        """Watchdog deadline (s; 0 = off): a collective that started on the comm stream and has not
        completed ``seconds`` later (P2P: twice that) prints which one, poisons the communicator,
        calls ncclCommAbort and ends the process with ``exit_status`` (default STALL_EXIT; 0:
        poison and abort only)."""
        code = self.STALL_EXIT if exit_status is None else int(exit_status)
        lib().comm_set_watchdog(self.id, float(seconds), code)

    @property
    def watchdog_s(self) -> float:
        return lib().comm_watchdog(self.id)

    def inject_stall(self, seconds: float):
        """Fault injection: the next collective is preceded on the comm stream (after its start
        marker) by a kernel that spins ``seconds`` -- what a dead peer looks like to the watchdog."""
        lib().comm_inject_stall(self.id, float(seconds))

    @property
    def error_word(self) -> int:
        """Device address of this rank's error word (the fused Adam skips its update while set)."""
        return lib().comm_error_word(self.id)

    def poll_error(self) -> int:
        """Cheap per-step failure check, no synchronisation: returns the error word copied
        asynchronously by the PREVIOUS call (0 on the first) and enqueues the next copy on the comm
        stream behind the collectives issued so far."""
        v = int(self._err_host[0]) if self._err_polled else 0
        lib().comm_error_async(self.id, self._err_host.data_ptr())
        self._err_polled = True
        return v

    def rccl_ranks(self) -> int:
        """Ranks of the RCCL communicator (ncclCommCount), 0 without one."""
        return lib().comm_rccl_ranks(self.id) if self.has_rccl else 0

    def close(self):
        if self.id is not None:
            lib().comm_destroy(self.id)
            self.id = None

    # ------------------------------------------------------------------ algorithm choice
    def available_algos(self) -> List[str]:
        out = []
        if self.has_rccl:
            out.append("rccl")
        if self.has_p2p:
            out += ["oneshot", "twoshot"]
        return out

    def set_timeout(self, seconds: float):
        """P2P barrier give-up (seconds) for collectives issued from now on."""
        lib().comm_set_timeout(self.id, float(seconds))
        self.timeout_s = float(seconds)

    def _agree(self, ok: bool) -> bool:
        if self.world == 1 or self.emulated:
            return ok
        return host_allreduce(torch.tensor([1.0 if ok else 0.0], dtype=torch.float64),
                              dist.ReduceOp.MIN).item() > 0

    def validate_p2p(self, timeout_s: float = 5.0) -> bool:
        """Exact-integer P2P all-reduce check (every rank contributes rank+1+i%7, one-shot and
        two-shot, fp32 and bf16 wire): True on every rank iff the staging was mapped and every
        call succeeded on every rank.  Agreement (default process group) before the first
        kernel and after each call, so a rank whose setup failed or a broken call costs at most
        one barrier timeout (shortened to ``timeout_s`` meanwhile), never a hang or a mismatch."""
        if self.emulated:
            return self.has_p2p
        if not self._agree(self.has_p2p and self.p2p_error is None):
            self.has_p2p = False
            return False
        n = 1 << 16
        keep = self.timeout_s
        self.set_timeout(timeout_s)
        try:
            base = torch.arange(n, device=self.device, dtype=torch.float32).remainder_(7)
            expect = base * self.world + self.world * (self.world + 1) / 2
            for algo in ("oneshot", "twoshot"):
                for bf in (False, True):
                    ok = True
                    try:
                        t = base + (self.rank + 1)
                        self.allreduce(t, algo, bf)
                        self.join()
                        torch.cuda.synchronize(self.device)
                        err = self.error()
                        if err:
                            self.p2p_error = f"error 0x{err:x}: {self.error_string()}"
                        ok = err == 0 and torch.equal(t, expect)
                    except Exception as e:   # noqa: BLE001 - reported, then P2P is off everywhere
                        self.p2p_error = repr(e)
                        ok = False
                    if not self._agree(ok):
                        self.has_p2p = False
                        # every rank abandons P2P: un-poison so the RCCL path stays usable
                        lib().comm_clear_error(self.id)
                        return False
        finally:
            self.set_timeout(keep)
        return True

    def validate_layout(self, sizes: Sequence[int], algos: Sequence[str], bf16_wire: bool = False,
                        bcast_n: int = 0, timeout_s: float = 5.0) -> bool:
        """The training step's own collectives at their real sizes, issued back to back as the
        step issues them: one all-reduce per bucket (``sizes`` / ``algos``; P2P buckets only --
        RCCL validates itself) followed by the per-step BN-buffer broadcast of ``bcast_n`` floats,
        each checked against an exact integer pattern.  True on every rank iff every result is
        exact on every rank (agreement over the default process group)."""
        p2p = [(n, a) for n, a in zip(sizes, algos) if a in ("oneshot", "twoshot")]
        if self.emulated or not self.has_p2p or (not p2p and not bcast_n):
            return True
        keep = self.timeout_s
        self.set_timeout(timeout_s)
        ok = True
        try:
            bufs, exps = [], []
            for n, a in p2p:
                base = torch.arange(n, device=self.device, dtype=torch.float32).remainder_(7)
                t = base + (self.rank + 1)
                self.allreduce(t, a, bf16_wire)
                bufs.append(t)
                exps.append(base * self.world + self.world * (self.world + 1) / 2)
            if bcast_n:
                pat = torch.arange(bcast_n, device=self.device, dtype=torch.float32).remainder_(11)
                t = pat + 1 if self.rank == 0 else torch.full_like(pat, -1.0)
                self.broadcast(t, 0, "oneshot")
                bufs.append(t)
                exps.append(pat + 1)
            self.join()
            torch.cuda.synchronize(self.device)
            err = self.error()
            if err:
                self.p2p_error = f"error 0x{err:x}: {self.error_string()}"
            ok = err == 0 and all(torch.equal(b, e) for b, e in zip(bufs, exps))
            if not ok and self.p2p_error is None:
                self.p2p_error = "a bucket-sized P2P collective miscomputed"
        except Exception as e:   # noqa: BLE001 - reported, then agreed on
            self.p2p_error, ok = repr(e), False
        finally:
            self.set_timeout(keep)
        ok = self._agree(ok)
        if not ok:
            lib().comm_clear_error(self.id)
        return ok

    def autotune(self, sizes: Sequence[int], candidates: Optional[Sequence[str]] = None, bf16_wire=False,
                 iters: int = 10, measure: bool = False) -> Dict[int, str]:
        """Fastest algorithm per all-reduce size (elements), by the MAX over ranks of the measured
        time, identical on every rank (``self.tuning``: the times; with a single candidate they
        are measured only when ``measure``)."""
        cands = [c for c in (candidates or self.available_algos()) if c in self.available_algos()]
        if bf16_wire:
            cands = [c for c in cands if c != "rccl"]
        if not cands:
            raise RuntimeError("autotune: no algorithm available")
        if len(cands) == 1 and not measure:
            return {int(s): cands[0] for s in sizes}
        uniq = sorted({int(s) for s in sizes})
        scratch = torch.zeros(max(uniq), dtype=torch.float32, device=self.device)
        times = torch.zeros(len(uniq), len(cands), dtype=torch.float64)
        for i, s in enumerate(uniq):
            for j, c in enumerate(cands):
                times[i, j] = self.time_allreduce(scratch[:s], c, bf16_wire, iters)
        if self.world > 1 and not self.emulated:
            times = host_allreduce(times, dist.ReduceOp.MAX)
        self.tuning = {s: {c: float(times[i, j]) for j, c in enumerate(cands)} for i, s in enumerate(uniq)}
        return {s: cands[int(times[i].argmin())] for i, s in enumerate(uniq)}
