"""Data-parallel gradient synchronisation over RCCL (xGMI inside an MI355X node).

Reference: ``DistributedDataParallel(model, device_ids=[local_rank])`` with all
defaults (``cifar10_mpi_mobilenet_224.py:142-145``): rank-0 parameter broadcast
at construction, BN-buffer broadcast every forward, bucketed (1 MiB then 25 MiB)
asynchronous all-reduce AVG hooked into autograd.

Re-design for MI355X:

* gradients are written by the wgrad kernels straight into ONE flat fp32
  buffer laid out in backward-completion order, so a bucket is a contiguous
  slice and needs no packing copy;
* the executor reports which parameters are final after every backward layer;
  when a bucket is complete its all-reduce is enqueued immediately
  (``async_op=True``: RCCL runs on its own HIP stream, ordered after the
  kernels that produced the bucket), overlapping the rest of backward;
* the whole MobileNetV2 gradient is only 8.95 MB, so on 7 point-to-point xGMI
  links a bucket is latency-bound, not bandwidth-bound: the default is a small
  first bucket (classifier + last layers become ready first, ~1 MiB) followed by
  ~4 MiB buckets — few collectives, started early;
* averaging (1/world) is folded into the fused Adam kernel's gradient read,
  so there is no separate divide pass;
* optional bf16 wire format (``reduce_dtype=bfloat16``) halves the bytes.

The same class works with the ``gloo`` backend on CPU (multi-process tests).
"""
import os
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


def build_buckets(ranges: Sequence[Tuple[str, int, int]], cap_bytes: int, first_cap_bytes: int,
                  elem_size: int = 4, last_cap_bytes: int = 0) -> List[Tuple[int, int, List[str]]]:
    """Greedy contiguous bucketing of (name, start, end) ranges given in buffer order.

    ``last_cap_bytes`` > 0: the trailing ranges that fit in it (at least one) form a last bucket
    of their own -- the stem side of the network, whose gradients are final only at the very
    end of the backward, so that bucket's all-reduce is exposed and should be small."""
    ranges = list(ranges)
    tail: List[Tuple[str, int, int]] = []
    if last_cap_bytes > 0 and len(ranges) > 1:
        k = len(ranges) - 1
        while k > 1 and (ranges[-1][2] - ranges[k - 1][1]) * elem_size <= last_cap_bytes:
            k -= 1
        ranges, tail = ranges[:k], ranges[k:]
    buckets: List[Tuple[int, int, List[str]]] = []
    cur_names: List[str] = []
    cur_start: Optional[int] = None
    cur_end = 0
    for name, s, e in ranges:
        if cur_start is None:
            cur_start = s
        cur_names.append(name)
        cur_end = e
        cap = first_cap_bytes if not buckets else cap_bytes
        if (cur_end - cur_start) * elem_size >= cap:
            buckets.append((cur_start, cur_end, cur_names))
            cur_names, cur_start = [], None
    if cur_names:
        buckets.append((cur_start, cur_end, cur_names))
    if tail:
        buckets.append((tail[0][1], tail[-1][2], [n for n, _, _ in tail]))
    return buckets


# main-stream cost of one bucket launch (us): the side-stream join and the event waits of the
# collective put barrier packets on the main stream (~5-8 us of idle each, docs/PERF_NOTES.md)
BUCKET_JOIN_US = 8.0


def simulate_buckets(buckets, ready_us: Dict[str, float], t_bwd_us: float, t_ar,
                     join_us: float = BUCKET_JOIN_US) -> float:
    """Exposed data-parallel cost (us) of a bucket layout: bucket b's all-reduce starts when its
    last gradient is final (``ready_us``: offset from the backward's start) and the comm stream is
    free, and takes ``t_ar(elements)``; what runs past the end of the backward (``t_bwd_us``) is
    exposed, and every bucket launch costs the main stream ``join_us``.  This is the quantity
    the bucket size trades off: small buckets start early (overlap) but each pays a launch."""
    t = 0.0
    for s, e, names in buckets:
        r = max((ready_us.get(n, t_bwd_us) for n in names), default=t_bwd_us)
        t = max(r, t) + join_us + t_ar(e - s)
    return max(0.0, t - t_bwd_us) + join_us * len(buckets)


BUCKET_CAPS_MB = (0.25, 0.5, 1.0, 2.0, 4.0, 8.0, 16.0, 32.0)
LAST_CAPS_MB = (0.0, 0.125, 0.25, 0.5, 1.0, 1.5)


def candidate_layouts(ranges, first_mb: float, grad_mb: float, aligned=lambda b: b):
    """{(cap MiB, last cap MiB): buckets} over the candidate grid (caps up to twice the gradient)."""
    out = {}
    for c in BUCKET_CAPS_MB:
        if c > 2 * max(grad_mb, 0.25):
            continue
        for lc in LAST_CAPS_MB:
            out[(c, lc)] = aligned(build_buckets(ranges, int(c * 2 ** 20), int(first_mb * 2 ** 20),
                                                 last_cap_bytes=int(lc * 2 ** 20)))
    return out


def choose_layout(cands, ready_us, t_bwd_us, t_ar, join_us: float = BUCKET_JOIN_US):
    """(cost table, best key): the candidate with the least simulated exposed cost (ties: fewer
    buckets, then the larger cap)."""
    cost = {k: simulate_buckets(b, ready_us, t_bwd_us, t_ar, join_us) for k, b in cands.items()}
    best = min(cost, key=lambda k: (round(cost[k], 3), len(cands[k]), -k[0], -k[1]))
    return cost, best


def estimate_ready_times(model: torch.nn.Module, img_size: int, t_bwd_us: float) -> Dict[str, float]:
    """Model of when every parameter's gradient becomes final during the backward (us after its
    start), used to size the gradient buckets before the step can be measured: the backward
    visits the layers in reverse forward order and a layer costs ~ its input + output activation
    elements (the network is memory-bound on MI355X).  Shapes from one forward of
    a CPU copy at a quarter of the resolution (every map scales alike)."""
    import copy
    m = copy.deepcopy(model).cpu().float().eval()
    order: List[Tuple[str, float]] = []
    hooks = []
    for name, mod in m.named_modules():
        if any(True for _ in mod.parameters(recurse=False)):
            def hook(mod_, inp, out, name=name):
                n_in = sum(t.numel() for t in inp if torch.is_tensor(t))
                order.append((name, float(n_in + out.numel())))
            hooks.append(mod.register_forward_hook(hook))
    S = max(32, (img_size // 4 + 31) // 32 * 32)
    with torch.no_grad():
        m(torch.zeros(1, 3, S, S))
    for h in hooks:
        h.remove()
    total = sum(c for _, c in order) or 1.0
    ready, acc = {}, 0.0
    for name, c in reversed(order):
        acc += c
        for pn, _ in dict(m.named_modules())[name].named_parameters(recurse=False):
            ready[f"{name}.{pn}" if name else pn] = acc / total * t_bwd_us
    return ready


def auto_bucket_mb(grad_bytes: int) -> float:
    """Bucket cap for a gradient of ``grad_bytes``: ~6 buckets (1-32 MiB).  The bucket holding the
    stem-side parameters completes last and its all-reduce is exposed after the backward, so it
    should be small; too many buckets pay RCCL's per-call latency (MobileNetV2: 8.95 MB ->
    1.5 MiB buckets, the last one 0.3 MiB; ResNet-50: 102 MB -> 16 MiB)."""
    return min(32.0, max(1.0, grad_bytes / 2 ** 20 / 6))


class BucketedGradReducer:
    def __init__(self, flat_grad: torch.Tensor, ranges: Sequence[Tuple[str, int, int]],
                 bucket_cap_mb: Optional[float] = None, first_bucket_mb: float = 1.0,
                 reduce_dtype: torch.dtype = torch.float32, group=None):
        if bucket_cap_mb is None:
            bucket_cap_mb = auto_bucket_mb(flat_grad.numel() * flat_grad.element_size())
        self.grad = flat_grad
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.reduce_dtype = reduce_dtype
        self.bucket_cap_mb = float(bucket_cap_mb)
        self._set_buckets(build_buckets(ranges, int(bucket_cap_mb * 2 ** 20), int(first_bucket_mb * 2 ** 20)))

    def _set_buckets(self, buckets):
        # a bucket covers [start, end) of the flat buffer; extend the last bucket to the
        # buffer end so alignment padding is reduced too (it is zero on every rank)
        self.buckets = buckets
        self.owner: Dict[str, int] = {}
        for bi, (_, _, names) in enumerate(self.buckets):
            for n in names:
                self.owner[n] = bi
        self._pending = [len(b[2]) for b in self.buckets]
        self._next = 0
        self._ready = [False] * len(self.buckets)
        self._works = []
        self._casts = {}
        if self.reduce_dtype != torch.float32:
            for bi, (s, e, _) in enumerate(self.buckets):
                self._casts[bi] = torch.empty(e - s, dtype=self.reduce_dtype, device=self.grad.device)

    @property
    def enabled(self) -> bool:
        return self.world > 1

    def begin(self):
        self._pending = [len(b[2]) for b in self.buckets]
        self._ready = [False] * len(self.buckets)
        self._next = 0
        self._works = []

    def would_launch(self, names: Sequence[str]) -> bool:
        """True if ``mark_ready(names)`` would launch at least one bucket (buckets launch in
        order, so exactly when the next unlaunched bucket becomes complete).  Lets the executor
        skip the side-stream join for the ~100 per-layer calls that launch nothing."""
        if not self.enabled or self._next >= len(self.buckets):
            return False
        if self._ready[self._next]:
            return True
        hit = sum(1 for n in names if self.owner.get(n) == self._next)
        return self._pending[self._next] - hit == 0

    def mark_ready(self, names: Sequence[str]):
        if not self.enabled:
            return
        for n in names:
            bi = self.owner.get(n)
            if bi is None:
                continue
            self._pending[bi] -= 1
            if self._pending[bi] == 0:
                self._ready[bi] = True
        # launch in bucket order (identical on every rank -> matching collectives)
        while self._next < len(self.buckets) and self._ready[self._next]:
            self._launch(self._next)
            self._next += 1

    def _launch(self, bi: int):
        s, e, _ = self.buckets[bi]
        view = self.grad[s:e]
        if self.reduce_dtype != torch.float32:
            buf = self._casts[bi]
            buf.copy_(view)
            w = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            self._works.append((w, bi))
        else:
            w = dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
            self._works.append((w, None))

    def finish(self):
        """Flush any bucket not yet launched and make the current stream wait for all."""
        if not self.enabled:
            return
        while self._next < len(self.buckets):
            self._launch(self._next)
            self._next += 1
        for w, bi in self._works:
            w.wait()
            if bi is not None:
                s, e, _ = self.buckets[bi]
                self.grad[s:e].copy_(self._casts[bi])
        self._works = []


class NativeBucketReducer(BucketedGradReducer):
    """The same bucket schedule as :class:`BucketedGradReducer`, issued through a
    :class:`~pgdist.parallel.comm.NativeComm`: every bucket launch is a native op (the comm
    stream waits for the current stream and the executor's side stream, then RCCL or a P2P
    xGMI kernel reduces the bucket in place) and ``finish`` makes the current stream wait for
    the comm stream.  Nothing here needs Python at replay time: the bookkeeping runs once while
    a launch plan records the step, and the recorded ops are the whole data-parallel part of
    every replayed step (``native = True`` tells the executor to call the hooks directly
    instead of wrapping them in ``plan_py``).

    ``algo``: ``rccl`` | ``oneshot`` | ``twoshot`` | ``auto`` (per bucket: validated P2P
    kernels and RCCL timed on this node at construction, fastest on the slowest rank)."""
    native = True

    def __init__(self, comm, flat_grad: torch.Tensor, ranges: Sequence[Tuple[str, int, int]],
                 bucket_cap_mb: Optional[float] = None, first_bucket_mb: float = 1.0, algo: str = "auto",
                 bf16_wire: bool = False, force: bool = False, ready_us: Optional[Dict[str, float]] = None,
                 t_bwd_us: Optional[float] = None):
        tune_cap = bucket_cap_mb is None
        self.last_bucket_mb = 0.0
        super().__init__(flat_grad, ranges, bucket_cap_mb, first_bucket_mb)
        self.comm = comm
        self.world = comm.world
        self.force = force   # run the bucket collectives even at world size 1 (tests)
        self.side = None     # the executor's side stream (weight-gradient producers)
        self.bf16_wire = bf16_wire
        self._ranges, self._first_mb = list(ranges), first_bucket_mb
        self._set_buckets(self._aligned(self.buckets))
        sizes = [e - s for s, e, _ in self.buckets]
        self.bucket_tuning = None
        if algo == "auto":
            if comm.region > 0 and comm.world > 1 and not comm.validate_p2p():
                print(f"[pgdist] P2P all-reduce unavailable or failed validation ({comm.p2p_error}): RCCL only",
                      flush=True)
            if bf16_wire and comm.world > 1 and not comm.has_p2p:
                if not comm.has_rccl:
                    raise RuntimeError("bf16 gradient wire format: neither the P2P path nor RCCL is available")
                # the bf16 wire is a P2P-kernel option; RCCL reduces fp32 (same result up to the
                # bf16 rounding of the summands; twice the bytes)
                print("[pgdist] bf16 gradient wire needs the P2P path: reducing fp32 over RCCL instead", flush=True)
                bf16_wire = self.bf16_wire = False
            self.tunable = comm.world > 1 and tune_cap and os.environ.get("PGDIST_BUCKET_TUNE", "1") == "1"
            if self.tunable:
                self._tune_bucket_cap(bf16_wire, ready_us, t_bwd_us)
                sizes = [e - s for s, e, _ in self.buckets]
            choice = comm.autotune(sizes, bf16_wire=bf16_wire) if comm.world > 1 else {}
            self.algos = [choice.get(sz, "rccl" if comm.has_rccl else "oneshot") for sz in sizes]
        else:
            self.tunable = False
            self.algos = [algo] * len(sizes)
        if bf16_wire and "rccl" in self.algos:
            raise ValueError("bf16 wire format: P2P algorithms only")

    def _aligned(self, buckets):
        """P2P kernels take multiples of 8 elements: bucket ends move to the next 64-element
        boundary (flat-buffer alignment padding, zero on every rank), the last to the end."""
        n = self.grad.numel()
        return [(s, n if i == len(buckets) - 1 else min(n, (e + 63) // 64 * 64), names)
                for i, (s, e, names) in enumerate(buckets)]

    def _tune_bucket_cap(self, bf16_wire: bool, ready_us: Optional[Dict[str, float]] = None,
                         t_bwd_us: Optional[float] = None):
        """Bucket layout from measurements on this node, scored by EXPOSED communication
        (:func:`simulate_buckets`): every bucket size of every candidate
        layout (cap x last-bucket cap, :func:`candidate_layouts`) is timed with every algorithm
        (NativeComm.autotune: MAX over ranks, so every rank scores identically), the layouts are
        simulated against the gradients' ready times (``ready_us``: measured by
        NativeTrainStep on a warm-up step, else :func:`estimate_ready_times` or a uniform model)
        and the one with the least exposed time wins."""
        grad_mb = self.grad.numel() * 4 / 2 ** 20
        cands = candidate_layouts(self._ranges, self._first_mb, grad_mb, self._aligned)
        sizes = sorted({e - s for b in cands.values() for s, e, _ in b})
        missing = [sz for sz in sizes if sz not in getattr(self.comm, "tuning", {}) or {}]
        if missing:
            self.comm.autotune(sizes, bf16_wire=bf16_wire, iters=5, measure=True)
        best_t = {sz: min(t.values()) for sz, t in self.comm.tuning.items()}
        if ready_us is None:
            # uniform model: parameters become ready evenly over a backward of 3 ms
            n = max(1, len(self._ranges))
            t_bwd_us = 3000.0
            ready_us = {name: (i + 1) / n * t_bwd_us for i, (name, _, _) in enumerate(self._ranges)}
        cost, key = choose_layout(cands, ready_us, float(t_bwd_us), lambda n: best_t[n])
        self.bucket_tuning = {f"{c}/{lc}": round(v, 1) for (c, lc), v in cost.items()}
        self.bucket_cap_mb, self.last_bucket_mb = key
        self._set_buckets(cands[key])

    def retune(self, ready_us: Dict[str, float], t_bwd_us: float):
        """Re-choose the bucket layout from MEASURED gradient ready times (collective: every
        rank calls it with the same, rank-agreed values) and re-pick the algorithms."""
        self._tune_bucket_cap(self.bf16_wire, ready_us, t_bwd_us)
        sizes = [e - s for s, e, _ in self.buckets]
        choice = self.comm.autotune(sizes, bf16_wire=self.bf16_wire) if self.comm.world > 1 else {}
        self.algos = [choice.get(sz, "rccl" if self.comm.has_rccl else "oneshot") for sz in sizes]

    def validate_layout(self, bcast_n: int = 0):
        """Check the chosen buckets' P2P collectives (and the BN broadcast) at their real sizes on
        every rank; on a failure every rank falls back to RCCL for every bucket (or raises
        without RCCL)."""
        if not (self.comm.world > 1 and getattr(self.comm, "has_p2p", False)):
            return True
        sizes = [e - s for s, e, _ in self.buckets]
        if self.comm.validate_layout(sizes, self.algos, self.bf16_wire, bcast_n):
            return True
        if not self.comm.has_rccl or self.bf16_wire:
            raise RuntimeError(f"P2P collectives failed validation at the bucket sizes ({self.comm.p2p_error}) "
                               "and RCCL cannot take over")
        print(f"[pgdist] P2P collectives failed validation at the bucket sizes ({self.comm.p2p_error}): "
              "RCCL for every bucket", flush=True)
        self.comm.has_p2p = False
        self.algos = ["rccl"] * len(sizes)
        return False

    @property
    def enabled(self) -> bool:
        return self.world > 1 or self.force

    def _launch(self, bi: int):
        s, e, _ = self.buckets[bi]
        cur = torch.cuda.current_stream(self.grad.device)
        wait = [cur] if self.side is None or self.side.cuda_stream == cur.cuda_stream else [cur, self.side]
        self.comm.allreduce(self.grad[s:e], self.algos[bi], self.bf16_wire, wait=wait)

    def finish(self):
        if not self.enabled:
            return
        while self._next < len(self.buckets):
            self._launch(self._next)
            self._next += 1
        self.comm.join(torch.cuda.current_stream(self.grad.device))


def broadcast_parameters(tensors: Sequence[torch.Tensor], src: int = 0, group=None):
    """Rank-0 broadcast of parameters/buffers (reference DDP ctor)."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return
    for t in tensors:
        dist.broadcast(t, src=src, group=group)


def verify_shapes(shapes: Sequence[Tuple[int, ...]], group=None):
    """Cross-rank parameter-shape check (reference DDP ctor)."""
    if not (dist.is_initialized() and dist.get_world_size(group) > 1):
        return
    mine = [tuple(s) for s in shapes]
    allv = [None] * dist.get_world_size(group)
    dist.all_gather_object(allv, mine, group=group)
    for r, v in enumerate(allv):
        if v != mine:
            raise RuntimeError(f"parameter shapes differ between this rank and rank {r}")


def replica_digest(tensors: Sequence[torch.Tensor]) -> List[float]:
    """Bitwise digest of a list of tensors: per tensor a position-weighted sum of its raw 32-bit
    words (int64 arithmetic, exact) folded into one number, plus the fp64 value sum.  Two
    replicas with equal digests hold the same bits with overwhelming probability."""
    h, s = 0, 0.0
    for i, t in enumerate(tensors):
        t = t.detach().contiguous()
        raw = t.view(-1).view(torch.uint8)
        pad = (-raw.numel()) % 4
        if pad:
            raw = torch.cat([raw, raw.new_zeros(pad)])
        w = raw.view(torch.int32).to(torch.int64)
        pos = torch.arange(w.numel(), device=w.device, dtype=torch.int64) % 65521 + 1
        h = (h * 1000003 + int((w * pos).sum().item()) + i) % (1 << 52)
        s += float(t.double().sum().item()) if t.is_floating_point() else float(t.sum().item())
    return [float(h), s]


def replicas_identical(tensors: Sequence[torch.Tensor], device, group=None):
    """(identical, digest): the digests of every rank agree (MIN == MAX all-reduce)."""
    d = replica_digest(tensors)
    lo = all_reduce_scalars(d, device, op=dist.ReduceOp.MIN, group=group)
    hi = all_reduce_scalars(d, device, op=dist.ReduceOp.MAX, group=group)
    return lo == hi, d


def all_reduce_scalars(values: Sequence[float], device, op=None, group=None) -> List[float]:
    """fp64 metric all-reduce (reference :187-196, :215-224)."""
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=op or dist.ReduceOp.SUM, group=group)
    return t.tolist()
