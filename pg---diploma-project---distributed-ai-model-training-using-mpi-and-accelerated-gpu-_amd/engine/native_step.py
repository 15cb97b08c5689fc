"""One native training step = GPU augmentation + fused forward/backward +
bucketed RCCL gradient all-reduce + fused Adam + device-side metrics,
optionally captured once into a hipGraph and replayed.

Reference per-batch body (``cifar10_mpi_mobilenet_224.py:173-185``):
``imgs.to(device); zero_grad(); out = ddp_model(imgs); loss = criterion(...);
loss.backward(); optimizer.step(); torch.max(...); loss.item(); (...).item()``
— two host syncs per batch and a CPU/PIL data pipeline.  Here the only host
work per step is one 1 KB index copy and a graph replay.
"""
import contextlib
import os
from typing import Optional

import torch
import torch.distributed as dist

from ..models import build_model
from ..ops import kernels as K
from ..parallel.comm import NativeComm
from ..parallel.ddp import BucketedGradReducer, NativeBucketReducer, broadcast_parameters, estimate_ready_times
from .executor import MobileNetV2Executor


def executor_class(model):
    """Static-plan executor of a model family (MobileNetV2 or ResNet)."""
    from ..models.resnet import ResNet
    if isinstance(model, ResNet):
        from .resnet_executor import ResNet50Executor
        return ResNet50Executor
    return MobileNetV2Executor


def coalesce_bn_buffers(model: torch.nn.Module):
    """Re-home every BatchNorm running_mean / running_var into one flat fp32 tensor and every
    num_batches_tracked into one int64 tensor (module buffers become views), so the per-step
    buffer broadcast of the reference's DDP is two collectives instead of 156."""
    mods = [m for m in model.modules() if isinstance(m, torch.nn.BatchNorm2d)]
    dev = mods[0].running_mean.device
    n = sum(m.running_mean.numel() + m.running_var.numel() for m in mods)
    # padded (zeros) so either buffer is a whole number of 16-B vectors (P2P broadcast)
    flat = torch.zeros((n + 63) // 64 * 64, dtype=torch.float32, device=dev)
    nbt = torch.zeros((len(mods) + 1) // 2 * 2, dtype=torch.int64, device=dev)
    o = 0
    for i, m in enumerate(mods):
        for name in ("running_mean", "running_var"):
            b = getattr(m, name)
            v = flat[o:o + b.numel()]
            v.copy_(b)
            setattr(m, name, v)
            o += b.numel()
        nbt[i:i + 1].copy_(m.num_batches_tracked.view(1))
        m.num_batches_tracked = nbt[i]
    return flat, nbt


def _dist_backend(group=None) -> str:
    try:
        return str(dist.get_backend(group)) if dist.is_available() and dist.is_initialized() else ""
    except Exception:   # no default group
        return ""


# augment(epoch_ctr=...) offset that makes the kernel's RNG key for step t that of step t + 1
# (key = mix(step * 0x100000001B3 + epoch_ctr), csrc/kernels/augment.hip)
AUG_NEXT_STEP = 0x100000001B3


class NativeTrainStep:
    def __init__(self, model, batch: int, device: torch.device, img_size: int = 224, lr: float = 1e-4,
                 betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0, world_size: int = 1,
                 rank: int = 0, use_graph: bool = True, seed: int = 0, bucket_mb: Optional[float] = None,
                 first_bucket_mb: float = 1.0, reduce_dtype: torch.dtype = torch.float32,
                 double_resize: bool = True, augment: bool = True, train_augment: bool = True,
                 side_stream: bool = True, bn_broadcast: bool = False, fp8: bool = False,
                 graph_forward: bool = False, comm: Optional[str] = None, force_ddp: bool = False,
                 allreduce_algo: Optional[str] = None, comm_watchdog_s: Optional[float] = None):
        self.device, self.B, self.S = device, batch, img_size
        self.world, self.rank = world_size, rank
        # deadline of the native communicator's collective watchdog (None: PGDIST_COMM_TIMEOUT);
        # the trainer passes its dist_timeout_s, so rank-0-only epoch work (checkpoints) that
        # keeps the peers waiting inside a collective is not mistaken for a dead peer
        self.comm_watchdog_s = comm_watchdog_s
        self.exe = executor_class(model)(model, batch, img_size, device, dropout_seed=(seed * 7919) ^ rank,
                                         side_stream=side_stream, fp8=fp8)
        self.flat = self.exe.flat
        self.betas, self.eps, self.wd = betas, eps, weight_decay
        self.seed = seed
        self.double_resize = double_resize
        self.augment_enabled = augment
        self.train_augment = train_augment   # False: deterministic Resize+Normalize (test transform)
        self.hyper = self.exe.hyper
        self.hyper[0] = lr
        self.metrics = torch.zeros(3, dtype=torch.float64, device=device)
        self.idx = torch.zeros(batch, dtype=torch.int64, device=device)
        self.aug_params = torch.zeros(batch, K.AUG_NPARAMS, dtype=torch.float32, device=device)
        self.src = None
        self.src_labels = None
        self.epoch_ctr = 0
        # fault injection (tests of the end-to-end evidence): the gradients of
        # the named parameters (PGDIST_FAULT_ZERO_GRAD, comma-separated names, or @dw / @pw / @bn:
        # every depthwise / 1x1 conv weight / BatchNorm affine parameter, i.e. a broken kernel
        # family) are zeroed after every backward: a planted "broken weight gradient" bug
        self.fault_zero = [self.flat.range_of(n) for n in self._fault_names(model)]
        # ---- data parallel
        # PGDIST_COMM: auto (native communicator when the process group is RCCL's, c10d with gloo)
        # | rccl | p2p (IPC xGMI kernels only; also over a gloo default group) | native (both) | c10d
        self.reducer = None
        self.comm = None
        self._measure_ready = False
        self.bucket_ready_us = None   # measured gradient ready times (us into the backward)
        self.comm_mode = comm or os.environ.get("PGDIST_COMM", "auto")
        force_ddp = force_ddp or os.environ.get("PGDIST_FORCE_DDP", "0") == "1"
        if world_size > 1 or force_ddp:
            ranges = [(n,) + self.flat.range_of(n) for n in self.flat.order]
            backend = _dist_backend()
            mode = self.comm_mode
            if mode == "auto":
                mode = "native" if (backend == "nccl" or world_size == 1) else "c10d"
            if mode == "c10d":
                self.reducer = BucketedGradReducer(self.flat.grad, ranges, bucket_mb, first_bucket_mb, reduce_dtype)
            else:
                self.comm = self._make_comm(mode, world_size)
                algo = allreduce_algo or os.environ.get("PGDIST_AR_ALGO", "auto")
                # bucket layout: modelled gradient ready times first, re-chosen from the times
                # measured on the second warm-up step (_back) before the step is recorded
                ready = (estimate_ready_times(model, img_size, 3000.0)
                         if bucket_mb is None and algo == "auto" and world_size > 1 else None)
                self.reducer = NativeBucketReducer(self.comm, self.flat.grad, ranges, bucket_mb, first_bucket_mb,
                                                   algo=algo, bf16_wire=reduce_dtype == torch.bfloat16,
                                                   force=force_ddp, ready_us=ready, t_bwd_us=3000.0)
                self._measure_ready = getattr(self.reducer, "tunable", False)
                self.exe.ready_native = True
            self.exe.on_params_ready = self.reducer.mark_ready
            self.exe.ready_probe = self.reducer.would_launch
            self.sync_from_rank0()
        # reference DDP default (broadcast_buffers=True): rank 0's BN running statistics are
        # broadcast before every training forward; the buffers are coalesced into one flat
        # fp32 tensor (+ one int64 tensor of num_batches_tracked) so that is two collectives
        self.bn_broadcast = bn_broadcast and (world_size > 1 or (self.reducer is not None and self.comm is not None))
        if self.bn_broadcast:
            self.bn_flat, self.bn_nbt = coalesce_bn_buffers(self.exe.model)
            if hasattr(self.exe, "refresh_bn_fin"):
                self.exe.refresh_bn_fin()   # fused BN finalize: descriptors point at the re-homed buffers
        self._validate_collectives()
        # RCCL collectives are issued eagerly between graph segments; a single-graph
        # capture is used on one GPU
        self.use_graph = use_graph and world_size == 1
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self._eager_runs = 0
        # forward-only graph: augment + forward (+ fused head backward) are one main-stream
        # chain of ~170 short kernels whose eager launch is host-bound on the small late layers;
        # replaying them as one graph lets the host run ahead and queue the (eager, two-stream)
        # backward while the GPU is still in the forward.  No collective is captured, so it
        # applies to data-parallel runs too (not with the per-step BN buffer broadcast).
        self.graph_forward = graph_forward and not self.use_graph and not self.bn_broadcast
        self.fwd_graph: Optional[torch.cuda.CUDAGraph] = None
        # eager steps replayed from a native launch plan (csrc/runtime/plan.h): same two-stream
        # schedule as eager launching, none of its Python host cost (PGDIST_PLAN=0: off)
        # Not with host-side (gloo) collectives on GPU tensors: their bucket launches and the
        # step-end wait block the host inside the replay (2 ranks on one MI355X over gloo: 560 ms
        # per step replayed vs 117 ms eager); RCCL collectives are stream-ordered and replay fine.
        # PGDIST_PLAN=force: replay with gloo too (tests of the replayed data-parallel step)
        plan_env = os.environ.get("PGDIST_PLAN", "1")
        gloo = (isinstance(self.reducer, BucketedGradReducer) and not getattr(self.reducer, "native", False)
                and self.reducer.enabled and _dist_backend(self.reducer.group) == "gloo" and plan_env != "force")
        self.use_plan = (not self.use_graph and not self.graph_forward and not gloo
                         and getattr(self.exe, "PLAN_SAFE", False) and plan_env in ("1", "force"))
        self.plan: Optional[K.LaunchPlan] = None
        # augmentation prefetch (PGDIST_AUG_PREFETCH=0: off): when the caller passes the NEXT
        # batch's indices, that batch is rendered on the weight-gradient side stream during this
        # step's backward into the other half of a double buffer (images, labels, indices), so
        # the GPU augmentation (~0.1 ms) leaves the critical path.  Its RNG stream is the one the
        # main-stream augmentation of that step would use (step counter + 1), so a prefetched
        # batch is bitwise the batch a non-prefetched step renders.  One launch plan per buffer
        # parity; steps that neither have a prefetched batch nor prefetch one run eagerly.
        self.prefetch = (self.use_plan and self.augment_enabled and self.train_augment and self.exe.side is not None
                         and os.environ.get("PGDIST_AUG_PREFETCH", "1") == "1")
        self._cur, self._have, self._next = 0, False, False
        # (rendered beside the backward's weight gradients; beside the forward, where the side
        # stream is otherwise idle, measured 4.556-4.572 vs 4.553-4.557 ms/step: the augmentation's
        # VALU competes with the bandwidth-bound forward)
        self._plans = {}
        if self.prefetch:
            self._imgs = [self.exe.img, torch.empty_like(self.exe.img)]
            self._labs = [self.exe.labels, torch.empty_like(self.exe.labels)]
            self._idxs = [self.idx, torch.empty_like(self.idx)]
            self._prms = [self.aug_params, torch.empty_like(self.aug_params)]

    def _validate_collectives(self):
        """The step's P2P collectives at their real sizes, back to back with the per-step BN
        broadcast (collective: every rank), before any training step (and again after a retune)."""
        if isinstance(self.reducer, NativeBucketReducer) and self.world > 1:
            bcast = self.bn_flat.numel() if getattr(self, "bn_broadcast", False) else 0
            self.reducer.validate_layout(bcast)

    @staticmethod
    def _fault_names(model):
        out = []
        params = dict(model.named_parameters())
        bn = {f"{m}.{k}" for m, mod in model.named_modules() if isinstance(mod, torch.nn.BatchNorm2d)
              for k in ("weight", "bias")}
        for tok in [x for x in os.environ.get("PGDIST_FAULT_ZERO_GRAD", "").split(",") if x]:
            if tok == "@dw":
                out += [n for n, p in params.items() if p.dim() == 4 and p.shape[1] == 1 and p.shape[2] == 3]
            elif tok == "@pw":
                out += [n for n, p in params.items() if p.dim() == 4 and p.shape[2] == 1]
            elif tok == "@bn":
                out += [n for n in params if n in bn]
            else:
                out.append(tok)
        return out

    def _make_comm(self, mode: str, world_size: int) -> NativeComm:
        """Native communicator of this data-parallel step: RCCL (modes rccl / native) and the P2P
        xGMI path (modes p2p / native, when every rank is on this node)."""
        local_world = int(os.environ.get("LOCAL_WORLD_SIZE", world_size))
        use_p2p = mode in ("p2p", "native") and local_world == world_size and world_size <= 8
        if mode == "p2p" and not use_p2p:
            raise RuntimeError("PGDIST_COMM=p2p needs every rank on this node (at most 8)")
        grad_bytes = self.flat.grad.numel() * 4
        return NativeComm.for_process_group(self.device, use_rccl=mode in ("rccl", "native"),
                                            p2p_bytes=grad_bytes if use_p2p else 0,
                                            watchdog_s=self.comm_watchdog_s) \
            if world_size > 1 else NativeComm(0, 1, self.device, use_rccl=mode in ("rccl", "native"),
                                              p2p_bytes=grad_bytes if use_p2p else 0)

    # ------------------------------------------------------------------ setup
    @classmethod
    def for_benchmark(cls, model_name: str, batch: int, device, img_size=224, use_graph=True,
                      world_size=1, rank=0, n_data=50000, side_stream=True, fp8=False, graph_forward=False,
                      bn_broadcast=False):
        if model_name not in ("mobilenet_v2", "resnet50"):
            raise NotImplementedError(f"native executors: mobilenet_v2, resnet50 (not {model_name}); "
                                      "use --backend torch")
        torch.manual_seed(42)  # identical random-init weights on every rank (then rank-0 broadcast)
        g = torch.Generator(device=device).manual_seed(1234 + rank)
        if model_name == "resnet50":
            # BASELINE config 4: ImageNet-shaped synthetic data (uint8 224x224x3 pool, 1000 classes)
            model = build_model("resnet50", num_classes=1000)
            n_data = min(n_data, 2048)
            src = torch.randint(0, 256, (n_data, img_size, img_size, 3), dtype=torch.uint8, device=device,
                                generator=g)
            labels = torch.randint(0, 1000, (n_data,), dtype=torch.int64, device=device, generator=g)
        else:
            model = build_model("mobilenet_v2", num_classes=10)
            src = torch.randint(0, 256, (n_data, 32, 32, 3), dtype=torch.uint8, device=device, generator=g)
            labels = torch.randint(0, 10, (n_data,), dtype=torch.int64, device=device, generator=g)
        st = cls(model, batch, device, img_size=img_size, world_size=world_size, rank=rank,
                 use_graph=use_graph, seed=42, side_stream=side_stream, fp8=fp8, graph_forward=graph_forward,
                 bn_broadcast=bn_broadcast)
        st.set_data(src, labels)
        st._perm = torch.randperm(n_data, device=device, generator=g)
        st._pos = 0
        return st

    def sibling(self, batch: int) -> "NativeTrainStep":
        """A step object for another batch size sharing weights, optimizer state, lr/step
        counter, metrics, data and gradient reducer (used for the short last batch of an
        epoch, which the reference's DataLoader keeps).  Runs eagerly."""
        st = NativeTrainStep.__new__(NativeTrainStep)
        st.__dict__.update(self.__dict__)
        st.B = batch
        st.exe = type(self.exe)(self.exe.model, batch, self.S, self.device, flat=self.flat,
                                dropout_seed=self.exe.dropout_seed, hyper=self.hyper)
        st.exe.on_params_ready = self.exe.on_params_ready
        st.exe.ready_probe = self.exe.ready_probe
        st.exe.ready_native = getattr(self.exe, "ready_native", False)
        st.idx = torch.zeros(batch, dtype=torch.int64, device=self.device)
        st.aug_params = torch.zeros(batch, K.AUG_NPARAMS, dtype=torch.float32, device=self.device)
        st.use_graph, st.graph, st._eager_runs = False, None, 0
        st.use_plan, st.plan = False, None
        st.graph_forward, st.fwd_graph = False, None
        st.prefetch, st._have, st._next, st._plans = False, False, False, {}
        return st

    def set_data(self, src_u8: torch.Tensor, labels: torch.Tensor):
        """Device-resident uint8 NHWC images: CIFAR-shaped [N,32,32,3] (GPU augmentation to
        the training resolution) or full-resolution [N,S,S,3] (flip + normalise only)."""
        assert src_u8.is_cuda and src_u8.dtype == torch.uint8 and src_u8.dim() == 4 and src_u8.shape[3] == 3
        assert tuple(src_u8.shape[1:3]) in ((32, 32), (self.S, self.S)), "source images: 32x32 or SxS"
        self.src = src_u8.contiguous()
        self.src_labels = labels.to(self.device, torch.int64).contiguous()
        if getattr(self, "plan", None) is not None:   # the recorded augment launch reads the old pool
            self.plan.free()
            self.plan, self._eager_runs = None, 0
        for p in getattr(self, "_plans", {}).values():
            p.free()
        self._plans, self._have = {}, False

    def sync_from_rank0(self):
        mods = [m for m in self.exe.model.modules() if isinstance(m, torch.nn.BatchNorm2d)]
        bufs = [b for m in mods for b in (m.running_mean, m.running_var, m.num_batches_tracked)]
        broadcast_parameters([self.flat.master] + bufs)
        self.flat.refresh_shadow()

    def set_lr(self, lr: float):
        self.hyper[0:1].fill_(float(lr))

    # ------------------------------------------------------------------ step
    def _body(self):
        self._front()
        self._back()

    def _front(self):
        """Step counter, augmentation and the training forward (main stream only)."""
        exe = self.exe
        # step counter + this step's BatchNorm statistics arena cleared in one launch
        arena = getattr(exe, "bn_arena", None)
        K.step_begin(self.hyper, zero=arena)
        exe.arena_cleared = arena is not None
        if self.augment_enabled and self.src.shape[1] != 32:
            s2d = getattr(exe, "stem_s2d", False)   # ResNet space-to-depth stem: render its input directly
            if s2d:
                exe.img_s2d_external = True
            K.image_prep(self.src, self.idx, self.src_labels, exe.img2 if s2d else exe.img, exe.labels,
                         seed=self.seed + 17 * self.rank if self.train_augment else 0,
                         hyper=self.hyper if self.train_augment else None, s2d=s2d)
        elif self.augment_enabled and not self._have:   # (a prefetched batch is already rendered)
            K.augment(self.src, self.idx, self.src_labels, exe.img, exe.labels, self.aug_params,
                      train=self.train_augment,
                      double_resize=self.double_resize, seed=self.seed + 17 * self.rank, hyper=self.hyper,
                      epoch_ctr=0, out_hw=self.S)
        if self.bn_broadcast:
            if self.comm is not None:   # native: recorded collectives, no Python at replay
                # P2P broadcast (one barrier, all links) when validated, else RCCL.  Issued on the
                # comm stream after the previous step (which wrote the running statistics) and
                # joined only where this forward first updates them (exe.join_stats: the batched
                # forward finalize in lazy mode): training-mode BN normalises with batch
                # statistics, so the broadcast overlaps the forward instead of delaying its head.
                algo = "oneshot" if self.comm.has_p2p else "rccl"
                cur = torch.cuda.current_stream(self.device)
                self.comm.broadcast(self.bn_flat, 0, algo, wait=[cur])
                self.comm.broadcast(self.bn_nbt.view(torch.float32), 0, algo, wait=[cur])
                exe.stats_wait = lambda cur=cur: self.comm.join(cur)
            else:
                K.plan_py(lambda: broadcast_parameters([self.bn_flat, self.bn_nbt]))
        try:
            exe.forward(train=True)
        finally:
            exe.__dict__.pop("stats_wait", None)

    def _prefetch_next(self):
        """Render the next batch into the other buffer on the side stream: after this step's
        main-stream work so far (the previous step, which last read that buffer, is before it);
        the backward's final join orders it before the next step's forward."""
        exe = self.exe
        nb = 1 - self._cur
        K.stream_wait(exe.side, torch.cuda.current_stream(self.device))
        with torch.cuda.stream(exe.side):
            K.augment(self.src, self._idxs[nb], self.src_labels, self._imgs[nb], self._labs[nb], self._prms[nb],
                      train=True, double_resize=self.double_resize, seed=self.seed + 17 * self.rank,
                      hyper=self.hyper, epoch_ctr=AUG_NEXT_STEP, out_hw=self.S)

    def _back(self):
        """Backward (+ bucketed all-reduce), Adam and metrics."""
        exe = self.exe
        if self._next:
            self._prefetch_next()
        native = getattr(self.reducer, "native", False)
        if native:   # host bookkeeping at record time only; the collectives are native plan ops
            self.reducer.side = exe.side
            self.reducer.begin()
        elif self.reducer is not None:
            K.plan_py(self.reducer.begin)
        probe = self._measure_ready and self._eager_runs == 2 and not K.plan_recording()
        if probe:
            t_ready, orig = [], exe.on_params_ready
            cur = torch.cuda.current_stream(self.device)
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record(cur)

            def on_ready(names, orig=orig, cur=cur):
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(cur)
                t_ready.append((list(names), ev))
                orig(names)
            exe.on_params_ready = on_ready
        try:
            exe.backward()
        finally:
            if probe:
                exe.on_params_ready = orig
        if probe:
            ev1 = torch.cuda.Event(enable_timing=True)
            ev1.record(torch.cuda.current_stream(self.device))
        if native:
            self.reducer.finish()
        elif self.reducer is not None:
            K.plan_py(self.reducer.finish)
        for a, b in self.fault_zero:
            K.memset(self.flat.grad[a:b])
        # a failed P2P collective or a poisoned communicator (comm_poison) leaves the device error
        # word set: Adam then skips the update, so no replica applies un-reduced gradients (the
        # job fails at the next check).  An RCCL stall ends the process (the collective watchdog's
        # default exit status); an RCCL asynchronous error is only seen by the host poll.
        K.adam_flat(self.flat.master, self.flat.grad, self.flat.exp_avg, self.flat.exp_avg_sq,
                    self.flat.shadow, self.hyper, self.betas[0], self.betas[1], self.eps, self.wd,
                    1.0 / self.world, skip=self.comm.error_word if self.comm is not None else 0,
                    metrics=(exe.loss, exe.correct, self.B, self.metrics))   # (+ the step's metrics)
        if probe:
            self._retune_buckets(t_ready, ev0, ev1)

    def _retune_buckets(self, t_ready, ev0, ev1):
        """Gradient ready times measured on this (eager warm-up) step -> the bucket layout of the
        recorded step: MAX over ranks (every rank must choose the same buckets), then
        NativeBucketReducer.retune (collective)."""
        from ..parallel.comm import host_allreduce
        torch.cuda.synchronize(self.device)
        names = [n for n, _, _ in self.reducer._ranges]
        at = {}
        for ns, ev in t_ready:
            t = ev0.elapsed_time(ev) * 1e3
            for n in ns:
                at[n] = t
        t_bwd = ev0.elapsed_time(ev1) * 1e3
        vec = torch.tensor([at.get(n, t_bwd) for n in names] + [t_bwd], dtype=torch.float64)
        vec = host_allreduce(vec, dist.ReduceOp.MAX)
        ready = {n: float(v) for n, v in zip(names, vec[:-1].tolist())}
        self.bucket_ready_us = ready
        self.reducer.retune(ready, float(vec[-1]))
        self._measure_ready = False
        self._validate_collectives()

    def run(self, idx: torch.Tensor, next_idx: Optional[torch.Tensor] = None):
        """One training step on the caller's current stream (a high-priority critical-path stream
        measured slower: 5.36-5.37 vs 5.30 ms/step, docs/PERF_NOTES.md round 4)."""
        return self._run(idx, next_idx)

    def _run(self, idx: torch.Tensor, next_idx: Optional[torch.Tensor] = None):
        """One training step on the batch ``src[idx]`` (idx: int64 [B] on device).  With
        ``next_idx`` (the next step's full batch) and prefetch enabled, that batch is augmented
        during this step's backward on the side stream (the next ``run`` then ignores its idx
        argument's contents only in the sense that the batch was already rendered from
        ``next_idx``: callers pass the same indices again)."""
        # (the 32x32 augmentation chain only: full-resolution sources take the short image_prep)
        if self.prefetch and (next_idx is not None or self._have) and self.src.shape[1] == 32:
            return self._run_prefetch(idx, next_idx)
        self.idx.copy_(idx, non_blocking=True)
        if self.graph_forward:
            if self.fwd_graph is None:
                if self._eager_runs < 2:
                    self._eager_runs += 1
                    self._body()
                    return
                torch.cuda.synchronize(self.device)
                self.fwd_graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.fwd_graph):
                    self._front()
            self.fwd_graph.replay()
            self._back()
            return
        if self.use_plan:
            if self.plan is None:
                if self._eager_runs < 2:   # warm-up: module loading / first-touch outside recording
                    self._eager_runs += 1
                    self._body()
                    return
                self.plan = K.LaunchPlan()
                self.plan.record(self._body)   # runs this step eagerly while recording it
                return
            self.plan.replay()
            return
        if not self.use_graph:
            self._body()
            return
        if self.graph is None:
            if self._eager_runs < 2:   # warm-up: module loading / first-touch outside capture
                self._eager_runs += 1
                self._body()
                return
            torch.cuda.synchronize(self.device)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self._body()
        self.graph.replay()

    def _run_prefetch(self, idx, next_idx):
        cur = self._cur
        self.exe.img, self.exe.labels = self._imgs[cur], self._labs[cur]
        self.idx, self.aug_params = self._idxs[cur], self._prms[cur]
        if not self._have:
            self.idx.copy_(idx, non_blocking=True)
        self._next = next_idx is not None and next_idx.numel() == self.B
        if self._next:
            # on the side stream, which reads it (the next batch's augmentation during this step's
            # backward) and last read that buffer: off the main stream's step head
            with torch.cuda.stream(self.exe.side) if self.exe.side is not None else contextlib.nullcontext():
                self._idxs[1 - cur].copy_(next_idx, non_blocking=True)
        if self._have and self._next and self._eager_runs >= 2:
            plan = self._plans.get(cur)
            if plan is None:
                plan = self._plans[cur] = K.LaunchPlan()
                plan.record(self._body)   # runs this step eagerly while recording it
            else:
                plan.replay()
            self.plan = plan
        else:   # first / last step of a prefetch chain, and warm-up: eager
            self._eager_runs += 1
            self._body()
        self._have = self._next
        if self._next:
            self._cur = 1 - cur

    @property
    def graph_enabled(self) -> bool:
        return self.use_graph

    def bench_step(self):
        n = self._perm.numel()
        if self._pos + self.B > n:
            self._pos = 0
        nxt = self._pos + self.B
        nxt = nxt if nxt + self.B <= n else 0
        self.run(self._perm[self._pos:self._pos + self.B], self._perm[nxt:nxt + self.B])
        self._pos += self.B

    # ------------------------------------------------------------------ metrics
    def read_metrics(self, reset: bool = True):
        """(sum loss, sum correct, count) accumulated on device since the last reset."""
        v = self.metrics.tolist()
        if reset:
            self.metrics.zero_()
        return v
