"""Static-plan executor: MobileNetV2 training step on the fused gfx950 kernels.

Instead of tracing autograd through ~150 forward / ~300 backward library ops
(reference call stack: SURVEY.md §3.3), the network is compiled once into a
fixed schedule of fused HIP kernels over preallocated NHWC bf16 buffers:

forward, per inverted-residual block (BN = training-mode BatchNorm)
  expand   pw_gemm(ACT_BN_RELU6 | ACT_NONE prologue)  -> y_e + BN_e partials
  finalize BN_e                                        -> scale/shift (+running stats)
  dw       dw_fwd(relu6(BN_e(y_e)) prologue)           -> y_d + BN_d partials
  finalize BN_d
  project  pw_gemm(relu6(BN_d(y_d)) prologue)          -> y_p + BN_p partials
  finalize BN_p
  output   o = BN_p(y_p) (+ o_in)                      (materialised, bf16)
head: BN_18/ReLU6 + avgpool + dropout + linear + CE + its backward (one kernel)

backward walks the schedule in reverse; every BN backward is split into a
partial-sum epilogue in the kernel that produces the gradient and a per-channel
finalize, and the BN-backward elementwise step is fused into the prologues of
both the dgrad and the wgrad kernels that consume it.  Weight gradients are
written straight into the flat gradient buffer; after each layer the gradient
bucket reducer is told which parameters are final so the RCCL all-reduce of a
complete bucket starts while backward continues.

Every buffer is allocated once, so the whole step can be captured in a hipGraph.
"""
import os
from dataclasses import dataclass, field
from typing import Callable, List, Optional

import torch

from ..models.mobilenet_v2 import MobileNetV2, InvertedResidual
from ..ops import kernels as K
from .flat import FlatParams


class BNState:
    """Buffers of one training-mode BatchNorm over an [M, C] activation."""

    def __init__(self, flat: FlatParams, module: torch.nn.BatchNorm2d, prefix: str, M: int, C: int,
                 device, need_g: bool = True):
        self.prefix, self.M, self.C = prefix, M, C
        self.module = module
        self.eps, self.momentum = module.eps, module.momentum if module.momentum is not None else 0.1
        self.gamma, self.beta = flat.w(prefix + ".weight"), flat.w(prefix + ".bias")
        self.dgamma, self.dbeta = flat.g(prefix + ".weight"), flat.g(prefix + ".bias")
        f32 = dict(dtype=torch.float32, device=device)
        self.mean = torch.zeros(C, **f32)
        self.rstd = torch.ones(C, **f32)
        self.scale = torch.ones(C, **f32)
        self.shift = torch.zeros(C, **f32)
        self.coef = torch.zeros(3, C, **f32)
        self.y = torch.empty(M, C, dtype=torch.bfloat16, device=device)   # pre-BN activation
        self.g = torch.empty(M, C, dtype=torch.bfloat16, device=device) if need_g else None
        self.act: Optional[torch.Tensor] = None   # relu(BN(y)) when a consumer wants it materialised
        self.param_names = [prefix + ".weight", prefix + ".bias"]
        # atomic statistics accumulators [rows][2][C] of this BN's forward / backward producer
        # (views into the executor's arena, zeroed once per training step)
        self.acc_f: Optional[torch.Tensor] = None
        self.acc_b: Optional[torch.Tensor] = None

    def finalize_fwd(self, part, P):
        K.bn_fwd_finalize(part, P, self.C, self.M, self.gamma, self.beta, self.eps, self.momentum,
                          self.module.running_mean, self.module.running_var,
                          self.module.num_batches_tracked, self.mean, self.rstd, self.scale, self.shift)

    def finalize_bwd(self, part, P):
        K.bn_bwd_finalize(part, P, self.C, self.M, self.mean, self.rstd, self.gamma, self.coef,
                          self.dgamma, self.dbeta)

    def eval_prepare(self):
        with torch.no_grad():
            rs = torch.rsqrt(self.module.running_var + self.eps)
            self.scale.copy_(self.gamma * rs)
            self.shift.copy_(self.beta - self.module.running_mean * self.gamma * rs)

    @property
    def a(self):
        return self.coef[0]

    @property
    def b(self):
        return self.coef[1]

    @property
    def c(self):
        return self.coef[2]


class AtomicBNState(BNState):
    """BN of the MobileNetV2 executor: its producers accumulate the statistics atomically into
    min(P, bn_rep) replica rows of ``acc_f`` / ``acc_b`` (P = the producer's partial rows), so a
    finalize reduces those rows only (deterministic mode: bn_rep unbounded, one row per
    producer workgroup).  ``rows_f`` / ``rows_b``: rows the accumulators were sized for.

    The finalize itself has three modes (``MobileNetV2Executor.bn_mode``):

    * ``lazy`` (default): ``lz_f`` / ``lz_b`` are device descriptors (ops.kernels.bn_fin_desc)
      passed to the CONSUMERS of this BN's parameters, which compute the scale / shift (or
      the backward coefficients) they need from the accumulator rows in their prologue
      (bnfin.h bn_lazy) -- no finalize launch between producer and consumer.  The side
      outputs are written off the critical path: every forward BN by one batched finalize at
      the end of the forward, the backward ones on the weight-gradient side stream.
    * (``fused``: the producers' last workgroup finalizing in their tail -- bnfin.h bn_fin_tail,
      kept as a kernel feature -- measured 5.93 vs 5.60 ms/step and is not an executor mode.)
    * ``launch`` (deterministic mode, or PGDIST_BN_LAZY=0): a separate finalize launch on
      the main stream after every producer."""
    rows_f = rows_b = 0
    fin_f = fin_b = None
    lz_f = lz_b = None
    desc_f = desc_b = None

    def build_desc(self, ctr_f, ctr_b):
        """(Re)write the fused-finalize descriptors (in place once built, so captured graphs
        keep valid pointers): call again after the module's running buffers were re-homed."""
        m = self.module
        df = K.bn_fin_desc(self.acc_f, ctr_f, self.rows_f, self.C, self.M, 0, gamma=self.gamma, beta=self.beta,
                           eps=self.eps, momentum=self.momentum, rmean=m.running_mean, rvar=m.running_var,
                           nbt=m.num_batches_tracked, mean=self.mean, rstd=self.rstd, scale=self.scale,
                           shift=self.shift)
        db = K.bn_fin_desc(self.acc_b, ctr_b, self.rows_b, self.C, self.M, 1, gamma=self.gamma, mean=self.mean,
                           rstd=self.rstd, coef=self.coef, dgamma=self.dgamma, dbeta=self.dbeta)
        if self.desc_f is None:
            self.desc_f, self.desc_b = df, db
        else:
            self.desc_f.copy_(df)
            self.desc_b.copy_(db)

    def finalize_fwd(self, part, P):
        r = K.bn_rows(P)
        assert r <= self.rows_f, f"{self.prefix}: forward producer has {r} rows > {self.rows_f} allocated"
        if self.fin_f is None and self.lz_f is None:
            super().finalize_fwd(part, r)

    def finalize_bwd(self, part, P, force=False):
        """Backward finalize launch; skipped when fused into the producer, and in lazy mode
        unless ``force`` (the executor forces it where the side outputs are needed: on the
        side stream, or for a main-stream consumer without a lazy prologue)."""
        r = K.bn_rows(P)
        assert r <= self.rows_b, f"{self.prefix}: backward producer has {r} rows > {self.rows_b} allocated"
        if self.fin_b is None and (self.lz_b is None or force):
            super().finalize_bwd(part, r)


@dataclass
class BlockPlan:
    idx: int
    prefix: str
    cin: int
    cout: int
    hidden: int
    stride: int
    expand: bool
    residual: bool
    H: int
    W: int
    Ho: int
    Wo: int
    w_e: Optional[str]
    w_d: str
    w_p: str
    bn_e: Optional[BNState]
    bn_d: BNState
    bn_p: BNState
    o: torch.Tensor = None          # block output (materialised)
    G: torch.Tensor = None          # gradient w.r.t. o


class MobileNetV2Executor:
    # every host-side action of a training step goes through recordable native ops
    # (ops.kernels: launches, stream_wait, memset, plan_py): the step can be a LaunchPlan
    PLAN_SAFE = True
    # on_params_ready issues only recordable native ops (NativeBucketReducer): called directly
    ready_native = False
    # depthwise dgrad+wgrad fused on maps >= this size.  Round 2: 14 / 28 / 56 / 112 / never =
    # 4.92 / 4.89 / 4.80-4.85 / 4.85 / 4.94 ms/step.  Round 5, after the fused kernel's ring
    # pipelined (inline-asm DMA): 28 = 4.365-4.375 vs 56 = 4.382-4.394 (7 / 14: 4.39-4.40),
    # same box (docs/PERF_NOTES.md round 5)
    DW_FUSE_MIN_H = 28
    # fused 1x1 dgrad+wgrad (pw_bwd) wherever supported (only M >= 500k / never: 5.06 / 5.27 vs 4.80)
    PW_BWD_FUSE_MIN_M = 0
    # block outputs of the maps with at most this many pixels per image (the latency-bound 14x14 /
    # 7x7 stages) are materialised by their consumer (next GEMM's prologue) instead of a BN-apply launch: bs128 4.517-4.530 vs 4.540-4.581 ms/step; the 28x28 stage
    # too (784): 4.527-4.559; every block: neutral (scripts/gpu_r4_aug.sh)
    FUSE_BLOCK_OUTPUT_HW = 196
    # expand-conv backward re-forms its BN input h1 = x We^T from the staged block input instead of
    # reading it (pw_bwd ``We``), on the shapes that support it
    PW_BWD_RECOMPUTE = True
    # side-stream joins batched per this many weight gradients (1 / 2 / 3 / 4 / 6: 5.28 / 5.23 /
    # 5.15 / 5.22 / 5.21 ms/step, docs/PERF_NOTES.md round 2)
    SIDE_BATCH = 3
    # fp8 mode: the forward 1x1 convs with K >= FP8_MIN_K run on e4m3 MFMA (weights per output
    # channel, activations scaled by ops.kernels.FP8_ASC); the K = 16 / 24 / 32 expand convs, the
    # backward and depthwise / BN stay bf16 / fp32

    def __init__(self, model: MobileNetV2, batch: int, img_size: int, device: torch.device,
                 flat: Optional[FlatParams] = None, dropout_seed: int = 0,
                 hyper: Optional[torch.Tensor] = None, side_stream: bool = True, fp8: bool = False):
        assert device.type == "cuda", "the native executor runs on the GPU"
        self.fp8 = fp8
        self.model = model.to(device)
        self.B, self.S, self.device = batch, img_size, device
        self.flat = flat or FlatParams(self.model, device)
        self.dropout_seed = dropout_seed
        self.drop_p = float(model.classifier[0].p)
        B = batch
        feats = model.features
        # ---------------- stem
        H = (img_size - 1) // 2 + 1
        self.H0 = H
        self.stem_w = "features.0.0.weight"
        self.bn0 = AtomicBNState(self.flat, feats[0][1], "features.0.1", B * H * H, feats[0][0].out_channels, device)
        wg = [K.stem_wgrad_workspace(B, img_size, img_size, 32)]   # side-stream weight gradients
        wparts = {}   # fused dgrad+wgrad: one split-M partial buffer per layer, reduced on the side stream
        # ---------------- blocks
        self.blocks: List[BlockPlan] = []
        cur_h = H
        for i in range(1, len(feats) - 1):
            blk: InvertedResidual = feats[i]
            pre = f"features.{i}.conv"
            Hin = cur_h
            Ho = (Hin - 1) // blk.stride + 1
            Min, Mout = B * Hin * Hin, B * Ho * Ho
            expand = blk.expand_ratio != 1
            if expand:
                bn_e = AtomicBNState(self.flat, blk.conv[0][1], f"{pre}.0.1", Min, blk.hidden, device)
                dwm, w_e = blk.conv[1], f"{pre}.0.0.weight"
                w_d, bn_d_pre = f"{pre}.1.0.weight", f"{pre}.1.1"
                w_p, bn_p_mod, bn_p_pre = f"{pre}.2.weight", blk.conv[3], f"{pre}.3"
            else:
                bn_e, w_e, dwm = None, None, blk.conv[0]
                w_d, bn_d_pre = f"{pre}.0.0.weight", f"{pre}.0.1"
                w_p, bn_p_mod, bn_p_pre = f"{pre}.1.weight", blk.conv[2], f"{pre}.2"
            bn_d = AtomicBNState(self.flat, dwm[1], bn_d_pre, Mout, blk.hidden, device)
            bn_p = AtomicBNState(self.flat, bn_p_mod, bn_p_pre, Mout, blk.oup, device, need_g=False)
            bp = BlockPlan(i, pre, blk.inp, blk.oup, blk.hidden, blk.stride, expand, blk.use_res_connect,
                           Hin, Hin, Ho, Ho, w_e, w_d, w_p, bn_e, bn_d, bn_p)
            bp.o = torch.empty(Mout, blk.oup, dtype=torch.bfloat16, device=device)
            bp.G = torch.empty(Mout, blk.oup, dtype=torch.bfloat16, device=device)
            self.blocks.append(bp)
            if expand:
                wg.append(K.pw_wgrad_workspace(Min, blk.hidden, blk.inp))
                if self._pw_bwd_ok(Min, blk.hidden, blk.inp):
                    wparts[(i, "e")] = K.pw_bwd_wgrad_workspace(Min, blk.hidden, blk.inp)
            if Hin >= self.DW_FUSE_MIN_H:
                wparts[(i, "d")] = K.dw_dgrad_wgrad_workspace(B, Hin, Hin, blk.hidden, blk.stride)
            else:
                wg.append(K.dw_wgrad_workspace(B, Hin, Hin, blk.hidden, blk.stride))
            wg.append(K.pw_wgrad_workspace(Mout, blk.oup, blk.hidden))
            if self._pw_bwd_ok(Mout, blk.oup, blk.hidden):
                wparts[(i, "p")] = K.pw_bwd_wgrad_workspace(Mout, blk.oup, blk.hidden)
            cur_h = Ho
        # ---------------- final 1x1 conv + head
        last = feats[-1]
        self.Hf = cur_h
        Mf = B * cur_h * cur_h
        self.C_last_in = self.blocks[-1].cout
        self.C_last = last[0].out_channels
        self.w_last = f"features.{len(feats) - 1}.0.weight"
        self.bn_last = AtomicBNState(self.flat, last[1], f"features.{len(feats) - 1}.1", Mf, self.C_last, device)
        wg.append(K.pw_wgrad_workspace(Mf, self.C_last, self.C_last_in))
        self.NC = model.classifier[1].out_features
        self.w_lin, self.b_lin = "classifier.1.weight", "classifier.1.bias"
        f32 = dict(dtype=torch.float32, device=device)
        self.logits = torch.zeros(B, self.NC, **f32)
        self.loss = torch.zeros(B, **f32)
        self.correct = torch.zeros(B, **f32)
        self.dlogits = torch.zeros(B, self.NC, **f32)
        self.pd = torch.zeros(B, self.C_last, **f32)
        # ---------------- workspaces (stream-ordered reuse)
        # BN statistics: one accumulator pair per BN ([rows][2][C] forward and backward, rows =
        # min(producer partial rows, bn_rep)), all in one arena so a training step zeroes them
        # with a single memset
        o, spans = 0, []
        self.bn_rep = K.bn_rep()   # the producers' replica rows the arena is sized for
        for bn, (pf, pb) in self._bn_producer_rows().items():
            bn.rows_f, bn.rows_b = K.bn_rows(pf), K.bn_rows(pb)
            nf, nb = K.bn_part_floats(bn.rows_f, bn.C), K.bn_part_floats(bn.rows_b, bn.C)
            spans.append((bn, o, nf, nb))
            o += (nf + nb + 63) // 64 * 64
        self.bn_arena = torch.zeros(o + 64, **f32)
        for bn, o, nf, nb in spans:
            bn.acc_f = self.bn_arena[o:o + nf]
            bn.acc_b = self.bn_arena[o + nf:o + nf + nb]
        # (finalize fused into the statistics producers' tails: measured on MI355X at bs128 5.93
        # ms/step vs 5.60 with separate launches -- every producer workgroup must wait for its
        # statistics atomics before arriving -- so not a mode of the executor)
        self.fused_bn = False
        # lazy finalize (default; PGDIST_BN_LAZY=0: a finalize launch after every producer): the
        # consumers compute the BN parameters from the accumulator rows (bnfin.h bn_lazy); one
        # batched forward finalize, backward finalizes on the side stream
        self.lazy_bn = not K.deterministic() and os.environ.get("PGDIST_BN_LAZY", "1") == "1"
        self.bn_mode = "lazy" if self.lazy_bn else ("fused" if self.fused_bn else "launch")
        self.bn_ctr = torch.zeros(8 * len(spans) + 16, dtype=torch.int32, device=device)   # 16-B apart
        self.refresh_bn_fin()
        if self.lazy_bn:
            bns = self.all_bns()
            self.fwd_fin_tab = K.bn_desc_table([bn.desc_f for bn in bns])
            self.fwd_fin_n, self.fwd_fin_maxc = len(bns), max(bn.C for bn in bns)
        self.ws_wgrad = torch.zeros(max(wg) + 1024, **f32)
        # one split-partial workspace per weight gradient of a flushed side-stream group (their
        # reductions are launched together after the group); ws_wgrad is the first
        nws = self.SIDE_BATCH
        self.ws_wgrad_pool = [self.ws_wgrad] + [torch.zeros_like(self.ws_wgrad) for _ in range(nws - 1)]
        # the stem weight gradient may run on the main stream concurrently with side-stream
        # weight gradients: its own split-M workspace
        self.ws_stem = torch.zeros(K.stem_wgrad_workspace(B, img_size, img_size, 32) + 1024, **f32)
        self._wpart = {k: torch.zeros(v + 1024, **f32) for k, v in wparts.items()}
        # weight gradients that are not fused into a dgrad run on a side stream, overlapping
        # the dgrad -> BN-finalize chain (the backward's critical path)
        self.side = None
        self._side_pending = []   # deferred (BN finalizes, weight-gradient callable) pairs
        self._fin_tabs = {}       # batched backward-finalize descriptor tables by BN group
        self.side_batch = self.SIDE_BATCH
        self.batch_reductions = True   # a group's split-M reductions in one launch (5.016 -> 5.003 ms)
        if device.type == "cuda" and side_stream:
            self.side = K.side_stream(device)
            K.register_side_stream(self.side)
        self.img = torch.zeros(B, img_size, img_size, 4, dtype=torch.bfloat16, device=device)
        self.labels = torch.zeros(B, dtype=torch.int64, device=device)
        self.hyper = hyper if hyper is not None else torch.zeros(2, **f32)   # [lr, step] (device)
        self.on_params_ready: Optional[Callable[[List[str]], None]] = None
        # ready_probe(names) -> True when marking ``names`` launches a gradient bucket; other
        # calls only do host bookkeeping (no side-stream event record / wait per layer)
        self.ready_probe: Optional[Callable[[List[str]], bool]] = None
        # 1x1 weights transposed for dgrad: table rows (offset, Cout, Cin)
        tab = []
        for bp in self.blocks:
            if bp.expand:
                tab.append((self.flat.offsets[bp.w_e][0], bp.hidden, bp.cin))
            tab.append((self.flat.offsets[bp.w_p][0], bp.cout, bp.hidden))
        tab.append((self.flat.offsets[self.w_last][0], self.C_last, self.C_last_in))
        self.wt_tab = torch.tensor(tab, dtype=torch.int32, device=device).contiguous()
        self.wt_n = len(tab)
        # fp8 forward (BASELINE config 5): per-output-channel e4m3 copies of every 1x1 weight,
        # re-quantised from the fp32 master at the start of each forward (one batched launch)
        self.w8 = {}
        if fp8:
            names = [n for bp in self.blocks for n in ((bp.w_e, bp.w_p) if bp.expand else (bp.w_p,))]
            names.append(self.w_last)
            qtab, qnames, dst, sc = [], [], 0, 0
            for name, (off, n, k) in zip(names, tab):
                if k < self.FP8_MIN_K:   # bf16 layer (see FP8_MIN_K)
                    continue
                qtab.append((off, n, k, dst, sc))
                qnames.append(name)
                dst += n * K.fp8_pitch(k)
                sc += n
            self.w8_buf = torch.zeros(dst + 64, dtype=torch.uint8, device=device)
            self.w8_scale = torch.ones(sc + 1, dtype=torch.float32, device=device)
            self.w8_tab = torch.tensor(qtab, dtype=torch.int32, device=device).contiguous()
            for name, (off, n, k, d0, c0) in zip(qnames, qtab):
                self.w8[name] = (self.w8_buf[d0:d0 + n * K.fp8_pitch(k)], self.w8_scale[c0:c0 + n])

    # ------------------------------------------------------------------ helpers
    def refresh_bn_fin(self):
        """(Re)build the BN-finalize descriptors of the fused / lazy modes (after BN running
        buffers were re-homed, e.g. coalesced for the per-step buffer broadcast): in place, so
        recorded plans, captured graphs and the batched-finalize table stay valid."""
        if not (self.fused_bn or self.lazy_bn):
            return
        for i, bn in enumerate(self.all_bns()):
            bn.build_desc(self.bn_ctr[8 * i:8 * i + 1], self.bn_ctr[8 * i + 4:8 * i + 5])
            if self.fused_bn:
                bn.fin_f, bn.fin_b = bn.desc_f, bn.desc_b
            else:
                bn.lz_f, bn.lz_b = bn.desc_f, bn.desc_b

    def _bn_producer_rows(self):
        """{bn: (forward P, backward P)}: partial rows of the kernels that produce each BN's
        statistics, in the order forward()/backward() launch them (the finalize asserts the
        launched P fits)."""
        B, S = self.B, self.S
        rows = {bn: [1, 1] for bn in self.all_bns()}
        rows[self.bn0][0] = K.stem_num_partials(B, S, S)
        for bi, bp in enumerate(self.blocks):
            prev = self.blocks[bi - 1] if bi > 0 else None
            Min, Mout = B * bp.H * bp.H, B * bp.Ho * bp.Wo
            dw_in = bp.bn_e if bp.expand else self.bn0
            if bp.expand:
                rows[bp.bn_e][0] = K.pw_num_partials(Min, bp.hidden, bp.cin)
                rows[prev.bn_p][1] = (K.pw_bwd_num_partials(Min, bp.hidden, bp.cin)
                                      if self._pw_bwd_ok(Min, bp.hidden, bp.cin)
                                      else K.pw_num_partials(Min, bp.cin, bp.hidden))
            rows[bp.bn_d][0] = K.dw_num_partials("fwd", B, bp.H, bp.H, bp.hidden, bp.stride)
            rows[dw_in][1] = K.dw_num_partials("dgrad", B, bp.H, bp.H, bp.hidden, bp.stride)
            rows[bp.bn_p][0] = K.pw_num_partials(Mout, bp.cout, bp.hidden)
            rows[bp.bn_d][1] = (K.pw_bwd_num_partials(Mout, bp.cout, bp.hidden)
                                if self._pw_bwd_ok(Mout, bp.cout, bp.hidden)
                                else K.pw_num_partials(Mout, bp.hidden, bp.cout))
        Mf = B * self.Hf * self.Hf
        rows[self.bn_last][0] = K.pw_num_partials(Mf, self.C_last, self.C_last_in)
        rows[self.bn_last][1] = B
        rows[self.blocks[-1].bn_p][1] = K.pw_num_partials(Mf, self.C_last_in, self.C_last)
        return {bn: tuple(r) for bn, r in rows.items()}

    def _pw_bwd_ok(self, M, Kg, Ng):
        """Use the fused 1x1 dgrad+wgrad kernel for this backward (else dgrad on the main
        stream, weight gradient on the side stream)."""
        return M >= self.PW_BWD_FUSE_MIN_M and K.pw_bwd_supported(M, Kg, Ng)

    def _check_bn_mode(self):
        # the producers write min(P, bn_rep()) rows: a mode switch after construction would
        # overrun the accumulators sized here
        if K.bn_rep() != self.bn_rep:
            raise RuntimeError(f"BN replica rows changed from {self.bn_rep} to {K.bn_rep()} after the executor "
                               "was built (ops.kernels.set_deterministic before building it)")

    def _ready(self, names):
        """Gradients of ``names`` are final once the work enqueued so far completes.  With a
        side stream the callback (DDP bucket launch) runs on it after it has joined the main
        stream, so the collective is ordered after both streams' producers.  Host-side Python
        (the reducer's bookkeeping and collectives): a launch-plan op (ops.kernels.plan_py).
        A call that launches a bucket first flushes the deferred side-stream work (the probe
        is a pure function of this step's reducer state, identical at record and replay)."""
        if self.on_params_ready is None:
            return
        if self.side is not None and (self.ready_probe is None or self.ready_probe(names)):
            self._flush_side()
        if self.ready_native:
            # native reducer: the bucket launch is a native op that waits for both streams
            # itself; its bookkeeping runs at record time only
            self.on_params_ready(names)
            return
        K.plan_py(lambda: self._ready_now(names))

    def _ready_now(self, names):
        if self.side is None or (self.ready_probe is not None and not self.ready_probe(names)):
            self.on_params_ready(names)
            return
        self.side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.side):
            self.on_params_ready(names)

    def _wgrad(self, fn, fins=()):
        """Enqueue a weight-gradient launch on the side stream (after the main stream's
        work so far, which produced its inputs).  Deferred in groups of ``side_batch``: every
        side-stream join is an event record on the main stream, whose barrier packet keeps the
        next main kernel from overlapping the previous one's completion (~5-6 us of main-stream
        idle per join on MI355X); one join per group instead of one per layer."""
        if self.side is None:
            self._side_fins(fins)
            fn(self.ws_wgrad)
            return
        self._side_pending.append((fins, fn))
        if len(self._side_pending) >= min(self.side_batch, len(self.ws_wgrad_pool)):
            self._flush_side()

    def _flush_side(self):
        """Join the side stream to the main stream's work so far and enqueue the deferred
        weight-gradient work on it."""
        if self.side is None or not self._side_pending:
            return
        K.stream_wait(self.side, torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.side):
            self._side_fins([f for fins, _ in self._side_pending for f in fins])
            # the group's split-M reductions in one multi-segment launch: each weight gradient
            # of the group writes its split partials into its own workspace
            K.wgrad_reduce_defer(self.batch_reductions)
            try:
                for j, (_, fn) in enumerate(self._side_pending):
                    fn(self.ws_wgrad_pool[j])
            finally:
                K.wgrad_reduce_defer(False)
            if self.batch_reductions:
                K.wgrad_reduce_flush()
        self._side_pending.clear()

    def _consume_output(self, pend, W, out, ws, M, N, K_, fin=None, lz=None):
        """Forward 1x1 conv whose input is a pending block output: prologue BN_p (+ residual),
        side-writes the block output o."""
        bn, res, o = pend
        if res is not None:
            K.pw_gemm(K.PRO_BNRES, K.EPI_FWD, bn.y, W, out, ws, M, N, K_, A2=res, pa=bn.scale, pb=bn.shift, Aout=o,
                      fin=fin, lz=lz)
        else:
            K.pw_gemm(K.ACT_BN, K.EPI_FWD, bn.y, W, out, ws, M, N, K_, pa=bn.scale, pb=bn.shift, Aout=o, fin=fin,
                      lz=lz)

    # fp8 mode: the e4m3 GEMM only for reduction depths >= this (PGDIST_FP8_MIN_K; 0: every
    # forward 1x1 conv).  The K = 16 / 24 / 32 expand convs of the 112 / 56 / 28 maps are pure
    # bandwidth (A read, C write) with nothing for the e4m3 MFMA to save, and on the e4m3 path
    # they lose the whole-row bf16 expand tiles: bs512 roofline 112x112 K=16 359 -> 518 us,
    # 56x56 K=24 280 -> 549 us (profiles/r4_roofline_bs512_fp8_vs_bf16.txt)
    FP8_MIN_K = int(os.environ.get("PGDIST_FP8_MIN_K", "64"))

    def _fp8_layer(self, K_):
        return self.fp8 and K_ >= self.FP8_MIN_K

    def _pw_fwd(self, pro, A, wname, out, ws, M, N, K_, pa=None, pb=None, fin=None, lz=None):
        """Forward 1x1 conv: bf16 MFMA GEMM, or the e4m3 one in fp8 mode (K >= FP8_MIN_K)."""
        if self._fp8_layer(K_):
            W8, wsc = self.w8[wname]
            K.pw_gemm_f8(pro, A, W8, wsc, out, ws, M, N, K_, pa=pa, pb=pb, fin=fin, lz=lz)
        else:
            K.pw_gemm(pro, K.EPI_FWD, A, self.flat.b(wname), out, ws, M, N, K_, pa=pa, pb=pb, fin=fin, lz=lz)

    def _side_fins(self, fins):
        """Lazy mode: the backward finalizes of the (bn, P) pairs of a flushed group of weight
        gradients -- coef for the side-stream weight gradients, dgamma / dbeta for the gradient
        buckets and the optimizer -- as ONE batched launch ahead of the group's weight
        gradients (main-stream consumers computed the coefficients themselves)."""
        if not self.lazy_bn or not fins:
            return
        for bn, P in fins:
            assert K.bn_rows(P) <= bn.rows_b, f"{bn.prefix}: backward producer rows exceed the accumulator"
        if len(fins) == 1:
            bn, P = fins[0]
            bn.finalize_bwd(bn.acc_b, P, force=True)
            return
        key = tuple(id(bn) for bn, _ in fins)
        tab = self._fin_tabs.get(key)
        if tab is None:
            tab = self._fin_tabs[key] = K.bn_desc_table([bn.desc_b for bn, _ in fins])
        K.bn_finalize_batch(tab, len(fins), max(bn.C for bn, _ in fins))

    def _fin_fwd(self, bn: BNState, P: int, train: bool):
        if train:
            if not self.lazy_bn:
                self.join_stats()   # this finalize launch updates the running statistics
            bn.finalize_fwd(bn.acc_f, P)

    def join_stats(self):
        """Before the first op of a training forward that writes BatchNorm running statistics:
        run the pending wait the step installed (``stats_wait``: the main stream joins the
        per-step rank-0 BN-buffer broadcast, which overlaps the forward until here; in training
        mode nothing before this point reads the running buffers).  Once per forward."""
        w = self.__dict__.pop("stats_wait", None)
        if w is not None:
            w()

    # ------------------------------------------------------------------ forward
    def forward(self, train: bool = True):
        """Runs the forward pass on ``self.img`` (and, when training, the head backward)."""
        f, B, S = self.flat, self.B, self.S
        self._check_bn_mode()
        if train and not self.__dict__.pop("arena_cleared", False):   # (else cleared by step_begin)
            K.memset(self.bn_arena)   # every BN statistics accumulator of this step
        # transposed 1x1 weights for the backward's dgrad GEMMs: on the (idle during the forward)
        # side stream, off the critical path; the main stream joins it at the end of the forward,
        # before the step enqueues anything else on the side stream
        self._wt_pending = train and self.side is not None
        if self._wt_pending:
            K.stream_wait(self.side, torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.side):
                K.wt_transpose(f.shadow, f.shadow_t, self.wt_tab, self.wt_n)
        if self.fp8:
            K.w8_quant(f.master, self.w8_buf, self.w8_scale, self.w8_tab, self.w8_tab.shape[0])
        # stem
        F = (lambda bn: bn.fin_f) if train else (lambda bn: None)   # fused forward finalize  # noqa: E731
        L = (lambda bn: bn.lz_f) if train else (lambda bn: None)    # lazy: consumer-side  # noqa: E731
        K.stem_fwd(self.img, f.b(self.stem_w), self.bn0.y, self.bn0.acc_f, B, S, S, fin=F(self.bn0))
        self._fin_fwd(self.bn0, K.stem_num_partials(B, S, S), train)
        inp_bn, inp_t = self.bn0, None   # block input: virtual relu6(bn0(y0))
        # A block output o = BN_p(y_p) (+ residual) is not materialised by a separate pass: its
        # consumer GEMM (next expand conv, or the final 1x1 conv) applies BN_p (+ residual) in
        # its prologue and writes o (needed for the next residual and the backward) on the way.
        pend = None      # (bn_p, residual tensor or None, o) of the previous block
        for bp in self.blocks:
            Hin = bp.H
            Min = B * Hin * Hin
            if bp.expand:
                if pend is not None:
                    self._consume_output(pend, f.b(bp.w_e), bp.bn_e.y, bp.bn_e.acc_f, Min, bp.hidden, bp.cin,
                                         fin=F(bp.bn_e), lz=L(pend[0]))
                elif inp_t is None:
                    self._pw_fwd(K.ACT_BN_RELU6, inp_bn.y, bp.w_e, bp.bn_e.y, bp.bn_e.acc_f, Min, bp.hidden, bp.cin,
                                 pa=inp_bn.scale, pb=inp_bn.shift, fin=F(bp.bn_e), lz=L(inp_bn))
                else:
                    self._pw_fwd(K.ACT_NONE, inp_t, bp.w_e, bp.bn_e.y, bp.bn_e.acc_f, Min, bp.hidden, bp.cin,
                                 fin=F(bp.bn_e))
                self._fin_fwd(bp.bn_e, K.pw_num_partials(Min, bp.hidden, bp.cin), train)
                dw_in = bp.bn_e
            else:
                assert inp_t is None and pend is None, "t=1 block expects the (virtual) stem output"
                dw_in = inp_bn
            K.dw_fwd(dw_in.y, dw_in.scale, dw_in.shift, K.ACT_BN_RELU6, f.b(bp.w_d), bp.bn_d.y, bp.bn_d.acc_f, B, Hin, Hin,
                     bp.hidden, bp.stride, fin=F(bp.bn_d), lz=L(dw_in))
            self._fin_fwd(bp.bn_d, K.dw_num_partials("fwd", B, Hin, Hin, bp.hidden, bp.stride), train)
            Mout = B * bp.Ho * bp.Wo
            self._pw_fwd(K.ACT_BN_RELU6, bp.bn_d.y, bp.w_p, bp.bn_p.y, bp.bn_p.acc_f, Mout, bp.cout, bp.hidden,
                         pa=bp.bn_d.scale, pb=bp.bn_d.shift, fin=F(bp.bn_p), lz=L(bp.bn_d))
            self._fin_fwd(bp.bn_p, K.pw_num_partials(Mout, bp.cout, bp.hidden), train)
            # (the consumer -- next expand conv or the final conv, K = bp.cout -- must be a bf16
            # GEMM: the e4m3 one has no BN + residual prologue)
            if bp.Ho * bp.Wo <= self.FUSE_BLOCK_OUTPUT_HW and not self._fp8_layer(bp.cout):
                pend = (bp.bn_p, inp_t if bp.residual else None, bp.o)
            else:
                pend = None   # (a previous block's output was consumed by this block's expand)
                K.bn_apply(bp.bn_p.y, bp.bn_p.scale, bp.bn_p.shift, bp.o, relu6=False,
                           res=inp_t if bp.residual else None, lz=L(bp.bn_p))
            inp_bn, inp_t = bp.bn_p, bp.o
        # final 1x1 conv (materialises the last block output o_17)
        Mf = B * self.Hf * self.Hf
        if pend is not None:
            self._consume_output(pend, f.b(self.w_last), self.bn_last.y, self.bn_last.acc_f, Mf, self.C_last,
                                 self.C_last_in, fin=F(self.bn_last), lz=L(pend[0]))
        else:
            self._pw_fwd(K.ACT_NONE, inp_t, self.w_last, self.bn_last.y, self.bn_last.acc_f, Mf, self.C_last,
                         self.C_last_in, fin=F(self.bn_last))
        self._fin_fwd(self.bn_last, K.pw_num_partials(Mf, self.C_last, self.C_last_in), train)
        if train and self.lazy_bn:
            # side outputs of every forward BN (mean / rstd / scale / shift for the backward
            # and the head, running statistics) in one launch
            self.join_stats()
            K.bn_finalize_batch(self.fwd_fin_tab, self.fwd_fin_n, self.fwd_fin_maxc)
        self.join_stats()   # (no statistics update at all: still joined within the forward)
        # head (+ its backward when training)
        K.head(self.bn_last.y, self.bn_last.scale, self.bn_last.shift, f.w(self.w_lin), f.w(self.b_lin),
               self.labels, B, self.Hf * self.Hf, self.C_last, self.NC, self.drop_p, self.dropout_seed,
               self.hyper, train, 1.0 / B, logits=self.logits, loss=self.loss, correct=self.correct,
               dlogits=self.dlogits if train else None, pd=self.pd,
               g_out=self.bn_last.g if train else None, part=self.bn_last.acc_b if train else None,
               dW=f.g(self.w_lin) if train else None, db=f.g(self.b_lin) if train else None,
               fin=self.bn_last.fin_b if train else None)
        if self._wt_pending:
            K.stream_wait(torch.cuda.current_stream(self.device), self.side)

    # ------------------------------------------------------------------ backward
    def backward(self):
        f, B, S = self.flat, self.B, self.S
        self._check_bn_mode()
        # transposed 1x1 weights for the dgrad GEMMs (one batched launch; done on the side stream
        # during a training forward)
        if not getattr(self, "_wt_pending", False):
            K.wt_transpose(f.shadow, f.shadow_t, self.wt_tab, self.wt_n)
        self._wt_pending = False
        self._ready([self.w_lin, self.b_lin])
        # BN of the final conv (g produced by the head kernel)
        bnl = self.bn_last
        bnl.finalize_bwd(bnl.acc_b, B)
        if not self.lazy_bn:
            self._ready(bnl.param_names)
        Mf = B * self.Hf * self.Hf
        last_blk = self.blocks[-1]
        # dgrad of the final conv -> gradient w.r.t. o_17 (feeds BN_p of block 17, linear)
        K.pw_gemm(K.PRO_BNBWD, K.EPI_BWD_LIN, bnl.g, f.bt(self.w_last), last_blk.G, last_blk.bn_p.acc_b, Mf,
                  self.C_last_in,
                  self.C_last, A2=bnl.y, pa=bnl.a, pb=bnl.b, pc=bnl.c, Yt=last_blk.bn_p.y, R=None,
                  fin=last_blk.bn_p.fin_b, lz=bnl.lz_b)
        P_g = K.pw_num_partials(Mf, self.C_last_in, self.C_last)
        last_blk.bn_p.finalize_bwd(last_blk.bn_p.acc_b, P_g)

        def last_wgrad(ws):
            K.pw_wgrad(bnl.g, bnl.y, bnl.a, bnl.b, bnl.c, last_blk.o, None, None, K.ACT_NONE,
                       ws, f.g(self.w_last), Mf, self.C_last, self.C_last_in)
        self._wgrad(last_wgrad, fins=((bnl, B), (last_blk.bn_p, P_g)))
        self._ready((bnl.param_names if self.lazy_bn else []) + [self.w_last] + last_blk.bn_p.param_names)

        for bi in range(len(self.blocks) - 1, -1, -1):
            bp = self.blocks[bi]
            prev = self.blocks[bi - 1] if bi > 0 else None
            Hin = bp.H
            Min, Mout = B * Hin * Hin, B * bp.Ho * bp.Wo
            bnp, bnd = bp.bn_p, bp.bn_d
            # bn_p backward coefficients were finalised by whoever produced bp.G
            # project dgrad -> g_d (relu6 mask of BN_d) + BN_d partials
            if self._pw_bwd_ok(Mout, bp.cout, bp.hidden):
                # fused dgrad + wgrad (x = relu6(BN_d(y_d)) rebuilt from the mask operand)
                wpm = self._wpart[(bp.idx, "p")]
                K.pw_bwd(K.EPI_BWD_RELU6, bp.G, bnp.y, bnp.a, bnp.b, bnp.c, f.bt(bp.w_p), bnd.g, bnd.y, bnd.acc_b, wpm,
                         None, Mout, bp.cout, bp.hidden, es=bnd.scale, et=bnd.shift, fin=bnd.fin_b, lz=bnp.lz_b)
                Pb = K.pw_bwd_num_partials(Mout, bp.cout, bp.hidden)

                def prj_wgrad(ws, Pb=Pb, wpm=wpm, bp=bp):   # deferred: bind this layer's values
                    K.wgrad_reduce(wpm, Pb, bp.cout * bp.hidden, f.g(bp.w_p))
                self._wgrad(prj_wgrad, fins=((bnd, Pb),))
                bnd.finalize_bwd(bnd.acc_b, Pb)
            else:
                K.pw_gemm(K.PRO_BNBWD, K.EPI_BWD_RELU6, bp.G, f.bt(bp.w_p), bnd.g, bnd.acc_b, Mout, bp.hidden, bp.cout,
                          A2=bnp.y, pa=bnp.a, pb=bnp.b, pc=bnp.c, Yt=bnd.y, es=bnd.scale, et=bnd.shift,
                          fin=bnd.fin_b, lz=bnp.lz_b)
                Pb = K.pw_num_partials(Mout, bp.hidden, bp.cout)
                bnd.finalize_bwd(bnd.acc_b, Pb)

                def prj_wgrad(ws, bnd=bnd, bnp=bnp, bp=bp, Mout=Mout):   # project wgrad (deferred)
                    K.pw_wgrad(bp.G, bnp.y, bnp.a, bnp.b, bnp.c, bnd.y, bnd.scale, bnd.shift,
                               K.ACT_BN_RELU6, ws, f.g(bp.w_p), Mout, bp.cout, bp.hidden)
                self._wgrad(prj_wgrad, fins=((bnd, Pb),))
            self._ready([bp.w_p] + bnd.param_names)
            # depthwise: input BN is BN_e (expand) or the stem BN0 (t=1 block)
            dw_in = bp.bn_e if bp.expand else self.bn0
            Pd = K.dw_num_partials("dgrad", B, Hin, Hin, bp.hidden, bp.stride)
            wpd = self._wpart.get((bp.idx, "d"))
            # the stem BN0's coefficients feed the stem weight gradient on the MAIN stream: its
            # finalize stays there; every other input BN is finalized on the side stream (lazy)
            main_fin = dw_in is self.bn0
            side_fins = () if main_fin else ((dw_in, Pd),)
            if wpd is not None:
                # large maps (bandwidth-bound): fused dgrad + wgrad, one pass over (g, y, yprev);
                # the wgrad partials are reduced on the side stream
                K.dw_dgrad(bnd.g, bnd.y, bnd.coef, f.b(bp.w_d), dw_in.y, dw_in.scale, dw_in.shift, dw_in.g,
                           dw_in.acc_b,
                           B, Hin, Hin, bp.hidden, bp.stride, wpart=wpd, fin=dw_in.fin_b, lz=bnd.lz_b)
                dw_in.finalize_bwd(dw_in.acc_b, Pd, force=main_fin)

                def dw_wg(ws, wpd=wpd, Pd=Pd, bp=bp):   # deferred: bind this layer's values
                    K.wgrad_reduce(wpd, Pd, 9 * bp.hidden, f.g(bp.w_d))
                self._wgrad(dw_wg, fins=side_fins)
            else:
                # small maps (latency-bound): lean dgrad on the critical path, wgrad on the side stream
                K.dw_dgrad(bnd.g, bnd.y, bnd.coef, f.b(bp.w_d), dw_in.y, dw_in.scale, dw_in.shift, dw_in.g,
                           dw_in.acc_b,
                           B, Hin, Hin, bp.hidden, bp.stride, fin=dw_in.fin_b, lz=bnd.lz_b)
                dw_in.finalize_bwd(dw_in.acc_b, Pd, force=main_fin)

                def dw_wg(ws, bnd=bnd, dw_in=dw_in, bp=bp, Hin=Hin):   # deferred
                    K.dw_wgrad(bnd.g, bnd.y, bnd.coef, dw_in.y, dw_in.scale, dw_in.shift, ws,
                               f.g(bp.w_d), B, Hin, Hin, bp.hidden, bp.stride)
                self._wgrad(dw_wg, fins=side_fins)
            self._ready([bp.w_d] + dw_in.param_names)
            if bp.expand:
                bne = bp.bn_e
                assert prev is not None
                # expand dgrad -> gradient w.r.t. the block input o_prev (+ skip gradient)
                if self._pw_bwd_ok(Min, bp.hidden, bp.cin):
                    wpe = self._wpart[(bp.idx, "e")]
                    # (h1 = BN_e's input is re-formed from the staged block input where the kernel can:
                    # Cin <= 32, i.e. the 112x112 / 56x56 / 28x28 blocks)
                    rc = (self.PW_BWD_RECOMPUTE and not self._fp8_layer(bp.cin)   # (bf16 forward GEMM)
                          and K.pw_bwd_recompute_supported(Min, bp.hidden, bp.cin))
                    K.pw_bwd(K.EPI_BWD_LIN, bne.g, None if rc else bne.y, bne.a, bne.b, bne.c, f.bt(bp.w_e), prev.G,
                             prev.bn_p.y, prev.bn_p.acc_b, wpe, None, Min, bp.hidden, bp.cin,
                             R=bp.G if bp.residual else None, X=prev.o, fin=prev.bn_p.fin_b, lz=bne.lz_b,
                             We=f.b(bp.w_e) if rc else None)
                    Pe = K.pw_bwd_num_partials(Min, bp.hidden, bp.cin)

                    def exp_wgrad(ws, Pe=Pe, wpe=wpe, bp=bp):   # deferred: bind this layer's values
                        K.wgrad_reduce(wpe, Pe, bp.hidden * bp.cin, f.g(bp.w_e))
                    self._wgrad(exp_wgrad, fins=((prev.bn_p, Pe),))
                    prev.bn_p.finalize_bwd(prev.bn_p.acc_b, Pe)
                else:
                    K.pw_gemm(K.PRO_BNBWD, K.EPI_BWD_LIN, bne.g, f.bt(bp.w_e), prev.G, prev.bn_p.acc_b, Min, bp.cin,
                              bp.hidden,
                              A2=bne.y, pa=bne.a, pb=bne.b, pc=bne.c, Yt=prev.bn_p.y,
                              R=bp.G if bp.residual else None, fin=prev.bn_p.fin_b, lz=bne.lz_b)
                    Pe = K.pw_num_partials(Min, bp.cin, bp.hidden)
                    prev.bn_p.finalize_bwd(prev.bn_p.acc_b, Pe)

                    def exp_wgrad(ws, prev=prev, bne=bne, bp=bp, Min=Min):   # deferred
                        K.pw_wgrad(bne.g, bne.y, bne.a, bne.b, bne.c, prev.o, None, None,
                                   K.ACT_NONE, ws, f.g(bp.w_e), Min, bp.hidden, bp.cin)
                    self._wgrad(exp_wgrad, fins=((prev.bn_p, Pe),))
                self._ready([bp.w_e] + prev.bn_p.param_names)
            else:
                # t=1 block: its input is relu6(BN0(stem)) -> stem weight gradient.  It is the last
                # work of the backward: on the main stream it runs beside the side stream's backlog
                # instead of queueing behind it (5.95 vs 5.97 ms/step on the side stream, round 1)
                bn0 = self.bn0
                K.stem_wgrad(bn0.g, bn0.y, bn0.a, bn0.b, bn0.c, self.img, self.ws_stem, f.g(self.stem_w), B, S, S, 32)
                self._ready([self.stem_w])
        self._flush_side()
        if self.side is not None:   # join: the optimizer (main stream) needs every gradient
            K.stream_wait(torch.cuda.current_stream(self.device), self.side)

    # ------------------------------------------------------------------ eval
    def eval_prepare(self):
        for bn in self.all_bns():
            bn.eval_prepare()

    def all_bns(self):
        out = [self.bn0]
        for bp in self.blocks:
            if bp.bn_e is not None:
                out.append(bp.bn_e)
            out += [bp.bn_d, bp.bn_p]
        out.append(self.bn_last)
        return out
