"""Static-plan executor: ResNet-50 training step on the gfx950 dense-conv kernels
(BASELINE.json config 4, "ResNet-50 ImageNet-shape 224x224 synthetic DDP").

Same design as the MobileNetV2 executor (engine/executor.py): the network is compiled
once into a fixed schedule of HIP kernels over preallocated NHWC bf16 buffers, BN
statistics come out of the producing conv's epilogue as per-tile partial sums and a
per-channel finalize, and BN-apply + ReLU is fused into the consumer's operand staging:

forward, per bottleneck (x = block input, materialised)
  conv1 1x1       y1 = conv(x)                           + BN1 partials -> finalize
  conv2 3x3 s     y2 = conv(relu(BN1(y1)))               + BN2 partials -> finalize
  conv3 1x1       y3 = conv(relu(BN2(y2)))               + BN3 partials -> finalize
  [projection]    yd = conv_s(x)                         + BNd partials -> finalize
  output          o = relu(BN3(y3) + (BNd(yd) | x))      (materialised, bf16)
stem: 7x7 s2 conv on the 4-channel image, BN0, fused relu + 3x3 s2 max-pool (arg-max kept)
head: average pool -> fc (fp32 split-K GEMM kernels, csrc/kernels/fc.hip) -> softmax CE kernel

backward walks the schedule in reverse.  Gz = dL/d(BN3(y3) + shortcut) is produced by
the NEXT block's conv1 dgrad epilogue ((dx + shortcut grad) * 1[o > 0], with the BN3 and
BNd partial sums of the previous block computed on the way), each dgrad applies its
layer's BN backward (a*G + b*Y + c) while staging dy and the producer's ReLU mask in its
epilogue, and weight gradients (split-M, BN-backward / BN+ReLU fused in the staging)
run on a side stream, reporting finished parameters to the DDP bucket reducer.

LDS-DMA convs (default, ``ops.kernels.conv_set_glds``): the operand tiles of a conv are
streamed global -> LDS by buffer_load ... lds, which needs operands without a prologue.  So
every backward conv first materialises its dy = a*G + b*Y + c once (``bn_mat``; read by both
the dgrad and the side-stream wgrad, which then skip the BN-backward prologue), and the
forward materialises relu(BN(y)) of every conv2 / conv3 input (class attributes RN_DY / RN_ACT
= all|none|auto select the policy; "auto" applies the per-layer rules ``mat_dy_pays`` /
``mat_act_pays`` measured with scripts/conv_bench.py).

Reference call stack for the model forward: SURVEY.md §3.3 (cuDNN conv / BN / ReLU
launches per layer); this executor replaces all of them.
"""
import os
from dataclasses import dataclass
from typing import Callable, List, Optional

import torch

from ..models.resnet import ResNet, Bottleneck
from ..ops import kernels as K
from .executor import AtomicBNState, BNState
from .flat import FlatParams


@dataclass
class ConvSpec:
    name: str       # weight parameter name
    cin: int
    cout: int
    k: int          # kernel size (square)
    stride: int
    pad: int
    H: int          # input spatial size (square)
    dy: Optional[torch.Tensor] = None   # materialised BN-backward output gradient (bn_mat)
    act: bool = False                   # input relu(BN(y)) materialised for this conv (bn_mat)
    w2: Optional[torch.Tensor] = None   # folded BN-backward dgrad: per-step [a.W | b.W] (conv_fold_w)
    fbias: Optional[torch.Tensor] = None

    @property
    def Ho(self) -> int:
        return (self.H + 2 * self.pad - self.k) // self.stride + 1


@dataclass
class BlockPlan:
    prefix: str
    cin: int
    planes: int
    cout: int
    stride: int
    H: int
    Ho: int
    c1: ConvSpec
    c2: ConvSpec
    c3: ConvSpec
    cd: Optional[ConvSpec]
    bn1: BNState
    bn2: BNState
    bn3: BNState
    bnd: Optional[BNState]
    x_in: torch.Tensor = None     # block input (previous output or max-pool output)
    out: torch.Tensor = None      # block output o (materialised)
    out_mask: torch.Tensor = None  # 1[o > 0] as bits, uint8 [M, C/8] (the next block's conv1 dgrad)
    Rd: torch.Tensor = None       # projection-shortcut data gradient (dgrad of cd)


class ResNet50Executor:
    # a training step is native launches, stream joins and plan_py callbacks only (the fc head
    # included: csrc/kernels/fc.hip), so NativeTrainStep replays it from a launch plan
    PLAN_SAFE = True
    # on_params_ready issues only recordable native ops (NativeBucketReducer): called directly
    ready_native = False
    # stem form: "s2d" (space-to-depth 4x4 s1 LDS-DMA conv, 12.13 -> 11.95 ms/step) | "direct"
    STEM = "s2d"
    # which convs get a materialised dy / relu(BN(y)) (all | none | auto): every dy materialised
    # 12.48 -> 12.28 ms/step (all wgrads on the LDS-DMA kernel); activations per layer (auto)
    RN_DY = "all"
    # relu(BN) of every conv2 / conv3 input materialised (LDS-DMA convs only): with those BNs
    # finalized lazily by the bn_mat pass ("act" lazy mode) this beats the per-layer policy
    # ("auto", which kept the register-prologue conv on the large 1x1 inputs): 11.093-11.141 vs
    # 11.190-11.233 ms/step, same box (profiles/r6_resnet50_act_all_ab.txt)
    RN_ACT = "all"

    def __init__(self, model: ResNet, batch: int, img_size: int, device: torch.device,
                 flat: Optional[FlatParams] = None, hyper: Optional[torch.Tensor] = None,
                 side_stream: bool = True, dropout_seed: int = 0, fp8: bool = False):
        assert device.type == "cuda", "the native executor runs on the GPU"
        if fp8:
            raise NotImplementedError("fp8 is implemented for the MobileNetV2 executor")
        self.model = model.to(device)
        self.B, self.S, self.device = batch, img_size, device
        self.dropout_seed = dropout_seed
        self.flat = flat or FlatParams(self.model, device, conv_nhwc=True)
        assert self.flat.nhwc, "ResNet executor needs FlatParams(conv_nhwc=True)"
        B = batch
        f32 = dict(dtype=torch.float32, device=device)
        bf16 = dict(dtype=torch.bfloat16, device=device)
        wgs = []

        def wg_space(c: ConvSpec):
            ci = 4 if c.cin == 3 else c.cin
            wgs.append(K.conv_wgrad_workspace(B, c.H, c.H, ci, c.cout, c.k, c.k, c.stride, c.pad))

        # ---------------- stem + max-pool
        self.stem = ConvSpec("conv1.weight", 3, 64, 7, 2, 3, img_size)
        H0 = self.stem.Ho
        self.H0 = H0
        self.bn0 = AtomicBNState(self.flat, model.bn1, "bn1", B * H0 * H0, 64, device)
        wg_space(self.stem)
        self.Hp = (H0 - 1) // 2 + 1
        self.pool = torch.empty(B * self.Hp * self.Hp, 64, **bf16)
        self.pool_idx = torch.empty(B * self.Hp * self.Hp, 64, dtype=torch.uint8, device=device)
        self.Gpool = torch.empty(B * self.Hp * self.Hp, 64, **bf16)
        # ---------------- bottlenecks
        self.blocks: List[BlockPlan] = []
        H, x_in = self.Hp, self.pool
        for li, layer in enumerate((model.layer1, model.layer2, model.layer3, model.layer4)):
            for bi, blk in enumerate(layer):
                blk: Bottleneck
                pre = f"layer{li + 1}.{bi}"
                cin, planes, cout, s = blk.conv1.in_channels, blk.conv1.out_channels, blk.conv3.out_channels, blk.stride
                Ho = (H - 1) // s + 1
                Min, Mout = B * H * H, B * Ho * Ho
                c1 = ConvSpec(f"{pre}.conv1.weight", cin, planes, 1, 1, 0, H)
                c2 = ConvSpec(f"{pre}.conv2.weight", planes, planes, 3, s, 1, H)
                c3 = ConvSpec(f"{pre}.conv3.weight", planes, cout, 1, 1, 0, Ho)
                cd = ConvSpec(f"{pre}.downsample.0.weight", cin, cout, 1, s, 0, H) if blk.downsample is not None else None
                bn1 = AtomicBNState(self.flat, blk.bn1, f"{pre}.bn1", Min, planes, device)
                bn2 = AtomicBNState(self.flat, blk.bn2, f"{pre}.bn2", Mout, planes, device)
                bn3 = AtomicBNState(self.flat, blk.bn3, f"{pre}.bn3", Mout, cout, device)
                bnd = (AtomicBNState(self.flat, blk.downsample[1], f"{pre}.downsample.1", Mout, cout, device,
                                     need_g=False)
                       if cd is not None else None)
                bp = BlockPlan(pre, cin, planes, cout, s, H, Ho, c1, c2, c3, cd, bn1, bn2, bn3, bnd)
                bp.x_in = x_in
                bp.out = torch.empty(Mout, cout, **bf16)
                if cd is not None:
                    bp.Rd = torch.empty(Min, cin, **bf16)
                for c in (c1, c2, c3) + ((cd,) if cd else ()):
                    wg_space(c)
                self.blocks.append(bp)
                H, x_in = Ho, bp.out
        # ReLU mask of every block output but the last as bits (res_out writes it, the next block's
        # conv1 dgrad epilogue reads 1/16 of the bytes of re-reading o: 12.11 -> 11.98 ms/step)
        for bp in self.blocks[:-1]:
            bp.out_mask = torch.empty(bp.out.shape[0], bp.cout // 8, dtype=torch.uint8, device=device)
        # ---------------- materialised operands of the LDS-DMA convs
        self.mat = K.conv_get_glds() != 0
        act_mode = self.RN_ACT
        # every dy materialised: the weight gradients then run on the LDS-DMA kernel
        # (conv_wgrad_dma_kernel), which the extra bn_mat pass more than pays for
        # (bench step 12.48 -> 12.28 ms on MI355X vs the per-layer "auto" policy)
        dy_mode = self.RN_DY
        if self.mat:
            for bp in self.blocks:
                for c in (bp.c1, bp.c2, bp.c3) + ((bp.cd,) if bp.cd else ()):
                    if c is bp.c3 and self.fold_pays(c):
                        # the BN backward folded into the data gradient's GEMM (no dy pass)
                        c.w2 = torch.empty(2 * c.cin * c.cout, **bf16)
                        c.fbias = torch.empty(c.cin, device=device, dtype=torch.float32)
                        continue
                    if dy_mode == "all" or (dy_mode == "auto" and self.mat_dy_pays(c, B)):
                        c.dy = torch.empty(B * c.Ho * c.Ho, c.cout, **bf16)
                for c, bn in ((bp.c2, bp.bn1), (bp.c3, bp.bn2)):
                    c.act = act_mode == "all" or (act_mode == "auto" and self.mat_act_pays(c, B))
                    if c.act:
                        bn.act = torch.empty(B * c.H * c.H, c.cin, **bf16)
        # ---------------- head
        self.Hf = H
        self.C_last = self.blocks[-1].cout
        self.NC = model.fc.out_features
        self.pooled = torch.zeros(B, self.C_last, **f32)
        self.logits = torch.zeros(B, self.NC, **f32)
        self.dlogits = torch.zeros(B, self.NC, **f32)
        self.dpool = torch.zeros(B, self.C_last, **f32)
        self.loss = torch.zeros(B, **f32)
        self.correct = torch.zeros(B, **f32)
        self.fc_w = self.flat.w("fc.weight").view(self.NC, self.C_last)
        self.fc_b = self.flat.w("fc.bias")
        self.fc_gw = self.flat.g("fc.weight").view(self.NC, self.C_last)
        self.fc_gb = self.flat.g("fc.bias")
        C, NC = self.C_last, self.NC
        self.ws_fc = torch.zeros(max(K.fc_gemm_workspace_floats(B, NC, C), K.fc_gemm_workspace_floats(NC, C, B),
                                     K.fc_gemm_workspace_floats(B, C, NC), 1), **f32)
        # ---------------- BN statistics accumulators
        # every producer (conv forward / dgrad epilogues, max-pool backward, head backward) adds
        # its per-tile partial sums into min(P, bn_rep) replica rows of its BN's zeroed
        # accumulator (common.h bn_part_add), so a finalize reduces <= 8 rows instead of one row
        # per output tile (up to 3136 at 56x56: 5-37 us per finalize launch); one arena, one
        # memset per step.  Deterministic mode: one plainly stored row per tile (bn_rep >= P).
        o, spans = 0, []
        for bn, (pf_, pb_) in self._bn_producer_rows().items():
            bn.rows_f, bn.rows_b = K.bn_rows(pf_), K.bn_rows(pb_)
            nf, nb = K.bn_part_floats(bn.rows_f, bn.C), K.bn_part_floats(bn.rows_b, bn.C)
            spans.append((bn, o, nf, nb))
            o += (nf + nb + 63) // 64 * 64
        self.bn_arena = torch.zeros(o + 64, **f32)
        for bn, o, nf, nb in spans:
            bn.acc_f = self.bn_arena[o:o + nf]
            bn.acc_b = self.bn_arena[o + nf:o + nf + nb]
        # lazy BN finalize (outside deterministic mode; else a finalize launch after every
        # producer): the consumers that support it -- max-pool, the bn_mat passes
        # (relu(BN(y)) forward, dy = a*G + b*Y + c backward) and the block output res_out --
        # compute the BN parameters they need from the replica rows in their prologue, so no
        # finalize launch sits between producer and consumer on the main stream.  The side
        # outputs (mean / rstd / scale / shift / running statistics) come from one batched
        # finalize at the end of the forward; the backward ones (coef, dgamma / dbeta) from
        # batched finalizes on the weight-gradient side stream ahead of the gradient buckets.
        # A BN whose consumer needs materialised parameters (a conv with the BN+ReLU prologue, a
        # dgrad / wgrad with the BN-backward prologue) keeps its finalize launch.
        # PGDIST_BN_LAZY: "act" (default) makes only bn1 / bn2 lazy where a forward relu(BN)
        # materialisation (bn_mat) consumes them; "1" every consumer above; "0" none.  Measured on
        # MI355X at bs128 (same box, profiles/r6_resnet50_lazy_act_ab.txt): act 11.256-11.267,
        # off 11.275-11.306, all 11.393-11.422 ms/step.  Per kernel (rocprofv3 traces of both):
        # a lazy backward bn_mat costs +9 us per launch against a 5 us finalize launch, a lazy
        # max-pool / res_out +28 / +140 us in total, while the forward bn_mat saves ~2.6 us each.
        lazy_mode = os.environ.get("PGDIST_BN_LAZY", "act")
        self.lazy_bn = not K.deterministic() and lazy_mode in ("1", "act")
        lazy_all = lazy_mode == "1"   # "act": only the forward BNs consumed by a bn_mat pass are lazy
        bns = self.all_bns()
        self.bn_ctr = torch.zeros(8 * len(bns) + 16, dtype=torch.int32, device=device)
        self._fin_tabs = {}
        self.fwd_lazy: List[AtomicBNState] = []
        if self.lazy_bn:
            self.refresh_bn_fin()
            # forward: consumers bn0 -> max-pool, bn1 -> conv2 input, bn2 -> conv3 input, bn3 / bnd
            # -> res_out; backward: each BN's coefficients -> bn_mat of its conv's dy (the stem's
            # on the side stream, after its side finalize)
            if lazy_all:
                self.bn0.lz_f, self.bn0.lz_b = self.bn0.desc_f, self.bn0.desc_b
            for bp in self.blocks:
                for bn, c_in, c_dy in ((bp.bn1, bp.c2, bp.c1), (bp.bn2, bp.c3, bp.c2), (bp.bn3, None, bp.c3),
                                       (bp.bnd, None, bp.cd)):
                    if bn is None:
                        continue
                    if (c_in is None and lazy_all) or (c_in is not None and c_in.act):
                        bn.lz_f = bn.desc_f
                    if lazy_all and c_dy.dy is not None:
                        bn.lz_b = bn.desc_b
            self.fwd_lazy = [bn for bn in bns if bn.lz_f is not None]
            self.fwd_fin_tab = K.bn_desc_table([bn.desc_f for bn in self.fwd_lazy])
            self.fwd_fin_maxc = max(bn.C for bn in self.fwd_lazy)
        self.ws_wgrad = torch.zeros(max(wgs) + 1024, **f32)
        # one split-partial workspace per weight gradient of a flushed side-stream group: the
        # group's split-M reductions then run as one multi-segment launch after its wgrads
        # -- measured 11.89-11.93 ms/step batched vs 11.80 with a reduction launch per wgrad (the
        # batch delays the next group's start on the side stream), so per-wgrad reductions here
        self.batch_reductions = False
        nws = 1
        self.ws_wgrad_pool = [self.ws_wgrad] + [torch.zeros_like(self.ws_wgrad) for _ in range(nws - 1)]
        self.side = None
        self._side_pending = []
        self.side_batch = 3   # side-stream joins per 3 weight gradients (2 / 5 / 8: within noise, round 6)
        if side_stream:
            self.side = K.side_stream(device)
            K.register_side_stream(self.side)
        self.img = torch.zeros(B, img_size, img_size, 4, **bf16)
        # space-to-depth stem (default; STEM = "direct": the 7x7 implicit GEMM over the
        # 4-channel image): the 7x7 s2 conv runs as a 4x4 s1 conv over img2 [B,S/2,S/2,16]
        # (K = 256 in four 64-wide LDS-DMA k-steps of 128 contiguous bytes per row instead of 49
        # 8-byte tap gathers), its weight re-laid out each step (stem_w_s2d) and its gradient
        # permuted back to the 7x7 layout.  img2 is written by image_prep(s2d=True) when the
        # training step renders the batch (img_s2d_external), else converted from img.
        self.stem_s2d = self.STEM == "s2d" and img_size % 2 == 0
        self.img_s2d_external = False
        if self.stem_s2d:
            self.img2 = torch.zeros(B, img_size // 2, img_size // 2, 16, **bf16)
            self.w2 = torch.zeros(64 * 256, **bf16)
            self.ws_stem = torch.zeros(K.conv_wgrad_s2d_workspace(B, img_size // 2) + 1024, **f32)
        self.labels = torch.zeros(B, dtype=torch.int64, device=device)
        self.hyper = hyper if hyper is not None else torch.zeros(2, **f32)
        self.on_params_ready: Optional[Callable[[List[str]], None]] = None
        # ready_probe(names) -> True when marking ``names`` launches a gradient bucket; other
        # calls only do host bookkeeping (no side-stream event record / wait per layer)
        self.ready_probe: Optional[Callable[[List[str]], bool]] = None
        # dgrad weights: every conv but the stem transposed to [Cin][R][S][Cout] (one launch)
        tab = []
        for bp in self.blocks:
            for c in (bp.c1, bp.c2, bp.c3) + ((bp.cd,) if bp.cd else ()):
                off = self.flat.offsets[c.name][0]
                tab.append((off, off, c.cout, c.k * c.k, c.cin))
        self.wt_tab = torch.tensor(tab, dtype=torch.int32, device=device).contiguous()

    # ------------------------------------------------------------------ helpers
    def refresh_bn_fin(self):
        """(Re)build the lazy-finalize descriptors in place (after the BN running buffers were
        re-homed, e.g. coalesced for the per-step buffer broadcast), so recorded plans and the
        batched-finalize tables keep valid pointers."""
        if not self.lazy_bn:
            return
        for i, bn in enumerate(self.all_bns()):
            bn.build_desc(self.bn_ctr[8 * i:8 * i + 1], self.bn_ctr[8 * i + 4:8 * i + 5])

    def _bn_producer_rows(self):
        """{bn: (forward P, backward P)}: partial rows of the kernels producing each BN's
        statistics (forward: its conv's epilogue; backward: the dgrad of the conv that consumes
        it, the next block's conv1 dgrad for bn3 / bnd, head_bwd and maxpool_bwd)."""
        B = self.B

        def pf(c: ConvSpec):
            ci = 4 if c.cin == 3 else c.cin
            return K.conv_fwd_num_partials(B, c.Ho, c.Ho, c.cout, c.k * c.k * ci, ci)

        def pd(c: ConvSpec):
            return K.conv_dgrad_num_partials(B, c.H, c.H, c.cin, c.cout, c.k, c.k, c.stride)

        rows = {self.bn0: (pf(self.stem), K.maxpool_bwd_num_partials(B, self.H0, self.H0))}
        for i, bp in enumerate(self.blocks):
            nxt = self.blocks[i + 1] if i + 1 < len(self.blocks) else None
            rows[bp.bn1] = (pf(bp.c1), pd(bp.c2))
            rows[bp.bn2] = (pf(bp.c2), pd(bp.c3))
            rows[bp.bn3] = (pf(bp.c3), pd(nxt.c1) if nxt is not None else B)
            if bp.bnd is not None:
                assert nxt is not None, "a projection shortcut's BN gets its gradient from the next block"
                rows[bp.bnd] = (pf(bp.cd), pd(nxt.c1))
        return rows

    # Materialisation policy, from per-layer timings of every ResNet-50 conv on MI355X at bs 128
    # (scripts/conv_bench.py: dgrad vs bn_mat + dgrad on the materialised dy, fwdbn vs bn_mat +
    # fwd).  A 3x3 conv re-stages each operand element up to 9x per N tile, so its BN prologue is
    # expensive and one materialising pass pays; a 1x1 conv stages each element once per N tile,
    # so the extra pass pays only while the tensor is small (launch-bound maps).
    MAT_ELEMS = 16 * 2 ** 20

    # conv3 data gradients with the BN backward folded into the GEMM (conv_dgrad_fold: K = 2 Cout
    # over [G | Y], no materialised dy) where the GEMM output fits one N tile (Cin <= FOLD_MAX_CIN),
    # so G and Y are each read once: the main stream drops the dy pass (read G, Y, write dy) and
    # reads two tensors instead of one; the side-stream weight gradient applies the BN backward in
    # its prologue (0: off)
    # (measured: 128 -> 11.308-11.327, off 11.346-11.363, 256 11.391-11.423, 512 11.515-11.550 ms/step;
    # profiles/r6_resnet50_fold_ab.txt)
    FOLD_MAX_CIN = 128

    @classmethod
    def fold_pays(cls, c: ConvSpec) -> bool:
        return c.k == 1 and c.stride == 1 and c.cin <= cls.FOLD_MAX_CIN and c.cout % 64 == 0

    @classmethod
    def mat_dy_pays(cls, c: ConvSpec, B: int) -> bool:
        return c.k == 3 or B * c.Ho * c.Ho * c.cout <= cls.MAT_ELEMS

    @classmethod
    def mat_act_pays(cls, c: ConvSpec, B: int) -> bool:
        n = B * c.H * c.H * c.cin
        return n <= 2 * cls.MAT_ELEMS if c.k == 3 else n <= cls.MAT_ELEMS // 2

    def _ready(self, names):
        """Gradients of ``names`` are final once the work enqueued so far completes (same
        contract as MobileNetV2Executor._ready): a call that launches a bucket first flushes the
        deferred side-stream work; a native reducer's bucket launch is itself a recorded native
        op, a host-side reducer runs as a launch-plan Python callback on the side stream."""
        if self.on_params_ready is None:
            return
        if self.side is not None and (self.ready_probe is None or self.ready_probe(names)):
            self._flush_side()
        if self.ready_native:
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
        """Weight-gradient work on the side stream, deferred in groups of ``side_batch`` (one
        side-stream join per group: each join's event record idles the main stream ~5 us;
        see MobileNetV2Executor._wgrad).  ``fins``: (bn, P) backward finalizes of lazy BNs whose
        statistics are complete by now, run (batched) ahead of the group's weight gradients."""
        if self.side is None:
            self._side_fins(list(fins))
            fn(self.ws_wgrad)
            return
        self._side_pending.append((fins, fn))
        if len(self._side_pending) >= min(self.side_batch, len(self.ws_wgrad_pool)):
            self._flush_side()

    def _flush_side(self):
        if self.side is None or not self._side_pending:
            return
        K.stream_wait(self.side, torch.cuda.current_stream(self.device))
        with torch.cuda.stream(self.side):
            self._side_fins([f for fins, _ in self._side_pending for f in fins])
            K.wgrad_reduce_defer(self.batch_reductions)
            try:
                for j, (_, fn) in enumerate(self._side_pending):
                    fn(self.ws_wgrad_pool[j])
            finally:
                K.wgrad_reduce_defer(False)
            if self.batch_reductions:
                K.wgrad_reduce_flush()
        self._side_pending.clear()

    def _side_fins(self, fins):
        """Backward finalizes (coef, dgamma / dbeta) of lazy BNs as one batched launch."""
        fins = [(bn, P) for bn, P in fins if bn.lz_b is not None]
        if not fins:
            return
        if len(fins) == 1:
            bn, P = fins[0]
            bn.finalize_bwd(bn.acc_b, P, force=True)
            return
        key = tuple(id(bn) for bn, _ in fins)
        tab = self._fin_tabs.get(key)
        if tab is None:
            tab = self._fin_tabs[key] = K.bn_desc_table([bn.desc_b for bn, _ in fins])
        K.bn_finalize_batch(tab, len(fins), max(bn.C for bn, _ in fins))

    def _fin(self, bn: AtomicBNState, P: int, train: bool):
        if train:
            if bn.lz_f is None:
                self.join_stats()   # this finalize launch updates the running statistics
            bn.finalize_fwd(bn.acc_f, P)

    def join_stats(self):
        """Main stream joins the per-step BN-buffer broadcast before the first running-statistics
        update of a training forward (MobileNetV2Executor.join_stats)."""
        w = self.__dict__.pop("stats_wait", None)
        if w is not None:
            w()

    def _conv(self, c: ConvSpec, pro, x, y, train, bn_out: BNState, bn_in: Optional[BNState] = None):
        B = self.B
        ci = 4 if c.cin == 3 else c.cin
        if c.act and pro == K.CP_BN_RELU:   # relu(BN(x)) materialised once: plain LDS-DMA conv
            K.bn_mat(K.BN_MAT_ACT, x, bn_in.scale, bn_in.shift, bn_in.act, lz=bn_in.lz_f if train else None)
            pro, x, bn_in = K.CP_NONE, bn_in.act, None
        K.conv_fwd(pro, x, self.flat.b(c.name), y, bn_out.acc_f, B, c.H, c.H, ci, c.cout, c.k, c.k, c.stride,
                   c.pad, pa=bn_in.scale if bn_in is not None else None,
                   pb=bn_in.shift if bn_in is not None else None)
        self._fin(bn_out, K.conv_fwd_num_partials(B, c.Ho, c.Ho, c.cout, c.k * c.k * ci, ci), train)

    def _dy(self, c: ConvSpec, G, bn: BNState):
        """(G, Y) operands of conv ``c``'s dgrad / wgrad: dy = a*G + b*Y + c materialised once
        into c.dy (LDS-DMA kernels, Y = None), or the pair for the fused BN-backward prologue."""
        if c.dy is None:
            return G, bn.y
        K.bn_mat(K.BN_MAT_BWD, bn.y, bn.a, bn.b, c.dy, G=G, c=bn.c, lz=bn.lz_b)
        return c.dy, None

    @staticmethod
    def _wx(c: ConvSpec, x, bn_in: Optional[BNState]):
        """wgrad input operand: the materialised relu(BN(x)) when the forward made one"""
        if bn_in is None:
            return dict(x=x, xpro=K.CP_NONE)
        if c.act:
            return dict(x=bn_in.act, xpro=K.CP_NONE)
        return dict(x=x, xpro=K.CP_BN_RELU, xs=bn_in.scale, xt=bn_in.shift)

    # ------------------------------------------------------------------ forward
    def forward(self, train: bool = True):
        B = self.B
        if not self.__dict__.pop("arena_cleared", False):   # (else cleared by the step's step_begin)
            K.memset(self.bn_arena)   # every BN statistics accumulator of this step
        # the dgrad weight transposes of a training step on the side stream, idle during the
        # forward (as in the MobileNetV2 executor); the main stream joins it at the end of the forward
        self._wt_pending = train and self.side is not None
        if self._wt_pending:
            K.stream_wait(self.side, torch.cuda.current_stream(self.device))
            with torch.cuda.stream(self.side):
                K.conv_wt(self.flat.shadow, self.flat.shadow_t, self.wt_tab, self.wt_tab.shape[0])
        if self.stem_s2d:
            st, H2 = self.stem, self.S // 2
            if not self.img_s2d_external:
                K.s2d_image(self.img, self.img2, B, self.S, self.S)
            K.stem_w_s2d(self.flat.b(st.name), self.w2)
            K.conv_fwd_s2d(self.img2, self.w2, self.bn0.y, self.bn0.acc_f, B, H2)
            self._fin(self.bn0, K.conv_fwd_num_partials(B, H2, H2, 64, 256, 16), train)
        else:
            self._conv(self.stem, K.CP_NONE, self.img, self.bn0.y, train, self.bn0)
        L = (lambda bn: bn.lz_f) if train else (lambda bn: None)   # lazy consumers (training only)  # noqa: E731
        K.maxpool_fwd(self.bn0.y, self.bn0.scale, self.bn0.shift, self.pool, self.pool_idx, B, self.H0, self.H0, 64,
                      lz=L(self.bn0))
        for bp in self.blocks:
            self._conv(bp.c1, K.CP_NONE, bp.x_in, bp.bn1.y, train, bp.bn1)
            self._conv(bp.c2, K.CP_BN_RELU, bp.bn1.y, bp.bn2.y, train, bp.bn2, bp.bn1)
            self._conv(bp.c3, K.CP_BN_RELU, bp.bn2.y, bp.bn3.y, train, bp.bn3, bp.bn2)
            if bp.cd is not None:
                self._conv(bp.cd, K.CP_NONE, bp.x_in, bp.bnd.y, train, bp.bnd)
                lz = (L(bp.bn3), L(bp.bnd)) if L(bp.bn3) is not None and L(bp.bnd) is not None else (None, None)
                K.res_out(bp.bn3.y, bp.bn3.scale, bp.bn3.shift, bp.bnd.y, bp.out, rs=bp.bnd.scale, rt=bp.bnd.shift,
                          lz=lz[0], lz2=lz[1], mask=bp.out_mask if train else None)
            else:
                K.res_out(bp.bn3.y, bp.bn3.scale, bp.bn3.shift, bp.x_in, bp.out, lz=L(bp.bn3),
                          mask=bp.out_mask if train else None)
        if train and self.fwd_lazy:   # side outputs of the lazily consumed BNs, one launch
            self.join_stats()
            K.bn_finalize_batch(self.fwd_fin_tab, len(self.fwd_lazy), self.fwd_fin_maxc)
        self.join_stats()
        # head
        HW = self.Hf * self.Hf
        K.avgpool(self.blocks[-1].out, self.pooled, B, HW, self.C_last)
        C, NC = self.C_last, self.NC
        # logits[b][j] = fc_b[j] + sum_c pooled[b][c] * fc_w[j][c]
        K.fc_gemm(self.pooled, C, 1, self.fc_w, 1, C, self.logits, B, NC, C, bias=self.fc_b, ws=self.ws_fc)
        K.softmax_ce(self.logits, self.labels, self.loss, self.correct, self.dlogits if train else None,
                     scale=1.0 / B)
        if self._wt_pending:   # join the side stream's weight transposes
            K.stream_wait(torch.cuda.current_stream(self.device), self.side)

    # ------------------------------------------------------------------ backward
    def backward(self):
        f, B = self.flat, self.B
        if not getattr(self, "_wt_pending", False):   # (else transposed on the side stream in the forward)
            K.conv_wt(f.shadow, f.shadow_t, self.wt_tab, self.wt_tab.shape[0])
        self._wt_pending = False
        # head: fc gradients (fp32 GEMMs) and the pooled gradient through the last ReLU
        C, NC = self.C_last, self.NC
        # fc_gw[j][c] = sum_b dlogits[b][j] * pooled[b][c];  fc_gb[j] = sum_b dlogits[b][j]
        # dpool[b][c] = sum_j dlogits[b][j] * fc_w[j][c]
        K.fc_gemm(self.dlogits, 1, NC, self.pooled, C, 1, self.fc_gw, NC, C, B, ws=self.ws_fc)
        K.col_sum(self.dlogits, B, NC, self.fc_gb)
        K.fc_gemm(self.dlogits, NC, 1, self.fc_w, C, 1, self.dpool, B, C, NC, ws=self.ws_fc)
        self._ready(["fc.weight", "fc.bias"])
        last = self.blocks[-1]
        HW = self.Hf * self.Hf
        K.head_bwd(self.dpool, last.out, last.bn3.y, last.bn3.g, last.bn3.acc_b, B, HW, self.C_last)
        last.bn3.finalize_bwd(last.bn3.acc_b, B)
        pend_fins = [(last.bn3, B)]   # lazy: finalized on the side stream with the next wgrad group
        if last.bn3.lz_b is None:
            self._ready(last.bn3.param_names)
        for i in range(len(self.blocks) - 1, -1, -1):
            bp = self.blocks[i]
            prev = self.blocks[i - 1] if i > 0 else None
            bn1, bn2, bn3, bnd = bp.bn1, bp.bn2, bp.bn3, bp.bnd
            H, Ho = bp.H, bp.Ho
            c1, c2, c3, cd = bp.c1, bp.c2, bp.c3, bp.cd
            # conv3 dgrad -> G2 (ReLU mask of BN2) + BN2 partials
            g3, y3 = self._dy(c3, bn3.g, bn3)
            if c3.w2 is not None:
                K.conv_fold_w(f.bt(c3.name), bn3.a, bn3.b, bn3.c, bn3.mean, c3.w2, c3.fbias, c3.cin, c3.cout)
                K.conv_dgrad_fold(g3, y3, c3.w2, c3.fbias, bn2.g, bn2.acc_b, B, Ho, Ho, c3.cin, c3.cout,
                                  Yt=bn2.y, es=bn2.scale, et=bn2.shift)
            else:
                K.conv_dgrad(K.CE_BWD_RELU, g3, y3, bn3.a, bn3.b, bn3.c, f.bt(c3.name), bn2.g, bn2.acc_b, B, Ho,
                             Ho, c3.cin, c3.cout, 1, 1, 1, 0, Yt=bn2.y, es=bn2.scale, et=bn2.shift)
            P2 = K.conv_dgrad_num_partials(B, Ho, Ho, c3.cin, c3.cout, 1, 1, 1)
            bn2.finalize_bwd(bn2.acc_b, P2)
            self._wgrad(lambda ws, bp=bp, g3=g3, y3=y3: K.conv_wgrad(
                g3, y3, bp.bn3.a, bp.bn3.b, bp.bn3.c, ws=ws, grad=f.g(bp.c3.name), B=B, H=bp.Ho, W=bp.Ho,
                Ci=bp.c3.cin, N=bp.c3.cout, R=1, S=1, stride=1, pad=0, **self._wx(bp.c3, bp.bn2.y, bp.bn2)),
                fins=pend_fins + [(bn2, P2)])
            self._ready([c3.name] + bn2.param_names + [n for bn_, _ in pend_fins for n in bn_.param_names
                                                       if bn_.lz_b is not None])
            pend_fins = []
            # projection shortcut: data gradient (summed in conv1's dgrad epilogue) + weight gradient
            if cd is not None:
                gd, yd = self._dy(cd, bn3.g, bnd)
                K.conv_dgrad(K.CE_BWD_RES, gd, yd, bnd.a, bnd.b, bnd.c, f.bt(cd.name), bp.Rd, None, B, H, H,
                             cd.cin, cd.cout, 1, 1, cd.stride, 0)
                self._wgrad(lambda ws, bp=bp, gd=gd, yd=yd: K.conv_wgrad(
                    gd, yd, bp.bnd.a, bp.bnd.b, bp.bnd.c, ws=ws, grad=f.g(bp.cd.name), B=B, H=bp.H, W=bp.H,
                    Ci=bp.cd.cin, N=bp.cd.cout, R=1, S=1, stride=bp.cd.stride, pad=0, **self._wx(bp.cd, bp.x_in, None)))
                self._ready([cd.name])
            # conv2 dgrad -> G1 (ReLU mask of BN1) + BN1 partials
            g2, y2 = self._dy(c2, bn2.g, bn2)
            K.conv_dgrad(K.CE_BWD_RELU, g2, y2, bn2.a, bn2.b, bn2.c, f.bt(c2.name), bn1.g, bn1.acc_b, B, H, H,
                         c2.cin, c2.cout, 3, 3, c2.stride, 1, Yt=bn1.y, es=bn1.scale, et=bn1.shift)
            P1b = K.conv_dgrad_num_partials(B, H, H, c2.cin, c2.cout, 3, 3, c2.stride)
            bn1.finalize_bwd(bn1.acc_b, P1b)
            self._wgrad(lambda ws, bp=bp, g2=g2, y2=y2: K.conv_wgrad(
                g2, y2, bp.bn2.a, bp.bn2.b, bp.bn2.c, ws=ws, grad=f.g(bp.c2.name), B=B, H=bp.H, W=bp.H,
                Ci=bp.c2.cin, N=bp.c2.cout, R=3, S=3, stride=bp.c2.stride, pad=1, **self._wx(bp.c2, bp.bn1.y, bp.bn1)),
                fins=[(bn1, P1b)])
            self._ready([c2.name] + bn1.param_names)
            # conv1 dgrad + shortcut gradient -> gradient of the block input:
            #   previous block: Gz_prev = (dx + sc) * 1[o_prev > 0], BN3 (+BNd) partials of that block
            #   first block: gradient of the max-pool output (no ReLU in between)
            sc = bp.Rd if cd is not None else bn3.g
            P1 = K.conv_dgrad_num_partials(B, H, H, c1.cin, c1.cout, 1, 1, 1)
            g1, y1 = self._dy(c1, bn1.g, bn1)
            if prev is not None:
                pds = prev.bnd is not None
                K.conv_dgrad(K.CE_BWD_RES, g1, y1, bn1.a, bn1.b, bn1.c, f.bt(c1.name), prev.bn3.g, prev.bn3.acc_b, B,
                             H, H, c1.cin, c1.cout, 1, 1, 1, 0, Yt=prev.bn3.y, Rg=sc,
                             X=prev.out if prev.out_mask is None else None, Xm=prev.out_mask,
                             Yt2=prev.bnd.y if pds else None, part2=prev.bnd.acc_b if pds else None)
                prev.bn3.finalize_bwd(prev.bn3.acc_b, P1)
                if pds:
                    prev.bnd.finalize_bwd(prev.bnd.acc_b, P1)
            else:
                K.conv_dgrad(K.CE_BWD_RES, g1, y1, bn1.a, bn1.b, bn1.c, f.bt(c1.name), self.Gpool, None, B,
                             H, H, c1.cin, c1.cout, 1, 1, 1, 0, Rg=sc)
            fins1 = [] if prev is None else [(prev.bn3, P1)] + ([(prev.bnd, P1)] if prev.bnd is not None else [])
            self._wgrad(lambda ws, bp=bp, g1=g1, y1=y1: K.conv_wgrad(
                g1, y1, bp.bn1.a, bp.bn1.b, bp.bn1.c, ws=ws, grad=f.g(bp.c1.name), B=B, H=bp.H, W=bp.H,
                Ci=bp.c1.cin, N=bp.c1.cout, R=1, S=1, stride=1, pad=0, **self._wx(bp.c1, bp.x_in, None)),
                fins=fins1)
            names = [c1.name]
            if prev is not None:
                names += prev.bn3.param_names + (prev.bnd.param_names if prev.bnd is not None else [])
            self._ready(names)
        # max-pool + stem
        bn0 = self.bn0
        K.maxpool_bwd(self.Gpool, self.pool_idx, bn0.y, bn0.scale, bn0.shift, bn0.g, bn0.acc_b, B, self.H0, self.H0,
                      64)
        P0 = K.maxpool_bwd_num_partials(B, self.H0, self.H0)
        bn0.finalize_bwd(bn0.acc_b, P0)
        st = self.stem
        # the stem weight gradient reads bn0's materialised coefficients (lazy: its side finalize
        # runs first in the same group).  In the s2d form it runs on the MAIN stream (own
        # split-M workspace), concurrently with the side stream's remaining layer-1 weight
        # gradients: the main stream is otherwise idle from here to the optimizer, which waits
        # for the side stream (~0.5 ms measured)
        if self.stem_s2d:
            stem_wg = lambda ws=None: K.conv_wgrad_s2d(bn0.g, bn0.y, bn0.a, bn0.b, bn0.c, self.img2,  # noqa: E731
                                                       self.ws_stem, f.g(st.name), B, self.S // 2)
            if bn0.lz_b is None:
                self._flush_side()
                stem_wg()
            else:
                self._wgrad(stem_wg, fins=[(bn0, P0)])
        else:
            self._wgrad(lambda ws: K.conv_wgrad(bn0.g, bn0.y, bn0.a, bn0.b, bn0.c, self.img, ws, f.g(st.name), B,
                                                st.H, st.H, 4, st.cout, 7, 7, 2, 3), fins=[(bn0, P0)])
        self._ready([st.name] + bn0.param_names)
        self._flush_side()
        if self.side is not None:
            K.stream_wait(torch.cuda.current_stream(self.device), self.side)

    # ------------------------------------------------------------------ eval
    def all_bns(self):
        out = [self.bn0]
        for bp in self.blocks:
            out += [bp.bn1, bp.bn2, bp.bn3] + ([bp.bnd] if bp.bnd is not None else [])
        return out

    def eval_prepare(self):
        for bn in self.all_bns():
            bn.eval_prepare()
