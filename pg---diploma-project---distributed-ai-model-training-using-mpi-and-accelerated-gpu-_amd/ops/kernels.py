"""Typed, validated Python entry points of the gfx950 HIP kernels.

Each wrapper checks device / dtype / contiguity / shape invariants the kernel
and its launch grid assume (a kernel that reads out of bounds can reset the
whole GPU node, so the checks run on the host before every launch), then calls
the native launcher on the current HIP stream (graph-capture safe: no
allocation, no synchronisation inside).

Activations are NHWC bf16 tensors viewed as [M, C]; per-channel BN vectors are
fp32 [C]; BN partial-sum buffers are fp32 [P, 2, C].
"""
import os
from typing import Optional

import torch

from ._lib import lib

ACT_NONE, ACT_BN_RELU6, ACT_BN, PRO_BNBWD, PRO_BNRES = 0, 1, 2, 3, 5   # PRO_BNRES: A*s + t + A2
EPI_FWD, EPI_BWD_RELU6, EPI_BWD_LIN = 0, 1, 2
AUG_NPARAMS = 16


def _s() -> int:
    return torch.cuda.current_stream().cuda_stream


MAX_KERNEL_BYTES = 1 << 31


def _p(t: Optional[torch.Tensor]) -> int:
    """Device address of a kernel operand.  The kernels address operands through raw buffer
    descriptors with 32-bit byte offsets and mask lanes with the offset 0x80000000
    (common.h kOOB), so every operand must stay below 2 GiB: a larger one would let masked
    lanes read / write real data."""
    if t is None:
        return 0
    if t.numel() * t.element_size() >= MAX_KERNEL_BYTES:
        raise ValueError(f"kernel operand of {t.numel() * t.element_size()} bytes: the HIP kernels take "
                         "operands below 2 GiB (32-bit buffer offsets); reduce the batch size")
    return t.data_ptr()


def _chk(t: Optional[torch.Tensor], dtype, numel=None, name="tensor"):
    if t is None:
        return
    if not t.is_cuda:
        raise ValueError(f"{name}: expected a device tensor")
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name}: must be contiguous")
    if numel is not None and t.numel() < numel:
        raise ValueError(f"{name}: has {t.numel()} elements, kernel needs {numel}")
    if t.data_ptr() % 16:
        raise ValueError(f"{name}: must be 16-byte aligned")


BF16, F32 = torch.bfloat16, torch.float32


# --------------------------------------------------------------------------- BN
def register_side_stream(stream):
    """Reductions launched on ``stream`` get their own arrival counters (they may run
    concurrently with reductions on the main stream)."""
    lib().register_side_stream(stream.cuda_stream)


BN_REP_DETERMINISTIC = 1 << 30   # > any producer's partial rows: one row per workgroup


def bn_rep():
    """Replica rows of the atomic BN-statistics accumulators of the MobileNetV2 producers."""
    return lib().bn_rep()


def set_deterministic(on: bool = True):
    """Bitwise run-to-run reproducible BN statistics.  By default the producers add their
    per-workgroup partial sums into ``bn_rep()`` (8) replica rows with float atomics, whose
    order varies between runs (a few ulp, which a deep net at a tiny batch can amplify);
    deterministic mode gives every workgroup its own row and the finalize sums the rows in a
    fixed order (slightly slower: more rows to reduce, larger accumulators).  Affects
    executors built afterwards (their accumulators are sized for the mode)."""
    lib().bn_set_rep(BN_REP_DETERMINISTIC if on else 8)


def deterministic() -> bool:
    return bn_rep() >= BN_REP_DETERMINISTIC


BN_FIN_BYTES = None


def bn_fin_desc(acc, ctr, rows, C, count, bwd, gamma=None, beta=None, eps=1e-5, momentum=0.1, rmean=None,
                rvar=None, nbt=None, mean=None, rstd=None, scale=None, shift=None, coef=None, dgamma=None,
                dbeta=None):
    """Device descriptor of a BN finalize fused into the tail of its statistics producer
    (bnfin.h): ``acc`` the producer's [rows][2][C] atomic accumulator (rows <= bn_rep()),
    ``ctr`` one int32 arrival counter (zero; re-armed by the kernel).  Forward (bwd=0) writes
    mean / rstd / scale / shift and the running statistics; backward (bwd=1) reads mean / rstd
    and writes coef [3][C], dgamma, dbeta.  Pass the returned tensor as ``fin=`` to the
    producer wrapper (stem_fwd, pw_gemm, pw_gemm_f8, pw_bwd, dw_fwd, dw_dgrad, head)."""
    _chk(acc, F32, 2 * rows * C, "acc")
    _chk(ctr, torch.int32, 1, "ctr")
    for t, n in ((gamma, C), (beta, C), (rmean, C), (rvar, C), (mean, C), (rstd, C), (scale, C), (shift, C),
                 (coef, 3 * C), (dgamma, C), (dbeta, C)):
        _chk(t, F32, n)
    raw = lib().bn_fin_pack(_p(acc), _p(ctr), int(rows), int(C), float(count), int(bwd), _p(gamma), _p(beta),
                            float(eps), float(momentum), _p(rmean), _p(rvar), _p(nbt), _p(mean), _p(rstd),
                            _p(scale), _p(shift), _p(coef), _p(dgamma), _p(dbeta))
    host = torch.frombuffer(bytearray(raw), dtype=torch.uint8)
    return host.to(acc.device)


def _arm(fin):
    """Arm a fused-finalize descriptor for the launch that immediately follows."""
    if fin is not None:
        if not (fin.is_cuda and fin.dtype == torch.uint8):
            raise TypeError("fin: a device descriptor from bn_fin_desc")
        lib().bn_fin_arm(fin.data_ptr())


def _arm_lz(lz):
    """Arm a lazy-finalize descriptor (bn_fin_desc of the BN whose parameters the next launch
    consumes): the consumer computes them from the accumulator rows in its prologue
    (bnfin.h bn_lazy) instead of reading materialised scale / shift / coef."""
    if lz is not None:
        if not (lz.is_cuda and lz.dtype == torch.uint8):
            raise TypeError("lz: a device descriptor from bn_fin_desc")
        lib().bn_lz_arm(lz.data_ptr())


def bn_desc_table(descs):
    """Device table (int64 pointers) of bn_fin_desc descriptors for :func:`bn_finalize_batch`."""
    return torch.tensor([d.data_ptr() for d in descs], dtype=torch.int64, device=descs[0].device)


def bn_finalize_batch(tab, n, max_c):
    """Finalize the n BNs of a descriptor table in one launch (forward descriptors: mean /
    rstd / scale / shift / running statistics; backward: coef / dgamma / dbeta)."""
    assert tab.dtype == torch.int64 and tab.is_contiguous() and tab.numel() >= n
    lib().bn_finalize_batch(_p(tab), int(n), int(max_c), _s())


def bn_rows(P):
    """Rows a BN finalize reduces after a producer with P partial rows accumulated atomically
    (rows = min(P, bn_rep()); the accumulator must be zeroed before the producer runs)."""
    return min(int(P), bn_rep())


def bn_part_floats(P, C):
    """Workspace a BN finalize over P partial rows needs ([P][2][C] + level-1 fold scratch)."""
    return lib().bn_part_floats(P, C)


def bn_fwd_finalize(part, P, C, count, gamma, beta, eps, momentum, rmean, rvar, nbt, mean, rstd,
                    scale, shift):
    _chk(part, F32, bn_part_floats(P, C), "part")
    for n, t in (("gamma", gamma), ("beta", beta), ("rmean", rmean), ("rvar", rvar), ("mean", mean),
                 ("rstd", rstd), ("scale", scale), ("shift", shift)):
        if t is not None and t.numel() < C:
            raise ValueError(f"{n}: too small")
    lib().bn_fwd_finalize(_p(part), P, C, float(count), _p(gamma), _p(beta), float(eps), float(momentum),
                          _p(rmean), _p(rvar), _p(nbt), _p(mean), _p(rstd), _p(scale), _p(shift), _s())


def bn_bwd_finalize(part, P, C, count, mean, rstd, gamma, coef, dgamma=None, dbeta=None):
    _chk(part, F32, bn_part_floats(P, C), "part")
    _chk(coef, F32, 3 * C, "coef")
    lib().bn_bwd_finalize(_p(part), P, C, float(count), _p(mean), _p(rstd), _p(gamma), _p(coef),
                          _p(dgamma), _p(dbeta), _s())


def bn_apply(y, scale, shift, out, relu6=False, res=None, lz=None):
    M, C = y.shape
    assert C % 8 == 0
    _chk(y, BF16, M * C, "y")
    _chk(out, BF16, M * C, "out")
    _chk(res, BF16, M * C, "res")
    if lz is not None and C > 8192:
        raise ValueError("bn_apply: lazy finalize stages 2*C floats in LDS (C <= 8192)")
    _arm_lz(lz)
    lib().bn_apply(_p(y), _p(res), _p(scale), _p(shift), _p(out), M, C, bool(relu6), _s())


# --------------------------------------------------------------------------- optimizer
def adam_flat(p, g, m, v, pb, hyper, beta1, beta2, eps, weight_decay=0.0, grad_scale=1.0, skip=0, metrics=None):
    """Fused Adam over the flat buffers.  ``skip``: device address of a data-parallel
    communicator's error word (NativeComm.error_word) -- the update is skipped while it is set.
    ``metrics``: (loss [B], correct [B], B, acc fp64 [3]) -- the same launch also folds the step's
    metrics into acc, as reduce_metrics would."""
    n = p.numel()
    loss = correct = acc = None
    B = 0
    if metrics is not None:
        loss, correct, B, acc = metrics
        _chk(acc, torch.float64, 3, "acc")
        _chk(loss, F32, B, "loss")
        _chk(correct, F32, B, "correct")
    assert n % 4 == 0 and g.numel() == n and m.numel() == n and v.numel() == n
    for t, nm in ((p, "p"), (g, "g"), (m, "m"), (v, "v")):
        _chk(t, F32, n, nm)
    _chk(pb, BF16, n, "pb")
    lib().adam_flat(_p(p), _p(g), _p(m), _p(v), _p(pb), n, _p(hyper), float(beta1), float(beta2),
                    float(eps), float(weight_decay), float(grad_scale), int(skip), _p(loss), _p(correct), int(B),
                    _p(acc), _s())


def f32_to_bf16(x, y):
    assert x.numel() == y.numel()
    lib().f32_to_bf16(_p(x), _p(y), x.numel(), _s())


def step_begin(hyper, zero=None):
    """hyper[1] += 1 (step counter); with ``zero`` (fp32, 16-byte aligned) the same launch also
    clears that buffer (a step's BatchNorm statistics arena)."""
    n = 0
    if zero is not None:
        assert zero.dtype == F32 and zero.is_contiguous() and zero.data_ptr() % 16 == 0, "step_begin: zero buffer"
        n = zero.numel()
    lib().step_begin(_p(hyper), _p(zero), n, _s())


def reduce_metrics(loss, correct, B, acc):
    _chk(acc, torch.float64, 3, "acc")
    lib().reduce_metrics(_p(loss), _p(correct), B, _p(acc), _s())


# --------------------------------------------------------------------------- depthwise
def dw_out_hw(H, W, stride):
    return (H - 1) // stride + 1, (W - 1) // stride + 1


def dw_num_partials(kind, B, H, W, C, stride):
    f = {"fwd": lib().dw_fwd_num_partials, "dgrad": lib().dw_dgrad_num_partials,
         "wgrad": lib().dw_wgrad_num_partials}[kind]
    return f(B, H, W, C, stride)


def dw_set_geom_mode(mask):
    """Occupancy-aware depthwise tile geometry per kernel kind (bit 1 fwd, 2 dgrad, 4 wgrad;
    default 3: stride-1 forward / dgrad on >= 56-row maps).  Partial counts and workspaces depend on it: switch only
    before sizing them (tests / tuning)."""
    lib().dw_set_geom_mode(int(mask))


def dw_geom_mode():
    return lib().dw_geom_mode()


def dw_set_tall_rows(rows):
    """Tall depthwise geometry (stride-1 forward / dgrad, maps <= 14 rows): the batch is walked
    as one B*H-row image in strips of `rows` rows (0: off; default 14).  Like
    dw_set_geom_mode it changes partial counts: switch only before sizing workspaces."""
    lib().dw_set_tall_rows(int(rows))


def dw_tall_rows():
    return lib().dw_tall_rows()


def dw_set_small_dgrad(on):
    """Round-aware slab / strip choice of the small-map stride-1 dgrad (tall geometry on;
    default on).  Changes partial counts like dw_set_tall_rows."""
    lib().dw_set_small_dgrad(int(on))


def dw_small_dgrad():
    return lib().dw_small_dgrad()


def _dw_check(B, H, W, C, stride):
    if C % 8 or C // 8 > 256:
        raise ValueError(f"depthwise: C={C} must be a multiple of 8 and <= 2048")
    if stride not in (1, 2):
        raise ValueError("depthwise: stride must be 1 or 2")


def dw_fwd(x, in_s, in_t, act, w, y, part, B, H, W, C, stride, fin=None, lz=None):
    _dw_check(B, H, W, C, stride)
    Ho, Wo = dw_out_hw(H, W, stride)
    _chk(x, BF16, B * H * W * C, "x")
    _chk(w, BF16, C * 9, "w")
    _chk(y, BF16, B * Ho * Wo * C, "y")
    _chk(part, F32, bn_rows(dw_num_partials("fwd", B, H, W, C, stride)) * 2 * C, "part")
    _arm(fin)
    _arm_lz(lz)
    lib().dw_fwd(_p(x), _p(in_s), _p(in_t), int(act), _p(w), _p(y), _p(part), B, H, W, C, stride, _s())


def dw_dgrad_wgrad_workspace(B, H, W, C, stride):
    """Floats of wpart a fused depthwise dgrad + wgrad needs ([P][9][C] + reduction rows)."""
    return lib().dw_dgrad_wgrad_workspace_floats(B, H, W, C, stride)


def dw_dgrad(g, yself, coef, w, yprev, ps, pt, gout, part, B, H, W, C, stride, wpart=None, fin=None, lz=None):
    """Depthwise dgrad (+ BN partials of gout).  With ``wpart`` the layer's weight gradient is
    accumulated in the same pass into split partials wpart[P][9][C] (P = dw_num_partials
    ("dgrad", ...)); reduce them with ``wgrad_reduce(wpart, P, 9 * C, grad)``."""
    _dw_check(B, H, W, C, stride)
    Ho, Wo = dw_out_hw(H, W, stride)
    _chk(g, BF16, B * Ho * Wo * C, "g")
    _chk(yself, BF16, B * Ho * Wo * C, "yself")
    _chk(yprev, BF16, B * H * W * C, "yprev")
    _chk(gout, BF16, B * H * W * C, "gout")
    _chk(part, F32, bn_rows(dw_num_partials("dgrad", B, H, W, C, stride)) * 2 * C, "part")
    _chk(wpart, F32, dw_dgrad_wgrad_workspace(B, H, W, C, stride), "wpart")
    _arm(fin)
    _arm_lz(lz)
    lib().dw_dgrad(_p(g), _p(yself), _p(coef), _p(w), _p(yprev), _p(ps), _p(pt), _p(gout), _p(part),
                   B, H, W, C, stride, _p(wpart), _s())


def dw_wgrad_workspace(B, H, W, C, stride):
    P = dw_num_partials("wgrad", B, H, W, C, stride)
    return (P + lib().colsum_rows(P)) * 9 * C


def dw_wgrad(g, yself, coef, yprev, ps, pt, part, grad, B, H, W, C, stride):
    _dw_check(B, H, W, C, stride)
    Ho, Wo = dw_out_hw(H, W, stride)
    _chk(g, BF16, B * Ho * Wo * C, "g")
    _chk(yprev, BF16, B * H * W * C, "yprev")
    _chk(part, F32, dw_wgrad_workspace(B, H, W, C, stride), "part")
    _chk(grad, F32, 9 * C, "grad")
    lib().dw_wgrad(_p(g), _p(yself), _p(coef), _p(yprev), _p(ps), _p(pt), _p(part), _p(grad),
                   B, H, W, C, stride, _s())


# --------------------------------------------------------------------------- pointwise
def pw_num_partials(M, N, K):
    return lib().pw_gemm_num_partials(M, N, K)


def pw_gemm(pro, epi, A, W, out, part, M, N, K, A2=None, pa=None, pb=None, pc=None, Yt=None,
            es=None, et=None, R=None, Aout=None, fin=None, lz=None):
    """out[M,N] = prologue(A)[M,K] @ W^T with W [N,K] in GEMM terms for every mode.

    For the dgrad (pro == PRO_BNBWD) W is the TRANSPOSED conv weight ([Cin][Cout],
    see :func:`wt_transpose`)."""
    if K % 8 or N % 8:
        raise ValueError(f"pw_gemm: K={K}, N={N} must be multiples of 8")
    _chk(A, BF16, M * K, "A")
    _chk(A2, BF16, M * K, "A2")
    _chk(W, BF16, N * K, "W")
    _chk(out, BF16, M * N, "out")
    _chk(Yt, BF16, M * N, "Yt")
    _chk(R, BF16, M * N, "R")
    _chk(part, F32, bn_rows(pw_num_partials(M, N, K)) * 2 * N, "part")
    if pro in (ACT_BN_RELU6, ACT_BN, PRO_BNBWD, PRO_BNRES):
        assert pa is not None and pb is not None and pa.numel() >= K
    if pro == PRO_BNBWD:
        assert A2 is not None and pc is not None
    if pro == PRO_BNRES:
        assert A2 is not None and epi == EPI_FWD
    if Aout is not None and (pro not in (ACT_BN, PRO_BNRES) or epi != EPI_FWD):
        raise ValueError("pw_gemm: Aout (block output) needs the ACT_BN / PRO_BNRES forward prologue")
    if epi in (EPI_BWD_RELU6, EPI_BWD_LIN):
        assert Yt is not None
    if epi == EPI_BWD_RELU6:
        assert es is not None and et is not None
    _chk(Aout, BF16, M * K, "Aout")
    _arm(fin)
    _arm_lz(lz)
    lib().pw_gemm(int(pro), int(epi), _p(A), _p(A2), _p(pa), _p(pb), _p(pc), _p(W), _p(out), _p(Yt),
                  _p(es), _p(et), _p(R), _p(part), M, N, K, _p(Aout), _s())


def pwt_trace_set(buf):
    """Diagnostics (builds with PGDIST_DEFINES=PGDIST_PWT_TRACE): the small-M pointwise GEMM
    (pw_tile) stamps the wall clock at its phase boundaries into ``buf`` (int64 [grid][8])."""
    if buf is not None:
        _chk(buf, torch.int64, buf.numel(), "buf")
    lib().pwt_trace_set(0 if buf is None else buf.data_ptr())


def pwb_trace_set(buf):
    """Diagnostics (PGDIST_PWT_TRACE builds): the fused large-M pointwise backward (pw_bwd) sums
    its per-phase wall clock over its tiles into ``buf`` (int64 [grid][8])."""
    if buf is not None:
        _chk(buf, torch.int64, buf.numel(), "buf")
    lib().pwb_trace_set(0 if buf is None else buf.data_ptr())


def pwg_trace_set(buf):
    """Diagnostics (PGDIST_PWT_TRACE builds): the 1x1 weight gradient (pw_wgrad) stamps the
    wall clock at its phase boundaries into ``buf`` (int64 [grid][8])."""
    if buf is not None:
        _chk(buf, torch.int64, buf.numel(), "buf")
    lib().pwg_trace_set(0 if buf is None else buf.data_ptr())


FP8 = torch.uint8   # raw OCP e4m3fn bytes (torch.float8_e4m3fn views share the encoding)

# activation scale applied before the e4m3 conversion of a GEMM's A operand: ReLU6 outputs
# lie in [0, 6] (x64 -> [0, 384], inside the normal e4m3 range up to 448); BN-linear /
# materialised block outputs are O(1) after BatchNorm (x8 -> saturation only beyond |x| = 56)
FP8_ASC = {ACT_BN_RELU6: 64.0, ACT_BN: 8.0, ACT_NONE: 8.0}


def fp8_pitch(K: int) -> int:
    """Row pitch (bytes) of an e4m3 weight matrix: K rounded up to 64, zero padded."""
    return (K + 63) // 64 * 64


def pw_gemm_f8(pro, A, W8, wsc, out, part, M, N, K, pa=None, pb=None, asc=None, fin=None, lz=None):
    """fp8 forward 1x1 conv: out[M,N] = bf16( (e4m3(asc*prologue(A)) . W8^T) * wsc[n] / asc ).

    W8 is the per-output-channel e4m3 weight copy [N][fp8_pitch(K)] (see :func:`w8_quant`),
    wsc[n] its dequantisation scale; the BN statistics partials are those of the
    dequantised output (same contract as :func:`pw_gemm` with EPI_FWD)."""
    if K % 8 or N % 8:
        raise ValueError(f"pw_gemm_f8: K={K}, N={N} must be multiples of 8")
    if pro not in (ACT_NONE, ACT_BN, ACT_BN_RELU6):
        raise ValueError("pw_gemm_f8: forward prologues only")
    ld = fp8_pitch(K)
    _chk(A, BF16, M * K, "A")
    _chk(W8, FP8, N * ld, "W8")
    _chk(wsc, F32, N, "wsc")
    _chk(out, BF16, M * N, "out")
    _chk(part, F32, bn_rows(pw_num_partials(M, N, K)) * 2 * N, "part")
    if pro != ACT_NONE:
        assert pa is not None and pb is not None and pa.numel() >= K
    a = float(FP8_ASC[pro] if asc is None else asc)
    _arm(fin)
    _arm_lz(lz)
    lib().pw_gemm_f8(int(pro), _p(A), _p(pa), _p(pb), _p(W8), ld, _p(wsc), a, _p(out), _p(part), M, N, K, _s())


def pw_f8_set_mx(on):
    """fp8 tile GEMMs (small M or K > 192) on the block-scaled double-rate
    v_mfma_scale_f32_16x16x128_f8f6f4: 2 (default) on the <= 64-row tiles,
    1 on every tile, 0: the 16x16x32 fp8 MFMA everywhere."""
    lib().pw_f8_set_mx(int(on))


def pw_f8_mx():
    return lib().pw_f8_mx()


def w8_quant(src, dst, wsc, tab, n):
    """Per-output-channel e4m3 quantisation of fp32 1x1 weights, batched over the int32
    table ``tab`` [n,5] = (src offset, N, K, dst byte offset, scale offset)."""
    _chk(src, F32, 1, "src")
    _chk(dst, FP8, 1, "dst")
    _chk(wsc, F32, 1, "wsc")
    assert tab.dtype == torch.int32 and tab.is_contiguous() and tab.numel() >= 5 * n
    lib().w8_quant(_p(src), _p(dst), _p(wsc), _p(tab), int(n), _s())


def wt_transpose(src, dst, tab, n):
    """Batched bf16 transpose of 1x1 conv weights: for each row (off, R, C) of the int32
    table ``tab`` [n,3], dst[off + c*R + r] = src[off + r*C + c]."""
    _chk(src, BF16, 1, "src")
    _chk(dst, BF16, src.numel(), "dst")
    assert tab.dtype == torch.int32 and tab.is_contiguous() and tab.numel() >= 3 * n
    lib().wt_transpose(_p(src), _p(dst), _p(tab), int(n), _s())


def pw_bwd_set_min_m(m):
    """Smallest M (rows) the fused 1x1 dgrad + wgrad kernel takes (set before building an executor)."""
    lib().pw_bwd_set_min_m(int(m))


def pw_bwd_supported(M, Kg, Ng):
    """True when the fused dgrad+wgrad kernel handles this 1x1 conv backward (large M)."""
    return bool(lib().pw_bwd_supported(M, Kg, Ng))


def pw_bwd_num_partials(M, Kg, Ng):
    return lib().pw_bwd_num_partials(M, Kg, Ng)


def pw_bwd_wgrad_workspace(M, Kg, Ng):
    return lib().pw_bwd_wgrad_workspace_floats(M, Kg, Ng)


def pw_bwd_recompute_supported(M, Kg, Ng):
    """True when pw_bwd can re-form Y = X We^T instead of reading it (expand convs, Cin <= 32)."""
    return bool(lib().pw_bwd_recompute_supported(M, Kg, Ng))


def pw_bwd(epi, G, Y, ca, cb, cc, WT, out, Yt, part, wpart, grad, M, Kg, Ng, es=None, et=None, R=None,
           X=None, fin=None, lz=None, We=None):
    """Fused 1x1-conv backward (one read of G, Y):

    dy = ca*G + cb*Y + cc                      [M, Kg]   (this conv's BN backward)
    out = epi(dy @ WT^T)                       [M, Ng]   WT = transposed conv weight [Ng, Kg]
      EPI_BWD_RELU6: out *= 1[0 < Yt*es+et < 6];  EPI_BWD_LIN: out += R
    grad[Kg, Ng] = dy^T @ x,  x = relu6(Yt*es+et) (RELU6) or X (LIN)
    part <- BN partials (sum out, sum out*Yt) per workgroup.
    ``We`` (EPI_BWD_LIN only; the forward weight [Kg, Ng]): Y is not read but re-formed as
    bf16(X @ We^T) from the X tile the wgrad stages anyway (``Y`` may then be None).
    """
    if not pw_bwd_supported(M, Kg, Ng):
        raise ValueError(f"pw_bwd: unsupported shape M={M} Kg={Kg} Ng={Ng}")
    _chk(G, BF16, M * Kg, "G")
    if We is not None:
        if epi != EPI_BWD_LIN or not pw_bwd_recompute_supported(M, Kg, Ng):
            raise ValueError(f"pw_bwd: no Y-recompute form for epi={epi} M={M} Kg={Kg} Ng={Ng}")
        _chk(We, BF16, Kg * Ng, "We")
        if Y is not None:
            _chk(Y, BF16, M * Kg, "Y")
    else:
        if Y is None:
            raise ValueError("pw_bwd: Y (or We for the recompute form) is required")
        _chk(Y, BF16, M * Kg, "Y")
    _chk(WT, BF16, Ng * Kg, "WT")
    _chk(out, BF16, M * Ng, "out")
    _chk(Yt, BF16, M * Ng, "Yt")
    _chk(R, BF16, M * Ng, "R")
    _chk(X, BF16, M * Ng, "X")
    _chk(part, F32, bn_rows(pw_bwd_num_partials(M, Kg, Ng)) * 2 * Ng, "part")
    _chk(wpart, F32, pw_bwd_wgrad_workspace(M, Kg, Ng), "wpart")
    _chk(grad, F32, Kg * Ng, "grad")   # grad=None: reduce wpart later with wgrad_reduce()
    for t, nm in ((ca, "ca"), (cb, "cb"), (cc, "cc")):
        _chk(t, F32, Kg, nm)
    if epi == EPI_BWD_RELU6:
        assert es is not None and et is not None
    elif epi == EPI_BWD_LIN:
        assert X is not None
    else:
        raise ValueError(f"pw_bwd: bad epilogue {epi}")
    _arm(fin)
    _arm_lz(lz)
    lib().pw_bwd(int(epi), _p(G), _p(Y), _p(ca), _p(cb), _p(cc), _p(WT), _p(out), _p(Yt), _p(es), _p(et),
                 _p(R), _p(X), _p(We), _p(part), _p(wpart), _p(grad), M, Kg, Ng, _s())


def wgrad_reduce(part, S, n, grad):
    """grad[n] = sum of the S split rows of part (part holds S + colsum_rows(S) rows of n)."""
    _chk(part, F32, (S + lib().colsum_rows(S)) * n, "part")
    _chk(grad, F32, n, "grad")
    lib().wgrad_reduce(_p(part), int(S), int(n), _p(grad), _s())


def wgrad_reduce_defer(on: bool):
    """While on, every weight-gradient split reduction (wgrad_reduce and the reductions inside
    pw_wgrad / dw_wgrad) is recorded instead of launched; :func:`wgrad_reduce_flush` then
    launches them together (one multi-segment launch per up to 8).  Their partial buffers
    must stay untouched until the flush."""
    lib().wgrad_reduce_defer(bool(on))


def wgrad_reduce_flush():
    lib().wgrad_reduce_flush(_s())


def pw_wgrad_workspace(M, N, K):
    return lib().pw_wgrad_workspace_floats(M, N, K)


def pw_wgrad(G, Y, ga, gb, gc, X, xs, xt, xact, part, grad, M, N, K):
    _chk(G, BF16, M * N, "G")
    _chk(Y, BF16, M * N, "Y")
    _chk(X, BF16, M * K, "X")
    _chk(part, F32, pw_wgrad_workspace(M, N, K), "part")
    _chk(grad, F32, N * K, "grad")
    lib().pw_wgrad(_p(G), _p(Y), _p(ga), _p(gb), _p(gc), _p(X), _p(xs), _p(xt), int(xact), _p(part),
                   _p(grad), M, N, K, _s())


# --------------------------------------------------------------------------- stem
def stem_num_partials(B, H, W):
    return lib().stem_fwd_num_partials(B, H, W)


def stem_fwd(img, w, y, part, B, H, W, px=None, fin=None):
    """Stem 3x3 s2 conv forward; ``px``: 0 = MFMA implicit GEMM (default: MobileNetV2 bs128 on
    MI355X 4.81 vs 4.88 ms/step with the best VALU variant), else output pixels per thread of
    the VALU kernel (1, 2 or 4)."""
    px = 0 if px is None else int(px)
    if px not in (0, 1, 2, 4):
        raise ValueError(f"stem_fwd: px={px} must be 0, 1, 2 or 4")
    Ho, Wo = dw_out_hw(H, W, 2)
    _chk(img, BF16, B * H * W * 4, "img")
    _chk(w, BF16, 32 * 27, "w")
    _chk(y, BF16, B * Ho * Wo * 32, "y")
    _chk(part, F32, bn_rows(stem_num_partials(B, H, W)) * 2 * 32, "part")
    _arm(fin)
    lib().stem_fwd(_p(img), _p(w), _p(y), _p(part), B, H, W, px, _s())


def stem_wgrad_workspace(B, H, W, O=32):
    Ho, Wo = dw_out_hw(H, W, 2)
    return lib().stem_wgrad_workspace_floats(B * Ho * Wo, O)


def stem_wgrad(G, Y, ga, gb, gc, img, part, grad, B, H, W, O=32):
    Ho, Wo = dw_out_hw(H, W, 2)
    _chk(G, BF16, B * Ho * Wo * O, "G")
    _chk(img, BF16, B * H * W * 4, "img")
    _chk(part, F32, stem_wgrad_workspace(B, H, W, O), "part")
    _chk(grad, F32, O * 27, "grad")
    lib().stem_wgrad(_p(G), _p(Y), _p(ga), _p(gb), _p(gc), _p(img), _p(part), _p(grad), B, H, W, O, _s())


# --------------------------------------------------------------------------- head
def head(y, s, t, Wl, bl, labels, B, HW, C, NC, drop_p, seed, hyper, train, loss_scale,
         logits=None, loss=None, correct=None, dlogits=None, pd=None, g_out=None, part=None,
         dW=None, db=None, fin=None):
    if NC > 16 or C % 8 or C // 8 > 256:
        raise ValueError("head kernel supports NC <= 16 and C <= 2048 (C % 8 == 0)")
    _chk(y, BF16, B * HW * C, "y")
    _chk(Wl, F32, NC * C, "Wl")
    if pd is None:
        raise ValueError("head needs pd [B, C] (pooled features; the CE launch reads them)")
    _chk(pd, F32, B * C, "pd")
    if train:
        for t_, n in ((dlogits, "dlogits"), (pd, "pd"), (g_out, "g_out"), (part, "part"), (dW, "dW"),
                      (db, "db")):
            if t_ is None:
                raise ValueError(f"head(train=True) needs {n}")
        _chk(g_out, BF16, B * HW * C, "g_out")
        _chk(part, F32, bn_rows(B) * 2 * C, "part")
    if labels is not None:
        _chk(labels, torch.int64, B, "labels")
    _arm(fin if train else None)
    lib().head(_p(y), _p(s), _p(t), _p(Wl), _p(bl), _p(labels), B, HW, C, NC, float(drop_p),
               int(seed) & ((1 << 64) - 1), _p(hyper), int(bool(train)), float(loss_scale), _p(logits),
               _p(loss), _p(correct), _p(dlogits), _p(pd), _p(g_out), _p(part), _p(dW), _p(db), _s())


# --------------------------------------------------------------------------- data
def augment(src, idx, labels_src, out, labels_out, params_out, train=True, double_resize=True,
            seed=0, hyper=None, epoch_ctr=0, given_params=None, out_hw=224):
    """uint8 [N,32,32,3] (device) gathered by idx [B] -> normalised NHWC4 bf16 [B,S,S,4]."""
    B = idx.numel()
    if src.dtype != torch.uint8 or tuple(src.shape[1:]) != (32, 32, 3) or not src.is_contiguous():
        raise ValueError("augment: src must be contiguous uint8 [N,32,32,3]")
    _chk(idx, torch.int64, B, "idx")
    _chk(out, BF16, B * out_hw * out_hw * 4, "out")
    _chk(params_out, F32, B * AUG_NPARAMS, "params_out")
    _chk(given_params, F32, B * AUG_NPARAMS, "given_params")
    lib().augment(_p(src), _p(idx), _p(labels_src), src.shape[0], B, out_hw, int(bool(train)),
                  int(bool(double_resize)), _p(given_params), int(seed) & ((1 << 64) - 1), _p(hyper),
                  int(epoch_ctr), _p(out), _p(labels_out), _p(params_out), _s())


# --------------------------------------------------------------------------- dense conv (ResNet-50)
CP_NONE, CP_BN_RELU, CP_BNBWD = 0, 1, 3
CE_BWD_RELU, CE_BWD_RES = 1, 2


def conv_set_glds(mode):
    """Operand staging of the dense convs without a prologue: 0 = register-staged kernel,
    2 = LDS-DMA kernel with two LDS buffers (default)."""
    lib().conv_set_glds(int(mode))


def conv_get_glds():
    return lib().conv_get_glds()


def conv_out_hw(H, W, R, S, stride, pad):
    return (H + 2 * pad - R) // stride + 1, (W + 2 * pad - S) // stride + 1


def _conv_check(Ci, N, what):
    if not (Ci % 8 == 0 or Ci == 4) or N % 8:
        raise ValueError(f"{what}: Ci={Ci} must be a multiple of 8 (or 4 for the padded stem input) and "
                         f"N={N} a multiple of 8")


def conv_fwd_num_partials(B, Ho, Wo, N, K, Ci):
    """BN partial rows a forward conv with output [B,Ho,Wo,N] and GEMM depth K writes."""
    return lib().conv_fwd_num_partials(B, Ho, Wo, N, K, Ci)


def conv_dgrad_num_partials(B, H, W, Cin, Cout, R, S, stride):
    return lib().conv_dgrad_num_partials(B, H, W, Cin, Cout, R, S, stride)


def conv_fwd(pro, x, w, y, part, B, H, W, Ci, N, R, S, stride, pad, pa=None, pb=None):
    """NHWC implicit-GEMM convolution  y = conv(pro(x), w)  on MFMA, plus per-tile BN
    partial sums of y.  x [B,H,W,Ci] bf16, w [N,R,S,Ci] bf16, y [B,Ho,Wo,N] bf16;
    pro = CP_BN_RELU applies relu(x*pa + pb) to in-bounds taps (padding stays 0)."""
    _conv_check(Ci, N, "conv_fwd")
    if Ci == 4 and pro != CP_NONE:
        raise ValueError("conv_fwd: the 4-channel (stem) path has no prologue")
    Ho, Wo = conv_out_hw(H, W, R, S, stride, pad)
    _chk(x, BF16, B * H * W * Ci, "x")
    _chk(w, BF16, N * R * S * Ci, "w")
    _chk(y, BF16, B * Ho * Wo * N, "y")
    # BN partial rows: min(P, bn_rep()) replica rows added atomically (zeroed accumulator), or
    # one stored row per M tile in deterministic mode
    _chk(part, F32, bn_rows(conv_fwd_num_partials(B, Ho, Wo, N, R * S * Ci, Ci)) * 2 * N, "part")
    if pro == CP_BN_RELU:
        _chk(pa, F32, Ci, "pa")
        _chk(pb, F32, Ci, "pb")
    lib().conv_fwd(int(pro), _p(x), _p(pa), _p(pb), _p(w), _p(y), _p(part), B, H, W, Ci, N, R, S, stride, pad,
                   _s())


def conv_fold_w(wt, a, b, c, mu, w2, fbias, Cin, Cout):
    """Per-step weights of :func:`conv_dgrad_fold`: w2 [Cin, 2, Cout] bf16 = [a*W | b*W] from the
    transposed 1x1 weight wt [Cin, Cout] and this layer's BN-backward coefficients (a, b, c, fp32
    [Cout]); fbias [Cin] fp32 = sum_k c_k W[n,k] + sum_k mu_k (b_k W[n,k] - bf16(b_k W[n,k]))."""
    if Cout % 8:
        raise ValueError("conv_fold_w: Cout % 8 == 0")
    _chk(wt, BF16, Cin * Cout, "wt")
    for t, nm in ((a, "a"), (b, "b"), (c, "c"), (mu, "mu")):
        _chk(t, F32, Cout, nm)
    _chk(w2, BF16, 2 * Cin * Cout, "w2")
    _chk(fbias, F32, Cin, "fbias")
    lib().conv_fold_w(_p(wt), _p(a), _p(b), _p(c), _p(mu), _p(w2), _p(fbias), Cin, Cout, _s())


def conv_dgrad_fold(G, Y, w2, fbias, dx, part, B, H, W, Cin, Cout, Yt, es, et):
    """1x1 stride-1 data gradient with this layer's BN backward folded into the GEMM:
    dx = [G | Y] . w2^T + fbias (w2 / fbias from :func:`conv_fold_w`), i.e. conv^T(a*G + b*Y + c)
    without materialising dy; epilogue CE_BWD_RELU (dx *= 1[Yt*es + et > 0], BN partials of dx
    against Yt into part, the rows of the unfolded dgrad)."""
    _conv_check(Cout, Cin, "conv_dgrad_fold")
    if Cout % 64 or conv_get_glds() == 0:
        raise ValueError("conv_dgrad_fold: Cout % 64 == 0 and the LDS-DMA kernel")
    for t, nm in ((G, "G"), (Y, "Y")):
        _chk(t, BF16, B * H * W * Cout, nm)
    _chk(w2, BF16, 2 * Cin * Cout, "w2")
    _chk(fbias, F32, Cin, "fbias")
    for t, nm in ((dx, "dx"), (Yt, "Yt")):
        _chk(t, BF16, B * H * W * Cin, nm)
    _chk(es, F32, Cin, "es")
    _chk(et, F32, Cin, "et")
    _chk(part, F32, bn_rows(conv_dgrad_num_partials(B, H, W, Cin, Cout, 1, 1, 1)) * 2 * Cin, "part")
    lib().conv_dgrad_fold(_p(G), _p(Y), _p(w2), _p(fbias), _p(dx), _p(Yt), _p(es), _p(et), _p(part), B, H, W, Cin,
                          Cout, _s())


def conv_dgrad(epi, G, Y, ga, gb, gc, wt, dx, part, B, H, W, Cin, Cout, R, S, stride, pad, Yt=None, es=None,
               et=None, Rg=None, X=None, Yt2=None, part2=None, Xm=None):
    """Data gradient of y = conv(x, w) with this layer's BN backward fused on the way in:
    dy = ga*G + gb*Y + gc  ([B,Ho,Wo,Cout]),  dx = conv^T(dy, wt)  ([B,H,W,Cin]), or with
    Y = None: G is dy itself, materialised by :func:`bn_mat` (LDS-DMA kernel, no prologue), where
    wt = w transposed to [Cin,R,S,Cout] (:func:`conv_wt`).  Epilogues:
      CE_BWD_RELU  dx *= 1[Yt*es + et > 0];  part <- (sum dx, sum dx*Yt)
      CE_BWD_RES   dx = (dx + Rg) * 1[X > 0]  (null operands skipped);
                   part <- (sum dx, sum dx*Yt), part2 <- (sum dx, sum dx*Yt2) when given.
    ``Xm`` instead of X: the ReLU mask as bits, uint8 [B*H*W, Cin/8] (res_out's ``mask``)."""
    _conv_check(Cout, Cin, "conv_dgrad")
    if Y is None and (Cout % 64 or conv_get_glds() == 0):
        raise ValueError("conv_dgrad: a materialised dy (Y=None) needs Cout % 64 == 0 and the LDS-DMA kernel "
                         "(conv_set_glds != 0)")
    if H % stride or W % stride:
        raise ValueError("conv_dgrad: H and W must be multiples of the stride")
    if R > 3 or S > 3:
        raise ValueError("conv_dgrad: filters up to 3x3")
    Ho, Wo = conv_out_hw(H, W, R, S, stride, pad)
    if G is None:
        raise ValueError("conv_dgrad: G is required")
    for t, nm in ((G, "G"), (Y, "Y")):
        _chk(t, BF16, B * Ho * Wo * Cout, nm)
    if Y is not None:
        for t, nm in ((ga, "ga"), (gb, "gb"), (gc, "gc")):
            if t is None:
                raise ValueError(f"conv_dgrad: {nm} is required with Y")
            _chk(t, F32, Cout, nm)
    _chk(wt, BF16, Cin * R * S * Cout, "wt")
    for t, nm in ((dx, "dx"), (Yt, "Yt"), (Rg, "Rg"), (X, "X"), (Yt2, "Yt2")):
        _chk(t, BF16, B * H * W * Cin, nm)
    P = bn_rows(conv_dgrad_num_partials(B, H, W, Cin, Cout, R, S, stride))   # rows written (see conv_fwd)
    if epi == CE_BWD_RELU:
        if Yt is None or es is None or et is None:
            raise ValueError("conv_dgrad(CE_BWD_RELU) needs Yt, es, et")
        _chk(part, F32, P * 2 * Cin, "part")
    if Xm is not None:
        if X is not None:
            raise ValueError("conv_dgrad: X or Xm, not both")
        _chk(Xm, torch.uint8, B * H * W * Cin // 8, "Xm")
    if epi == CE_BWD_RELU:
        pass
    elif epi == CE_BWD_RES:
        ops = (Rg is not None, X is not None or Xm is not None, Yt is not None, Yt2 is not None)
        if ops not in ((False, False, False, False), (True, False, False, False), (True, True, True, False),
                       (True, True, True, True)):
            raise ValueError("conv_dgrad(CE_BWD_RES): operand sets {} | {Rg} | {Rg,X,Yt} | {Rg,X,Yt,Yt2}")
        if Yt is not None:
            _chk(part, F32, P * 2 * Cin, "part")
        if Yt2 is not None:
            if Yt is None:
                raise ValueError("conv_dgrad: Yt2 needs Yt")
            _chk(part2, F32, P * 2 * Cin, "part2")
    else:
        raise ValueError(f"conv_dgrad: bad epilogue {epi}")
    lib().conv_dgrad(int(epi), _p(G), _p(Y), _p(ga), _p(gb), _p(gc), _p(wt), _p(dx), _p(Yt), _p(es), _p(et),
                     _p(Rg), _p(X), _p(Yt2), _p(part), _p(part2), B, H, W, Cin, Cout, R, S, stride, pad, _p(Xm),
                     _s())


def conv_wgrad_workspace(B, H, W, Ci, N, R, S, stride, pad):
    return lib().conv_wgrad_workspace_floats(B, H, W, Ci, N, R, S, stride, pad)


def conv_wgrad(G, Y, ga, gb, gc, x, ws, grad, B, H, W, Ci, N, R, S, stride, pad, xpro=CP_NONE, xs=None, xt=None):
    """grad [N,R,S,Ci] (fp32, overwritten) = sum_m dy[m] (x) im2col(x')[m] with
    dy = ga*G + gb*Y + gc (or G itself when Y is None: materialised by :func:`bn_mat`) and
    x' = relu(x*xs + xt) (xpro = CP_BN_RELU) or x."""
    _conv_check(Ci, N, "conv_wgrad")
    Ho, Wo = conv_out_hw(H, W, R, S, stride, pad)
    if G is None:
        raise ValueError("conv_wgrad: G is required")
    _chk(G, BF16, B * Ho * Wo * N, "G")
    _chk(Y, BF16, B * Ho * Wo * N, "Y")
    if Y is not None:
        for t, nm in ((ga, "ga"), (gb, "gb"), (gc, "gc")):
            if t is None:
                raise ValueError(f"conv_wgrad: {nm} is required with Y")
            _chk(t, F32, N, nm)
    _chk(x, BF16, B * H * W * Ci, "x")
    if xpro == CP_BN_RELU:
        _chk(xs, F32, Ci, "xs")
        _chk(xt, F32, Ci, "xt")
    _chk(ws, F32, conv_wgrad_workspace(B, H, W, Ci, N, R, S, stride, pad), "ws")
    _chk(grad, F32, N * R * S * Ci, "grad")
    lib().conv_wgrad(_p(G), _p(Y), _p(ga), _p(gb), _p(gc), _p(x), _p(xs), _p(xt), int(xpro), _p(ws), _p(grad),
                     B, H, W, Ci, N, R, S, stride, pad, _s())


BN_MAT_ACT, BN_MAT_BWD = 0, 1


def bn_mat(mode, Y, a, b, out, G=None, c=None, lz=None):
    """Materialise a BN-transformed [M, C] bf16 operand for the LDS-DMA convs:
    BN_MAT_ACT  out = relu(Y*a + b)        (producer BN + ReLU: the next conv's input)
    BN_MAT_BWD  out = a*G + b*Y + c        (this layer's BN backward: dgrad / wgrad dy)
    C/8 must divide 256 (C in 8, 16, ..., 2048 powers of two).  ``lz``: lazy finalize
    descriptor (bn_fin_desc of this BN, forward for ACT / backward for BWD): the kernel computes
    a, b (, c) from the producer's replica rows itself; a, b, c are then not read."""
    M, C = Y.shape
    if C % 8 or 256 % (C // 8):
        raise ValueError(f"bn_mat: C={C} (C/8 must divide 256)")
    _chk(Y, BF16, M * C, "Y")
    _chk(out, BF16, M * C, "out")
    _chk(a, F32, C, "a")
    _chk(b, F32, C, "b")
    if mode == BN_MAT_BWD:
        if G is None or c is None:
            raise ValueError("bn_mat(BN_MAT_BWD) needs G and c")
        _chk(G, BF16, M * C, "G")
        _chk(c, F32, C, "c")
    elif mode != BN_MAT_ACT:
        raise ValueError(f"bn_mat: bad mode {mode}")
    _arm_lz(lz)
    lib().bn_mat(int(mode), _p(G), _p(Y), _p(a), _p(b), _p(c), _p(out), M, C, _s())


def conv_wt(src, dst, tab, n):
    """Batched bf16 weight transpose for dgrad: for each row (src_off, dst_off, Cout, taps, Cin)
    of the int32 table ``tab`` [n,5], dst[ci][t][co] = src[co][t][ci]."""
    _chk(src, BF16, 1, "src")
    _chk(dst, BF16, 1, "dst")
    assert tab.dtype == torch.int32 and tab.is_contiguous() and tab.numel() >= 5 * n
    lib().conv_wt(_p(src), _p(dst), _p(tab), int(n), _s())


def res_out(y, s, t, r, out, rs=None, rt=None, lz=None, lz2=None, mask=None):
    """Bottleneck output out = relu(y*s + t + r'), r' = r*rs + rt (projection shortcut BN) or r.
    ``lz`` (, ``lz2`` with the projection): lazy finalize descriptors of the two BNs (s, t / rs,
    rt computed from the producers' replica rows in the kernel).  ``mask``: uint8 [M, C/8]
    also written, bit j of byte i = (out element 8i+j > 0) (conv_dgrad's ``Xm``)."""
    M, C = y.shape
    if C % 8:
        raise ValueError("res_out: C % 8")
    for x_, nm in ((y, "y"), (r, "r"), (out, "out")):
        _chk(x_, BF16, M * C, nm)
    ok = (lz is None and lz2 is None) or (lz is not None and (rs is None) == (lz2 is None))
    if not ok:
        raise ValueError("res_out: lz (and lz2 with the projection BN) both or neither")
    for d in (lz, lz2):
        if d is not None and not (d.is_cuda and d.dtype == torch.uint8):
            raise TypeError("res_out: lz descriptors from bn_fin_desc")
    _chk(mask, torch.uint8, M * C // 8, "mask")
    lib().res_out(_p(y), _p(s), _p(t), _p(r), _p(rs), _p(rt), _p(out), M, C, _p(lz), _p(lz2), _p(mask), _s())


def maxpool_fwd(y, s, t, out, idx, B, H, W, C, lz=None):
    """3x3 s2 p1 max-pool of relu(y*s+t) -> out [B,Ho,Wo,C] bf16 + arg-max tap (uint8);
    ``lz``: s, t from the producer's replica rows (lazy finalize descriptor)."""
    Ho, Wo = conv_out_hw(H, W, 3, 3, 2, 1)
    if C % 8:
        raise ValueError("maxpool: C % 8")
    _chk(y, BF16, B * H * W * C, "y")
    _chk(out, BF16, B * Ho * Wo * C, "out")
    _chk(idx, torch.uint8, B * Ho * Wo * C, "idx")
    _arm_lz(lz)
    lib().maxpool_fwd(_p(y), _p(s), _p(t), _p(out), _p(idx), B, H, W, C, _s())


def maxpool_bwd_num_partials(B, H, W):
    return lib().maxpool_bwd_num_partials(B, H, W)


def maxpool_bwd(gp, idx, y, s, t, g, part, B, H, W, C):
    """Max-pool backward fused with the stem BN's ReLU mask: g = route(gp) * 1[y*s+t > 0],
    part <- (sum g, sum g*y) per workgroup (C == 64), atomically into bn_rows(P) replica rows of a
    zeroed accumulator (deterministic mode: one stored row per workgroup)."""
    if C != 64:
        raise ValueError("maxpool_bwd: C must be 64")
    Ho, Wo = conv_out_hw(H, W, 3, 3, 2, 1)
    _chk(gp, BF16, B * Ho * Wo * C, "gp")
    _chk(idx, torch.uint8, B * Ho * Wo * C, "idx")
    _chk(y, BF16, B * H * W * C, "y")
    _chk(g, BF16, B * H * W * C, "g")
    _chk(part, F32, bn_rows(maxpool_bwd_num_partials(B, H, W)) * 2 * C, "part")
    lib().maxpool_bwd(_p(gp), _p(idx), _p(y), _p(s), _p(t), _p(g), _p(part), B, H, W, C, _s())


def avgpool(x, out, B, HW, C):
    if C % 8 or C // 8 > 256:
        raise ValueError("avgpool: C % 8 and C <= 2048")
    _chk(x, BF16, B * HW * C, "x")
    _chk(out, F32, B * C, "out")
    lib().avgpool(_p(x), _p(out), B, HW, C, _s())


def head_bwd(dpool, x, y, G, part, B, HW, C):
    """G = dpool/HW broadcast * 1[x > 0];  part <- (sum G, sum G*y) per image, atomically into
    bn_rows(B) replica rows of a zeroed accumulator (deterministic mode: row b = image b)."""
    if C % 8 or C // 8 > 256:
        raise ValueError("head_bwd: C % 8 and C <= 2048")
    _chk(dpool, F32, B * C, "dpool")
    for t, nm in ((x, "x"), (y, "y"), (G, "G")):
        _chk(t, BF16, B * HW * C, nm)
    _chk(part, F32, bn_rows(B) * 2 * C, "part")
    lib().head_bwd(_p(dpool), _p(x), _p(y), _p(G), _p(part), B, HW, C, _s())


def softmax_ce(logits, labels, loss, correct, dlogits=None, scale=1.0):
    B, NC = logits.shape
    _chk(logits, F32, B * NC, "logits")
    _chk(labels, torch.int64, B, "labels")
    _chk(loss, F32, B, "loss")
    _chk(correct, F32, B, "correct")
    _chk(dlogits, F32, B * NC, "dlogits")
    lib().softmax_ce(_p(logits), _p(labels), B, NC, float(scale), _p(loss), _p(correct), _p(dlogits), _s())


def fc_gemm_workspace_floats(M, N, K):
    return int(lib().fc_gemm_workspace_floats(M, N, K))


def _strided_span(t, rows, cols, s_row, s_col, nm):
    """the strided fp32 operand t(r, c) = t[r*s_row + c*s_col] must fit inside t"""
    if t.dtype != F32 or not t.is_contiguous():
        raise ValueError(f"fc_gemm: {nm} must be contiguous fp32")
    need = (rows - 1) * s_row + (cols - 1) * s_col + 1
    if s_row < 0 or s_col < 0 or t.numel() < need:
        raise ValueError(f"fc_gemm: {nm} has {t.numel()} elements, the strides address {need}")


def fc_gemm(A, sam, sak, B, sbk, sbn, C, M, N, K, bias=None, ws=None):
    """fp32 C[m][n] = sum_k A[m*sam + k*sak] * B[k*sbk + n*sbn] (+ bias[n]); deterministic
    (split-K partials in `ws`, fc_gemm_workspace_floats(M, N, K) floats, summed in a fixed order)."""
    if min(M, N, K) < 1:
        raise ValueError("fc_gemm: empty shape")
    _strided_span(A, M, K, sam, sak, "A")
    _strided_span(B, K, N, sbk, sbn, "B")
    _chk(C, F32, M * N, "C")
    _chk(bias, F32, N, "bias")
    nws = fc_gemm_workspace_floats(M, N, K)
    if nws:
        _chk(ws, F32, nws, "ws")
    lib().fc_gemm(_p(A), sam, sak, _p(B), sbk, sbn, _p(bias), _p(C), M, N, K, _p(ws) if nws else 0, _s())


def col_sum(X, M, N, out):
    """out[n] = sum over rows m of X[m][n] (fixed order)"""
    _chk(X, F32, M * N, "X")
    _chk(out, F32, N, "out")
    lib().col_sum(_p(X), M, N, _p(out), _s())


def image_prep(src, idx, labels_src, out, labels_out, seed=0, hyper=None, s2d=False):
    """uint8 [N,H,W,3] pool gathered by idx [B] -> random h-flip, ImageNet normalisation,
    NHWC bf16 [B,H,W,4] (4th channel 0); ``s2d``: space-to-depth by 2 instead,
    [B,H/2,W/2,16] with channel (dh*2 + dw)*4 + c (the input of :func:`conv_fwd_s2d`)."""
    B = idx.numel()
    if src.dtype != torch.uint8 or src.dim() != 4 or src.shape[3] != 3 or not src.is_contiguous():
        raise ValueError("image_prep: src must be contiguous uint8 [N,H,W,3]")
    H, W = src.shape[1], src.shape[2]
    _chk(idx, torch.int64, B, "idx")
    _chk(out, BF16, B * H * W * 4, "out")
    _chk(labels_out, torch.int64, B, "labels_out")
    if s2d and (H % 2 or W % 2):
        raise ValueError("image_prep: space-to-depth needs even H and W")
    lib().image_prep(_p(src), _p(idx), _p(labels_src), B, H, W, int(seed) & ((1 << 64) - 1), _p(hyper), _p(out),
                     _p(labels_out), int(bool(s2d)), _s())


# --------------------------------------------------------------------------- space-to-depth stem
def s2d_image(img, x2, B, H, W):
    """img [B,H,W,4] bf16 -> space-to-depth x2 [B,H/2,W/2,16] (layout of image_prep(s2d=True))."""
    if H % 2 or W % 2:
        raise ValueError("s2d_image: even H and W")
    _chk(img, BF16, B * H * W * 4, "img")
    _chk(x2, BF16, B * H * W * 4, "x2")
    lib().s2d_image(_p(img), _p(x2), B, H, W, _s())


def stem_w_s2d(w, w2, N=64):
    """w [N,7,7,4] bf16 (the 7x7 stem weight, 4-channel storage) -> w2 [N,4,4,16] bf16 with
    w2[n][r][s][(dh*2+dw)*4+c] = w[n][2r+dh-1][2s+dw-1][c] (zero outside the 7x7)."""
    _chk(w, BF16, N * 196, "w")
    _chk(w2, BF16, N * 256, "w2")
    lib().stem_w_s2d(_p(w), _p(w2), N, _s())


def conv_fwd_s2d(x2, w2, y, part, B, H2, N=64):
    """The 7x7 s2 p3 stem as a 4x4 s1 conv over the space-to-depth image x2 [B,H2,H2,16]
    (LDS-DMA kernel, multi-tap k-steps): y [B,H2,H2,N] bf16 + BN partial sums of y (rows as
    :func:`conv_fwd`)."""
    _chk(x2, BF16, B * H2 * H2 * 16, "x2")
    _chk(w2, BF16, N * 256, "w2")
    _chk(y, BF16, B * H2 * H2 * N, "y")
    _chk(part, F32, bn_rows(conv_fwd_num_partials(B, H2, H2, N, 256, 16)) * 2 * N, "part")
    lib().conv_fwd_s2d(_p(x2), _p(w2), _p(y), _p(part), B, H2, N, _s())


def conv_wgrad_s2d_workspace(B, H2, N=64):
    return lib().conv_wgrad_s2d_workspace_floats(B, H2, N)


def conv_wgrad_s2d(G, Y, ga, gb, gc, x2, ws, grad, B, H2, N=64):
    """Stem weight gradient grad [N,7,7,4] (fp32, overwritten) from dy = ga*G + gb*Y + gc
    ([B,H2,H2,N]; or G itself with Y None) and the space-to-depth image x2."""
    for t, nm in ((G, "G"), (Y, "Y")):
        _chk(t, BF16, B * H2 * H2 * N, nm)
    if Y is not None:
        for t, nm in ((ga, "ga"), (gb, "gb"), (gc, "gc")):
            _chk(t, F32, N, nm)
    _chk(x2, BF16, B * H2 * H2 * 16, "x2")
    _chk(ws, F32, conv_wgrad_s2d_workspace(B, H2, N), "ws")
    _chk(grad, F32, N * 196, "grad")
    lib().conv_wgrad_s2d(_p(G), _p(Y), _p(ga), _p(gb), _p(gc), _p(x2), _p(ws), _p(grad), B, H2, N, _s())


# --------------------------------------------------------------------------- launch plans
def stream_wait(waiter, signaler):
    """``waiter`` waits for the work enqueued so far on ``signaler`` (torch streams); unlike
    ``Stream.wait_stream`` it is recorded into an open launch plan."""
    lib().stream_wait(waiter.cuda_stream, signaler.cuda_stream)


def memset(t: torch.Tensor, value: int = 0):
    """Byte-wise fill of a contiguous device tensor on the current stream (recordable)."""
    if not (t.is_cuda and t.is_contiguous()):
        raise ValueError("memset: contiguous device tensor expected")
    lib().memset_async(t.data_ptr(), int(value), t.numel() * t.element_size(), _s())


def plan_py(fn):
    """Run ``fn()`` now and, while a launch plan is being recorded, again at this point of
    every replay (host-side Python work of a step, e.g. the DDP bucket hand-off)."""
    lib().plan_py(fn)


def plan_recording() -> bool:
    return lib().plan_recording()


class LaunchPlan:
    """One training step recorded as a native launch sequence (csrc/runtime/plan.h).

    ``record(fn)`` runs ``fn()`` eagerly and records every native launch, stream wait,
    memset and ``plan_py`` callback it issues; ``replay()`` re-issues them from C++ (no Python
    wrapper or validation in between).  Everything ``fn`` passes to the kernels must stay
    valid (fixed buffers; per-step values in device memory) — the hipGraph-capture contract."""

    def __init__(self):
        self.id = None

    def record(self, fn):
        lib().plan_record_begin()
        try:
            fn()
        except BaseException:
            lib().plan_record_abort()
            raise
        self.id = lib().plan_record_end()

    def replay(self):
        lib().plan_replay(self.id)

    def __len__(self):
        return 0 if self.id is None else lib().plan_size(self.id)

    def free(self):
        if self.id is not None:
            lib().plan_free(self.id)
            self.id = None


def side_stream(device):
    """The weight-gradient side stream of an executor: a plain stream.  (CU-masked streams
    (hipExtStreamCreateWithCUMask) measured 1.5-1.9x slower steps with every mask tried, even the
    full one -- docs/PERF_NOTES.md rounds 2-4 -- and were removed.)"""
    return torch.cuda.Stream(device)


# --------------------------------------------------------------------------- launch log (diagnostics)
# While a launch plan is recorded with the log on, every kernel wrapper call appends its op range
# in the plan, its tensor operands' bytes and its integer shape arguments: scripts/roofline.py
# then times each range in isolation (lib().plan_time_ops) for a per-op roofline table.
_LOG = None
_LOG_DEPTH = [0]
# operands that are workspaces / whole pools / tiny side tables, not per-op traffic
_LOG_SKIP = {"part", "wpart", "ws", "params_out", "given_params", "tab", "fin", "lz", "hyper", "src", "idx",
             "labels_src", "labels_out", "labels", "W8", "wsc"}


def launch_log_start():
    global _LOG
    _LOG = []


def launch_log_stop():
    global _LOG
    out, _LOG = _LOG, None
    return out


def _logged(fn):
    import functools
    import inspect
    sig = inspect.signature(fn)

    @functools.wraps(fn)
    def wrapper(*a, **kw):
        if _LOG is None or _LOG_DEPTH[0] > 0:
            return fn(*a, **kw)
        before = lib().plan_recording_size()
        _LOG_DEPTH[0] += 1
        try:
            r = fn(*a, **kw)
        finally:
            _LOG_DEPTH[0] -= 1
        after = lib().plan_recording_size()
        if after > before:
            ba = sig.bind(*a, **kw).arguments
            nb = sum(v.numel() * v.element_size() for k, v in ba.items()
                     if torch.is_tensor(v) and k not in _LOG_SKIP)
            ints = {k: v for k, v in ba.items() if isinstance(v, int) and not isinstance(v, bool)}
            _LOG.append(dict(op=fn.__name__, first=before, last=after, bytes=nb, shape=ints, stream=_s()))
        return r
    return wrapper


for _name in ("bn_fwd_finalize", "bn_bwd_finalize", "bn_apply", "bn_finalize_batch", "adam_flat", "f32_to_bf16",
              "step_begin", "reduce_metrics", "dw_fwd", "dw_dgrad", "dw_wgrad", "pw_gemm", "pw_gemm_f8", "w8_quant",
              "wt_transpose", "pw_bwd", "wgrad_reduce", "wgrad_reduce_flush", "pw_wgrad", "stem_fwd", "stem_wgrad",
              "head", "augment", "conv_fwd", "conv_dgrad", "conv_wgrad", "bn_mat", "conv_wt", "res_out", "maxpool_fwd",
              "maxpool_bwd", "avgpool", "head_bwd", "softmax_ce", "fc_gemm", "col_sum", "image_prep", "memset"):
    globals()[_name] = _logged(globals()[_name])
