"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op.

Inputs are bf16-representable (kernels read bf16 storage); the reference runs in
fp32 on those exact values, so the residual error is the kernels' own bf16
output rounding and fp32 accumulation order.
"""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from pgdist.ops import kernels as K  # noqa: E402


def bf(t):
    return t.to(torch.bfloat16)


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def rnd(*shape, dev, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dev)


def bn_params(C, dev, seed=1):
    g = torch.Generator(device="cpu").manual_seed(seed)
    s = (torch.rand(C, generator=g) + 0.5).to(dev)
    t = (torch.rand(C, generator=g) - 0.5).to(dev)
    return s.contiguous(), t.contiguous()


def relu6(x):
    return x.clamp(0, 6)


def tapmajor(w):
    """[C,1,3,3] depthwise weight -> the kernels' tap-major [9][C] storage."""
    return w.reshape(w.shape[0], 9).t().contiguous()


def bn_ws(part, P, C):
    """[P][2][C] partials padded to the workspace a BN finalize needs (level-1 scratch)."""
    flat = part.reshape(-1)
    extra = K.bn_part_floats(P, C) - flat.numel()
    return torch.cat([flat, torch.zeros(max(extra, 0), device=flat.device)]).contiguous()


def sum_parts(part, P, C, nv=2):
    return part[: P * nv * C].view(P, nv, C).sum(0)


# ----------------------------------------------------------------------------- BN
@pytest.mark.parametrize("P,C", [(40, 24), (700, 96), (10752, 32), (3001, 1280)])
def test_bn_reduce_two_level(dev, P, C):
    """Single-launch two-level reduction (last-workgroup hand-off), repeated launches with
    different data and uneven row counts: every launch must match an fp64 reference exactly
    enough and re-arm its counters."""
    gamma, beta = bn_params(C, dev, 3)
    for it in range(6):
        part = rnd(P, 2, C, dev=dev, seed=100 + it) + 1.0
        part[:, 1] = part[:, 1].abs() * 3 + 5
        ws = bn_ws(part, P, C)
        mean, rstd, scale, shift = [torch.empty(C, device=dev) for _ in range(4)]
        K.bn_fwd_finalize(ws, P, C, 1e6, gamma, beta, 1e-5, 0.1, None, None, None, mean, rstd, scale, shift)
        s = part.double().sum(0)
        m_ref = s[0] / 1e6
        assert torch.allclose(mean.double(), m_ref, rtol=1e-5, atol=1e-7)
        coef = torch.empty(3, C, device=dev)
        dg, db = torch.empty(C, device=dev), torch.empty(C, device=dev)
        K.bn_bwd_finalize(ws, P, C, 1e6, mean, rstd, gamma, coef, dg, db)
        assert torch.allclose(db.double(), s[0], rtol=1e-5, atol=1e-3)
    torch.cuda.synchronize()


def test_bn_finalize_and_apply(dev):
    M, C = 5000, 96
    y = bf(rnd(M, C, dev=dev) * 2 + 0.3)
    P = 7
    chunks = torch.tensor_split(y.float(), P, dim=0)
    part = torch.stack([torch.stack([c.sum(0), (c * c).sum(0)]) for c in chunks]).contiguous()
    gamma, beta = bn_params(C, dev, 3)
    rm, rv = torch.zeros(C, device=dev), torch.ones(C, device=dev)
    nbt = torch.zeros(1, dtype=torch.int64, device=dev)
    mean, rstd, scale, shift = [torch.empty(C, device=dev) for _ in range(4)]
    K.bn_fwd_finalize(bn_ws(part, P, C), P, C, M, gamma, beta, 1e-5, 0.1, rm, rv, nbt, mean, rstd, scale, shift)
    ref = torch.nn.BatchNorm2d(C).to(dev)
    with torch.no_grad():
        ref.weight.copy_(gamma)
        ref.bias.copy_(beta)
    out_ref = ref(y.float().t().reshape(1, C, M, 1)).reshape(C, M).t()
    torch.cuda.synchronize()
    assert torch.allclose(rm, ref.running_mean, rtol=1e-4, atol=1e-5)
    assert torch.allclose(rv, ref.running_var, rtol=1e-4, atol=1e-5)
    assert int(nbt.item()) == 1
    out = torch.empty_like(y)
    K.bn_apply(y, scale, shift, out, relu6=True)
    assert rel(out, relu6(out_ref)) < 1e-2
    res = bf(rnd(M, C, dev=dev, seed=5))
    K.bn_apply(y, scale, shift, out, relu6=False, res=res)
    assert rel(out, out_ref + res.float()) < 1e-2


def test_bn_bwd_finalize_matches_autograd(dev):
    M, C = 4096, 64
    y = bf(rnd(M, C, dev=dev) * 1.5 + 0.2).float()
    gamma, beta = bn_params(C, dev, 4)
    g = bf(rnd(M, C, dev=dev, seed=9)).float()
    yy = y.clone().requires_grad_(True)
    ga = gamma.clone().requires_grad_(True)
    be = beta.clone().requires_grad_(True)
    out = F.batch_norm(yy.t().reshape(1, C, M, 1), None, None, ga, be, training=True, eps=1e-5)
    out.backward(g.t().reshape(1, C, M, 1))
    mean = y.mean(0)
    rstd = torch.rsqrt(y.var(0, unbiased=False) + 1e-5)
    part = torch.stack([g.sum(0), (g * y).sum(0)]).unsqueeze(0).contiguous()
    coef = torch.empty(3, C, device=dev)
    dgam, dbet = torch.empty(C, device=dev), torch.empty(C, device=dev)
    K.bn_bwd_finalize(bn_ws(part, 1, C), 1, C, M, mean.contiguous(), rstd.contiguous(), gamma, coef, dgam, dbet)
    dy = coef[0] * g + coef[1] * y + coef[2]
    assert rel(dy, yy.grad) < 1e-4
    assert rel(dgam, ga.grad) < 1e-4
    assert rel(dbet, be.grad) < 1e-4


# ----------------------------------------------------------------------------- depthwise
DW_CASES = [(2, 14, 14, 32, 1), (2, 14, 14, 96, 2), (3, 28, 28, 144, 1), (2, 7, 7, 960, 1),
            (2, 56, 56, 96, 2), (1, 28, 28, 576, 2), (2, 9, 9, 24, 1), (2, 10, 10, 16, 2),
            # partial last column tile (W not a multiple of the tile width), odd sizes, full-size rows
            (1, 57, 57, 64, 2), (1, 45, 45, 192, 1), (1, 112, 112, 32, 1), (1, 112, 112, 96, 2),
            (1, 29, 31, 48, 2), (1, 13, 33, 40, 1),
            # narrow maps: widened channel slabs (dw_geom: CC up to 128, e.g. 120 for C = 960)
            (2, 14, 14, 576, 2), (2, 7, 7, 576, 1), (1, 5, 5, 120, 1), (2, 14, 14, 960, 2), (1, 7, 9, 480, 1),
            (2, 8, 8, 384, 2)]


@pytest.mark.parametrize("B,H,W,C,stride", DW_CASES)
def test_dw_fwd(dev, B, H, W, C, stride):
    x = bf(rnd(B, H, W, C, dev=dev, seed=B + C))
    s, t = bn_params(C, dev)
    w = bf(rnd(C, 1, 3, 3, dev=dev, seed=3) * 0.3)
    Ho, Wo = K.dw_out_hw(H, W, stride)
    y = torch.empty(B, Ho, Wo, C, dtype=torch.bfloat16, device=dev)
    P = K.dw_num_partials("fwd", B, H, W, C, stride)
    part = torch.zeros(P * 2 * C, device=dev)
    K.dw_fwd(x, s, t, K.ACT_BN_RELU6, tapmajor(w), y, part, B, H, W, C, stride)
    z = relu6(x.float() * s + t).permute(0, 3, 1, 2)
    ref = F.conv2d(z, w.float(), stride=stride, padding=1, groups=C).permute(0, 2, 3, 1)
    assert rel(y, ref) < 8e-3
    st = sum_parts(part, P, C)
    r2 = ref.reshape(-1, C)
    assert rel(st[0], r2.sum(0)) < 1e-3
    assert rel(st[1], (r2 * r2).sum(0)) < 1e-3


@pytest.mark.parametrize("B,H,W,C,stride", DW_CASES)
def test_dw_dgrad_wgrad(dev, B, H, W, C, stride):
    yprev = bf(rnd(B, H, W, C, dev=dev, seed=11))
    s, t = bn_params(C, dev, 2)
    w = bf(rnd(C, 1, 3, 3, dev=dev, seed=3) * 0.3)
    Ho, Wo = K.dw_out_hw(H, W, stride)
    g = bf(rnd(B, Ho, Wo, C, dev=dev, seed=12))
    yself = bf(rnd(B, Ho, Wo, C, dev=dev, seed=13))
    coef = torch.stack([torch.rand(C, device=dev) + 0.5, torch.rand(C, device=dev) - 0.5,
                        torch.rand(C, device=dev) - 0.5]).contiguous()
    dy = (coef[0] * g.float() + coef[1] * yself.float() + coef[2]).permute(0, 3, 1, 2)
    z = relu6(yprev.float() * s + t).permute(0, 3, 1, 2)
    dz = torch.nn.grad.conv2d_input(z.shape, w.float(), dy, stride=stride, padding=1, groups=C)
    a = yprev.float() * s + t
    mask = ((a > 0) & (a < 6)).float()
    gref = dz.permute(0, 2, 3, 1) * mask
    gout = torch.empty(B, H, W, C, dtype=torch.bfloat16, device=dev)
    P = K.dw_num_partials("dgrad", B, H, W, C, stride)
    part = torch.zeros(P * 2 * C, device=dev)
    K.dw_dgrad(g, yself, coef, tapmajor(w), yprev, s, t, gout, part, B, H, W, C, stride)
    assert rel(gout, gref) < 8e-3
    st = sum_parts(part, P, C)
    assert rel(st[0], gref.reshape(-1, C).sum(0)) < 2e-2
    assert rel(st[1], (gref * yprev.float()).reshape(-1, C).sum(0)) < 2e-2
    # wgrad
    wref = torch.nn.grad.conv2d_weight(z, w.shape, dy, stride=stride, padding=1, groups=C)
    wpart = torch.zeros(K.dw_wgrad_workspace(B, H, W, C, stride), device=dev)
    grad = torch.empty(C * 9, device=dev)
    K.dw_wgrad(g, yself, coef, yprev, s, t, wpart, grad, B, H, W, C, stride)
    assert rel(grad.view(9, C).t().reshape(C, 1, 3, 3), wref) < 1e-3
    # fused dgrad + wgrad (one pass): identical dgrad, same weight gradient
    gout2 = torch.empty_like(gout)
    part2 = torch.zeros(P * 2 * C, device=dev)
    wpart2 = torch.zeros(K.dw_dgrad_wgrad_workspace(B, H, W, C, stride), device=dev)
    K.dw_dgrad(g, yself, coef, tapmajor(w), yprev, s, t, gout2, part2, B, H, W, C, stride, wpart=wpart2)
    # identical dgrad; the BN partials are float-atomic sums (order-dependent in the last bits)
    assert torch.equal(gout2, gout) and torch.allclose(part2, part, rtol=1e-5, atol=1e-5)
    grad2 = torch.empty(C * 9, device=dev)
    K.wgrad_reduce(wpart2, P, 9 * C, grad2)
    assert rel(grad2.view(9, C).t().reshape(C, 1, 3, 3), wref) < 1e-3


def _dw_all(B, H, C, stride, dev):
    """fwd y, BN sums, fused dgrad gout, its BN sums and weight gradient, separate weight gradient"""
    x = bf(rnd(B, H, H, C, dev=dev, seed=21))
    s, t = bn_params(C, dev, 2)
    w = tapmajor(bf(rnd(C, 1, 3, 3, dev=dev, seed=3) * 0.3))
    Ho, _ = K.dw_out_hw(H, H, stride)
    y = torch.empty(B, Ho, Ho, C, dtype=torch.bfloat16, device=dev)
    Pf = K.dw_num_partials("fwd", B, H, H, C, stride)
    pf = torch.zeros(K.bn_rows(Pf) * 2 * C, device=dev)
    K.dw_fwd(x, s, t, K.ACT_BN_RELU6, w, y, pf, B, H, H, C, stride)
    g = bf(rnd(B, Ho, Ho, C, dev=dev, seed=12))
    gen = torch.Generator(device="cpu").manual_seed(7)
    coef = (torch.rand(3, C, generator=gen) + torch.tensor([[0.5], [-0.5], [-0.5]])).to(dev).contiguous()
    gout = torch.empty(B, H, H, C, dtype=torch.bfloat16, device=dev)
    Pd = K.dw_num_partials("dgrad", B, H, H, C, stride)
    pd = torch.zeros(K.bn_rows(Pd) * 2 * C, device=dev)
    wp = torch.zeros(K.dw_dgrad_wgrad_workspace(B, H, H, C, stride), device=dev)
    K.dw_dgrad(g, y, coef, w, x, s, t, gout, pd, B, H, H, C, stride, wpart=wp)
    gw1 = torch.empty(C * 9, device=dev)
    K.wgrad_reduce(wp, Pd, 9 * C, gw1)
    ws = torch.zeros(K.dw_wgrad_workspace(B, H, H, C, stride), device=dev)
    gw2 = torch.empty(C * 9, device=dev)
    K.dw_wgrad(g, y, coef, x, s, t, ws, gw2, B, H, H, C, stride)
    torch.cuda.synchronize()
    return (y, sum_parts(pf, K.bn_rows(Pf), C), gout, sum_parts(pd, K.bn_rows(Pd), C), gw1, gw2,
            (Pf, Pd, K.dw_num_partials("wgrad", B, H, H, C, stride)))


@pytest.mark.parametrize("H,C,stride", [(56, 144, 1), (56, 144, 2), (28, 192, 2), (112, 32, 1)])
def test_dw_occupancy_geometry(dev, H, C, stride):
    """The occupancy-aware tile geometry (dw_set_geom_mode 15: every kind, unrestricted; channel
    slab / strip length chosen per launch from the resident-workgroup count) computes the same convolution as the default
    geometry at the MobileNetV2 bs128 shapes: identical activations and dgrad, BN sums and
    weight gradients equal up to float summation order."""
    B = 128
    old = K.dw_geom_mode()
    try:
        K.dw_set_geom_mode(0)
        ref = _dw_all(B, H, C, stride, dev)
        K.dw_set_geom_mode(15)
        out = _dw_all(B, H, C, stride, dev)
    finally:
        K.dw_set_geom_mode(old)
    assert torch.equal(out[0], ref[0]) and torch.equal(out[2], ref[2])
    for a, b in zip(out[1:6], ref[1:6]):
        if a.dtype != torch.bfloat16:
            assert rel(a, b) < 1e-4
    if (H, C) == (56, 144):
        assert out[6] != ref[6]   # the model re-tiles these layers


@pytest.mark.parametrize("B,H,C,rows,small", [(128, 7, 960, 28, 0), (128, 14, 384, 28, 0), (128, 14, 576, 21, 0),
                                              (5, 7, 960, 10, 0), (3, 14, 384, 9, 0), (128, 14, 384, 14, 1),
                                              (128, 14, 576, 14, 1), (128, 7, 960, 14, 1)])
def test_dw_tall_geometry(dev, B, H, C, rows, small):
    """Tall geometry (dw_set_tall_rows: the batch walked as one B*H-row image in strips that
    cross image boundaries, here also strips starting mid-image and a partial last strip):
    the window taps across an image edge are masked, so forward activations and dgrad are
    identical to the per-image tiling and the BN sums / weight gradients (fused and separate)
    equal up to float summation order."""
    old, old_small = K.dw_tall_rows(), K.dw_small_dgrad()
    try:
        K.dw_set_tall_rows(0)
        K.dw_set_small_dgrad(0)
        ref = _dw_all(B, H, C, 1, dev)
        K.dw_set_tall_rows(rows)
        K.dw_set_small_dgrad(small)   # round-aware dgrad slab / strip choice
        out = _dw_all(B, H, C, 1, dev)
    finally:
        K.dw_set_tall_rows(old)
        K.dw_set_small_dgrad(old_small)
    assert torch.equal(out[0], ref[0]) and torch.equal(out[2], ref[2])
    for a, b in zip(out[1:6], ref[1:6]):
        if a.dtype != torch.bfloat16:
            assert rel(a, b) < 1e-4
    tiles_w = ref[6][0] // B   # column tiles per image row (unchanged)
    assert out[6][0] == -(-B * H // rows) * tiles_w
    if small:   # the dgrad tiling differs where one round of workgroups is reachable
        assert out[6][1] != ref[6][1] or C == 960


# ----------------------------------------------------------------------------- pointwise
# small M -> L2-direct weights with the K split over waves (KS 1/2/4); M >= 65536 -> LDS-resident weights
PW_CASES = [(1000, 16, 96), (4096, 24, 144), (777, 96, 24), (3000, 320, 1280), (2048, 160, 960),
            (513, 32, 32), (6272, 960, 160), (256, 64, 384), (70001, 16, 96), (65600, 144, 24),
            (66000, 192, 64), (68000, 24, 160)]


@pytest.mark.parametrize("M,K_,N", PW_CASES)
@pytest.mark.parametrize("pro", [K.ACT_NONE, K.ACT_BN_RELU6])
def test_pw_fwd(dev, M, K_, N, pro):
    A = bf(rnd(M, K_, dev=dev, seed=M))
    s, t = bn_params(K_, dev)
    W = bf(rnd(N, K_, dev=dev, seed=5) / math.sqrt(K_))
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    P = K.pw_num_partials(M, N, K_)
    part = torch.zeros(P * 2 * N, device=dev)
    K.pw_gemm(pro, K.EPI_FWD, A, W, out, part, M, N, K_, pa=s, pb=t)
    x = relu6(A.float() * s + t) if pro == K.ACT_BN_RELU6 else A.float()
    ref = x @ W.float().t()
    assert rel(out, ref) < 8e-3
    st = sum_parts(part, P, N)
    assert rel(st[0], ref.sum(0)) < 1e-2
    assert rel(st[1], (ref * ref).sum(0)) < 1e-2


@pytest.mark.parametrize("M,K_,N,epi", [(6272, 960, 160, K.EPI_FWD), (6272, 1280, 320, K.EPI_BWD_LIN),
                                        (25088, 576, 96, K.EPI_FWD), (1111, 1216, 200, K.EPI_BWD_RELU6)])
def test_pw_splitk_bitwise_repeatable(dev, M, K_, N, epi):
    """Small-M / long-K GEMMs split K over workgroups (pwtile.hip split-K): the last arriver sums
    the fp32 slabs in split order, so repeated launches (different arrival orders) are bitwise
    equal, the ticket counters re-arm (a second launch on the same workspace is correct), and the
    result matches the fp32 reference."""
    A = bf(rnd(M, K_, dev=dev, seed=M))
    W = bf(rnd(N, K_, dev=dev, seed=5) / math.sqrt(K_))
    P = K.pw_num_partials(M, N, K_)
    outs, parts = [], []
    for _ in range(3):
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        part = torch.zeros(P * 2 * N, device=dev)
        if epi == K.EPI_FWD:
            K.pw_gemm(K.ACT_NONE, epi, A, W, out, part, M, N, K_)
        else:
            ones, zeros = torch.ones(K_, device=dev), torch.zeros(K_, device=dev)
            Yt = bf(rnd(M, N, dev=dev, seed=6))
            es, et = torch.ones(N, device=dev), torch.full((N,), 3.0, device=dev)
            K.pw_gemm(K.PRO_BNBWD, epi, A, W, out, part, M, N, K_, A2=A, pa=ones, pb=zeros, pc=zeros,
                      Yt=Yt, es=es, et=et, R=torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
                      if epi == K.EPI_BWD_LIN else None)
        outs.append(out)
        parts.append(part)
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    ref = A.float() @ W.float().t()
    if epi == K.EPI_BWD_RELU6:
        a = Yt.float() + 3.0
        ref = ref * ((a > 0) & (a < 6)).float()
    assert rel(outs[0], ref) < 8e-3


def e4m3(x):
    """fp32 -> OCP e4m3fn (saturating) -> fp32, PyTorch's conversion as the reference."""
    return x.clamp(-448.0, 448.0).to(torch.float8_e4m3fn).float()


def test_w8_quant_matches_torch_e4m3(dev):
    """Per-output-channel e4m3 weight quantisation: bytes equal PyTorch's float8_e4m3fn
    encoding of w / (amax/448), rows zero-padded to the 64-byte pitch, two layers in one launch."""
    shapes = [(96, 24), (1280, 320)]
    ws = [rnd(n, k, dev=dev, seed=n) * 0.1 for n, k in shapes]
    ws[0][3].zero_()                                    # all-zero row -> scale 1, zero bytes
    src = torch.cat([w.flatten() for w in ws])
    tab, so, do, co = [], 0, 0, 0
    for n, k in shapes:
        tab.append([so, n, k, do, co])
        so += n * k
        do += n * K.fp8_pitch(k)
        co += n
    dst = torch.full((do,), 0xAB, dtype=torch.uint8, device=dev)
    wsc = torch.zeros(co, device=dev)
    K.w8_quant(src, dst, wsc, torch.tensor(tab, dtype=torch.int32, device=dev), len(tab))
    for (n, k), w, (_, _, _, d0, c0) in zip(shapes, ws, tab):
        ld = K.fp8_pitch(k)
        amax = w.abs().amax(1)
        s = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
        assert torch.allclose(wsc[c0:c0 + n], s)
        q = dst[d0:d0 + n * ld].view(n, ld)
        ref = (w / s[:, None]).clamp(-448, 448).to(torch.float8_e4m3fn).view(torch.uint8)
        assert torch.equal(q[:, :k], ref)
        assert int(q[:, k:].count_nonzero()) == 0


@pytest.mark.parametrize("M,K_,N,mx", [(70001, 16, 96, 1), (100352, 24, 144, 1), (66000, 192, 64, 1),
                                       (6272, 960, 160, 1), (6272, 960, 160, 0), (25088, 64, 384, 1),
                                       (25088, 64, 384, 0), (3000, 320, 1280, 1), (3000, 320, 1280, 0),
                                       (777, 96, 24, 1), (777, 96, 24, 0), (25088, 160, 960, 1), (4096, 576, 96, 1),
                                       (25088, 160, 960, 2), (6272, 960, 160, 2)])
@pytest.mark.parametrize("pro", [K.ACT_NONE, K.ACT_BN_RELU6, K.ACT_BN])
def test_pw_fwd_fp8(dev, M, K_, N, mx, pro):
    """fp8 forward GEMM: equals the fp32 GEMM of the e4m3-rounded operands (PyTorch
    float8_e4m3fn conversion) up to the bf16 output rounding.  mx = 1: the tile-path launches
    (M < 65536 or K > 192) on the block-scaled v_mfma_scale_f32_16x16x128_f8f6f4 (128-wide k
    steps, K zero-padded: K = 960 / 320 / 96 / 160 / 576); mx = 2: only the <= 64-row tiles
    (the default); mx = 0: v_mfma_f32_16x16x32_fp8_fp8."""
    old = K.pw_f8_mx()
    K.pw_f8_set_mx(mx)
    try:
        _pw_fwd_fp8(dev, M, K_, N, pro)
    finally:
        K.pw_f8_set_mx(old)


def _pw_fwd_fp8(dev, M, K_, N, pro):
    A = bf(rnd(M, K_, dev=dev, seed=M))
    s, t = bn_params(K_, dev)
    W = rnd(N, K_, dev=dev, seed=5) / math.sqrt(K_)
    ld = K.fp8_pitch(K_)
    W8 = torch.empty(N * ld, dtype=torch.uint8, device=dev)
    wsc = torch.empty(N, device=dev)
    K.w8_quant(W.flatten(), W8, wsc, torch.tensor([[0, N, K_, 0, 0]], dtype=torch.int32, device=dev), 1)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    P = K.pw_num_partials(M, N, K_)
    part = torch.zeros(P * 2 * N, device=dev)
    K.pw_gemm_f8(pro, A, W8, wsc, out, part, M, N, K_, pa=s, pb=t)
    asc = K.FP8_ASC[pro]
    x = A.float()
    if pro == K.ACT_BN_RELU6:
        x = relu6(x * s + t)
    elif pro == K.ACT_BN:
        x = x * s + t
    xq = e4m3(x * asc) / asc
    wq = W8.view(N, ld)[:, :K_].view(torch.float8_e4m3fn).float() * wsc[:, None]
    ref = xq @ wq.t()
    assert rel(out, ref) < 6e-3
    assert rel(ref, x @ W.t()) < 0.08          # e4m3 vs exact: a few % (3 mantissa bits)
    st = sum_parts(part, P, N)
    assert rel(st[0], ref.sum(0)) < 1e-2
    assert rel(st[1], (ref * ref).sum(0)) < 1e-2


@pytest.mark.parametrize("M,K_,N", [(70001, 24, 144), (25088, 64, 384), (6272, 320, 1280), (100352, 32, 192)])
@pytest.mark.parametrize("res", [False, True])
def test_pw_fwd_block_output(dev, M, K_, N, res):
    """Consumer GEMM of a block output: prologue BN (+ residual) and the block output o written
    on the way (replaces a separate BN-apply pass)."""
    A = bf(rnd(M, K_, dev=dev, seed=M))
    Rz = bf(rnd(M, K_, dev=dev, seed=M + 1)) if res else None
    s, t = bn_params(K_, dev)
    W = bf(rnd(N, K_, dev=dev, seed=5) / math.sqrt(K_))
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    o = torch.full((M, K_), 7.0, dtype=torch.bfloat16, device=dev)
    P = K.pw_num_partials(M, N, K_)
    part = torch.zeros(P * 2 * N, device=dev)
    pro = K.PRO_BNRES if res else K.ACT_BN
    K.pw_gemm(pro, K.EPI_FWD, A, W, out, part, M, N, K_, A2=Rz, pa=s, pb=t, Aout=o)
    x = A.float() * s + t + (Rz.float() if res else 0.0)
    assert rel(o, x) < 4e-3
    ref = bf(x).float() @ W.float().t()
    assert rel(out, ref) < 8e-3


@pytest.mark.parametrize("M,Kf,Nf", PW_CASES)
@pytest.mark.parametrize("epi", [K.EPI_BWD_RELU6, K.EPI_BWD_LIN])
def test_pw_dgrad(dev, M, Kf, Nf, epi):
    # forward conv: [M,Kf] -> [M,Nf], weight [Nf][Kf]; dgrad produces [M,Kf]
    G = bf(rnd(M, Nf, dev=dev, seed=1))
    Y = bf(rnd(M, Nf, dev=dev, seed=2))
    coef = torch.stack([torch.rand(Nf, device=dev) + 0.5, torch.rand(Nf, device=dev) - 0.5,
                        torch.rand(Nf, device=dev) - 0.5]).contiguous()
    W = bf(rnd(Nf, Kf, dev=dev, seed=5) / math.sqrt(Nf))
    Yt = bf(rnd(M, Kf, dev=dev, seed=6))
    es, et = bn_params(Kf, dev, 7)
    R = bf(rnd(M, Kf, dev=dev, seed=8)) if epi == K.EPI_BWD_LIN else None
    out = torch.empty(M, Kf, dtype=torch.bfloat16, device=dev)
    P = K.pw_num_partials(M, Kf, Nf)
    part = torch.zeros(P * 2 * Kf, device=dev)
    Wt = torch.empty_like(W)
    tab = torch.tensor([[0, Nf, Kf]], dtype=torch.int32, device=dev)
    K.wt_transpose(W, Wt, tab, 1)
    assert torch.equal(Wt.view(Kf, Nf), W.t())
    K.pw_gemm(K.PRO_BNBWD, epi, G, Wt, out, part, M, Kf, Nf, A2=Y, pa=coef[0], pb=coef[1], pc=coef[2],
              Yt=Yt, es=es, et=et, R=R)
    dy = coef[0] * G.float() + coef[1] * Y.float() + coef[2]
    ref = dy @ W.float()
    if epi == K.EPI_BWD_RELU6:
        a = Yt.float() * es + et
        ref = ref * ((a > 0) & (a < 6)).float()
    else:
        ref = ref + R.float()
    assert rel(out, ref) < 8e-3
    st = sum_parts(part, P, Kf)
    assert rel(st[0], ref.sum(0)) < 2e-2
    assert rel(st[1], (ref * Yt.float()).sum(0)) < 2e-2


@pytest.mark.parametrize("M,Kf,Nf", PW_CASES)
@pytest.mark.parametrize("xact", [K.ACT_NONE, K.ACT_BN_RELU6])
def test_pw_wgrad(dev, M, Kf, Nf, xact):
    G = bf(rnd(M, Nf, dev=dev, seed=1))
    Y = bf(rnd(M, Nf, dev=dev, seed=2))
    coef = torch.stack([torch.rand(Nf, device=dev) + 0.5, torch.rand(Nf, device=dev) - 0.5,
                        torch.rand(Nf, device=dev) - 0.5]).contiguous()
    X = bf(rnd(M, Kf, dev=dev, seed=3))
    xs, xt = bn_params(Kf, dev, 4)
    ws = torch.zeros(K.pw_wgrad_workspace(M, Nf, Kf), device=dev)
    grad = torch.empty(Nf * Kf, device=dev)
    K.pw_wgrad(G, Y, coef[0], coef[1], coef[2], X, xs, xt, xact, ws, grad, M, Nf, Kf)
    dy = coef[0] * G.float() + coef[1] * Y.float() + coef[2]
    x = relu6(X.float() * xs + xt) if xact == K.ACT_BN_RELU6 else X.float()
    # bf16 operands inside the MFMA: compare against the bf16-rounded operands
    ref = bf(dy).float().t() @ bf(x).float()
    assert rel(grad.view(Nf, Kf), ref) < 2e-3


# fused dgrad + wgrad of a 1x1 conv (large M): (M, Kg = conv Cout, Ng = conv Cin, epilogue, residual)
PW_BWD_CASES = [(70001, 96, 16, "lin", True), (66000, 24, 144, "relu6", False), (65600, 192, 32, "lin", False),
                (70000, 32, 192, "relu6", False), (65613, 144, 24, "lin", True), (65540, 16, 32, "relu6", False),
                (66001, 24, 96, "relu6", False), (401408, 32, 144, "relu6", False),
                # small maps with a narrow K (the 14x14 project convs at batch 128): 6 / 9 N tiles
                (25088, 64, 384, "relu6", False), (25088, 96, 576, "relu6", False)]


@pytest.mark.parametrize("M,Kg,Ng,mode,res,recompute", [c + (False,) for c in PW_BWD_CASES] + [
    (70001, 96, 16, "lin", True, True), (65613, 144, 24, "lin", False, True), (100352, 192, 32, "lin", True, True),
    (401408, 144, 24, "lin", True, True)])
def test_pw_bwd_fused(dev, M, Kg, Ng, mode, res, recompute):
    """recompute: the expand form that re-forms Y = bf16(X W^T) from the staged X tile (no Y
    operand); the reference is computed from that Y."""
    assert K.pw_bwd_supported(M, Kg, Ng)
    G = bf(rnd(M, Kg, dev=dev, seed=1))
    W = bf(rnd(Kg, Ng, dev=dev, seed=5) / math.sqrt(Kg))        # conv weight [Cout=Kg][Cin=Ng]
    X = bf(rnd(M, Ng, dev=dev, seed=9)) if mode == "lin" else None
    if recompute:
        assert K.pw_bwd_recompute_supported(M, Kg, Ng)
        Y = bf(X.float() @ W.float().t())
    else:
        Y = bf(rnd(M, Kg, dev=dev, seed=2))
    coef = torch.stack([torch.rand(Kg, device=dev) + 0.5, torch.rand(Kg, device=dev) - 0.5,
                        torch.rand(Kg, device=dev) - 0.5]).contiguous()
    WT = W.t().contiguous()
    Yt = bf(rnd(M, Ng, dev=dev, seed=6))
    es, et = bn_params(Ng, dev, 7)
    R = bf(rnd(M, Ng, dev=dev, seed=8)) if res else None
    out = torch.empty(M, Ng, dtype=torch.bfloat16, device=dev)
    P = K.pw_bwd_num_partials(M, Kg, Ng)
    part = torch.zeros(P * 2 * Ng, device=dev)
    wpart = torch.zeros(K.pw_bwd_wgrad_workspace(M, Kg, Ng), device=dev)
    grad = torch.empty(Kg * Ng, device=dev)
    epi = K.EPI_BWD_RELU6 if mode == "relu6" else K.EPI_BWD_LIN
    K.pw_bwd(epi, G, None if recompute else Y, coef[0], coef[1], coef[2], WT, out, Yt, part, wpart, grad, M, Kg,
             Ng, es=es, et=et, R=R, X=X, We=W if recompute else None)
    dy = bf(coef[0] * G.float() + coef[1] * Y.float() + coef[2]).float()
    ref = dy @ W.float()
    if mode == "relu6":
        a = Yt.float() * es + et
        ref = ref * ((a > 0) & (a < 6)).float()
        x = bf(relu6(a)).float()
    else:
        if res:
            ref = ref + R.float()
        x = X.float()
    assert rel(out, ref) < 8e-3
    st = sum_parts(part, P, Ng)
    assert rel(st[0], ref.sum(0)) < 2e-2
    assert rel(st[1], (ref * Yt.float()).sum(0)) < 2e-2
    assert rel(grad.view(Kg, Ng), dy.t() @ x) < 2e-3


# ----------------------------------------------------------------------------- stem
@pytest.mark.parametrize("px", [0, 1, 2, 4])
@pytest.mark.parametrize("B,S", [(2, 32), (3, 64), (2, 224), (3, 30), (1, 50)])
def test_stem(dev, B, S, px):
    """The MFMA implicit-GEMM kernel (px = 0) and every register-blocking VALU variant (px
    pixels per thread); (3, 30) / (1, 50) give B*Ho*Wo = 675 / 625, not a multiple of 16 or
    64*px, so the tail pixels are exercised."""
    img = torch.zeros(B, S, S, 4, dtype=torch.bfloat16, device=dev)
    img[..., :3] = bf(rnd(B, S, S, 3, dev=dev, seed=1))
    w = bf(rnd(32, 3, 3, 3, dev=dev, seed=2) * 0.2)
    Ho = (S - 1) // 2 + 1
    y = torch.empty(B, Ho, Ho, 32, dtype=torch.bfloat16, device=dev)
    P = K.stem_num_partials(B, S, S)
    part = torch.zeros(P * 2 * 32, device=dev)
    K.stem_fwd(img, w, y, part, B, S, S, px=px)
    x = img[..., :3].float().permute(0, 3, 1, 2)
    ref = F.conv2d(x, w.float(), stride=2, padding=1).permute(0, 2, 3, 1)
    # fp32 accumulation then one bf16 rounding: every element within half a bf16 ulp (+ fp32 noise)
    assert ((y.float() - ref).abs() <= ref.abs() * 2.0 ** -8 + 1e-4).all()
    st = sum_parts(part, P, 32)
    assert rel(st[0], ref.reshape(-1, 32).sum(0)) < 1e-3
    assert rel(st[1], (ref.reshape(-1, 32) ** 2).sum(0)) < 1e-3
    if px != 1:
        return
    # wgrad
    G = bf(rnd(B, Ho, Ho, 32, dev=dev, seed=3))
    Y = bf(rnd(B, Ho, Ho, 32, dev=dev, seed=4))
    coef = torch.stack([torch.rand(32, device=dev) + 0.5, torch.rand(32, device=dev) - 0.5,
                        torch.rand(32, device=dev) - 0.5]).contiguous()
    dy = coef[0] * G.float() + coef[1] * Y.float() + coef[2]
    ws = torch.zeros(K.stem_wgrad_workspace(B, S, S), device=dev)
    grad = torch.empty(32 * 27, device=dev)
    K.stem_wgrad(G, Y, coef[0], coef[1], coef[2], img, ws, grad, B, S, S)
    wref = torch.nn.grad.conv2d_weight(x, w.shape, bf(dy).float().permute(0, 3, 1, 2), stride=2, padding=1)
    assert rel(grad.view(32, 3, 3, 3), wref) < 2e-3


# ----------------------------------------------------------------------------- head
@pytest.mark.parametrize("train", [True, False])
@pytest.mark.parametrize("HW,C", [(49, 1280), (9, 1000)])
def test_head(dev, train, HW, C):
    B, NC = 6, 10
    y = bf(rnd(B, HW, C, dev=dev, seed=1) * 3)
    s, t = bn_params(C, dev, 2)
    Wl = (rnd(NC, C, dev=dev, seed=3) * 0.05).contiguous()
    bl = (rnd(NC, dev=dev, seed=4) * 0.1).contiguous()
    labels = torch.randint(0, NC, (B,), device=dev)
    f32 = dict(device=dev, dtype=torch.float32)
    logits, loss, correct = torch.zeros(B, NC, **f32), torch.zeros(B, **f32), torch.zeros(B, **f32)
    dlog, pd = torch.zeros(B, NC, **f32), torch.zeros(B, C, **f32)
    g = torch.empty(B, HW, C, dtype=torch.bfloat16, device=dev)
    part = torch.zeros(B * 2 * C, **f32)
    dW, db = torch.zeros(NC * C, **f32), torch.zeros(NC, **f32)
    K.head(y, s, t, Wl, bl, labels, B, HW, C, NC, 0.0, 0, None, train, 1.0 / B, logits=logits, loss=loss,
           correct=correct, dlogits=dlog, pd=pd, g_out=g, part=part, dW=dW, db=db)
    yy = y.float().clone().requires_grad_(True)
    W_ = Wl.clone().requires_grad_(True)
    b_ = bl.clone().requires_grad_(True)
    z = relu6(yy * s + t)
    pooled = z.mean(1)
    lg = pooled @ W_.t() + b_
    L = F.cross_entropy(lg, labels)
    assert rel(logits, lg) < 1e-4
    assert abs(loss.mean().item() - L.item()) < 1e-4
    assert torch.equal(correct.bool(), lg.argmax(1) == labels)
    if train:
        L.backward()
        # g is the gradient w.r.t. the pre-activation a (= relu6 mask applied)
        a = y.float() * s + t
        mask = ((a > 0) & (a < 6)).float()
        dpool = (torch.softmax(lg, 1) - F.one_hot(labels, NC)).detach() / B @ Wl
        gref = dpool[:, None, :] / HW * mask
        assert rel(g, gref) < 8e-3
        assert rel(dW.view(NC, C), W_.grad) < 1e-4
        assert rel(db, b_.grad) < 1e-4
        st = sum_parts(part, B, C).float()
        assert rel(st[0], gref.reshape(-1, C).sum(0)) < 1e-2


# ----------------------------------------------------------------------------- adam
def test_adam_matches_torch(dev):
    n = 4096
    p0 = rnd(n, dev=dev, seed=1)
    p = p0.clone()
    m, v = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    pb = torch.empty(n, dtype=torch.bfloat16, device=dev)
    ref = p0.clone().requires_grad_(True)
    opt = torch.optim.Adam([ref], lr=1e-3)
    hyper = torch.tensor([1e-3, 0.0], device=dev)
    for it in range(5):
        g = rnd(n, dev=dev, seed=10 + it)
        ref.grad = g.clone()
        opt.step()
        hyper[1] += 1
        K.adam_flat(p, g * 2.0, m, v, pb, hyper, 0.9, 0.999, 1e-8, 0.0, grad_scale=0.5)
    assert rel(p, ref.detach()) < 1e-6
    assert rel(pb, ref.detach()) < 5e-3


# ----------------------------------------------------------------------------- augment
def test_augment_eval_matches_bilinear_resize(dev):
    N, B, S = 10, 4, 224
    src = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8, device=dev)
    labels = torch.arange(N, device=dev)
    idx = torch.tensor([3, 1, 7, 3], device=dev)
    out = torch.empty(B, S, S, 4, dtype=torch.bfloat16, device=dev)
    lab = torch.empty(B, dtype=torch.int64, device=dev)
    prm = torch.empty(B, K.AUG_NPARAMS, device=dev)
    K.augment(src, idx, labels, out, lab, prm, train=False)
    x = src[idx].permute(0, 3, 1, 2).float() / 255
    ref = F.interpolate(x, size=(S, S), mode="bilinear", align_corners=False)
    mean = torch.tensor([0.485, 0.456, 0.406], device=dev).view(1, 3, 1, 1)
    std = torch.tensor([0.229, 0.224, 0.225], device=dev).view(1, 3, 1, 1)
    ref = ((ref - mean) / std).permute(0, 2, 3, 1)
    assert rel(out[..., :3], ref) < 5e-3
    assert torch.all(out[..., 3] == 0)
    assert torch.equal(lab, labels[idx])


def test_augment_train_param_distribution(dev):
    N, B, S = 64, 256, 224
    src = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8, device=dev)
    labels = torch.zeros(N, dtype=torch.int64, device=dev)
    idx = torch.randint(0, N, (B,), device=dev)
    out = torch.empty(B, S, S, 4, dtype=torch.bfloat16, device=dev)
    lab = torch.empty(B, dtype=torch.int64, device=dev)
    prm = torch.empty(B, K.AUG_NPARAMS, device=dev)
    hyper = torch.tensor([0.0, 5.0], device=dev)
    K.augment(src, idx, labels, out, lab, prm, train=True, seed=3, hyper=hyper)
    p = prm.cpu()
    area = p[:, 2] * p[:, 3] / (S * S)
    assert area.min() >= 0.69 and area.max() <= 1.0
    ratio = p[:, 3] / p[:, 2]
    assert ratio.min() >= 0.74 and ratio.max() <= 1.34
    assert (p[:, 0] + p[:, 2] <= S).all() and (p[:, 1] + p[:, 3] <= S).all()
    assert 0.3 < p[:, 4].mean() < 0.7
    for col in (5, 6, 7):
        assert p[:, col].min() >= 0.7 and p[:, col].max() <= 1.3
    assert p[:, 8].abs().max() <= 0.1 and p[:, 10].abs().max() <= 15
    assert torch.isfinite(out.float()).all()
    # same seed + step -> identical params; next step -> different
    prm2 = torch.empty_like(prm)
    K.augment(src, idx, labels, out, lab, prm2, train=True, seed=3, hyper=hyper)
    assert torch.equal(prm, prm2)
    hyper[1] += 1
    K.augment(src, idx, labels, out, lab, prm2, train=True, seed=3, hyper=hyper)
    assert not torch.equal(prm, prm2)


def test_augment_flip_identity(dev):
    N, B, S = 4, 2, 64
    src = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8, device=dev)
    labels = torch.zeros(N, dtype=torch.int64, device=dev)
    idx = torch.tensor([0, 2], device=dev)
    ev = torch.empty(B, S, S, 4, dtype=torch.bfloat16, device=dev)
    tr = torch.empty_like(ev)
    lab = torch.empty(B, dtype=torch.int64, device=dev)
    prm = torch.empty(B, K.AUG_NPARAMS, device=dev)
    K.augment(src, idx, labels, ev, lab, prm, train=False, out_hw=S)
    given = torch.zeros(B, K.AUG_NPARAMS, device=dev)
    given[:, 2] = S
    given[:, 3] = S
    given[:, 4] = 1.0                       # flip
    given[:, 5:8] = 1.0                     # identity jitter
    given[:, 9] = 0 | (1 << 2) | (2 << 4) | (3 << 6)
    K.augment(src, idx, labels, tr, lab, prm, train=True, given_params=given, out_hw=S)
    assert rel(tr, ev.flip(2)) < 1e-3


@pytest.mark.parametrize("train", [False, True])
def test_augment_unaligned_source_matches_aligned(dev, train):
    """The render / params kernels stage the 32x32x3 source with 16-B loads when the image is
    16-B aligned and with a byte loop otherwise: both must give identical output."""
    N, B, S = 6, 5, 224
    src = torch.randint(0, 256, (N, 32, 32, 3), dtype=torch.uint8, device=dev)
    buf = torch.empty(N * 3072 + 1, dtype=torch.uint8, device=dev)
    mis = buf[1:].view(N, 32, 32, 3)
    mis.copy_(src)
    assert mis.data_ptr() % 16 != 0
    labels = torch.arange(N, device=dev)
    idx = torch.tensor([5, 0, 3, 3, 1], device=dev)
    hyper = torch.tensor([0.0, 7.0], device=dev)
    outs = []
    for s_ in (src, mis):
        out = torch.empty(B, S, S, 4, dtype=torch.bfloat16, device=dev)
        lab = torch.empty(B, dtype=torch.int64, device=dev)
        prm = torch.empty(B, K.AUG_NPARAMS, device=dev)
        K.augment(s_, idx, labels, out, lab, prm, train=train, seed=11, hyper=hyper)
        outs.append((out, prm))
    assert torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(outs[0][0], outs[1][0])


def test_head_dropout_consistent(dev):
    """Dropout in the split head: the pool launch draws the mask, the backward launch redraws
    the same one (same seed / step counter), so g is zero exactly on dropped channels and
    scaled by 1/(1-p) elsewhere."""
    B, HW, C, NC, p = 4, 49, 1280, 10, 0.2
    y = bf(rnd(B, HW, C, dev=dev, seed=11) * 3)
    s, t = bn_params(C, dev, 12)
    Wl = (rnd(NC, C, dev=dev, seed=13) * 0.05).contiguous()
    bl = torch.zeros(NC, device=dev)
    labels = torch.randint(0, NC, (B,), device=dev)
    f32 = dict(device=dev, dtype=torch.float32)
    hyper = torch.tensor([1e-3, 7.0], **f32)
    logits, loss, correct = torch.zeros(B, NC, **f32), torch.zeros(B, **f32), torch.zeros(B, **f32)
    dlog, pd = torch.zeros(B, NC, **f32), torch.zeros(B, C, **f32)
    g = torch.empty(B, HW, C, dtype=torch.bfloat16, device=dev)
    part = torch.zeros(B * 2 * C, **f32)
    dW, db = torch.zeros(NC * C, **f32), torch.zeros(NC, **f32)
    K.head(y, s, t, Wl, bl, labels, B, HW, C, NC, p, 1234, hyper, True, 1.0 / B, logits=logits, loss=loss,
           correct=correct, dlogits=dlog, pd=pd, g_out=g, part=part, dW=dW, db=db)
    a = y.float() * s + t
    pooled = relu6(a).mean(1)
    keep = torch.where(pooled.abs() > 1e-6, pd / pooled, torch.ones_like(pd))
    dropped = (pd == 0) & (pooled.abs() > 1e-6)
    frac = dropped.float().mean().item()
    assert 0.1 < frac < 0.3, frac
    kept = ~dropped & (pooled.abs() > 1e-6)
    assert torch.allclose(keep[kept], torch.full_like(keep[kept], 1 / (1 - p)), rtol=1e-4)
    lg = pd @ Wl.t() + bl
    assert rel(logits, lg) < 1e-4
    mask = ((a > 0) & (a < 6)).float()
    keepm = torch.where(dropped, torch.zeros_like(pd), torch.full_like(pd, 1 / (1 - p)))
    dpool = ((torch.softmax(lg, 1) - F.one_hot(labels, NC)) / B) @ Wl * keepm
    gref = dpool[:, None, :] / HW * mask
    assert rel(g, gref) < 8e-3


# ----------------------------------------------------------------------------- split-M reductions
@pytest.mark.parametrize("segs", [
    [(40, 64), (700, 96 * 9), (3, 16)],                      # vectorised (n % 4 == 0)
    [(1024, 1296), (17, 30), (2000, 8)],                     # one odd n: scalar path for all
    [(i * 37 % 900 + 1, 64 * (i + 1)) for i in range(11)],   # > 8 segments: two multi launches
])
def test_wgrad_reduce_deferred_multi(dev, segs):
    """Deferred reductions flushed as multi-segment launches == one launch each == fp64 sums
    (row chunking differs: a multi launch splits its grid target over the segments);
    repeated to check the per-segment arrival counters are re-armed."""
    for it in range(3):
        parts, grads, refs = [], [], []
        for k, (S, n) in enumerate(segs):
            ws = torch.zeros((S + K.lib().colsum_rows(S)) * n + 64, device=dev)
            src = rnd(S, n, dev=dev, seed=100 * it + k)
            ws[:S * n] = src.reshape(-1)
            parts.append(ws)
            grads.append(torch.full((n,), float("nan"), device=dev))
            refs.append(src.double().sum(0))
        K.wgrad_reduce_defer(True)
        try:
            for (S, n), ws, g in zip(segs, parts, grads):
                K.wgrad_reduce(ws, S, n, g)
        finally:
            K.wgrad_reduce_defer(False)
        torch.cuda.synchronize()
        assert all(torch.isnan(g).all() for g in grads), "a deferred reduction ran before the flush"
        K.wgrad_reduce_flush()
        torch.cuda.synchronize()
        for (S, n), ws, g, r in zip(segs, parts, grads, refs):
            assert torch.allclose(g.double(), r, rtol=1e-5, atol=1e-3), (S, n)
            g1 = torch.empty(n, device=dev)
            K.wgrad_reduce(ws, S, n, g1)
            torch.cuda.synchronize()
            assert torch.allclose(g1, g, rtol=1e-5, atol=1e-3), "multi-segment and single reductions differ"
