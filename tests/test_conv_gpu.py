"""Numerics of the dense-convolution HIP kernels (ResNet-50 path, csrc/kernels/conv.hip)
against plain PyTorch fp32 references of the same ops.

Inputs are bf16-representable; references run in fp32 (F.conv2d and its autograd) on
those exact values, so what is left is the kernels' bf16 output rounding and fp32
accumulation order.  Weights are handed to the kernels in their NHWC storage layout
([Cout][R][S][Cin]); the stem runs on 4-channel input (3 real + 1 zero channel).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from pgdist.ops import kernels as K  # noqa: E402


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def rnd(*shape, dev, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dev)


def bfr(t):
    """round to bf16 and back (fp32 values the kernels see)"""
    return t.to(torch.bfloat16).float()


def bn_params(C, dev, seed=1):
    g = torch.Generator(device="cpu").manual_seed(seed)
    s = (torch.rand(C, generator=g) + 0.5).to(dev)
    t = (torch.rand(C, generator=g) - 0.5).to(dev)
    return s.contiguous(), t.contiguous()


def nchw(x_nhwc):
    return x_nhwc.permute(0, 3, 1, 2)


def nhwc(x_nchw):
    return x_nchw.permute(0, 2, 3, 1).contiguous()


def w_store(w):
    """[Cout,Cin,R,S] -> kernel storage [Cout][R][S][Cin] bf16"""
    return w.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)


# (B, H, Ci, N, R, stride, pad)
FWD_SHAPES = [
    (2, 8, 64, 64, 3, 1, 1),
    (2, 8, 64, 128, 3, 2, 1),
    (2, 7, 256, 64, 1, 1, 0),
    (2, 8, 64, 256, 1, 2, 0),
    (3, 14, 128, 128, 3, 1, 1),
    (2, 6, 512, 2048, 1, 1, 0),
    (8, 64, 64, 128, 3, 1, 1),     # 128 x 128 tiles (>= 256 workgroups)
    (4, 30, 128, 200, 3, 2, 1),    # N not a multiple of the N tile, M tail
    (4, 7, 512, 256, 3, 1, 1),     # K = 4608 (72 k steps)
]


@pytest.fixture
def glds_mode():
    """restores the dense-conv staging mode a test selects (ops.kernels.conv_set_glds)"""
    old = K.conv_get_glds()
    yield K.conv_set_glds
    K.conv_set_glds(old)


@pytest.mark.parametrize("shape", FWD_SHAPES)
@pytest.mark.parametrize("pro,glds", [(K.CP_NONE, 0), (K.CP_NONE, 2), (K.CP_BN_RELU, 2)])
def test_conv_fwd(dev, shape, pro, glds, glds_mode):
    """CP_NONE with Ci % 64 == 0 runs on the LDS-DMA kernel (2 or 3 LDS buffers) unless glds=0."""
    glds_mode(glds)
    B, H, Ci, N, R, st, pad = shape
    x = bfr(rnd(B, H, H, Ci, dev=dev, seed=1))
    w = bfr(rnd(N, Ci, R, R, dev=dev, scale=(Ci * R * R) ** -0.5, seed=2))
    s, t = bn_params(Ci, dev)
    xin = torch.relu(x * s + t) if pro == K.CP_BN_RELU else x
    ref = nhwc(F.conv2d(nchw(bfr(xin)), w, stride=st, padding=pad))
    Ho, Wo = K.conv_out_hw(H, H, R, R, st, pad)
    y = torch.empty(B, Ho, Wo, N, dtype=torch.bfloat16, device=dev)
    P = K.conv_fwd_num_partials(B, Ho, Wo, N, R * R * Ci, Ci)
    part = torch.zeros(P, 2, N, device=dev)   # replica rows are added to atomically (bn_part_add)
    K.conv_fwd(pro, x.to(torch.bfloat16).contiguous(), w_store(w), y, part, B, H, H, Ci, N, R, R, st, pad,
               pa=s if pro else None, pb=t if pro else None)
    torch.cuda.synchronize()
    assert rel(y, ref) < 1e-2, rel(y, ref)
    yf = y.float().reshape(-1, N)
    ps = part.sum(0)
    assert torch.allclose(ps[0], yf.sum(0), rtol=1e-3, atol=1e-2)
    assert torch.allclose(ps[1], (yf * yf).sum(0), rtol=1e-3, atol=1e-2)


def test_conv_fwd_stem(dev):
    """7x7 s2 p3 stem on 4-channel (3 + zero pad) input, 4-channel weight storage."""
    B, H, N = 2, 32, 64
    x3 = bfr(rnd(B, H, H, 3, dev=dev, seed=3))
    x4 = torch.cat([x3, torch.zeros(B, H, H, 1, device=dev)], 3).to(torch.bfloat16).contiguous()
    w = bfr(rnd(N, 3, 7, 7, dev=dev, scale=0.1, seed=4))
    w4 = torch.cat([w, torch.zeros(N, 1, 7, 7, device=dev)], 1)
    ref = nhwc(F.conv2d(nchw(x3), w, stride=2, padding=3))
    Ho = (H + 6 - 7) // 2 + 1
    y = torch.empty(B, Ho, Ho, N, dtype=torch.bfloat16, device=dev)
    P = K.conv_fwd_num_partials(B, Ho, Ho, N, 196, 4)
    part = torch.zeros(P, 2, N, device=dev)
    K.conv_fwd(K.CP_NONE, x4, w_store(w4), y, part, B, H, H, 4, N, 7, 7, 2, 3)
    torch.cuda.synchronize()
    assert rel(y, ref) < 1e-2, rel(y, ref)
    assert torch.allclose(part.sum(0)[0], y.float().reshape(-1, N).sum(0), rtol=1e-3, atol=1e-2)


# (B, H, Cin, Cout, R, stride, pad) ; H = input (dx) size
DGRAD_SHAPES = [
    (2, 8, 64, 64, 3, 1, 1),
    (2, 8, 64, 128, 3, 2, 1),
    (2, 8, 128, 64, 1, 1, 0),
    (2, 8, 64, 256, 1, 2, 0),
    (2, 14, 256, 256, 3, 2, 1),
    (2, 7, 2048, 512, 1, 1, 0),
    (8, 64, 128, 64, 3, 1, 1),     # 128 x 128 tiles
    (8, 64, 64, 128, 3, 2, 1),     # 128 x 64 tiles over 4 parity classes
    (4, 7, 512, 256, 3, 1, 1),     # K = 2304 per class
]


def _dgrad_ref(dy, w, H, st, pad, B, Cin):
    x = torch.zeros(B, Cin, H, H, device=dy.device, requires_grad=True)
    y = F.conv2d(x, w, stride=st, padding=pad)
    (gx,) = torch.autograd.grad(y, x, nchw(dy))
    return nhwc(gx)


def _mat_dy(G, Y, ga, gb, gc):
    """dy = ga*G + gb*Y + gc materialised by the bn_mat kernel (checked against fp32)"""
    C = G.shape[-1]
    bf = lambda t: t.to(torch.bfloat16).contiguous().view(-1, C)  # noqa: E731
    out = torch.empty_like(bf(G))
    K.bn_mat(K.BN_MAT_BWD, bf(Y), ga, gb, out, G=bf(G), c=gc)
    torch.cuda.synchronize()
    ref = ga * G.reshape(-1, C) + gb * Y.reshape(-1, C) + gc
    assert rel(out, ref) < 5e-3
    return out.view(G.shape)


@pytest.mark.parametrize("shape", DGRAD_SHAPES)
@pytest.mark.parametrize("epi", ["relu", "res", "plain"])
@pytest.mark.parametrize("mat", [False, True])
def test_conv_dgrad(dev, shape, epi, mat):
    """mat: dy materialised by bn_mat and consumed by the LDS-DMA dgrad kernel (Y=None)"""
    B, H, Cin, Cout, R, st, pad = shape
    Ho, Wo = K.conv_out_hw(H, H, R, R, st, pad)
    G = bfr(rnd(B, Ho, Wo, Cout, dev=dev, seed=5))
    Y = bfr(rnd(B, Ho, Wo, Cout, dev=dev, seed=6))
    ga, gb = bn_params(Cout, dev, 7)
    gc = (bn_params(Cout, dev, 8)[1] * 0.1).contiguous()
    w = bfr(rnd(Cout, Cin, R, R, dev=dev, scale=(Cout * R * R) ** -0.5, seed=9))
    dy = bfr(ga * G + gb * Y + gc)
    dx_ref = _dgrad_ref(dy, w, H, st, pad, B, Cin)
    # transposed weight [Cin][R][S][Cout] via the batched kernel
    ws = w_store(w).reshape(-1)
    wt = torch.empty_like(ws)
    tab = torch.tensor([[0, 0, Cout, R * R, Cin]], dtype=torch.int32, device=dev)
    K.conv_wt(ws, wt, tab, 1)
    assert torch.equal(wt.view(Cin, R, R, Cout), w.permute(1, 2, 3, 0).to(torch.bfloat16))
    bf = lambda t: t.to(torch.bfloat16).contiguous()  # noqa: E731
    if mat:
        Gk, Yk = _mat_dy(G, Y, ga, gb, gc), None
    else:
        Gk, Yk = bf(G), bf(Y)
    dx = torch.empty(B, H, H, Cin, dtype=torch.bfloat16, device=dev)
    P = K.conv_dgrad_num_partials(B, H, H, Cin, Cout, R, R, st)
    part = torch.zeros(P, 2, Cin, device=dev)
    part2 = torch.zeros(P, 2, Cin, device=dev)
    Yt = bfr(rnd(B, H, H, Cin, dev=dev, seed=10))
    if epi == "relu":
        es, et = bn_params(Cin, dev, 11)
        K.conv_dgrad(K.CE_BWD_RELU, Gk, Yk, ga, gb, gc, wt, dx, part, B, H, H, Cin, Cout, R, R, st, pad,
                     Yt=bf(Yt), es=es, et=et)
        ref = dx_ref * ((Yt * es + et) > 0)
        ref_b = bfr(ref)
        s_ref = [ref_b.reshape(-1, Cin).sum(0), (ref_b * Yt).reshape(-1, Cin).sum(0)]
    elif epi == "res":
        Rg = bfr(rnd(B, H, H, Cin, dev=dev, seed=12))
        X = bfr(rnd(B, H, H, Cin, dev=dev, seed=13))
        Yt2 = bfr(rnd(B, H, H, Cin, dev=dev, seed=14))
        K.conv_dgrad(K.CE_BWD_RES, Gk, Yk, ga, gb, gc, wt, dx, part, B, H, H, Cin, Cout, R, R, st, pad,
                     Yt=bf(Yt), Rg=bf(Rg), X=bf(X), Yt2=bf(Yt2), part2=part2)
        ref = (dx_ref + Rg) * (X > 0)
        ref_b = bfr(ref)
        s_ref = [ref_b.reshape(-1, Cin).sum(0), (ref_b * Yt).reshape(-1, Cin).sum(0),
                 (ref_b * Yt2).reshape(-1, Cin).sum(0)]
    else:
        K.conv_dgrad(K.CE_BWD_RES, Gk, Yk, ga, gb, gc, wt, dx, None, B, H, H, Cin, Cout, R, R, st, pad)
        ref, s_ref = dx_ref, None
    torch.cuda.synchronize()
    assert rel(dx, ref) < 1.5e-2, rel(dx, ref)
    if s_ref is not None:
        ps = part.sum(0)
        scale = ref_b.abs().reshape(-1, Cin).sum(0) + 1
        assert ((ps[0] - s_ref[0]).abs() / scale).max() < 2e-2
        assert ((ps[1] - s_ref[1]).abs() / (scale * 4)).max() < 2e-2
        if len(s_ref) == 3:
            ps2 = part2.sum(0)
            assert torch.allclose(ps2[0], ps[0])
            assert ((ps2[1] - s_ref[2]).abs() / (scale * 4)).max() < 2e-2


@pytest.mark.parametrize("B,H,Cin,Cout", [(4, 14, 64, 256), (2, 28, 128, 512), (3, 9, 64, 128), (2, 7, 128, 64)])
def test_conv_dgrad_fold(dev, B, H, Cin, Cout):
    """1x1 data gradient with the BN backward folded into the GEMM (conv_fold_w + conv_dgrad_fold:
    K = 2 Cout over [G | Y]) against the fp32 reference of conv^T(a*G + b*Y + c) with the ReLU-mask
    epilogue, and its BN partials.  Y carries channel means 4x its spread and c cancels them (as in a
    real BN backward), the case the mean-corrected bias is for."""
    G = bfr(rnd(B, H, H, Cout, dev=dev, seed=5))
    mu = (torch.rand(Cout, device=dev) * 8 - 4).contiguous()
    Y = bfr(rnd(B, H, H, Cout, dev=dev, seed=6) + mu)
    ga, gb = bn_params(Cout, dev, 7)
    gc = (-gb * mu + 0.1 * bn_params(Cout, dev, 8)[1]).contiguous()
    w = bfr(rnd(Cout, Cin, 1, 1, dev=dev, scale=Cout ** -0.5, seed=9))
    dy = ga * G + gb * Y + gc                      # fp32, no rounding of dy
    dx_ref = _dgrad_ref(dy, w, H, 1, 0, B, Cin)
    wt = w.reshape(Cout, Cin).t().contiguous().to(torch.bfloat16)
    w2 = torch.empty(2 * Cin * Cout, dtype=torch.bfloat16, device=dev)
    fb = torch.empty(Cin, device=dev)
    K.conv_fold_w(wt, ga, gb, gc, mu, w2, fb, Cin, Cout)
    torch.cuda.synchronize()
    wf = wt.float()
    assert torch.equal(w2.view(Cin, 2, Cout)[:, 0], (ga * wf).to(torch.bfloat16))
    assert torch.equal(w2.view(Cin, 2, Cout)[:, 1], (gb * wf).to(torch.bfloat16))
    fb_ref = (gc * wf).sum(1) + (mu * (gb * wf - w2.view(Cin, 2, Cout)[:, 1].float())).sum(1)
    assert rel(fb, fb_ref) < 1e-5
    bf = lambda t: t.to(torch.bfloat16).contiguous()  # noqa: E731
    Yt = bfr(rnd(B, H, H, Cin, dev=dev, seed=10))
    es, et = bn_params(Cin, dev, 11)
    dx = torch.empty(B, H, H, Cin, dtype=torch.bfloat16, device=dev)
    P = K.conv_dgrad_num_partials(B, H, H, Cin, Cout, 1, 1, 1)
    part = torch.zeros(P, 2, Cin, device=dev)
    K.conv_dgrad_fold(bf(G), bf(Y), w2, fb, dx, part, B, H, H, Cin, Cout, Yt=bf(Yt), es=es, et=et)
    torch.cuda.synchronize()
    ref = dx_ref * ((Yt * es + et) > 0)
    assert rel(dx, ref) < 1.5e-2, rel(dx, ref)
    ref_b = bfr(ref)
    ps = part.sum(0)
    scale = ref_b.abs().reshape(-1, Cin).sum(0) + 1
    assert ((ps[0] - ref_b.reshape(-1, Cin).sum(0)).abs() / scale).max() < 2e-2
    assert ((ps[1] - (ref_b * Yt).reshape(-1, Cin).sum(0)).abs() / (scale * 4)).max() < 2e-2
    # no worse than the materialised-dy path on the same operands
    dx_m = torch.empty_like(dx)
    part_m = torch.zeros_like(part)
    K.conv_dgrad(K.CE_BWD_RELU, _mat_dy(G, Y, ga, gb, gc), None, ga, gb, gc, wt.view(-1), dx_m, part_m, B, H, H,
                 Cin, Cout, 1, 1, 1, 0, Yt=bf(Yt), es=es, et=et)
    torch.cuda.synchronize()
    assert rel(dx, ref) < 2 * rel(dx_m, ref) + 1e-3, (rel(dx, ref), rel(dx_m, ref))


# (B, H, Ci, N, R, stride, pad)
WGRAD_SHAPES = [
    (2, 8, 64, 64, 3, 1, 1),
    (2, 8, 64, 128, 3, 2, 1),
    (4, 7, 256, 64, 1, 1, 0),
    (2, 8, 64, 256, 1, 2, 0),
    (8, 14, 128, 128, 3, 1, 1),
    (2, 7, 512, 2048, 1, 1, 0),
    (16, 28, 128, 256, 3, 1, 1),    # many m splits (LDS-DMA wgrad with materialised dy)
    (32, 14, 256, 64, 1, 1, 0),
    (8, 28, 64, 128, 3, 2, 1),
]


def _wgrad_ref(x_in, dy, w_shape, st, pad):
    w = torch.zeros(w_shape, device=dy.device, requires_grad=True)
    y = F.conv2d(nchw(x_in), w, stride=st, padding=pad)
    (gw,) = torch.autograd.grad(y, w, nchw(dy))
    return gw


@pytest.mark.parametrize("shape", WGRAD_SHAPES)
@pytest.mark.parametrize("xpro", [K.CP_NONE, K.CP_BN_RELU])
@pytest.mark.parametrize("mat", [False, True])
def test_conv_wgrad(dev, shape, xpro, mat):
    """mat: dy materialised by bn_mat (G = dy, Y = None)"""
    B, H, Ci, N, R, st, pad = shape
    Ho, Wo = K.conv_out_hw(H, H, R, R, st, pad)
    x = bfr(rnd(B, H, H, Ci, dev=dev, seed=21))
    G = bfr(rnd(B, Ho, Wo, N, dev=dev, seed=22))
    Y = bfr(rnd(B, Ho, Wo, N, dev=dev, seed=23))
    ga, gb = bn_params(N, dev, 24)
    gc = (bn_params(N, dev, 25)[1] * 0.1).contiguous()
    xs, xt = bn_params(Ci, dev, 26)
    dy = bfr(ga * G + gb * Y + gc)
    xin = bfr(torch.relu(x * xs + xt)) if xpro == K.CP_BN_RELU else x
    ref = _wgrad_ref(xin, dy, (N, Ci, R, R), st, pad).permute(0, 2, 3, 1)   # -> [N][R][S][Ci]
    ws = torch.zeros(max(K.conv_wgrad_workspace(B, H, H, Ci, N, R, R, st, pad), 1), device=dev)
    grad = torch.full((N, R, R, Ci), float("nan"), device=dev)
    bf = lambda t: t.to(torch.bfloat16).contiguous()  # noqa: E731
    Gk, Yk = (_mat_dy(G, Y, ga, gb, gc), None) if mat else (bf(G), bf(Y))
    K.conv_wgrad(Gk, Yk, ga, gb, gc, bf(x), ws, grad, B, H, H, Ci, N, R, R, st, pad, xpro=xpro,
                 xs=xs if xpro else None, xt=xt if xpro else None)
    torch.cuda.synchronize()
    assert rel(grad, ref) < 1e-2, rel(grad, ref)


def test_conv_wgrad_stem(dev):
    B, H, N = 2, 32, 64
    x3 = bfr(rnd(B, H, H, 3, dev=dev, seed=31))
    x4 = torch.cat([x3, torch.zeros(B, H, H, 1, device=dev)], 3)
    Ho = (H + 6 - 7) // 2 + 1
    G = bfr(rnd(B, Ho, Ho, N, dev=dev, seed=32))
    Y = bfr(rnd(B, Ho, Ho, N, dev=dev, seed=33))
    ga, gb = bn_params(N, dev, 34)
    gc = torch.zeros(N, device=dev)
    dy = bfr(ga * G + gb * Y + gc)
    ref = _wgrad_ref(x3, dy, (N, 3, 7, 7), 2, 3).permute(0, 2, 3, 1)
    ws = torch.zeros(max(K.conv_wgrad_workspace(B, H, H, 4, N, 7, 7, 2, 3), 1), device=dev)
    grad = torch.full((N, 7, 7, 4), float("nan"), device=dev)
    bf = lambda t: t.to(torch.bfloat16).contiguous()  # noqa: E731
    K.conv_wgrad(bf(G), bf(Y), ga, gb, gc, bf(x4), ws, grad, B, H, H, 4, N, 7, 7, 2, 3)
    torch.cuda.synchronize()
    assert rel(grad[..., :3], ref) < 1e-2
    assert grad[..., 3].abs().max().item() == 0.0


@pytest.mark.parametrize("B,H", [(2, 32), (3, 46), (2, 224)])
def test_stem_s2d_fwd_wgrad(dev, B, H):
    """Space-to-depth stem: the 7x7 s2 p3 conv as a 4x4 s1 conv over the s2d image (LDS-DMA
    kernel with multi-tap k-steps) and its weight gradient (permuted back to [N][7][7][4]) vs
    the fp32 PyTorch conv / autograd on the same bf16 values; image_prep(s2d=True) and
    s2d_image give the same layout."""
    N, H2 = 64, H // 2
    x3 = bfr(rnd(B, H, H, 3, dev=dev, seed=71))
    x4 = torch.cat([x3, torch.zeros(B, H, H, 1, device=dev)], 3).to(torch.bfloat16).contiguous()
    w = bfr(rnd(N, 3, 7, 7, dev=dev, scale=0.1, seed=72))
    w4 = torch.cat([w, torch.zeros(N, 1, 7, 7, device=dev)], 1)
    x2 = torch.empty(B, H2, H2, 16, dtype=torch.bfloat16, device=dev)
    K.s2d_image(x4, x2, B, H, H)
    ref_x2 = x4.view(B, H2, 2, H2, 2, 4).permute(0, 1, 3, 2, 4, 5).reshape(B, H2, H2, 16)
    assert torch.equal(x2, ref_x2)
    w2 = torch.empty(N * 256, dtype=torch.bfloat16, device=dev)
    K.stem_w_s2d(w_store(w4), w2)
    y = torch.empty(B, H2, H2, N, dtype=torch.bfloat16, device=dev)
    P = K.conv_fwd_num_partials(B, H2, H2, N, 256, 16)
    part = torch.zeros(P, 2, N, device=dev)
    K.conv_fwd_s2d(x2, w2, y, part, B, H2)
    torch.cuda.synchronize()
    ref = nhwc(F.conv2d(nchw(x3), w, stride=2, padding=3))
    assert rel(y, ref) < 1e-2, rel(y, ref)
    assert torch.allclose(part.sum(0)[0], y.float().reshape(-1, N).sum(0), rtol=1e-3, atol=1e-2)
    # weight gradient
    G = bfr(rnd(B, H2, H2, N, dev=dev, seed=73))
    Y = bfr(rnd(B, H2, H2, N, dev=dev, seed=74))
    ga, gb = bn_params(N, dev, 75)
    gc = torch.randn(N, device=dev) * 0.1
    dy = bfr(ga * G + gb * Y + gc)
    wref = _wgrad_ref(x3, dy, (N, 3, 7, 7), 2, 3).permute(0, 2, 3, 1)
    ws = torch.zeros(K.conv_wgrad_s2d_workspace(B, H2), device=dev)
    grad = torch.full((N, 7, 7, 4), float("nan"), device=dev)
    bf = lambda t: t.to(torch.bfloat16).contiguous()  # noqa: E731
    K.conv_wgrad_s2d(bf(G), bf(Y), ga, gb, gc, x2, ws, grad, B, H2)
    torch.cuda.synchronize()
    assert rel(grad[..., :3], wref) < 1e-2, rel(grad[..., :3], wref)
    assert grad[..., 3].abs().max().item() == 0.0


def test_image_prep_s2d(dev):
    src = torch.randint(0, 256, (4, 24, 24, 3), dtype=torch.uint8, device=dev)
    labels = torch.arange(4, device=dev)
    idx = torch.tensor([3, 1], device=dev)
    hyper = torch.tensor([0.0, 5.0], device=dev)
    out = torch.empty(2, 24, 24, 4, dtype=torch.bfloat16, device=dev)
    out2 = torch.empty(2, 12, 12, 16, dtype=torch.bfloat16, device=dev)
    lab = torch.empty(2, dtype=torch.int64, device=dev)
    K.image_prep(src, idx, labels, out, lab, seed=9, hyper=hyper)
    K.image_prep(src, idx, labels, out2, lab, seed=9, hyper=hyper, s2d=True)
    conv = torch.empty_like(out2)
    K.s2d_image(out, conv, 2, 24, 24)
    torch.cuda.synchronize()
    assert torch.equal(out2, conv)


@pytest.mark.parametrize("mat", [False, True])
def test_conv_dgrad_bitmask(dev, mat):
    """res_out's ReLU bit mask (uint8 [M, C/8]) as the dgrad's Xm gives bitwise the dx and BN
    partials of the bf16 X operand (CE_BWD_RXYM / RXYYM vs RXY / RXYY)."""
    B, H, Cin, Cout = 4, 14, 256, 64
    g = torch.Generator(device=dev).manual_seed(81)
    y = torch.randn(B * H * H, Cin, device=dev, generator=g).to(torch.bfloat16)
    r = torch.randn(B * H * H, Cin, device=dev, generator=g).to(torch.bfloat16)
    s3 = torch.rand(Cin, device=dev, generator=g) + 0.5
    t3 = torch.randn(Cin, device=dev, generator=g) * 0.3
    X = torch.empty_like(y)
    mask = torch.empty(B * H * H, Cin // 8, dtype=torch.uint8, device=dev)
    K.res_out(y, s3, t3, r, X, mask=mask)
    bits = torch.stack([(mask >> j) & 1 for j in range(8)], 2).reshape(-1, Cin).bool()
    assert torch.equal(bits, X.float() > 0)
    G = torch.randn(B * H * H, Cout, device=dev, generator=g).to(torch.bfloat16)
    Yv = torch.randn(B * H * H, Cout, device=dev, generator=g).to(torch.bfloat16)
    ga, gb = (torch.randn(Cout, device=dev, generator=g) * 0.1 for _ in range(2))
    gc = torch.randn(Cout, device=dev, generator=g) * 0.01
    wt = (torch.randn(Cin * Cout, device=dev, generator=g) * 0.05).to(torch.bfloat16)
    Rg = torch.randn(B * H * H, Cin, device=dev, generator=g).to(torch.bfloat16)
    Yt = torch.randn(B * H * H, Cin, device=dev, generator=g).to(torch.bfloat16)
    Yt2 = torch.randn(B * H * H, Cin, device=dev, generator=g).to(torch.bfloat16)
    if mat:
        Gk, Yk = _mat_dy(G.float().view(B, H, H, Cout), Yv.float().view(B, H, H, Cout), ga, gb, gc), None
    else:
        Gk, Yk = G, Yv
    P = K.conv_dgrad_num_partials(B, H, H, Cin, Cout, 1, 1, 1)
    res = []
    for use_mask in (False, True):
        dx = torch.empty(B * H * H, Cin, dtype=torch.bfloat16, device=dev)
        part = torch.zeros(P, 2, Cin, device=dev)
        part2 = torch.zeros(P, 2, Cin, device=dev)
        K.conv_dgrad(K.CE_BWD_RES, Gk, Yk, ga, gb, gc, wt, dx, part, B, H, H, Cin, Cout, 1, 1, 1, 0, Yt=Yt, Rg=Rg,
                     X=None if use_mask else X, Xm=mask if use_mask else None, Yt2=Yt2, part2=part2)
        torch.cuda.synchronize()
        res.append((dx, part.sum(0), part2.sum(0)))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.allclose(res[0][1], res[1][1], rtol=1e-5, atol=1e-4)
    assert torch.allclose(res[0][2], res[1][2], rtol=1e-5, atol=1e-4)


def test_res_out(dev):
    M, C = 1000, 256
    y, r = bfr(rnd(M, C, dev=dev, seed=41)), bfr(rnd(M, C, dev=dev, seed=42))
    s, t = bn_params(C, dev, 43)
    rs, rt = bn_params(C, dev, 44)
    out = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    bf = lambda a: a.to(torch.bfloat16).contiguous()  # noqa: E731
    K.res_out(bf(y), s, t, bf(r), out)
    assert rel(out, torch.relu(y * s + t + r)) < 5e-3
    K.res_out(bf(y), s, t, bf(r), out, rs=rs, rt=rt)
    assert rel(out, torch.relu(y * s + t + r * rs + rt)) < 5e-3


def test_maxpool_fwd_bwd(dev):
    B, H, C = 2, 16, 64
    y = bfr(rnd(B, H, H, C, dev=dev, seed=51))
    s, t = bn_params(C, dev, 52)
    z = torch.relu(y * s + t).requires_grad_(True)
    ref = F.max_pool2d(nchw(z), 3, 2, 1)
    Ho = (H - 1) // 2 + 1
    out = torch.empty(B, Ho, Ho, C, dtype=torch.bfloat16, device=dev)
    idx = torch.empty(B, Ho, Ho, C, dtype=torch.uint8, device=dev)
    bf = lambda a: a.to(torch.bfloat16).contiguous()  # noqa: E731
    K.maxpool_fwd(bf(y), s, t, out, idx, B, H, H, C)
    assert rel(out, nhwc(ref)) < 5e-3
    gp = bfr(rnd(B, Ho, Ho, C, dev=dev, seed=53))
    (gz,) = torch.autograd.grad(ref, z, nchw(gp))
    g_ref = bfr(gz * ((y * s + t) > 0))
    g = torch.empty(B, H, H, C, dtype=torch.bfloat16, device=dev)
    P = K.maxpool_bwd_num_partials(B, H, H)
    part = torch.zeros(P, 2, C, device=dev)
    K.maxpool_bwd(bf(gp), idx, bf(y), s, t, g, part, B, H, H, C)
    torch.cuda.synchronize()
    assert rel(g, g_ref) < 1e-2
    ps = part.sum(0)
    assert torch.allclose(ps[0], g_ref.reshape(-1, C).sum(0), rtol=1e-2, atol=1e-2)
    assert torch.allclose(ps[1], (g_ref * y).reshape(-1, C).sum(0), rtol=1e-2, atol=1e-2)


def test_head_pieces(dev):
    B, HW, C, NC = 4, 49, 2048, 1000
    x = torch.relu(bfr(rnd(B, HW, C, dev=dev, seed=61)))
    pooled = torch.empty(B, C, device=dev)
    K.avgpool(x.to(torch.bfloat16).contiguous(), pooled, B, HW, C)
    assert torch.allclose(pooled, x.mean(1), rtol=1e-4, atol=1e-5)
    logits = rnd(B, NC, dev=dev, seed=62).contiguous()
    labels = torch.tensor([3, 999, 0, 500], device=dev)
    loss, correct = torch.empty(B, device=dev), torch.empty(B, device=dev)
    dl = torch.empty(B, NC, device=dev)
    K.softmax_ce(logits, labels, loss, correct, dl, scale=1.0 / B)
    lg = logits.clone().requires_grad_(True)
    l_ref = F.cross_entropy(lg, labels, reduction="none")
    (dref,) = torch.autograd.grad(l_ref.mean(), lg)
    assert torch.allclose(loss, l_ref, rtol=1e-4, atol=1e-5)
    assert torch.allclose(dl, dref, rtol=1e-4, atol=1e-7)
    assert torch.equal(correct, (logits.argmax(1) == labels).float())
    dpool = rnd(B, C, dev=dev, seed=63).contiguous()
    y = bfr(rnd(B, HW, C, dev=dev, seed=64))
    G = torch.empty(B, HW, C, dtype=torch.bfloat16, device=dev)
    part = torch.zeros(B, 2, C, device=dev)
    K.head_bwd(dpool, x.to(torch.bfloat16).contiguous(), y.to(torch.bfloat16).contiguous(), G, part, B, HW, C)
    g_ref = bfr((dpool / HW)[:, None, :] * (x > 0))
    assert rel(G, g_ref) < 5e-3
    assert torch.allclose(part.sum(0)[1], (g_ref * y).reshape(-1, C).sum(0), rtol=1e-3, atol=1e-3)


def test_image_prep(dev):
    src = torch.randint(0, 256, (5, 24, 24, 3), dtype=torch.uint8, device=dev)
    labels = torch.arange(5, device=dev)
    idx = torch.tensor([4, 0, 2], device=dev)
    out = torch.empty(3, 24, 24, 4, dtype=torch.bfloat16, device=dev)
    lab = torch.empty(3, dtype=torch.int64, device=dev)
    K.image_prep(src, idx, labels, out, lab, seed=7)
    torch.cuda.synchronize()
    mean = torch.tensor([0.485, 0.456, 0.406], device=dev)
    std = torch.tensor([0.229, 0.224, 0.225], device=dev)
    ref = (src[idx].float() / 255 - mean) / std
    for b in range(3):
        o = out[b, ..., :3].float()
        ok = rel(o, ref[b]) < 1e-2 or rel(o, ref[b].flip(1)) < 1e-2
        assert ok
    assert out[..., 3].abs().max().item() == 0
    assert torch.equal(lab, labels[idx])


@pytest.mark.parametrize("S,n", [(1, 4096), (7, 1000), (3136, 512), (3000, 36864), (200, 4717), (5000, 64),
                                 (8, 2359296)])
def test_wgrad_reduce(dev, S, n):
    """Split-M weight-gradient reduction: grad = sum of the S partial rows, repeated launches
    (counters re-armed), fixed summation order (bitwise repeatable)."""
    rows = S + K.lib().colsum_rows(S)
    part = torch.zeros(rows * n, device=dev)
    for it in range(3):
        vals = rnd(S, n, dev=dev, seed=70 + it)
        part[: S * n] = vals.reshape(-1)
        grad = torch.full((n,), float("nan"), device=dev)
        K.wgrad_reduce(part, S, n, grad)
        g2 = torch.full((n,), float("nan"), device=dev)
        K.wgrad_reduce(part, S, n, g2)
        torch.cuda.synchronize()
        ref = vals.double().sum(0)
        assert torch.allclose(grad.double(), ref, rtol=1e-4, atol=1e-3 * (S ** 0.5))
        assert torch.equal(grad, g2)


@pytest.mark.parametrize("M,C", [(1000, 64), (333, 2048), (4096, 256), (7, 8)])
def test_bn_mat_act(dev, M, C):
    """BN_MAT_ACT: relu(y*s + t) materialised for the LDS-DMA forward conv"""
    y = bfr(rnd(M, C, dev=dev, seed=41))
    s, t = bn_params(C, dev, 42)
    out = torch.empty(M, C, dtype=torch.bfloat16, device=dev)
    K.bn_mat(K.BN_MAT_ACT, y.to(torch.bfloat16), s, t, out)
    torch.cuda.synchronize()
    assert rel(out, torch.relu(y * s + t)) < 5e-3
