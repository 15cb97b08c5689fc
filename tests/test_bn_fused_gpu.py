"""BN finalize fused into the tail of every statistics producer (csrc/bnfin.h).

Each producer runs with a fused-finalize descriptor; its accumulator is then finalized again
by the separate finalize kernel (same replica rows, same fixed summation order), and the two
results must agree to fp32 rounding.  Every producer is launched three times in a row to
check that the last arriver re-arms the arrival counter, and the running statistics /
num_batches_tracked updates are checked to happen exactly once per launch.
"""
import math

import pytest
import torch

from pgdist.ops import kernels as K

pytestmark = pytest.mark.gpu


def bf(t):
    return t.to(torch.bfloat16)


def rnd(*shape, dev, scale=1.0, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dev)


def bn_params(C, dev, seed=1):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.rand(C, generator=g) + 0.5).to(dev), (torch.rand(C, generator=g) - 0.5).to(dev)


class Fused:
    """Accumulator + descriptor + outputs of one BN for a producer with P partial rows."""

    def __init__(self, dev, P, C, count, bwd):
        self.rows, self.C, self.count, self.bwd = K.bn_rows(P), C, float(count), bwd
        f32 = dict(device=dev, dtype=torch.float32)
        self.acc = torch.zeros(K.bn_part_floats(self.rows, C) + 64, **f32)
        self.ctr = torch.zeros(4, device=dev, dtype=torch.int32)
        self.gamma, self.beta = bn_params(C, dev, 5)
        self.rm, self.rv = torch.zeros(C, **f32), torch.ones(C, **f32)
        self.nbt = torch.zeros(1, device=dev, dtype=torch.int64)
        self.mean = (torch.rand(C, **f32) - 0.5) if bwd else torch.zeros(C, **f32)
        self.rstd = (torch.rand(C, **f32) + 0.5) if bwd else torch.zeros(C, **f32)
        self.scale, self.shift = torch.zeros(C, **f32), torch.zeros(C, **f32)
        self.coef, self.dg, self.db = torch.zeros(3, C, **f32), torch.zeros(C, **f32), torch.zeros(C, **f32)
        if bwd:
            self.fin = K.bn_fin_desc(self.acc, self.ctr, self.rows, C, count, 1, gamma=self.gamma, mean=self.mean,
                                     rstd=self.rstd, coef=self.coef, dgamma=self.dg, dbeta=self.db)
        else:
            self.fin = K.bn_fin_desc(self.acc, self.ctr, self.rows, C, count, 0, gamma=self.gamma, beta=self.beta,
                                     eps=1e-5, momentum=0.1, rmean=self.rm, rvar=self.rv, nbt=self.nbt,
                                     mean=self.mean, rstd=self.rstd, scale=self.scale, shift=self.shift)

    def check(self, launch, reps=3):
        for it in range(reps):
            self.acc.zero_()
            rm0, rv0 = self.rm.clone(), self.rv.clone()
            launch(self.acc, self.fin)
            torch.cuda.synchronize()
            assert int(self.ctr[0].item()) == 0, "arrival counter not re-armed"
            C = self.C
            if self.bwd:
                coef, dg, db = torch.zeros_like(self.coef), torch.zeros_like(self.dg), torch.zeros_like(self.db)
                K.bn_bwd_finalize(self.acc, self.rows, C, self.count, self.mean, self.rstd, self.gamma, coef, dg, db)
                torch.cuda.synchronize()
                assert torch.allclose(self.coef, coef, rtol=1e-6, atol=1e-7)
                assert torch.allclose(self.dg, dg, rtol=1e-6, atol=1e-6)
                assert torch.allclose(self.db, db, rtol=1e-6, atol=1e-6)
                assert self.db.abs().sum() > 0
            else:
                mean, rstd, scale, shift = [torch.zeros(C, device=self.acc.device) for _ in range(4)]
                rm, rv = rm0.clone(), rv0.clone()
                nbt = torch.zeros(1, device=self.acc.device, dtype=torch.int64)
                K.bn_fwd_finalize(self.acc, self.rows, C, self.count, self.gamma, self.beta, 1e-5, 0.1, rm, rv, nbt,
                                  mean, rstd, scale, shift)
                torch.cuda.synchronize()
                for a, b in ((self.mean, mean), (self.rstd, rstd), (self.scale, scale), (self.shift, shift),
                             (self.rm, rm), (self.rv, rv)):
                    assert torch.allclose(a, b, rtol=1e-6, atol=1e-7)
                assert int(self.nbt.item()) == it + 1
                assert self.rstd.abs().sum() > 0


@pytest.mark.parametrize("B,H,C,stride", [(2, 14, 96, 2), (2, 56, 32, 1), (2, 7, 960, 1)])
def test_dw_fwd_fused_finalize(dev, B, H, C, stride):
    x = bf(rnd(B, H, H, C, dev=dev, seed=1))
    s, t = bn_params(C, dev)
    w = bf(rnd(9 * C, dev=dev, seed=3) * 0.3)
    Ho, _ = K.dw_out_hw(H, H, stride)
    y = torch.empty(B, Ho, Ho, C, dtype=torch.bfloat16, device=dev)
    P = K.dw_num_partials("fwd", B, H, H, C, stride)
    Fused(dev, P, C, B * Ho * Ho, 0).check(
        lambda acc, fin: K.dw_fwd(x, s, t, K.ACT_BN_RELU6, w, y, acc, B, H, H, C, stride, fin=fin))


@pytest.mark.parametrize("B,H,C,stride,fuse_w", [(2, 14, 96, 2, False), (2, 56, 32, 1, True), (2, 28, 144, 2, True)])
def test_dw_dgrad_fused_finalize(dev, B, H, C, stride, fuse_w):
    yprev = bf(rnd(B, H, H, C, dev=dev, seed=11))
    s, t = bn_params(C, dev, 2)
    w = bf(rnd(9 * C, dev=dev, seed=3) * 0.3)
    Ho, _ = K.dw_out_hw(H, H, stride)
    g = bf(rnd(B, Ho, Ho, C, dev=dev, seed=12))
    ys = bf(rnd(B, Ho, Ho, C, dev=dev, seed=13))
    coef = torch.stack([torch.rand(C, device=dev) + 0.5, torch.rand(C, device=dev) - 0.5,
                        torch.rand(C, device=dev) - 0.5]).contiguous()
    gout = torch.empty(B, H, H, C, dtype=torch.bfloat16, device=dev)
    P = K.dw_num_partials("dgrad", B, H, H, C, stride)
    wpart = torch.zeros(K.dw_dgrad_wgrad_workspace(B, H, H, C, stride), device=dev) if fuse_w else None
    Fused(dev, P, C, B * H * H, 1).check(
        lambda acc, fin: K.dw_dgrad(g, ys, coef, w, yprev, s, t, gout, acc, B, H, H, C, stride, wpart=wpart, fin=fin))


# small M: L2-direct-weight GEMM; M >= 65536: LDS-resident-weight tile kernel
@pytest.mark.parametrize("M,K_,N", [(1000, 16, 96), (3000, 320, 1280), (70001, 16, 96), (66000, 192, 64)])
@pytest.mark.parametrize("mode", ["fwd", "dgrad"])
def test_pw_gemm_fused_finalize(dev, M, K_, N, mode):
    A = bf(rnd(M, K_, dev=dev, seed=M))
    s, t = bn_params(K_, dev)
    W = bf(rnd(N, K_, dev=dev, seed=5) / math.sqrt(K_))
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    P = K.pw_num_partials(M, N, K_)
    if mode == "fwd":
        Fused(dev, P, N, M, 0).check(
            lambda acc, fin: K.pw_gemm(K.ACT_BN_RELU6, K.EPI_FWD, A, W, out, acc, M, N, K_, pa=s, pb=t, fin=fin))
    else:
        Y = bf(rnd(M, K_, dev=dev, seed=7))
        Yt = bf(rnd(M, N, dev=dev, seed=8))
        es, et = bn_params(N, dev, 9)
        c = torch.rand(3, K_, device=dev) - 0.25
        Fused(dev, P, N, M, 1).check(
            lambda acc, fin: K.pw_gemm(K.PRO_BNBWD, K.EPI_BWD_RELU6, A, W, out, acc, M, N, K_, A2=Y, pa=c[0], pb=c[1],
                                       pc=c[2], Yt=Yt, es=es, et=et, fin=fin))


@pytest.mark.parametrize("M,Kg,Ng,mode", [(70001, 96, 16, "lin"), (66000, 24, 144, "relu6")])
def test_pw_bwd_fused_finalize(dev, M, Kg, Ng, mode):
    G, Y = bf(rnd(M, Kg, dev=dev, seed=1)), bf(rnd(M, Kg, dev=dev, seed=2))
    c = torch.rand(3, Kg, device=dev) - 0.25
    WT = bf(rnd(Ng, Kg, dev=dev, seed=5) / math.sqrt(Kg))
    Yt = bf(rnd(M, Ng, dev=dev, seed=6))
    es, et = bn_params(Ng, dev, 7)
    X = bf(rnd(M, Ng, dev=dev, seed=9))
    out = torch.empty(M, Ng, dtype=torch.bfloat16, device=dev)
    P = K.pw_bwd_num_partials(M, Kg, Ng)
    wpart = torch.zeros(K.pw_bwd_wgrad_workspace(M, Kg, Ng), device=dev)
    epi = K.EPI_BWD_RELU6 if mode == "relu6" else K.EPI_BWD_LIN
    Fused(dev, P, Ng, M, 1).check(
        lambda acc, fin: K.pw_bwd(epi, G, Y, c[0], c[1], c[2], WT, out, Yt, acc, wpart, None, M, Kg, Ng, es=es, et=et,
                                  X=X if mode == "lin" else None, fin=fin))


def test_pw_gemm_f8_fused_finalize(dev):
    M, K_, N = 70001, 96, 24
    A = bf(rnd(M, K_, dev=dev, seed=1))
    w = rnd(N, K_, dev=dev, seed=2) * 0.1
    W8 = torch.zeros(N * K.fp8_pitch(K_), dtype=torch.uint8, device=dev)
    wsc = torch.ones(N, device=dev)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
    P = K.pw_num_partials(M, N, K_)
    Fused(dev, P, N, M, 0).check(lambda acc, fin: K.pw_gemm_f8(K.ACT_NONE, A, W8, wsc, out, acc, M, N, K_, fin=fin))


@pytest.mark.parametrize("B,S", [(2, 64), (3, 224)])
def test_stem_fused_finalize(dev, B, S):
    img = torch.zeros(B, S, S, 4, dtype=torch.bfloat16, device=dev)
    img[..., :3] = bf(rnd(B, S, S, 3, dev=dev, seed=1))
    w = bf(rnd(32 * 27, dev=dev, seed=2) * 0.2)
    Ho = (S - 1) // 2 + 1
    y = torch.empty(B, Ho, Ho, 32, dtype=torch.bfloat16, device=dev)
    P = K.stem_num_partials(B, S, S)
    Fused(dev, P, 32, B * Ho * Ho, 0).check(lambda acc, fin: K.stem_fwd(img, w, y, acc, B, S, S, fin=fin))


def test_head_fused_finalize(dev):
    B, HW, C, NC = 6, 49, 1280, 10
    y = bf(rnd(B, HW, C, dev=dev, seed=1) * 3)
    s, t = bn_params(C, dev, 2)
    Wl, bl = (rnd(NC, C, dev=dev, seed=3) * 0.05).contiguous(), (rnd(NC, dev=dev, seed=4) * 0.1).contiguous()
    labels = torch.randint(0, NC, (B,), device=dev)
    f32 = dict(device=dev, dtype=torch.float32)
    logits, loss, correct = torch.zeros(B, NC, **f32), torch.zeros(B, **f32), torch.zeros(B, **f32)
    dlog, pd = torch.zeros(B, NC, **f32), torch.zeros(B, C, **f32)
    g = torch.empty(B, HW, C, dtype=torch.bfloat16, device=dev)
    dW, db = torch.zeros(NC * C, **f32), torch.zeros(NC, **f32)
    Fused(dev, B, C, B * HW, 1).check(
        lambda acc, fin: K.head(y, s, t, Wl, bl, labels, B, HW, C, NC, 0.0, 0, None, True, 1.0 / B, logits=logits,
                                loss=loss, correct=correct, dlogits=dlog, pd=pd, g_out=g, part=acc, dW=dW, db=db,
                                fin=fin))
