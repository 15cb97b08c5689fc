"""Lazy (consumer-side) BN finalize (csrc/bnfin.h bn_lazy).

Every consumer of a BN's parameters (1x1 GEMM prologues, fused 1x1 backward, depthwise
forward / dgrad, BN-apply) can compute them from the producer's replica rows itself.  Each
consumer runs twice on the same accumulator: once with the parameters materialised by the
finalize kernel, once with a lazy descriptor and poisoned parameter buffers -- the outputs
must be bitwise identical (same accumulation order and rounding).  The batched finalize
(``bn_finalize_batch``) must write exactly what the per-BN finalize launches write, and the
executor in lazy mode must train like the launch mode.
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


class LazyBN:
    """A BN with a filled [rows][2][C] accumulator, its materialised parameters and a lazy
    descriptor (rows < kBnRep exercises the masked rows)."""

    def __init__(self, dev, C, count, bwd, rows=8, seed=0):
        g = torch.Generator(device="cpu").manual_seed(seed)
        f32 = dict(device=dev, dtype=torch.float32)
        self.C, self.count, self.rows, self.bwd = C, float(count), rows, bwd
        self.acc = torch.zeros(K.bn_part_floats(rows, C) + 64, **f32)
        n = float(count) / rows
        part = torch.empty(rows, 2, C)
        mu = torch.randn(C, generator=g) * 0.5
        if bwd:
            part[:, 0] = torch.randn(rows, C, generator=g) * n * 0.01
            part[:, 1] = torch.randn(rows, C, generator=g) * n * 0.01
        else:
            part[:, 0] = (mu + torch.randn(rows, C, generator=g) * 0.05) * n
            part[:, 1] = (mu * mu + torch.rand(rows, C, generator=g) + 0.2) * n
        self.acc[:rows * 2 * C] = part.reshape(-1).to(dev)
        self.gamma = (torch.rand(C, generator=g) + 0.5).to(dev)
        self.beta = (torch.rand(C, generator=g) - 0.5).to(dev)
        self.mean = (torch.randn(C, generator=g) * 0.3).to(dev)
        self.rstd = (torch.rand(C, generator=g) + 0.5).to(dev)
        self.rm, self.rv = torch.zeros(C, **f32), torch.ones(C, **f32)
        self.nbt = torch.zeros(1, device=dev, dtype=torch.int64)
        self.scale, self.shift = torch.zeros(C, **f32), torch.zeros(C, **f32)
        self.coef = torch.zeros(3, C, **f32)
        self.dg, self.db = torch.zeros(C, **f32), torch.zeros(C, **f32)
        self.ctr = torch.zeros(4, device=dev, dtype=torch.int32)
        if bwd:
            K.bn_bwd_finalize(self.acc, rows, C, self.count, self.mean, self.rstd, self.gamma, self.coef, self.dg,
                              self.db)
            self.lz = K.bn_fin_desc(self.acc, self.ctr, rows, C, count, 1, gamma=self.gamma, mean=self.mean,
                                    rstd=self.rstd, coef=self.coef, dgamma=self.dg, dbeta=self.db)
        else:
            K.bn_fwd_finalize(self.acc, rows, C, self.count, self.gamma, self.beta, 1e-5, 0.1, self.rm, self.rv,
                              self.nbt, self.mean, self.rstd, self.scale, self.shift)
            self.lz = K.bn_fin_desc(self.acc, self.ctr, rows, C, count, 0, gamma=self.gamma, beta=self.beta,
                                    eps=1e-5, momentum=0.1, rmean=self.rm, rvar=self.rv, nbt=self.nbt,
                                    mean=self.mean, rstd=self.rstd, scale=self.scale, shift=self.shift)
        torch.cuda.synchronize()
        assert (self.coef.abs().sum() if bwd else self.scale.abs().sum()) > 0

    def poisoned(self):
        """Parameter buffers full of NaN: the lazy consumer must not read them."""
        nan = float("nan")
        if self.bwd:
            c = torch.full_like(self.coef, nan)
            return c[0], c[1], c[2]
        return torch.full_like(self.scale, nan), torch.full_like(self.shift, nan)


def same(a, b):
    assert torch.equal(a.view(torch.int16) if a.dtype == torch.bfloat16 else a,
                       b.view(torch.int16) if b.dtype == torch.bfloat16 else b)


@pytest.mark.parametrize("M,K_,N", [(1000, 16, 96), (3000, 320, 1280), (70001, 16, 96), (66000, 192, 64)])
@pytest.mark.parametrize("rows", [8, 3])
def test_pw_gemm_lazy_fwd(dev, M, K_, N, rows):
    A = bf(rnd(M, K_, dev=dev, seed=M))
    W = bf(rnd(N, K_, dev=dev, seed=5) / math.sqrt(K_))
    bn = LazyBN(dev, K_, M, 0, rows=rows, seed=K_)
    ps, pt = bn.poisoned()
    P = K.pw_num_partials(M, N, K_)

    def mk():
        return (torch.empty(M, N, dtype=torch.bfloat16, device=dev),
                torch.zeros(K.bn_rows(P) * 2 * N + 64, device=dev))

    def launch(o, lazy):
        K.pw_gemm(K.ACT_BN_RELU6, K.EPI_FWD, A, W, o[0], o[1], M, N, K_, pa=ps if lazy else bn.scale,
                  pb=pt if lazy else bn.shift, lz=bn.lz if lazy else None)
    # BN partials are float atomics: compare the GEMM output bitwise, the statistics loosely
    o1, o2 = mk(), mk()
    launch(o1, False)
    launch(o2, True)
    torch.cuda.synchronize()
    same(o1[0], o2[0])
    assert torch.allclose(o1[1], o2[1], rtol=1e-4, atol=1e-2)
    assert o1[0].float().abs().sum() > 0


@pytest.mark.parametrize("M,K_,N", [(1000, 96, 16), (66000, 96, 24), (6272, 960, 160)])
def test_pw_gemm_lazy_dgrad(dev, M, K_, N):
    A, Y = bf(rnd(M, K_, dev=dev, seed=1)), bf(rnd(M, K_, dev=dev, seed=2))
    W = bf(rnd(N, K_, dev=dev, seed=5) / math.sqrt(K_))
    Yt = bf(rnd(M, N, dev=dev, seed=8))
    es, et = torch.rand(N, device=dev) + 0.5, torch.rand(N, device=dev) - 0.5
    bn = LazyBN(dev, K_, M, 1, seed=3)
    pa, pb, pc = bn.poisoned()
    P = K.pw_num_partials(M, N, K_)
    out1, out2 = (torch.empty(M, N, dtype=torch.bfloat16, device=dev) for _ in range(2))
    acc1, acc2 = (torch.zeros(K.bn_rows(P) * 2 * N + 64, device=dev) for _ in range(2))
    K.pw_gemm(K.PRO_BNBWD, K.EPI_BWD_RELU6, A, W, out1, acc1, M, N, K_, A2=Y, pa=bn.coef[0], pb=bn.coef[1],
              pc=bn.coef[2], Yt=Yt, es=es, et=et)
    K.pw_gemm(K.PRO_BNBWD, K.EPI_BWD_RELU6, A, W, out2, acc2, M, N, K_, A2=Y, pa=pa, pb=pb, pc=pc, Yt=Yt, es=es,
              et=et, lz=bn.lz)
    torch.cuda.synchronize()
    same(out1, out2)
    assert out1.float().abs().sum() > 0


@pytest.mark.parametrize("M,Kg,Ng,mode", [(70001, 96, 16, "lin"), (66000, 24, 144, "relu6")])
def test_pw_bwd_lazy(dev, M, Kg, Ng, mode):
    G, Y = bf(rnd(M, Kg, dev=dev, seed=1)), bf(rnd(M, Kg, dev=dev, seed=2))
    WT = bf(rnd(Ng, Kg, dev=dev, seed=5) / math.sqrt(Kg))
    Yt = bf(rnd(M, Ng, dev=dev, seed=6))
    es, et = torch.rand(Ng, device=dev) + 0.5, torch.rand(Ng, device=dev) - 0.5
    X = bf(rnd(M, Ng, dev=dev, seed=9))
    bn = LazyBN(dev, Kg, M, 1, seed=4)
    ca, cb, cc = bn.poisoned()
    P = K.pw_bwd_num_partials(M, Kg, Ng)
    epi = K.EPI_BWD_RELU6 if mode == "relu6" else K.EPI_BWD_LIN
    outs = []
    for lazy in (False, True):
        out = torch.empty(M, Ng, dtype=torch.bfloat16, device=dev)
        acc = torch.zeros(K.bn_rows(P) * 2 * Ng + 64, device=dev)
        wpart = torch.zeros(K.pw_bwd_wgrad_workspace(M, Kg, Ng), device=dev)
        grad = torch.zeros(Kg * Ng, device=dev)
        c = (ca, cb, cc) if lazy else (bn.coef[0], bn.coef[1], bn.coef[2])
        K.pw_bwd(epi, G, Y, *c, WT, out, Yt, acc, wpart, grad, M, Kg, Ng, es=es, et=et,
                 X=X if mode == "lin" else None, lz=bn.lz if lazy else None)
        outs.append((out, grad))
    torch.cuda.synchronize()
    same(outs[0][0], outs[1][0])
    same(outs[0][1], outs[1][1])   # the weight gradient uses the same coefficients
    assert outs[0][1].abs().sum() > 0


@pytest.mark.parametrize("B,H,C,stride", [(2, 14, 96, 2), (2, 56, 32, 1), (2, 7, 960, 1)])
def test_dw_fwd_lazy(dev, B, H, C, stride):
    x = bf(rnd(B, H, H, C, dev=dev, seed=1))
    w = bf(rnd(9 * C, dev=dev, seed=3) * 0.3)
    Ho, _ = K.dw_out_hw(H, H, stride)
    bn = LazyBN(dev, C, B * H * H, 0, seed=C)
    ps, pt = bn.poisoned()
    P = K.dw_num_partials("fwd", B, H, H, C, stride)
    ys = []
    for lazy in (False, True):
        y = torch.empty(B, Ho, Ho, C, dtype=torch.bfloat16, device=dev)
        acc = torch.zeros(K.bn_rows(P) * 2 * C + 64, device=dev)
        K.dw_fwd(x, ps if lazy else bn.scale, pt if lazy else bn.shift, K.ACT_BN_RELU6, w, y, acc, B, H, H, C,
                 stride, lz=bn.lz if lazy else None)
        ys.append(y)
    torch.cuda.synchronize()
    same(ys[0], ys[1])
    assert ys[0].float().abs().sum() > 0


@pytest.mark.parametrize("B,H,C,stride,fuse_w", [(2, 14, 96, 2, False), (2, 56, 32, 1, True), (2, 7, 960, 1, False)])
def test_dw_dgrad_lazy(dev, B, H, C, stride, fuse_w):
    yprev = bf(rnd(B, H, H, C, dev=dev, seed=11))
    s, t = torch.rand(C, device=dev) + 0.5, torch.rand(C, device=dev) - 0.5
    w = bf(rnd(9 * C, dev=dev, seed=3) * 0.3)
    Ho, _ = K.dw_out_hw(H, H, stride)
    g = bf(rnd(B, Ho, Ho, C, dev=dev, seed=12))
    ys = bf(rnd(B, Ho, Ho, C, dev=dev, seed=13))
    bn = LazyBN(dev, C, B * Ho * Ho, 1, seed=5)
    poison = torch.full_like(bn.coef, float("nan"))
    P = K.dw_num_partials("dgrad", B, H, H, C, stride)
    outs = []
    for lazy in (False, True):
        gout = torch.empty(B, H, H, C, dtype=torch.bfloat16, device=dev)
        acc = torch.zeros(K.bn_rows(P) * 2 * C + 64, device=dev)
        wpart = torch.zeros(K.dw_dgrad_wgrad_workspace(B, H, H, C, stride), device=dev) if fuse_w else None
        K.dw_dgrad(g, ys, poison if lazy else bn.coef, w, yprev, s, t, gout, acc, B, H, H, C, stride, wpart=wpart,
                   lz=bn.lz if lazy else None)
        outs.append((gout, wpart))
    torch.cuda.synchronize()
    same(outs[0][0], outs[1][0])
    if fuse_w:
        same(outs[0][1], outs[1][1])
    assert outs[0][0].float().abs().sum() > 0


@pytest.mark.parametrize("M,C,res", [(4096, 16, False), (6272, 320, True), (401408, 24, True)])
def test_bn_apply_lazy(dev, M, C, res):
    y = bf(rnd(M, C, dev=dev, seed=1))
    r = bf(rnd(M, C, dev=dev, seed=2)) if res else None
    bn = LazyBN(dev, C, M, 0, seed=6)
    ps, pt = bn.poisoned()
    o1, o2 = (torch.empty(M, C, dtype=torch.bfloat16, device=dev) for _ in range(2))
    K.bn_apply(y, bn.scale, bn.shift, o1, relu6=False, res=r)
    K.bn_apply(y, ps, pt, o2, relu6=False, res=r, lz=bn.lz)
    torch.cuda.synchronize()
    same(o1, o2)


def test_pw_gemm_f8_lazy(dev):
    M, K_, N = 70001, 96, 24
    A = bf(rnd(M, K_, dev=dev, seed=1))
    w = rnd(N, K_, dev=dev, seed=2) * 0.1
    W8 = torch.zeros(N * K.fp8_pitch(K_), dtype=torch.uint8, device=dev)
    wsc = torch.ones(N, device=dev)
    tab = torch.tensor([[0, N, K_, 0, 0]], dtype=torch.int32, device=dev)
    K.w8_quant(w.reshape(-1).contiguous(), W8, wsc, tab, 1)
    bn = LazyBN(dev, K_, M, 0, seed=7)
    ps, pt = bn.poisoned()
    P = K.pw_num_partials(M, N, K_)
    outs = []
    for lazy in (False, True):
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        acc = torch.zeros(K.bn_rows(P) * 2 * N + 64, device=dev)
        K.pw_gemm_f8(K.ACT_BN_RELU6, A, W8, wsc, out, acc, M, N, K_, pa=ps if lazy else bn.scale,
                     pb=pt if lazy else bn.shift, lz=bn.lz if lazy else None)
        outs.append(out)
    torch.cuda.synchronize()
    same(outs[0], outs[1])
    assert outs[0].float().abs().sum() > 0


@pytest.mark.parametrize("bwd", [0, 1])
def test_bn_finalize_batch(dev, bwd):
    """One batched launch over BNs of different widths == the per-BN finalize launches."""
    bns = [LazyBN(dev, C, 1000 + C, bwd, rows=r, seed=C) for C, r in ((16, 8), (1280, 8), (96, 2), (320, 5))]
    ref = [(b.mean.clone(), b.rstd.clone(), b.scale.clone(), b.shift.clone(), b.rm.clone(), b.rv.clone(),
            b.nbt.clone(), b.coef.clone(), b.dg.clone(), b.db.clone()) for b in bns]
    for b in bns:   # undo the constructor's finalize side effects, then redo them in one launch
        for t in (b.scale, b.shift, b.coef, b.dg, b.db):
            t.zero_()
        if not bwd:
            b.mean.zero_()
            b.rstd.zero_()
            b.rm.fill_(0.0)
            b.rv.fill_(1.0)
            b.nbt.zero_()
    tab = K.bn_desc_table([b.lz for b in bns])
    K.bn_finalize_batch(tab, len(bns), max(b.C for b in bns))
    torch.cuda.synchronize()
    for b, r in zip(bns, ref):
        got = (b.mean, b.rstd, b.scale, b.shift, b.rm, b.rv, b.nbt, b.coef, b.dg, b.db)
        for x, y in zip(got, r):
            assert torch.equal(x, y)


def test_executor_lazy_matches_launch_mode(dev, monkeypatch):
    """One MobileNetV2 training step with the lazy finalize vs separate finalize launches:
    same loss, BN statistics and running statistics up to float-atomic ordering, and a
    gradient difference within the float-atomic noise floor (two launch-mode runs: at this
    tiny batch the run-to-run difference of some gradients, e.g. the betas of linear BNs
    whose analytic gradient is ~0, is of the order of the gradients themselves);
    num_batches_tracked advances once per step in both modes."""
    from pgdist.models import mobilenet_v2
    from pgdist.engine.native_step import NativeTrainStep
    src = torch.randint(0, 256, (32, 32, 32, 3), dtype=torch.uint8, device=dev,
                        generator=torch.Generator(device=dev).manual_seed(7))
    labels = torch.randint(0, 10, (32,), device=dev, generator=torch.Generator(device=dev).manual_seed(8))
    res = {}
    for tag, lazy in (("lazy", "1"), ("launch", "0"), ("launch2", "0")):
        monkeypatch.setenv("PGDIST_BN_LAZY", lazy)
        torch.manual_seed(100)
        st = NativeTrainStep(mobilenet_v2(10), 16, dev, img_size=96, lr=1e-3, use_graph=False, train_augment=False)
        assert st.exe.bn_mode == ("lazy" if lazy == "1" else "launch")
        st.set_data(src, labels)
        st.run(torch.arange(16, device=dev))
        torch.cuda.synchronize()
        bns = st.exe.all_bns()
        stats = [torch.cat([b.mean, b.rstd, b.module.running_mean, b.module.running_var]) for b in bns[:6]]
        first = (stats, st.read_metrics()[0], st.flat.grad.clone())
        st.run(torch.arange(16, device=dev))
        torch.cuda.synchronize()
        res[tag] = first + ([int(b.module.num_batches_tracked) for b in bns],)
    for a, b in zip(res["lazy"][0], res["launch"][0]):
        assert torch.allclose(a, b, rtol=1e-3, atol=1e-4)
    assert abs(res["lazy"][1] - res["launch"][1]) < 1e-2 * max(1.0, abs(res["launch"][1]))
    g, g0, g2 = res["lazy"][2], res["launch"][2], res["launch2"][2]
    noise = (g2 - g0).norm()
    assert g0.norm() > 0 and (g - g0).norm() <= 3 * noise + 1e-3 * g0.norm()
    assert res["lazy"][3] == res["launch"][3] == [2] * len(res["lazy"][3])
