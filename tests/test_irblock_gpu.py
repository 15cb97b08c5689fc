"""Fused inverted-residual block forward (csrc/kernels/irblock.hip) against the three-launch
path it replaces and against fp32 torch.

The fused launch computes expand -> BN_e -> ReLU6 -> dw 3x3 -> BN_d -> ReLU6 -> project of a
stride-1 14x14 / 7x7 MobileNetV2 block with two grid barriers at the BatchNorm statistics
points.  Every tensor it writes (block input o, raw h1 / h2 / y, BN statistics) is compared
with the unfused executor on the same weights and images, per block; the whole training step
(gradients) must agree too, the barriers must never time out (error word), and a re-run must
reproduce the first run (the kernel re-arms its own barrier counters).
Reference body: cifar10_mpi_mobilenet_224.py:176-180.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

TOL = 2e-2


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-20)).item()


def _build(B, S, fuse, monkeypatch):
    from pgdist.models import mobilenet_v2
    from pgdist.engine.executor import MobileNetV2Executor
    monkeypatch.setattr(MobileNetV2Executor, "IR_FUSE", fuse)   # True / False / "fwd" / "bwd"
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = mobilenet_v2(10)
    model.classifier[0].p = 0.0
    with torch.no_grad():
        g = torch.Generator().manual_seed(1)
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.copy_(torch.rand(m.weight.shape, generator=g) + 0.5)
                m.bias.copy_(torch.rand(m.bias.shape, generator=g) - 0.5)
        for _, p in model.named_parameters():
            p.copy_(p.to(torch.bfloat16).float())
    exe = MobileNetV2Executor(model, B, S, dev)
    gi = torch.Generator(device=dev).manual_seed(2)
    img = torch.randn(B, S, S, 3, device=dev, generator=gi).to(torch.bfloat16)
    exe.img.zero_()
    exe.img[..., :3] = img
    exe.labels.copy_(torch.randint(0, 10, (B,), device=dev, generator=gi))
    return exe


def _run(exe):
    exe.forward(train=True)
    exe.backward()
    torch.cuda.synchronize()


@pytest.mark.parametrize("B", [8, 128])
def test_fused_blocks_match_unfused(B, monkeypatch):
    """Whole-network forward: the fused executor against the unfused one, per block tensor, in
    units of the run-to-run noise of the unfused path itself (float-atomic BN statistics make
    two identical runs differ, and a small batch amplifies that through 52 BatchNorms): blocks
    before the first fused one must stay at the noise level, the fused ones within it plus a
    bf16-rounding allowance (their depthwise input is the bf16-rounded activation; the
    unfused kernel keeps it in fp32).  Each fused block is checked strictly from its own input
    in test_fused_block_vs_torch."""
    S = 224
    ref = _build(B, S, False, monkeypatch)
    assert not ref.ir_grid
    _run(ref)
    ref2 = _build(B, S, False, monkeypatch)
    _run(ref2)
    exe = _build(B, S, True, monkeypatch)
    fused = sorted(exe.ir_grid)
    # every stride-1 14x14 / 7x7 block with expansion: features 8-13 and 15-17
    assert fused == [8, 9, 10, 11, 12, 13, 15, 16, 17], fused
    _run(exe)
    assert exe.ir_error() == 0, "grid barrier timed out"
    errs, table = [], []
    for bp, rp, rp2 in zip(exe.blocks, ref.blocks, ref2.blocks):
        allow = 0.005 if bp.idx < 8 else 0.03
        for name, get in (("h1", lambda b: b.bn_e.y if b.expand else None), ("h2", lambda b: b.bn_d.y),
                          ("y", lambda b: b.bn_p.y), ("o", lambda b: b.o),
                          ("mean_d", lambda b: b.bn_d.mean), ("rstd_d", lambda b: b.bn_d.rstd),
                          ("mean_p", lambda b: b.bn_p.mean), ("rstd_p", lambda b: b.bn_p.rstd)):
            a = get(bp)
            if a is None:
                continue
            e, noise = _rel(a, get(rp)), _rel(get(rp2), get(rp))
            table.append((bp.idx, name, round(e, 4), round(noise, 4)))
            if not e < 3 * noise + allow:
                errs.append((bp.prefix, name, round(e, 4), round(noise, 4)))
    print(table)
    assert not errs, errs
    lg_noise = _rel(ref2.logits, ref.logits)
    assert _rel(exe.logits, ref.logits) < 3 * lg_noise + 0.05
    # the training step's gradients (backward unchanged, fed by the fused forward's tensors)
    g_noise = _rel(ref2.flat.grad, ref.flat.grad)
    assert _rel(exe.flat.grad, ref.flat.grad) < 3 * g_noise + 0.1


def test_fused_block_vs_torch(monkeypatch):
    """One fused block recomputed in fp32 torch from the executor's own bf16 block input."""
    B, S = 8, 224
    exe = _build(B, S, True, monkeypatch)
    _run(exe)
    for bp in exe.blocks:
        if bp.idx not in exe.ir_grid:
            continue
        prev = exe.blocks[[b.idx for b in exe.blocks].index(bp.idx) - 1]
        x = prev.o.float().reshape(B, bp.H, bp.H, bp.cin).permute(0, 3, 1, 2)
        f = exe.flat
        we = f.view(f.master, bp.w_e, (bp.hidden, bp.cin, 1, 1))
        wd = f.view(f.master, bp.w_d, (bp.hidden, 1, 3, 3))
        wp = f.view(f.master, bp.w_p, (bp.cout, bp.hidden, 1, 1))

        def bn(t, st):
            return F.batch_norm(t, None, None, weight=st.gamma, bias=st.beta, training=True, eps=st.eps)
        h1 = F.conv2d(x, we)
        a1 = bn(h1, bp.bn_e).clamp(0, 6)
        h2 = F.conv2d(a1, wd, padding=1, groups=bp.hidden)
        a2 = bn(h2, bp.bn_d).clamp(0, 6)
        y = F.conv2d(a2, wp)

        def nchw(t, C):
            return t.float().reshape(B, bp.H, bp.H, C).permute(0, 3, 1, 2)
        assert _rel(nchw(bp.bn_e.y, bp.hidden), h1) < TOL, bp.prefix
        assert _rel(nchw(bp.bn_d.y, bp.hidden), h2) < TOL, bp.prefix
        assert _rel(nchw(bp.bn_p.y, bp.cout), y) < 3e-2, bp.prefix


def test_fused_rerun_reproduces(monkeypatch):
    """Two forwards of the same batch: the fused blocks' outputs differ only by the float-atomic
    run-to-run noise the unfused executor shows too (a barrier passing early -- counters not
    re-armed -- would leave statistics half-summed: O(1) errors)."""
    B, S = 16, 224
    diffs = {}
    for fuse in (True, False):
        exe = _build(B, S, fuse, monkeypatch)
        exe.forward(train=True)
        torch.cuda.synchronize()
        snap = [bp.bn_p.y.clone() for bp in exe.blocks]
        if fuse:
            assert all(int(t[0].item()) == 0 for t in exe.ir_bar.values()), "counters not re-armed"
        exe.forward(train=True)
        torch.cuda.synchronize()
        diffs[fuse] = [_rel(bp.bn_p.y, a) for bp, a in zip(exe.blocks, snap)]
        if fuse:
            assert exe.ir_error() == 0
    print([(i + 1, round(a, 4), round(b, 4)) for i, (a, b) in enumerate(zip(diffs[True], diffs[False]))])
    for a, b in zip(diffs[True], diffs[False]):
        assert a < 3 * b + 0.02


@pytest.mark.parametrize("B", [8, 128])
def test_fused_backward_matches_unfused(B, monkeypatch):
    """The fused block backward (one launch per block: project dgrad -> depthwise dgrad -> expand
    dgrad) against the three-launch chain on the same (fused) forward, per gradient tensor and for
    the whole flat gradient, in units of the unfused run-to-run noise.  The per-layer strict check
    against fp32 autograd from the executor's own tensors is test_executor_teacher_forced_gpu."""
    S = 224
    runs = {}
    for tag, mode in (("ref", "fwd"), ("ref2", "fwd"), ("fused", "1")):
        exe = _build(B, S, mode, monkeypatch)
        _run(exe)
        runs[tag] = exe
    exe, ref, ref2 = runs["fused"], runs["ref"], runs["ref2"]
    assert not ref.irb_grid and sorted(exe.irb_grid) == [8, 9, 10, 11, 12, 13, 15, 16], sorted(exe.irb_grid)
    assert exe.ir_error() == 0
    errs, table = [], []
    for bp, rp, rp2 in zip(exe.blocks, ref.blocks, ref2.blocks):
        for name, get in (("G", lambda b: b.G), ("gd", lambda b: b.bn_d.g),
                          ("ge", lambda b: b.bn_e.g if b.expand else None)):
            a = get(bp)
            if a is None:
                continue
            e, noise = _rel(a, get(rp)), _rel(get(rp2), get(rp))
            table.append((bp.idx, name, round(e, 4), round(noise, 4)))
            if not e < 3 * noise + 0.03:
                errs.append((bp.prefix, name, round(e, 4), round(noise, 4)))
    print(table)
    assert not errs, errs
    g_noise = _rel(ref2.flat.grad, ref.flat.grad)
    assert _rel(exe.flat.grad, ref.flat.grad) < 3 * g_noise + 0.05
