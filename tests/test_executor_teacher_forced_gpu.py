"""Teacher-forced, per-layer check of the MobileNetV2 executor's wiring (engine/executor.py).

After one native training step at 224x224, every op is recomputed in fp32 torch FROM THE
EXECUTOR'S OWN bf16 INPUTS of that op (so bf16 noise cannot accumulate across the 52 BN
layers and a wrong operand — wrong BN partner, residual, transposed weight, mask — shows up
as an O(1) error in exactly that layer), and compared per layer:

forward   stem / expand / depthwise / project / final conv outputs (pre-BN), BN batch
          statistics, block outputs (BN + residual), head logits
backward  for every BN-ReLU6-conv segment, torch autograd from the executor's saved
          activations with the executor's upstream gradient: the gradient the executor
          handed to the producing layer (bn.g, block G), the weight gradients and the BN
          gamma / beta gradients

Tolerance: relative L2 <= 2e-2 per tensor (bf16 storage of the compared tensors ~ 4e-3).
Reference: the training step body, cifar10_mpi_mobilenet_224.py:176-180.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

TOL = 2e-2


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-20)).item()


def _rel_sum(a, b, scale):
    """Relative error of a batch reduction (dgamma = sum g*xhat, dbeta = sum g) against
    max(|b|, scale): scale = the reduction's statistical magnitude sqrt(sum of squared terms).
    Some of these sums are zero in exact arithmetic (sum_m dL/do = 0 when o feeds a bias-free
    conv followed by BN), so both sides are rounding noise of that magnitude."""
    a, b = a.float(), b.float()
    return ((a - b).norm() / max(b.norm().item(), scale.norm().item(), 1e-20)).item()


def _nchw(t, B, H, C):
    return t.float().reshape(B, H, H, C).permute(0, 3, 1, 2)


def _bn(x, bn):
    return F.batch_norm(x, None, None, weight=bn.gamma, bias=bn.beta, training=True, eps=bn.eps)


@pytest.fixture(scope="module")
def stepped():
    from pgdist.models import mobilenet_v2
    from pgdist.engine.executor import MobileNetV2Executor
    dev = torch.device("cuda", 0)
    B, S = 8, 224
    torch.manual_seed(0)
    model = mobilenet_v2(10)
    model.classifier[0].p = 0.0
    with torch.no_grad():
        # non-trivial BN affine parameters: at gamma = 1, beta = 0 the scale invariance of a
        # BN -> ReLU6 -> conv -> BN chain makes sum(g * xhat) ~ 0 (pure rounding noise)
        g = torch.Generator().manual_seed(1)
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.weight.copy_(torch.rand(m.weight.shape, generator=g) + 0.5)
                m.bias.copy_(torch.rand(m.bias.shape, generator=g) - 0.5)
        # bf16-representable weights: master == the bf16 shadow the kernels read
        for n, p in model.named_parameters():
            p.copy_(p.to(torch.bfloat16).float())
    exe = MobileNetV2Executor(model, B, S, dev)
    img = torch.randn(B, S, S, 3, device=dev).to(torch.bfloat16)
    labels = torch.randint(0, 10, (B,), device=dev)
    exe.img.zero_()
    exe.img[..., :3] = img
    exe.labels.copy_(labels)
    exe.forward(train=True)
    exe.backward()
    torch.cuda.synchronize()
    return exe, img, labels, B, S


def _w(exe, name, shape):
    return exe.flat.view(exe.flat.master, name, shape).detach().clone()


def _g(exe, name, shape):
    return exe.flat.view(exe.flat.grad, name, shape).detach().clone()


def _seg_backward(exe, x_in, bn_in, conv, bn_out, grad_out, relu_out):
    """torch autograd of  z_in -> relu6 -> conv -> y -> BN_out -> (relu6)  from the executor's
    saved pre-BN input ``x_in`` (None: ``x_in`` is already the conv input, no BN/ReLU6 in
    front), with upstream gradient ``grad_out`` w.r.t. the BN_out output (pre-ReLU6 when
    relu_out).  Returns (grad of the conv input side: dL/dz_in or dL/dx, weight grad,
    dgamma, dbeta of BN_out, conv output y)."""
    gamma = bn_out.gamma.detach().clone().requires_grad_(True)
    beta = bn_out.beta.detach().clone().requires_grad_(True)
    w = conv["w"].clone().requires_grad_(True)
    if bn_in is not None:
        z_in = F.batch_norm(x_in, None, None, weight=bn_in.gamma, bias=bn_in.beta, training=True,
                            eps=bn_in.eps).detach().requires_grad_(True)
        a = z_in.clamp(0, 6)
    else:
        z_in = x_in.detach().clone().requires_grad_(True)
        a = z_in
    y = F.conv2d(a, w, stride=conv.get("stride", 1), padding=conv.get("pad", 0), groups=conv.get("groups", 1))
    z = F.batch_norm(y, None, None, weight=gamma, bias=beta, training=True, eps=bn_out.eps)
    z.backward(grad_out)
    with torch.no_grad():
        yd = y.detach()
        xhat = (yd - yd.mean((0, 2, 3), keepdim=True)) * torch.rsqrt(yd.var((0, 2, 3), unbiased=False, keepdim=True)
                                                                     + bn_out.eps)
        sg = (grad_out * xhat).pow(2).sum((0, 2, 3)).sqrt()
        sb = grad_out.pow(2).sum((0, 2, 3)).sqrt()
    return z_in.grad, w.grad, (gamma.grad, sg), (beta.grad, sb), yd


def test_stem_and_block_forward(stepped):
    exe, img, labels, B, S = stepped
    x = img.float().permute(0, 3, 1, 2)
    H = exe.H0
    y0 = F.conv2d(x, _w(exe, exe.stem_w, (32, 3, 3, 3)), stride=2, padding=1)
    assert _rel(_nchw(exe.bn0.y, B, H, 32), y0) < TOL
    errs = []
    prev_out = None   # block input (materialised o of the previous block), NCHW fp32
    for bp in exe.blocks:
        if bp.expand:
            xin = prev_out
            ye = F.conv2d(xin, _w(exe, bp.w_e, (bp.hidden, bp.cin, 1, 1)))
            errs.append((bp.prefix + " expand", _rel(_nchw(bp.bn_e.y, B, bp.H, bp.hidden), ye)))
            ye_exe = _nchw(bp.bn_e.y, B, bp.H, bp.hidden)
            a = _bn(ye_exe, bp.bn_e).clamp(0, 6)
            dw_in = bp.bn_e
        else:
            xin = None
            a = _bn(_nchw(exe.bn0.y, B, H, 32), exe.bn0).clamp(0, 6)
            dw_in = exe.bn0
        # BN statistics of the dw input (executor's finalize) vs torch over the same tensor
        yin = _nchw(dw_in.y, B, bp.H, bp.hidden)
        assert _rel(dw_in.mean, yin.mean((0, 2, 3))) < TOL, dw_in.prefix
        wd = _w(exe, bp.w_d, (bp.hidden, 1, 3, 3))
        yd = F.conv2d(a, wd, stride=bp.stride, padding=1, groups=bp.hidden)
        errs.append((bp.prefix + " dw", _rel(_nchw(bp.bn_d.y, B, bp.Ho, bp.hidden), yd)))
        ad = _bn(_nchw(bp.bn_d.y, B, bp.Ho, bp.hidden), bp.bn_d).clamp(0, 6)
        yp = F.conv2d(ad, _w(exe, bp.w_p, (bp.cout, bp.hidden, 1, 1)))
        errs.append((bp.prefix + " project", _rel(_nchw(bp.bn_p.y, B, bp.Ho, bp.cout), yp)))
        o = _bn(_nchw(bp.bn_p.y, B, bp.Ho, bp.cout), bp.bn_p)
        if bp.residual:
            o = o + xin
        errs.append((bp.prefix + " out", _rel(_nchw(bp.o, B, bp.Ho, bp.cout), o)))
        prev_out = _nchw(bp.o, B, bp.Ho, bp.cout)
    yl = F.conv2d(prev_out, _w(exe, exe.w_last, (exe.C_last, exe.C_last_in, 1, 1)))
    errs.append(("last", _rel(_nchw(exe.bn_last.y, B, exe.Hf, exe.C_last), yl)))
    bad = [(n, e) for n, e in errs if not e < TOL]
    assert not bad, bad
    # head from the executor's final activation
    z = _bn(_nchw(exe.bn_last.y, B, exe.Hf, exe.C_last), exe.bn_last).clamp(0, 6).mean((2, 3))
    logits = F.linear(z, exe.flat.w(exe.w_lin).view(exe.NC, -1), exe.flat.w(exe.b_lin))
    assert _rel(exe.logits, logits) < TOL


def test_head_and_last_conv_backward(stepped):
    exe, img, labels, B, S = stepped
    bnl = exe.bn_last
    y = _nchw(bnl.y, B, exe.Hf, exe.C_last).requires_grad_(False)
    z = _bn(y, bnl).detach().requires_grad_(True)
    W = exe.flat.w(exe.w_lin).view(exe.NC, -1).clone().requires_grad_(True)
    b = exe.flat.w(exe.b_lin).clone().requires_grad_(True)
    loss = F.cross_entropy(F.linear(z.clamp(0, 6).mean((2, 3)), W, b), labels)
    loss.backward()
    assert _rel(_nchw(bnl.g, B, exe.Hf, exe.C_last), z.grad) < TOL
    assert _rel(exe.flat.g(exe.w_lin).view(exe.NC, -1), W.grad) < TOL
    assert _rel(exe.flat.g(exe.b_lin), b.grad) < TOL
    # final 1x1 conv: input o_17, upstream gradient bnl.g (w.r.t. its BN output)
    last = exe.blocks[-1]
    gx, gw, gg, gb, _ = _seg_backward(exe, _nchw(last.o, B, exe.Hf, exe.C_last_in), None,
                                      {"w": _w(exe, exe.w_last, (exe.C_last, exe.C_last_in, 1, 1))}, bnl,
                                      _nchw(bnl.g, B, exe.Hf, exe.C_last), True)
    assert _rel(_nchw(last.G, B, exe.Hf, exe.C_last_in), gx) < TOL
    assert _rel(_g(exe, exe.w_last, (exe.C_last, exe.C_last_in, 1, 1)), gw) < TOL
    assert _rel_sum(bnl.dgamma, *gg) < TOL
    assert _rel_sum(bnl.dbeta, *gb) < TOL


def test_block_backward_per_layer(stepped):
    exe, img, labels, B, S = stepped
    errs = []
    for bi, bp in enumerate(exe.blocks):
        prev = exe.blocks[bi - 1] if bi > 0 else None
        dw_in = bp.bn_e if bp.expand else exe.bn0
        # project: z_d -> relu6 -> W_p -> y_p -> BN_p ; upstream G = dL/do (o = BN_p(y_p) + res)
        gz_d, gWp, ggp, gbp, _ = _seg_backward(
            exe, _nchw(bp.bn_d.y, B, bp.Ho, bp.hidden), bp.bn_d,
            {"w": _w(exe, bp.w_p, (bp.cout, bp.hidden, 1, 1))}, bp.bn_p, _nchw(bp.G, B, bp.Ho, bp.cout), False)
        mask_d = ((_bn(_nchw(bp.bn_d.y, B, bp.Ho, bp.hidden), bp.bn_d) > 0)
                  & (_bn(_nchw(bp.bn_d.y, B, bp.Ho, bp.hidden), bp.bn_d) < 6)).float()
        errs += [(bp.prefix + " project dgrad (bn_d.g)", _rel(_nchw(bp.bn_d.g, B, bp.Ho, bp.hidden), gz_d * mask_d)),
                 (bp.prefix + " project wgrad", _rel(_g(exe, bp.w_p, (bp.cout, bp.hidden, 1, 1)), gWp)),
                 (bp.prefix + " bn_p dgamma", _rel_sum(bp.bn_p.dgamma, *ggp)),
                 (bp.prefix + " bn_p dbeta", _rel_sum(bp.bn_p.dbeta, *gbp))]
        # depthwise: z_in -> relu6 -> dw -> y_d -> BN_d ; upstream bn_d.g = dL/dz_d
        gz_in, gWd, ggd, gbd, _ = _seg_backward(
            exe, _nchw(dw_in.y, B, bp.H, bp.hidden), dw_in,
            {"w": _w(exe, bp.w_d, (bp.hidden, 1, 3, 3)), "stride": bp.stride, "pad": 1, "groups": bp.hidden},
            bp.bn_d, _nchw(bp.bn_d.g, B, bp.Ho, bp.hidden), False)
        zin = _bn(_nchw(dw_in.y, B, bp.H, bp.hidden), dw_in)
        mask_in = ((zin > 0) & (zin < 6)).float()
        errs += [(bp.prefix + " dw dgrad (input bn.g)", _rel(_nchw(dw_in.g, B, bp.H, bp.hidden), gz_in * mask_in)),
                 (bp.prefix + " dw wgrad", _rel(_g(exe, bp.w_d, (bp.hidden, 1, 3, 3)), gWd)),
                 (bp.prefix + " bn_d dgamma", _rel_sum(bp.bn_d.dgamma, *ggd)),
                 (bp.prefix + " bn_d dbeta", _rel_sum(bp.bn_d.dbeta, *gbd))]
        if bp.expand:
            # expand: x (= o of the previous block) -> W_e -> y_e -> BN_e ; upstream bn_e.g
            gx, gWe, gge, gbe, _ = _seg_backward(
                exe, _nchw(prev.o, B, bp.H, bp.cin), None, {"w": _w(exe, bp.w_e, (bp.hidden, bp.cin, 1, 1))},
                bp.bn_e, _nchw(bp.bn_e.g, B, bp.H, bp.hidden), False)
            if bp.residual:
                gx = gx + _nchw(bp.G, B, bp.H, bp.cin)
            errs += [(bp.prefix + " expand dgrad (prev G)", _rel(_nchw(prev.G, B, bp.H, bp.cin), gx)),
                     (bp.prefix + " expand wgrad", _rel(_g(exe, bp.w_e, (bp.hidden, bp.cin, 1, 1)), gWe)),
                     (bp.prefix + " bn_e dgamma", _rel_sum(bp.bn_e.dgamma, *gge)),
                     (bp.prefix + " bn_e dbeta", _rel_sum(bp.bn_e.dbeta, *gbe))]
    bad = [(n, round(e, 4)) for n, e in errs if not e < TOL]
    assert not bad, bad


def test_stem_backward(stepped):
    exe, img, labels, B, S = stepped
    x = img.float().permute(0, 3, 1, 2)
    _, gW, gg, gb, _ = _seg_backward(exe, x, None, {"w": _w(exe, exe.stem_w, (32, 3, 3, 3)), "stride": 2, "pad": 1},
                                     exe.bn0, _nchw(exe.bn0.g, B, exe.H0, 32), False)
    assert _rel(_g(exe, exe.stem_w, (32, 3, 3, 3)), gW) < TOL
    assert _rel_sum(exe.bn0.dgamma, *gg) < TOL
    assert _rel_sum(exe.bn0.dbeta, *gb) < TOL
