"""Render parity of the fused GPU augmentation kernel (csrc/kernels/augment.hip) against the
torch oracle of the reference chain (data/augment_torch.py), with IDENTICAL parameters.

Reference transform: Resize(224) -> RandomResizedCrop(224, (0.7, 1)) -> RandomHorizontalFlip
-> ColorJitter(0.3, 0.3, 0.3, 0.1) -> RandomRotation(15) -> ToTensor -> Normalize
(cifar10_serial_mobilenet_224.py:28-40).  Both implementations share the 16-slot parameter
layout, so the kernel is driven with ``given_params`` and the oracle renders the same rows.

One documented deviation: the kernel takes the contrast op's grey mean over a 56 x 56
sub-grid of the 224 x 224 pre-contrast image (the oracle and torchvision use every pixel).
The frame is a bilinear upsample of a 32 x 32 source, so the sub-grid mean is within ~1e-3
of the full mean; ``test_contrast_mean_subsample_error_bound`` pins that bound, and the
rendered pixels (which move by (1 - c) * dmean <= 0.3 * dmean) stay below bf16 resolution.
"""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu

S = 224
IDENT_ORDER = 0 | (1 << 2) | (2 << 4) | (3 << 6)


def _setup(dev, B, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    src = torch.randint(0, 256, (B, 32, 32, 3), dtype=torch.uint8, device=dev, generator=g)
    # smoother, image-like content as well as noise: half of the batch is a blurred copy
    sm = torch.nn.functional.avg_pool2d(src.permute(0, 3, 1, 2).float(), 5, 1, 2).permute(0, 2, 3, 1)
    src[B // 2:] = sm[B // 2:].round().clamp(0, 255).to(torch.uint8)
    return src


def _params(B, crop=True, flip=None, b=1.0, c=1.0, s=1.0, hue=0.0, order=IDENT_ORDER, angle=0.0, seed=0):
    gen = torch.Generator().manual_seed(seed)
    p = torch.zeros(B, 16)
    for i in range(B):
        if crop:
            h = int(torch.randint(160, S + 1, (1,), generator=gen))
            w = int(torch.randint(160, S + 1, (1,), generator=gen))
            p[i, 0] = int(torch.randint(0, S - h + 1, (1,), generator=gen))
            p[i, 1] = int(torch.randint(0, S - w + 1, (1,), generator=gen))
            p[i, 2], p[i, 3] = h, w
        else:
            p[i, 2] = p[i, 3] = S
        p[i, 4] = float(i % 2) if flip is None else float(flip)
    p[:, 5], p[:, 6], p[:, 7], p[:, 8] = b, c, s, hue
    p[:, 9] = order
    p[:, 10] = angle
    p[:, 12] = S
    return p


def _render_both(dev, src, prm):
    from pgdist.ops import kernels as K
    from pgdist.data import augment_torch as A
    B = src.shape[0]
    idx = torch.arange(B, device=dev)
    labels = torch.zeros(B, dtype=torch.int64, device=dev)
    out = torch.empty(B, S, S, 4, dtype=torch.bfloat16, device=dev)
    lab = torch.empty(B, dtype=torch.int64, device=dev)
    pout = torch.empty(B, K.AUG_NPARAMS, device=dev)
    K.augment(src, idx, labels, out, lab, pout, train=True, given_params=prm.to(dev), out_hw=S)
    ref = A.render(src.cpu(), prm, S, train=True).permute(0, 2, 3, 1).to(dev)
    return out[..., :3].float(), ref, pout


def _rel(a, b):
    return ((a - b).norm() / b.norm()).item()


def test_crop_resize_and_flip(dev):
    src = _setup(dev, 8)
    got, ref, _ = _render_both(dev, src, _params(8))
    assert _rel(got, ref) < 1e-2
    assert (got - ref).abs().max().item() < 0.05     # bf16 of normalised values up to ~2.6


@pytest.mark.parametrize("op,kw", [("brightness", dict(b=1.27)), ("brightness_dark", dict(b=0.72)),
                                   ("contrast", dict(c=1.25)), ("contrast_low", dict(c=0.71)),
                                   ("saturation", dict(s=1.3)), ("saturation_low", dict(s=0.7)),
                                   ("hue", dict(hue=0.08)), ("hue_neg", dict(hue=-0.09))])
def test_each_jitter_op(dev, op, kw):
    src = _setup(dev, 6, seed=1)
    got, ref, _ = _render_both(dev, src, _params(6, seed=2, **kw))
    assert _rel(got, ref) < 1e-2, op


@pytest.mark.parametrize("order", [IDENT_ORDER, 3 | (1 << 2) | (0 << 4) | (2 << 6), 1 | (3 << 2) | (2 << 4) | (0 << 6),
                                   2 | (0 << 2) | (3 << 4) | (1 << 6)])
def test_all_jitter_ops_in_order(dev, order):
    src = _setup(dev, 6, seed=3)
    got, ref, _ = _render_both(dev, src, _params(6, b=1.2, c=0.8, s=1.25, hue=-0.06, order=order, seed=4))
    assert _rel(got, ref) < 1e-2


@pytest.mark.parametrize("angle", [7.5, -14.0, 15.0])
def test_rotation_nearest_fill0(dev, angle):
    """Nearest-neighbour rotation with fill 0: compared away from the boundary ring of the
    rotated frame (pixels whose source lies within 1 px of the frame edge may round either
    way), the rest must match; the fill region must be the normalised zero."""
    src = _setup(dev, 4, seed=5)
    got, ref, _ = _render_both(dev, src, _params(4, crop=False, flip=0, angle=angle, seed=6))
    th = math.radians(angle)
    y, x = torch.meshgrid(torch.arange(S, device=dev) + 0.5 - S / 2, torch.arange(S, device=dev) + 0.5 - S / 2,
                          indexing="ij")
    xin = math.cos(-th) * x + math.sin(-th) * y + S / 2
    yin = -math.sin(-th) * x + math.cos(-th) * y + S / 2
    interior = (xin >= 1.5) & (xin <= S - 1.5) & (yin >= 1.5) & (yin <= S - 1.5)
    outside = (xin < -0.5) | (xin > S + 0.5) | (yin < -0.5) | (yin > S + 0.5)
    m = interior[None, :, :, None].expand_as(ref)
    assert _rel(got[m], ref[m]) < 1e-2
    fill = ref[outside[None].expand(ref.shape[0], -1, -1)]
    assert torch.allclose(got[outside[None].expand(ref.shape[0], -1, -1)], fill, atol=0.02)


def test_full_random_params_from_the_kernels_sampler(dev):
    """Train-mode parameters drawn by the kernel's own sampler, rendered by both."""
    from pgdist.ops import kernels as K
    B = 8
    src = _setup(dev, B, seed=7)
    idx = torch.arange(B, device=dev)
    labels = torch.zeros(B, dtype=torch.int64, device=dev)
    out = torch.empty(B, S, S, 4, dtype=torch.bfloat16, device=dev)
    lab = torch.empty(B, dtype=torch.int64, device=dev)
    pout = torch.empty(B, K.AUG_NPARAMS, device=dev)
    K.augment(src, idx, labels, out, lab, pout, train=True, seed=11, hyper=torch.tensor([0.0, 3.0], device=dev))
    prm = pout.cpu().clone()
    prm[:, 11:16] = 0
    prm[:, 12] = S
    got, ref, _ = _render_both(dev, src, prm)
    th = torch.deg2rad(prm[:, 10]).to(dev).view(B, 1, 1)
    y, x = torch.meshgrid(torch.arange(S, device=dev) + 0.5 - S / 2, torch.arange(S, device=dev) + 0.5 - S / 2,
                          indexing="ij")
    xin = torch.cos(-th) * x + torch.sin(-th) * y + S / 2
    yin = -torch.sin(-th) * x + torch.cos(-th) * y + S / 2
    interior = (xin >= 1.5) & (xin <= S - 1.5) & (yin >= 1.5) & (yin <= S - 1.5)
    m = interior[..., None].expand_as(ref)
    assert _rel(got[m], ref[m]) < 1.5e-2


def test_contrast_mean_subsample_error_bound(dev):
    """The kernel's 56 x 56 sub-grid grey mean vs the full-frame mean of the oracle's
    pre-contrast image (contrast applied last, so the pre-contrast image is crop + flip +
    brightness + saturation + hue)."""
    from pgdist.data import augment_torch as A
    import torch.nn.functional as F
    B = 8
    src = _setup(dev, B, seed=9)
    order = 0 | (2 << 2) | (3 << 4) | (1 << 6)       # contrast last
    prm = _params(B, b=1.15, c=1.3, s=0.8, hue=0.05, order=order, seed=10)
    _, _, pout = _render_both(dev, src, prm)
    kmean = (pout[:, 11] + pout[:, 13] + pout[:, 14] + pout[:, 15]).cpu() / (56 * 56)
    x = src.cpu().permute(0, 3, 1, 2).float() / 255.0
    R = F.interpolate(x, size=(S, S), mode="bilinear", align_corners=False)
    full = []
    for b in range(B):
        i, j, h, w = (int(prm[b, k]) for k in range(4))
        img = F.interpolate(R[b:b + 1, :, i:i + h, j:j + w], size=(S, S), mode="bilinear", align_corners=False)
        if prm[b, 4] > 0.5:
            img = img.flip(3)
        img = (img * prm[b, 5]).clamp(0, 1)
        gy = A._gray(img)
        img = (gy + prm[b, 7] * (img - gy)).clamp(0, 1)
        hh, ss, vv = A._rgb_to_hsv(img)
        hh = hh + prm[b, 8]
        img = A._hsv_to_rgb(hh - torch.floor(hh), ss, vv)
        full.append(A._gray(img).mean().item())
    err = (kmean - torch.tensor(full)).abs().max().item()
    assert err < 2e-3, f"sub-grid contrast mean off by {err}"
