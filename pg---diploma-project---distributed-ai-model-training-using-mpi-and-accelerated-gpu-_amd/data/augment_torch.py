"""Reference-semantics augmentation in plain torch ops (CPU path / oracle).

Implements the reference chain (``cifar10_serial_mobilenet_224.py:28-47``)
batch-wise on tensors:

  train: Resize(224) -> RandomResizedCrop(224, (0.7, 1.0)) -> RandomHorizontalFlip
         -> ColorJitter(0.3, 0.3, 0.3, 0.1) -> RandomRotation(15) -> Normalize
  test:  Resize(224) -> Normalize

Parameters follow torchvision's ``get_params`` rules and use the same 16-slot
layout as the GPU kernel (``csrc/kernels/augment.hip``) so a parameter tensor
can be rendered by either implementation.
"""
import math
from typing import Optional

import torch
import torch.nn.functional as F

from .. import IMAGENET_MEAN, IMAGENET_STD

P_I, P_J, P_H, P_W, P_FLIP, P_B, P_C, P_S, P_HUE, P_ORDER, P_ANGLE, P_MEAN, P_SRC_HW = range(13)
NPARAMS = 16
IDENTITY_ORDER = 0 | (1 << 2) | (2 << 4) | (3 << 6)


def sample_params(B: int, size: int = 224, generator: Optional[torch.Generator] = None) -> torch.Tensor:
    g = generator
    p = torch.zeros(B, NPARAMS)
    area = float(size * size)
    lr0, lr1 = math.log(3 / 4), math.log(4 / 3)
    for b in range(B):
        found = False
        for _ in range(10):
            ta = area * torch.empty(1).uniform_(0.7, 1.0, generator=g).item()
            ar = math.exp(torch.empty(1).uniform_(lr0, lr1, generator=g).item())
            w = int(round(math.sqrt(ta * ar)))
            h = int(round(math.sqrt(ta / ar)))
            if 0 < w <= size and 0 < h <= size:
                p[b, P_I] = torch.randint(0, size - h + 1, (1,), generator=g).item()
                p[b, P_J] = torch.randint(0, size - w + 1, (1,), generator=g).item()
                p[b, P_H], p[b, P_W] = h, w
                found = True
                break
        if not found:
            p[b, P_H] = p[b, P_W] = size
        p[b, P_FLIP] = float(torch.rand(1, generator=g).item() < 0.5)
        perm = torch.randperm(4, generator=g).tolist()
        p[b, P_ORDER] = perm[0] | (perm[1] << 2) | (perm[2] << 4) | (perm[3] << 6)
        p[b, P_B] = torch.empty(1).uniform_(0.7, 1.3, generator=g).item()
        p[b, P_C] = torch.empty(1).uniform_(0.7, 1.3, generator=g).item()
        p[b, P_S] = torch.empty(1).uniform_(0.7, 1.3, generator=g).item()
        p[b, P_HUE] = torch.empty(1).uniform_(-0.1, 0.1, generator=g).item()
        p[b, P_ANGLE] = torch.empty(1).uniform_(-15.0, 15.0, generator=g).item()
        p[b, P_SRC_HW] = size
    return p


def _gray(x):
    return 0.299 * x[:, 0:1] + 0.587 * x[:, 1:2] + 0.114 * x[:, 2:3]


def _rgb_to_hsv(x):
    r, g, b = x[:, 0], x[:, 1], x[:, 2]
    mx, _ = x.max(1)
    mn, _ = x.min(1)
    d = mx - mn
    s = torch.where(mx > 0, d / mx.clamp_min(1e-12), torch.zeros_like(mx))
    dd = d.clamp_min(1e-12)
    h = torch.where(mx == r, (g - b) / dd, torch.where(mx == g, 2 + (b - r) / dd, 4 + (r - g) / dd))
    h = torch.where(d > 0, h / 6.0, torch.zeros_like(h))
    h = h - torch.floor(h)
    return h, s, mx


def _hsv_to_rgb(h, s, v):
    h6 = h * 6
    i = torch.floor(h6).long() % 6
    f = h6 - torch.floor(h6)
    p, q, t = v * (1 - s), v * (1 - s * f), v * (1 - s * (1 - f))
    r = torch.stack([v, q, p, p, t, v], 1).gather(1, i[:, None]).squeeze(1)
    g = torch.stack([t, v, v, q, p, p], 1).gather(1, i[:, None]).squeeze(1)
    b = torch.stack([p, p, t, v, v, q], 1).gather(1, i[:, None]).squeeze(1)
    return torch.stack([r, g, b], 1)


def _jitter(x, prm):
    order = int(prm[P_ORDER].item())
    for k in range(4):
        op = (order >> (2 * k)) & 3
        if op == 0:
            x = (x * prm[P_B]).clamp(0, 1)
        elif op == 1:
            m = _gray(x).mean()
            x = (m + prm[P_C] * (x - m)).clamp(0, 1)
        elif op == 2:
            gy = _gray(x)
            x = (gy + prm[P_S] * (x - gy)).clamp(0, 1)
        else:
            h, s, v = _rgb_to_hsv(x)
            h = h + prm[P_HUE]
            h = h - torch.floor(h)
            x = _hsv_to_rgb(h, s, v)
    return x


def render(src_u8: torch.Tensor, params: Optional[torch.Tensor], size: int = 224, train: bool = True,
           double_resize: bool = True) -> torch.Tensor:
    """uint8 NHWC [B,32,32,3] -> normalised float NCHW [B,3,size,size]."""
    x = src_u8.permute(0, 3, 1, 2).float() / 255.0
    R = F.interpolate(x, size=(size, size), mode="bilinear", align_corners=False) if double_resize else x
    mean = torch.tensor(IMAGENET_MEAN, device=x.device).view(1, 3, 1, 1)
    std = torch.tensor(IMAGENET_STD, device=x.device).view(1, 3, 1, 1)
    if not train:
        if not double_resize:
            R = F.interpolate(x, size=(size, size), mode="bilinear", align_corners=False)
        return (R - mean) / std
    outs = []
    for b in range(x.shape[0]):
        prm = params[b]
        i, j, h, w = (int(prm[k].item()) for k in (P_I, P_J, P_H, P_W))
        crop = R[b:b + 1, :, i:i + h, j:j + w]
        img = F.interpolate(crop, size=(size, size), mode="bilinear", align_corners=False)
        if prm[P_FLIP] > 0.5:
            img = img.flip(3)
        img = _jitter(img, prm)
        ang = float(prm[P_ANGLE].item())
        if ang != 0.0:
            th = math.radians(ang)
            # output pixel -> source pixel: rotate by -angle about the centre (PIL convention)
            cos, sin = math.cos(-th), math.sin(-th)
            theta = torch.tensor([[cos, sin, 0.0], [-sin, cos, 0.0]], dtype=img.dtype, device=img.device)
            grid = F.affine_grid(theta[None], img.shape, align_corners=False)
            img = F.grid_sample(img, grid, mode="nearest", padding_mode="zeros", align_corners=False)
        outs.append(img)
    return (torch.cat(outs) - mean) / std
