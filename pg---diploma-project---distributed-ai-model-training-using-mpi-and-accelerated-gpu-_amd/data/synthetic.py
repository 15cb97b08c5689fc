"""Synthetic CIFAR-shaped data (no network / no dataset in this environment).

Produces uint8 NHWC 32x32x3 images and int64 labels in [0, num_classes), with
the same container layout as :class:`pgdist.data.cifar10.CIFAR10Arrays` so the
trainer, the GPU augmentation kernel and the benchmark consume either source.
Images carry a weak class-dependent signal (per-class colour tint + pattern) so
a few training steps visibly reduce the loss in integration tests.
"""
import numpy as np
import torch


def synthetic_cifar(n: int, num_classes: int = 10, seed: int = 0, signal: bool = True):
    g = np.random.default_rng(seed)
    labels = g.integers(0, num_classes, size=n, dtype=np.int64)
    imgs = g.integers(0, 256, size=(n, 32, 32, 3), dtype=np.int64)
    if signal:
        tint = np.random.default_rng(1234).integers(0, 256, size=(num_classes, 3))
        yy, xx = np.meshgrid(np.arange(32), np.arange(32), indexing="ij")
        freq = (np.arange(num_classes) % 5 + 1)[:, None, None]
        pattern = (np.sin(xx[None] * freq * 0.2 + yy[None] * 0.1 * freq) * 60)  # [C,32,32]
        imgs = imgs // 2 + tint[labels][:, None, None, :] // 2 + pattern[labels][..., None].astype(np.int64)
    imgs = np.clip(imgs, 0, 255).astype(np.uint8)
    return imgs, labels


def synthetic_images_224(batch: int, device, dtype=torch.bfloat16, seed: int = 0, channels_last=True):
    """Random normalised 224x224x3 batch (used by the torch-backend baseline)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = torch.randn(batch, 3, 224, 224, generator=g).to(device=device, dtype=dtype)
    if channels_last:
        x = x.contiguous(memory_format=torch.channels_last)
    return x


def _smooth_fields(g, n: int, freqs: int = 4, amp: float = 1.0) -> np.ndarray:
    """n random low-frequency RGB fields [n,32,32,3] in about [-amp, amp] (a few random Fourier
    modes per channel): spatially spread structure, no single discriminative pixel.  The mode
    parameters come from ``g`` (numpy, reproducible); the fields are evaluated separably in
    float32 with torch (cos(a + b) = cos a cos b - sin a sin b, a over rows, b over columns)."""
    t = torch.arange(32, dtype=torch.float32) / 32.0
    out = torch.zeros(n, 32, 32, 3)
    for _ in range(freqs):
        fy, fx = g.integers(0, 4, size=(2, n))
        ph = torch.from_numpy(g.uniform(0, 2 * np.pi, size=(n, 3)).astype(np.float32))
        a = torch.from_numpy(g.normal(0, 1, size=(n, 3)).astype(np.float32))
        ay = 2 * np.pi * torch.from_numpy(fy.astype(np.float32))[:, None, None] * t[None, :, None] + ph[:, None, :]
        bx = 2 * np.pi * torch.from_numpy(fx.astype(np.float32))[:, None] * t[None, :]            # [n,32]
        cy, sy = torch.cos(ay), torch.sin(ay)                                                     # [n,32,3]
        cx, sx = torch.cos(bx), torch.sin(bx)                                                     # [n,32]
        out += a[:, None, None, :] * (cy[:, :, None, :] * cx[:, None, :, None] - sy[:, :, None, :] * sx[:, None, :, None])
    return (amp * out / np.sqrt(freqs)).numpy()


def synthetic_cifar_hard(n: int, num_classes: int = 10, seed: int = 0, split: str = "train",
                         signal: float = 0.7, label_noise: float = 0.1, protos: int = 3):
    """A CIFAR-shaped synthetic set whose learning curve does NOT saturate in one epoch (VERDICT r3:
    the plain synthetic set reaches test accuracy 1.0000 after epoch 1, so it cannot reveal a
    broken gradient).  Each class owns ``protos`` fixed low-frequency colour templates (seeded
    independently of ``seed``: train and test share them); an image is a random low-frequency
    background of larger amplitude + ONE of its class's templates at ``signal`` relative strength,
    shifted by up to +-4 px and randomly mirrored, + pixel noise.  A fraction ``label_noise`` of
    the labels (train and test alike) is replaced by a uniformly random class, so the best
    achievable test accuracy is about 1 - label_noise * (1 - 1/num_classes) (0.91 by default)
    and a model that memorises noise does not reach it.  ``signal`` = 0.7 was calibrated on an
    MI355X (profiles/r4_synthetic_hard_calibration.txt): the gpu128 preset from random init reaches
    test accuracy 0.21 / 0.43 / 0.74 after epochs 1 / 3 / 10 (0.35: 0.32 after 20 epochs; 1.5: 0.86
    after epoch 3, saturating)."""
    g = np.random.default_rng(seed * 7919 + (0 if split == "train" else 104729))
    tg = np.random.default_rng(20241017)
    templ = _smooth_fields(tg, num_classes * protos, freqs=6, amp=1.0).reshape(num_classes, protos, 32, 32, 3)
    true = g.integers(0, num_classes, size=n, dtype=np.int64)
    which = g.integers(0, protos, size=n)
    dy, dx = g.integers(-4, 5, size=(2, n))
    flip = g.random(n) < 0.5
    ar = np.arange(32)
    rows = (ar[None, :] - dy[:, None]) % 32                            # cyclic shift
    cols = np.where(flip[:, None], 31 - ar[None, :], ar[None, :])      # mirror, then shift
    cols = (cols - dx[:, None]) % 32
    sig = templ[true[:, None, None], which[:, None, None], rows[:, :, None], cols[:, None, :]]   # [n,32,32,3]
    bg = _smooth_fields(g, n, freqs=5, amp=1.0)
    noise = torch.from_numpy(g.integers(0, 2 ** 31, size=1)).item()
    x = torch.from_numpy(bg + signal * sig).mul_(60).add_(128)
    x += torch.randn(x.shape, generator=torch.Generator().manual_seed(noise)) * 12
    imgs = x.clamp_(0, 255).to(torch.uint8).numpy()
    labels = true.copy()
    noisy = g.random(n) < label_noise
    labels[noisy] = g.integers(0, num_classes, size=int(noisy.sum()))
    return imgs, labels
