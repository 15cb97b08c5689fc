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
