"""Flat parameter / gradient / optimizer-state storage.

All trainable tensors of a model live in ONE contiguous fp32 master buffer (the
module's ``Parameter`` objects are re-pointed to views of it, so
``state_dict()`` / checkpointing / the torch oracle path see the same memory),
with a parallel fp32 gradient buffer, Adam ``m``/``v`` buffers and a bf16
shadow copy that the HIP kernels read.

Layout is *backward-completion order* (reverse of ``named_parameters``: the
classifier first, the stem last) with every tensor 64-element aligned, so the
gradient all-reduce buckets are contiguous prefixes/ranges of the gradient
buffer that become ready in order while backward is still running
(reference DDP buckets: SURVEY.md §2.7 N6).

Depthwise 3x3 weights ``[C,1,3,3]`` are stored *tap-major* ``[9][C]`` so the
depthwise kernels read the 4 channels of one tap with a single 8-byte load; the
Parameter is a strided view of that storage, so ``state_dict()`` still yields
torchvision-layout tensors.

With ``conv_nhwc=True`` (dense-conv networks, ResNet-50) every dense R x S (R*S > 1)
conv weight ``[Cout,Cin,R,S]`` is stored ``[Cout][R][S][Cp]`` — the implicit-GEMM
kernels' K order (r, s, ci) — with Cp = 4 for a 3-channel input (the zero 4th
channel matches the 4-channel NHWC image; its gradient is exactly zero, so it stays 0).
"""
from typing import Dict, List, Tuple

import torch

ALIGN = 64


def _align(n: int, a: int = ALIGN) -> int:
    return (n + a - 1) // a * a


def is_depthwise3x3(p: torch.Tensor) -> bool:
    return p.dim() == 4 and p.shape[1] == 1 and tuple(p.shape[2:]) == (3, 3) and p.shape[0] % 4 == 0


class FlatParams:
    def __init__(self, model: torch.nn.Module, device: torch.device, with_shadow: bool = True,
                 conv_nhwc: bool = False):
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        order = list(reversed(named))
        # dense R x S conv weights in NHWC storage: name -> (Cout, R, S, Cin, Cp)
        self.nhwc = {}
        if conv_nhwc:
            for n, p in order:
                if p.dim() == 4 and p.shape[2] * p.shape[3] > 1 and not is_depthwise3x3(p):
                    co, ci, r, s_ = p.shape
                    self.nhwc[n] = (co, r, s_, ci, 4 if ci == 3 else ci)
        self.offsets: Dict[str, Tuple[int, int]] = {}
        self.order: List[str] = []
        off = 0
        for name, p in order:
            off = _align(off)
            numel = p.numel()
            if name in self.nhwc:
                co, r, s_, ci, cp = self.nhwc[name]
                numel = co * r * s_ * cp
            self.offsets[name] = (off, numel)
            self.order.append(name)
            off += numel
        self.numel = _align(off)
        self.device = device
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.grad = torch.zeros_like(self.master)
        self.exp_avg = torch.zeros_like(self.master)
        self.exp_avg_sq = torch.zeros_like(self.master)
        self.shadow = torch.zeros(self.numel, dtype=torch.bfloat16, device=device) if with_shadow else None
        # transposed bf16 copies of the 1x1 conv weights (same offsets; filled by the executor)
        self.shadow_t = torch.zeros_like(self.shadow) if with_shadow else None
        self.params = {}
        self.tap_major = {n for n, p in order if is_depthwise3x3(p)} - set(self.nhwc)
        with torch.no_grad():
            for name, p in order:
                w_view, g_view = self.view(self.master, name, p.shape), self.view(self.grad, name, p.shape)
                w_view.copy_(p.detach().to(device))
                p.data = w_view
                p.grad = g_view
                self.params[name] = p
        self.refresh_shadow()

    # views ---------------------------------------------------------------
    def view(self, buf: torch.Tensor, name: str, shape) -> torch.Tensor:
        """Parameter-shaped view of ``name`` inside a flat buffer (strided for tap-major weights)."""
        o, n = self.offsets[name]
        if name in self.tap_major:
            C = shape[0]
            return buf[o:o + n].view(9, C).t().view(*shape)
        if name in self.nhwc:
            co, r, s_, ci, cp = self.nhwc[name]
            return buf[o:o + n].view(co, r, s_, cp)[..., :ci].permute(0, 3, 1, 2)
        return buf[o:o + n].view(shape)

    def w(self, name: str) -> torch.Tensor:
        o, n = self.offsets[name]
        return self.master[o:o + n]

    def g(self, name: str) -> torch.Tensor:
        o, n = self.offsets[name]
        return self.grad[o:o + n]

    def b(self, name: str) -> torch.Tensor:
        o, n = self.offsets[name]
        return self.shadow[o:o + n]

    def bt(self, name: str) -> torch.Tensor:
        o, n = self.offsets[name]
        return self.shadow_t[o:o + n]

    def range_of(self, name: str) -> Tuple[int, int]:
        o, n = self.offsets[name]
        return o, o + n

    def refresh_shadow(self):
        if self.shadow is None:
            return
        if self.device.type == "cuda":
            from ..ops import kernels as K
            K.f32_to_bf16(self.master, self.shadow)
        else:
            self.shadow.copy_(self.master.to(torch.bfloat16))

    def optimizer_state(self):
        return {"exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq}
