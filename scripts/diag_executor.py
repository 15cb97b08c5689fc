#!/usr/bin/env python3
"""Per-layer diagnostic: native executor vs fp32 PyTorch autograd on the same input.

Prints, for every BatchNorm input (conv output) the relative error of the
executor's bf16 buffer against the reference activation, then the gradient
cosine per parameter.  Used to localise numerical problems layer by layer.
"""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import pgdist  # noqa: E402,F401
from pgdist.models import mobilenet_v2  # noqa: E402
from pgdist.engine.executor import MobileNetV2Executor  # noqa: E402


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def main(B=8, S=64, fp64=False):
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = mobilenet_v2(10)
    model.classifier[0].p = 0.0
    with torch.no_grad():
        for n, p in model.named_parameters():
            if p.dim() > 1 and not n.startswith("classifier"):
                p.copy_(p.to(torch.bfloat16).float())
    ref = copy.deepcopy(model).to(dev).train()
    if fp64:
        ref = ref.double()
    exe = MobileNetV2Executor(model, B, S, dev)
    img = torch.randn(B, S, S, 3, device=dev).to(torch.bfloat16)
    labels = torch.randint(0, 10, (B,), device=dev)
    exe.img.zero_()
    exe.img[..., :3] = img
    exe.labels.copy_(labels)
    exe.forward(train=True)
    exe.backward()
    torch.cuda.synchronize()

    acts = {}

    def hook(name):
        def f(mod, inp, out):
            acts[name] = inp[0].detach()
        return f

    for n, m in ref.named_modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.register_forward_hook(hook(n))
    x = img.float().permute(0, 3, 1, 2).contiguous()
    if fp64:
        x = x.double()
    out = ref(x)
    loss = F.cross_entropy(out, labels)
    loss.backward()
    # torch's own bf16 path (autocast) against the same fp32 reference: the noise floor
    ref16 = copy.deepcopy(model).to(dev).train()
    acts16 = {}

    def hook16(name):
        def f(mod, inp, out):
            acts16[name] = inp[0].detach()
        return f

    for n, m in ref16.named_modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.register_forward_hook(hook16(n))
    with torch.autocast("cuda", dtype=torch.bfloat16):
        out16 = ref16(img.float().permute(0, 3, 1, 2).contiguous())
        loss16 = F.cross_entropy(out16.float(), labels)
    loss16.backward()
    print(f"loss native {exe.loss.mean().item():.5f} ref {loss.item():.5f} torch-bf16 {loss16.item():.5f}")
    print(f"torch-bf16 logits rel err {rel(out16.float().detach(), out.detach()):.4f}")
    print(f"logits rel err {rel(exe.logits, out.detach()):.4f}")
    for bn in exe.all_bns():
        a = acts[bn.prefix]                     # NCHW
        y = bn.y.view(a.shape[0], a.shape[2], a.shape[3], a.shape[1]).permute(0, 3, 1, 2)
        print(f"{bn.prefix:28s} M={bn.M:8d} C={bn.C:5d}  y rel {rel(y, a):.4f}  "
              f"torch-bf16 rel {rel(acts16[bn.prefix].float(), a):.4f}")
    res = []
    for name, p in ref.named_parameters():
        g = exe.flat.view(exe.flat.grad, name, p.shape)
        res.append((F.cosine_similarity(g.flatten().float(), p.grad.flatten().float(), dim=0).item(),
                    rel(g, p.grad), name))
    res.sort()
    p16 = dict(ref16.named_parameters())
    for c, r, n in res[:20]:
        c16 = F.cosine_similarity(p16[n].grad.flatten().float(), dict(ref.named_parameters())[n].grad.flatten().float(), dim=0).item()
        print(f"grad {n:36s} cos {c:.4f} rel {r:.4f}   torch-bf16 cos {c16:.4f}")
    print("median grad cos", sorted(r[0] for r in res)[len(res) // 2])
    c16all = sorted(F.cosine_similarity(p16[n].grad.flatten().float(), p.grad.flatten().float(), dim=0).item()
                    for n, p in ref.named_parameters())
    print("torch-bf16 median grad cos", c16all[len(c16all) // 2])


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 8, int(sys.argv[2]) if len(sys.argv) > 2 else 64)
