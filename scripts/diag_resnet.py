"""Diagnostics for the native ResNet-50 executor: run-to-run determinism of the forward
and per-layer distance to the fp32 PyTorch reference (which BN input diverges first)."""
import copy
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, ".")
import pgdist  # noqa: F401,E402
from pgdist.models import build_model  # noqa: E402
from pgdist.engine.resnet_executor import ResNet50Executor  # noqa: E402


def rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def main():
    dev = torch.device("cuda", 0)
    B, S, NC = 4, 64, 10
    torch.manual_seed(0)
    model = build_model("resnet50", num_classes=NC)
    with torch.no_grad():
        for n, p in model.named_parameters():
            if p.dim() > 1:
                p.copy_(p.to(torch.bfloat16).float())
    ref = copy.deepcopy(model).to(dev).train()
    exe = ResNet50Executor(model, B, S, dev)
    g = torch.Generator(device="cpu").manual_seed(5)
    img = torch.randn(B, S, S, 3, generator=g).to(dev).to(torch.bfloat16)
    labels = torch.tensor([1, 2, 3, 4], device=dev)
    exe.img.zero_()
    exe.img[..., :3] = img
    exe.labels.copy_(labels)
    snaps = []
    for rep in range(3):
        exe.forward(train=True)
        torch.cuda.synchronize()
        snaps.append([bn.y.clone() for bn in exe.all_bns()] + [exe.logits.clone()])
    names = [bn.prefix for bn in exe.all_bns()] + ["logits"]
    for i, n in enumerate(names):
        d1 = (snaps[0][i].float() - snaps[1][i].float()).abs().max().item()
        d2 = (snaps[0][i].float() - snaps[2][i].float()).abs().max().item()
        if d1 or d2:
            print(f"NONDETERMINISTIC {n}: max diff {d1} {d2}")
    acts = {}

    def hook(name):
        def f(mod, inp, out):
            acts[name] = inp[0].detach().float()
        return f

    for n, m in ref.named_modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.register_forward_hook(hook(n))
    x = img.float().permute(0, 3, 1, 2).contiguous()
    with torch.no_grad():
        out = ref(x)
    for bn in exe.all_bns():
        a = acts[bn.prefix]
        y = bn.y.view(a.shape[0], a.shape[2], a.shape[3], a.shape[1]).permute(0, 3, 1, 2)
        print(f"{bn.prefix:24s} rel {rel(y, a):.4f}")
    print("logits rel", rel(exe.logits, out), "loss", exe.loss.mean().item(),
          F.cross_entropy(out, labels).item())


if __name__ == "__main__":
    main()
