"""fp8 vs bf16 executor step against fp32 autograd: loss, gradient cosines per layer."""
import copy
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import pgdist  # noqa: E402,F401
from pgdist.engine.executor import MobileNetV2Executor  # noqa: E402
from pgdist.models import mobilenet_v2  # noqa: E402


def cos(a, b):
    a, b = a.flatten().float(), b.flatten().float()
    return float(a @ b / (a.norm() * b.norm() + 1e-30))


def main(B=8, S=64):
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = mobilenet_v2(10)
    model.classifier[0].p = 0.0
    ref = copy.deepcopy(model).to(dev).train()
    img = torch.randn(B, S, S, 3, device=dev).to(torch.bfloat16)
    labels = torch.randint(0, 10, (B,), device=dev)
    x = img.float().permute(0, 3, 1, 2).contiguous()
    out = ref(x)
    loss = F.cross_entropy(out, labels)
    loss.backward()
    print("ref loss", loss.item())
    res = {}
    for fp8 in (False, True):
        exe = MobileNetV2Executor(copy.deepcopy(model), B, S, dev, fp8=fp8)
        exe.img.zero_()
        exe.img[..., :3] = img
        exe.labels.copy_(labels)
        exe.forward(train=True)
        exe.backward()
        torch.cuda.synchronize()
        cs = {n: cos(exe.flat.view(exe.flat.grad, n, p.shape), p.grad) for n, p in ref.named_parameters()}
        res[fp8] = cs
        print("fp8" if fp8 else "bf16", "loss", exe.loss.mean().item(), "logits cos", cos(exe.logits, out.detach()),
              "median grad cos", sorted(cs.values())[len(cs) // 2])
    for n in list(res[False])[::6]:
        print(f"{n:40s} bf16 {res[False][n]:7.4f} fp8 {res[True][n]:7.4f}")


if __name__ == "__main__":
    main(*[int(a) for a in sys.argv[1:]])
