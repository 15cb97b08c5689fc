"""End-to-end: one ResNet-50 training step through the native dense-conv executor vs
PyTorch autograd in fp32 on the same (bf16-representable) input and weights.

Acceptance is relative to the bf16 noise floor (same criterion as the MobileNetV2
executor test): per BatchNorm input, logits and parameter gradients the native path
must be about as close to fp32 as PyTorch's own bf16 autocast step is."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from pgdist.models import build_model  # noqa: E402
from pgdist.engine.resnet_executor import ResNet50Executor  # noqa: E402


def _cos(a, b):
    return F.cosine_similarity(a.float().flatten(), b.float().flatten(), dim=0).item()


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _run_ref(model, x, labels, autocast):
    acts = {}

    def hook(name):
        def f(mod, inp, out):
            acts[name] = inp[0].detach().float()
        return f

    for n, m in model.named_modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.register_forward_hook(hook(n))
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        out = model(x)
        loss = F.cross_entropy(out.float(), labels)
    loss.backward()
    return out.detach().float(), loss.item(), acts


@pytest.mark.parametrize("B,S,NC", [(8, 128, 10), (4, 224, 1000)])
def test_resnet_step_matches_autograd(dev, B, S, NC):
    torch.manual_seed(0)
    model = build_model("resnet50", num_classes=NC)
    with torch.no_grad():
        for n, p in model.named_parameters():
            if p.dim() > 1:
                p.copy_(p.to(torch.bfloat16).float())
    ref = copy.deepcopy(model).to(dev).train()
    ref16 = copy.deepcopy(model).to(dev).train()
    exe = ResNet50Executor(model, B, S, dev)
    img = torch.randn(B, S, S, 3, device=dev).to(torch.bfloat16)
    labels = torch.randint(0, NC, (B,), device=dev)
    exe.img.zero_()
    exe.img[..., :3] = img
    exe.labels.copy_(labels)
    exe.flat.refresh_shadow()
    exe.forward(train=True)
    exe.backward()
    torch.cuda.synchronize()

    x = img.float().permute(0, 3, 1, 2).contiguous()
    out, loss, acts = _run_ref(ref, x, labels, autocast=False)
    out16, loss16, acts16 = _run_ref(ref16, x, labels, autocast=True)

    assert abs(exe.loss.mean().item() - loss) < 0.05 + 2 * abs(loss16 - loss)
    assert _rel(exe.logits, out) <= 1.5 * _rel(out16, out) + 0.02
    for bn in exe.all_bns():
        a = acts[bn.prefix]
        y = bn.y.view(a.shape[0], a.shape[2], a.shape[3], a.shape[1]).permute(0, 3, 1, 2)
        assert _rel(y, a) <= 1.5 * _rel(acts16[bn.prefix], a) + 0.02, bn.prefix
    p16 = dict(ref16.named_parameters())
    cos_native, cos16 = [], []
    for name, p in ref.named_parameters():
        cos_native.append(_cos(exe.flat.view(exe.flat.grad, name, p.shape), p.grad))
        cos16.append(_cos(p16[name].grad, p.grad))
    med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
    assert med(cos_native) >= med(cos16) - 0.05, (med(cos_native), med(cos16))
    fc16 = _cos(p16["fc.weight"].grad, ref.fc.weight.grad)
    assert _cos(exe.flat.g("fc.weight"), ref.fc.weight.grad) > min(0.98, fc16 - 0.03), fc16
    assert _cos(exe.flat.view(exe.flat.grad, "conv1.weight", ref.conv1.weight.shape), ref.conv1.weight.grad) > \
        min(0.9, _cos(p16["conv1.weight"].grad, ref.conv1.weight.grad) - 0.05)
    # the stem weight's padding channel (4-channel NHWC storage) never moves off zero
    o, n = exe.flat.offsets["conv1.weight"]
    assert exe.flat.grad[o:o + n].view(64, 7, 7, 4)[..., 3].abs().max().item() == 0.0
    for m in exe.model.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            assert int(m.num_batches_tracked) == 1
    assert _rel(exe.model.bn1.running_mean, ref.bn1.running_mean) < 0.02


def test_resnet_native_step_loss_decreases(dev):
    from pgdist.engine.native_step import NativeTrainStep
    torch.manual_seed(0)
    model = build_model("resnet50", num_classes=10)
    st = NativeTrainStep(model, 8, dev, img_size=64, lr=1e-3, use_graph=False, train_augment=False)
    src = torch.randint(0, 256, (4, 64, 64, 3), dtype=torch.uint8, device=dev)
    labels = torch.tensor([0, 3, 5, 7], device=dev)
    st.set_data(src, labels)
    idx = torch.arange(8, device=dev) % 4
    losses = []
    for i in range(30):
        st.run(idx)
        if i % 5 == 4:
            l, c, n = st.read_metrics()
            losses.append(l / n)
    assert losses[-1] < losses[0] * 0.5, losses
    assert torch.isfinite(st.flat.master).all()
