"""End-to-end: one MobileNetV2 training step through the native executor vs
PyTorch autograd in fp32 on the same (bf16-representable) input and weights."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from pgdist.models import mobilenet_v2  # noqa: E402
from pgdist.engine.executor import MobileNetV2Executor  # noqa: E402


def _cos(a, b):
    return F.cosine_similarity(a.float().flatten(), b.float().flatten(), dim=0).item()


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("B,S", [(8, 64), (4, 224)])
def test_executor_step_matches_autograd(dev, B, S):
    torch.manual_seed(0)
    model = mobilenet_v2(10)
    model.classifier[0].p = 0.0                  # deterministic comparison
    # weights exactly representable in bf16 so both paths see the same values
    with torch.no_grad():
        for n, p in model.named_parameters():
            if p.dim() > 1 and not n.startswith("classifier"):
                p.copy_(p.to(torch.bfloat16).float())
    ref = copy.deepcopy(model).to(dev).train()
    exe = MobileNetV2Executor(model, B, S, dev)
    img = torch.randn(B, S, S, 3, device=dev).to(torch.bfloat16)
    labels = torch.randint(0, 10, (B,), device=dev)
    exe.img.zero_()
    exe.img[..., :3] = img
    exe.labels.copy_(labels)
    exe.forward(train=True)
    exe.backward()
    torch.cuda.synchronize()

    x = img.float().permute(0, 3, 1, 2).contiguous()
    out = ref(x)
    loss = F.cross_entropy(out, labels)
    loss.backward()

    assert abs(exe.loss.mean().item() - loss.item()) < 0.05 * max(1.0, abs(loss.item()))
    assert _cos(exe.logits, out.detach()) > 0.995
    worst = []
    for name, p in ref.named_parameters():
        g_native = exe.flat.g(name).view_as(p)
        c = _cos(g_native, p.grad)
        worst.append((c, name, _rel(g_native, p.grad)))
    worst.sort()
    assert worst[0][0] > 0.97, worst[:5]
    # BN running statistics updated like torch
    for (n, m), (_, mr) in zip(exe.model.named_modules(), ref.named_modules()):
        if isinstance(m, torch.nn.BatchNorm2d):
            assert _rel(m.running_mean, mr.running_mean) < 0.05, n
            assert _rel(m.running_var, mr.running_var) < 0.05, n
            assert int(m.num_batches_tracked) == 1


def test_native_train_step_loss_decreases(dev):
    from pgdist.engine.native_step import NativeTrainStep
    torch.manual_seed(0)
    model = mobilenet_v2(10)
    st = NativeTrainStep(model, 16, dev, img_size=64, lr=1e-3, use_graph=True)
    # 4 images x 16 copies: memorisation task
    src = torch.randint(0, 256, (4, 32, 32, 3), dtype=torch.uint8, device=dev)
    labels = torch.tensor([0, 3, 5, 7], device=dev)
    st.set_data(src, labels)
    st.augment_enabled = True
    idx = torch.arange(16, device=dev) % 4
    losses = []
    for i in range(30):
        st.run(idx)
        if i % 5 == 4:
            l, c, n = st.read_metrics()
            losses.append(l / n)
    assert losses[-1] < losses[0] * 0.7, losses
    assert st.graph is not None
