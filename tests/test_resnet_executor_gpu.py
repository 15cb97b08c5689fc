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


@pytest.mark.parametrize("M,N,K_,orient", [
    (128, 1000, 2048, "fwd"), (128, 2048, 1000, "dpool"), (1000, 2048, 128, "dw"),
    (5, 37, 100, "fwd"), (3, 70, 33, "dpool"), (37, 65, 7, "dw"), (64, 10, 2048, "fwd")])
def test_fc_gemm_matches_fp32(dev, M, N, K_, orient):
    """Native fp32 head GEMMs (csrc/kernels/fc.hip) vs torch fp32 matmul (TF32 off), in the three
    operand orientations of the classifier forward / backward; split-K is deterministic."""
    from pgdist.ops import kernels as K
    torch.backends.cuda.matmul.allow_tf32 = False
    g = torch.Generator(device=dev).manual_seed(M * 7 + N)
    bias = None
    if orient == "fwd":       # C = A[M,K] . W[N,K]^T + b
        A = torch.randn(M, K_, device=dev, generator=g)
        B = torch.randn(N, K_, device=dev, generator=g)
        bias = torch.randn(N, device=dev, generator=g)
        ref = A @ B.t() + bias
        args = (A, K_, 1, B, 1, K_)
    elif orient == "dpool":   # C = A[M,K] . B[K,N]
        A = torch.randn(M, K_, device=dev, generator=g)
        B = torch.randn(K_, N, device=dev, generator=g)
        ref = A @ B
        args = (A, K_, 1, B, N, 1)
    else:                     # C = A[K,M]^T . B[K,N]
        A = torch.randn(K_, M, device=dev, generator=g)
        B = torch.randn(K_, N, device=dev, generator=g)
        ref = A.t() @ B
        args = (A, 1, M, B, N, 1)
    ws = torch.empty(max(K.fc_gemm_workspace_floats(M, N, K_), 1), device=dev)
    outs = []
    for _ in range(2):
        C = torch.full((M, N), float("nan"), device=dev)
        K.fc_gemm(*args, C, M, N, K_, bias=bias, ws=ws)
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    err = (outs[0] - ref).abs().max().item()
    assert err <= 1e-5 * (K_ ** 0.5) * ref.abs().max().item() + 1e-5, err
    X = torch.randn(M, N, device=dev, generator=g)
    s = torch.empty(N, device=dev)
    K.col_sum(X, M, N, s)
    ref_s = X.double().sum(0).float()   # fp32 summation error ~ sqrt(M) ulp
    assert (s - ref_s).abs().max().item() <= 2e-6 * M ** 0.5 * X.abs().max().item() * 4


def test_fc_gemm_rejects_bad_operands(dev):
    from pgdist.ops import kernels as K
    A = torch.zeros(4, 8, device=dev)
    B = torch.zeros(6, 8, device=dev)
    C = torch.zeros(4, 6, device=dev)
    with pytest.raises(ValueError, match="strides address"):
        K.fc_gemm(A, 8, 1, B, 1, 8, C, 4, 6, 9)            # K beyond the operands
    with pytest.raises(ValueError):
        K.fc_gemm(A.double(), 8, 1, B, 1, 8, C, 4, 6, 8)
    with pytest.raises(ValueError):
        K.fc_gemm(A, 8, 1, B, 1, 8, C[:3], 4, 6, 8)


def test_resnet_launch_plan_matches_eager(dev, deterministic, monkeypatch):
    """The ResNet-50 step replayed from a native launch plan (recorded on the 3rd step; head
    GEMMs native) gives bitwise the weights, Adam state and metrics of eager launching."""
    from pgdist.engine.native_step import NativeTrainStep
    src = torch.randint(0, 256, (16, 64, 64, 3), dtype=torch.uint8, device=dev,
                        generator=torch.Generator(device=dev).manual_seed(3))
    labels = torch.arange(16, device=dev) % 10
    out = {}
    for plan in ("1", "0"):
        monkeypatch.setenv("PGDIST_PLAN", plan)
        torch.manual_seed(0)
        st = NativeTrainStep(build_model("resnet50", num_classes=10), 8, dev, img_size=64, lr=1e-3,
                             use_graph=False)
        assert st.use_plan == (plan == "1")
        st.set_data(src, labels)
        for i in range(5):
            st.run((torch.arange(8, device=dev) + 3 * i) % 16)
        torch.cuda.synchronize()
        if plan == "1":
            assert st.plan is not None and len(st.plan) > 300
        out[plan] = (st.flat.master.clone(), st.flat.exp_avg.clone(), st.read_metrics())
    assert torch.equal(out["1"][0], out["0"][0])
    assert torch.equal(out["1"][1], out["0"][1])
    assert out["1"][2] == out["0"][2]


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


@pytest.mark.parametrize("mode", ["1", "act"])
@pytest.mark.parametrize("stem", ["s2d", "direct"])
def test_resnet_lazy_bn_matches_launch(dev, monkeypatch, stem, mode):
    """Lazy BN finalize (consumers compute the parameters from the replica rows; side outputs
    batched at the end of the forward / on the side stream) vs a finalize launch after every
    producer: after 4 replayed training steps the weights, Adam moments, BN running statistics
    and metrics agree within the float-atomic noise floor of the replica rows (both modes add the
    statistics atomically; estimated as the median pairwise spread of three launch-mode runs, and
    the lazy run is compared with its closest launch-mode run).  mode "1": every consumer that
    can is lazy; "act" (the default): only the forward relu(BN) materialisations."""
    from pgdist.engine.native_step import NativeTrainStep
    from pgdist.engine.resnet_executor import ResNet50Executor
    monkeypatch.setattr(ResNet50Executor, "STEM", stem)
    src = torch.randint(0, 256, (16, 64, 64, 3), dtype=torch.uint8, device=dev,
                        generator=torch.Generator(device=dev).manual_seed(5))
    labels = torch.arange(16, device=dev) % 10
    out = []
    for lazy in ("0", "0", "0", mode):
        monkeypatch.setenv("PGDIST_BN_LAZY", lazy)
        torch.manual_seed(0)
        st = NativeTrainStep(build_model("resnet50", num_classes=10), 8, dev, img_size=64, lr=1e-3,
                             use_graph=False)
        assert st.exe.lazy_bn == (lazy != "0")
        st.set_data(src, labels)
        losses = []
        for i in range(4):
            st.run((torch.arange(8, device=dev) + 3 * i) % 16)
            lsum, _, n = st.read_metrics()
            losses.append(lsum / n)
        torch.cuda.synchronize()
        rs = torch.cat([m.running_var.flatten() for m in st.exe.model.modules()
                        if isinstance(m, torch.nn.BatchNorm2d)])
        nbt = [int(m.num_batches_tracked) for m in st.exe.model.modules() if isinstance(m, torch.nn.BatchNorm2d)]
        out.append((st.flat.master.clone(), st.flat.exp_avg.clone(), rs, nbt, losses))
    ref, lz = out[:3], out[3]
    (w0, m0, r0, n0, k0) = ref[0]
    (w2, m2, r2, n2, k2) = lz
    assert n2 == n0 and set(n2) == {4}
    pairs = [(a, b) for i, a in enumerate(ref) for b in ref[i + 1:]]

    def spread(f):   # median pairwise spread of the three reference runs
        return sorted(f(a, b) for a, b in pairs)[len(pairs) // 2]

    def dist(f):     # lazy run vs the closest reference run (the same statistic as a pair)
        return min(f(lz, r) for r in ref)
    # the first step's forward sees identical weights: its loss agrees to the atomic noise (a
    # consumer reading stale BN parameters would be off by far more).  The noise is chaotic: the
    # float-atomic order of the replica rows flips bf16 roundings that 50 BN layers at batch 8 and
    # 16-pixel maps amplify -- identically configured launch-mode runs in one process differ by up
    # to 0.05 in this loss (scripts/diag_resnet_lazy_act.py), so three of them can under-estimate
    # it; hence the 3 % floor
    lnoise = spread(lambda a, b: abs(a[4][0] - b[4][0]))
    assert dist(lambda a, b: abs(a[4][0] - b[4][0])) <= max(10 * lnoise, 0.03 * abs(k0[0])), \
        ([r[4] for r in ref], k2)
    noise = max(spread(lambda a, b: _rel(a[0], b[0])), 1e-6)
    assert dist(lambda a, b: _rel(a[0], b[0])) < max(20 * noise, 1e-4), (_rel(w2, w0), noise)
    assert dist(lambda a, b: _rel(a[1], b[1])) < max(20 * max(spread(lambda a, b: _rel(a[1], b[1])), 1e-6), 1e-3)
    assert dist(lambda a, b: _rel(a[2], b[2])) < max(20 * max(spread(lambda a, b: _rel(a[2], b[2])), 1e-6), 1e-4)
