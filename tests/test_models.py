"""Model definitions: torchvision-compatible structure, parameter counts and keys."""
import torch

from pgdist.models import mobilenet_v2, resnet50, build_model


def test_mobilenet_v2_param_count_matches_reference_log():
    m = mobilenet_v2(10)
    # logs_cifar10_cpu_27299.out:28 "Total parameters: 2236682"
    assert sum(p.numel() for p in m.parameters()) == 2236682
    assert len(list(m.parameters())) == 158


def test_mobilenet_v2_state_dict_layout():
    sd = mobilenet_v2(10).state_dict()
    assert len(sd) == 314
    assert sd["features.0.0.weight"].shape == (32, 3, 3, 3)
    assert sd["features.1.conv.0.0.weight"].shape == (32, 1, 3, 3)        # t=1 dw
    assert sd["features.1.conv.1.weight"].shape == (16, 32, 1, 1)         # t=1 project
    assert sd["features.2.conv.0.0.weight"].shape == (96, 16, 1, 1)       # expand
    assert sd["features.2.conv.1.0.weight"].shape == (96, 1, 3, 3)        # dw
    assert sd["features.2.conv.2.weight"].shape == (24, 96, 1, 1)         # project
    assert sd["features.2.conv.3.running_var"].shape == (24,)
    assert sd["features.18.0.weight"].shape == (1280, 320, 1, 1)
    assert sd["classifier.1.weight"].shape == (10, 1280)
    n_bn = sum(1 for k in sd if k.endswith("num_batches_tracked"))
    assert n_bn == 52


def test_mobilenet_v2_forward_shapes_and_residuals():
    m = mobilenet_v2(10).eval()
    res = [i for i, f in enumerate(m.features) if getattr(f, "use_res_connect", False)]
    assert res == [3, 5, 6, 8, 9, 10, 12, 13, 15, 16]
    with torch.no_grad():
        out = m(torch.randn(2, 3, 224, 224))
    assert out.shape == (2, 10)


def test_pretrained_head_swap(tmp_path):
    src = mobilenet_v2(1000)
    p = tmp_path / "imagenet.pth"
    torch.save(src.state_dict(), p)
    m = mobilenet_v2(10, pretrained=str(p))
    assert m.classifier[1].out_features == 10
    assert torch.equal(m.features[5].conv[1][0].weight, src.features[5].conv[1][0].weight)


def test_resnet50_param_count():
    assert sum(p.numel() for p in resnet50(1000).parameters()) == 25557032
    assert build_model("resnet50", 10).fc.out_features == 10


def test_coalesce_bn_buffers_views_and_values():
    from pgdist.engine.native_step import coalesce_bn_buffers
    torch.manual_seed(0)
    m = mobilenet_v2(10)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_mean.uniform_()
            mod.running_var.uniform_(1, 2)
            mod.num_batches_tracked.fill_(3)
    before = {k: v.clone() for k, v in m.state_dict().items()}
    flat, nbt = coalesce_bn_buffers(m)
    after = m.state_dict()
    assert set(before) == set(after)
    for k in before:
        assert torch.equal(before[k], after[k]), k
    assert flat.numel() == 2 * 17056 and nbt.numel() == 52
    flat.zero_()
    nbt.zero_()
    bn = m.features[0][1]
    assert float(bn.running_mean.abs().sum()) == 0.0 and int(bn.num_batches_tracked) == 0
