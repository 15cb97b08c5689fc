"""Inference helper and web demo (reference predict_cifar10_image + Gradio predict())."""
import io

import numpy as np
import pytest
import torch

from pgdist.models import mobilenet_v2
from pgdist.serve.predict import Predictor, predict_cifar10_image, eval_transform


def _png(tmp_path, color=(200, 30, 30)):
    from PIL import Image
    arr = np.zeros((32, 32, 3), dtype=np.uint8)
    arr[...] = color
    p = tmp_path / "img.png"
    Image.fromarray(arr).save(p)
    return p


@pytest.fixture
def ckpt(tmp_path):
    torch.manual_seed(0)
    m = mobilenet_v2(10)
    p = tmp_path / "best.pth"
    torch.save({"module." + k: v for k, v in m.state_dict().items()}, p)   # DDP-style prefix accepted
    return p, m


def test_predict_format_and_threshold(tmp_path, ckpt, capsys):
    p, m = ckpt
    pred = Predictor(str(p), device="cpu")
    res = predict_cifar10_image(str(_png(tmp_path)), topk=3, conf_threshold=0.99, predictor=pred)
    out = capsys.readouterr().out
    assert "Top-3 predictions:" in out and "Prediction uncertain" in out
    assert len(res) == 3 and all(isinstance(l, str) and 0 <= c <= 1 for l, c in res)
    assert res[0][1] >= res[1][1] >= res[2][1]
    res2 = predict_cifar10_image(str(_png(tmp_path)), topk=3, conf_threshold=0.0, predictor=pred)
    assert "Predicted:" in capsys.readouterr().out and res2 == res


def test_matches_module_forward(tmp_path, ckpt):
    p, m = ckpt
    pred = Predictor(str(p), device="cpu")
    img = _png(tmp_path, (10, 200, 90))
    from PIL import Image
    arr = np.asarray(Image.open(img).convert("RGB"))
    with torch.no_grad():
        ref = torch.softmax(m.eval()(eval_transform(arr)), 1)[0]
    got = pred.probs([str(img)])[0]
    assert torch.allclose(got, ref, atol=1e-5)


def test_fastapi_app(tmp_path, ckpt):
    pytest.importorskip("fastapi")
    from fastapi.testclient import TestClient
    from pgdist.serve.app import build_fastapi
    p, _ = ckpt
    client = TestClient(build_fastapi(Predictor(str(p), device="cpu")))
    data = _png(tmp_path).read_bytes()
    r = client.post("/predict", content=data)
    assert r.status_code == 200
    lab = r.json()["label"]
    assert len(lab) == 3 and abs(sum(lab.values())) <= 1.0 + 1e-6
    assert client.get("/").status_code == 200


@pytest.mark.gpu
def test_native_predictor_matches_torch(tmp_path, ckpt):
    p, m = ckpt
    img = str(_png(tmp_path, (90, 10, 240)))
    ref = Predictor(str(p), device="cpu").probs([img, img])
    nat = Predictor(str(p), device="cuda", backend="hip", max_batch=4).probs([img, img])
    # bf16 noise floor: the same fp32 module under torch bf16 autocast on the GPU
    tp = Predictor(str(p), device="cuda")
    from PIL import Image
    x = eval_transform(np.asarray(Image.open(img).convert("RGB"))).cuda()
    x = x if x.dim() == 4 else x.unsqueeze(0)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        p16 = torch.softmax(tp.model(x).float(), 1).cpu()
    floor = (p16[0] - ref[0]).abs().max().item()
    err = (nat - ref).abs().max().item()
    assert err <= 2 * floor + 5e-3, (err, floor)
    assert nat.argmax(1).tolist() == ref.argmax(1).tolist()


@pytest.mark.gpu
def test_native_predictor_resnet50(tmp_path):
    """ResNet-50 checkpoint served through its native eval executor (BN from running stats)."""
    from pgdist.models import build_model
    torch.manual_seed(0)
    m = build_model("resnet50", num_classes=10)
    with torch.no_grad():   # non-trivial running statistics
        for mod in m.modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.uniform_(-0.1, 0.1)
                mod.running_var.uniform_(0.5, 1.5)
    p = tmp_path / "r50.pth"
    torch.save(m.state_dict(), p)
    img = str(_png(tmp_path, (20, 180, 60)))
    ref = Predictor(str(p), device="cpu", model_name="resnet50").probs([img])
    nat = Predictor(str(p), device="cuda", backend="hip", max_batch=2, model_name="resnet50").probs([img])
    assert torch.allclose(nat, ref, atol=0.05)
