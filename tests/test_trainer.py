"""Training engine: reference log formats, best-model export, full-state resume."""
import re

import pytest
import torch

from pgdist.config import TrainConfig, preset
from pgdist.engine.trainer import Trainer, step_lr

SERIAL_RE = re.compile(r"^Epoch (\d+)/(\d+) Time: [\d.]+s Train Loss: [\d.]+ Train Acc: [\d.]+ "
                       r"Test Loss: [\d.]+ Test Acc: [\d.]+$")


def test_step_lr_matches_torch():
    p = torch.nn.Parameter(torch.zeros(1))
    opt = torch.optim.Adam([p], lr=1e-4)
    sch = torch.optim.lr_scheduler.StepLR(opt, step_size=10, gamma=0.1)
    for e in range(25):
        assert abs(opt.param_groups[0]["lr"] - step_lr(1e-4, e, 10, 0.1)) < 1e-12
        opt.step()
        sch.step()


def test_presets_match_reference_constants():
    s, g, m = preset("serial"), preset("gpu128"), preset("mpi")
    assert (s.batch_size, s.device, s.epochs, s.lr) == (64, "cpu", 20, 1e-4)
    assert (g.batch_size, g.save_path) == (128, "best_mobilenetv2_cifar10_224.pth")
    assert (m.batch_size, m.seed, m.save_path) == (128, 42, "best_mobilenetv2_cifar10_224_mpi.pth")
    # DDP default broadcast_buffers=True (cifar10_mpi_mobilenet_224.py:142-145): BN buffers every step
    assert m.bn_sync == "broadcast"
    assert (s.step_size, s.gamma, s.img_size) == (10, 0.1, 224)


def _cfg(tmp_path, **kw):
    base = dict(data="synthetic", synthetic_train_size=40, synthetic_test_size=16, batch_size=16, epochs=2,
                img_size=32, device="cpu", backend="torch", precision="fp32", augment="torch",
                save_path=str(tmp_path / "best.pth"), seed=0)
    base.update(kw)
    return TrainConfig(**base)


def test_cpu_training_log_and_checkpoint(tmp_path, capsys):
    tr = Trainer(_cfg(tmp_path, ckpt_dir=str(tmp_path / "ck")))
    hist = tr.fit()
    out = capsys.readouterr().out.splitlines()
    assert "Device: cpu" in out and "Train samples: 40" in out and "Total parameters: 2236682" in out
    epoch_lines = [l for l in out if l.startswith("Epoch ")]
    assert len(epoch_lines) == 2 and all(SERIAL_RE.match(l) for l in epoch_lines)
    assert any(l.startswith("Best test accuracy: ") for l in out)
    assert any(re.match(r"^Total training time: [\d.]+s \([\d.]+ min\)$", l) for l in out)
    assert f"Saved {tmp_path / 'best.pth'}" in out
    sd = torch.load(tmp_path / "best.pth", weights_only=True)
    assert len(sd) == 314 and sd["features.2.conv.1.0.weight"].shape == (96, 1, 3, 3)
    assert (tmp_path / "ck" / "ckpt_epoch2.pt").exists()
    assert hist[-1]["train_images"] == 40   # short last batch kept (drop_last=False)


def test_resume_continues_epochs(tmp_path, capsys):
    Trainer(_cfg(tmp_path, epochs=1, ckpt_dir=str(tmp_path / "ck"))).fit()
    tr = Trainer(_cfg(tmp_path, epochs=2, ckpt_dir=str(tmp_path / "ck"), resume="auto"))
    assert tr.start_epoch == 1
    st = next(iter(tr.opt.state.values()))
    assert int(st["step"]) == 3                     # 40 samples / bs 16 -> 3 steps in epoch 1
    hist = tr.fit()
    assert [h["epoch"] for h in hist] == [2]


@pytest.mark.gpu
def test_native_training_hip_backend(tmp_path, capsys):
    cfg = _cfg(tmp_path, device="cuda", backend="hip", precision="bf16", augment="gpu",
               synthetic_train_size=300, synthetic_test_size=70, batch_size=32, epochs=3, img_size=64,
               lr=1e-3, ckpt_dir=str(tmp_path / "ck"))
    tr = Trainer(cfg)
    hist = tr.fit()
    out = capsys.readouterr().out.splitlines()
    assert "Device: cuda" in out
    assert sum(1 for l in out if SERIAL_RE.match(l)) == 3
    assert hist[-1]["train_images"] == 300          # 9 full batches + a native tail batch of 12
    assert hist[-1]["train_loss"] < hist[0]["train_loss"]
    assert all(h["test_loss"] == h["test_loss"] for h in hist)
    sd = torch.load(tmp_path / "best.pth", weights_only=True)
    assert len(sd) == 314
    # resume from the last full checkpoint
    tr2 = Trainer(cfg.replace(epochs=4, resume="auto"))
    assert tr2.start_epoch == 3
    assert int(tr2.step.hyper[1].item()) == 30


@pytest.mark.gpu
def test_native_training_resnet50(tmp_path, capsys):
    """ResNet-50 (BASELINE config 4) through the same trainer on the native dense-conv executor:
    CIFAR-shaped data GPU-augmented to 64x64, tail batch, eval, torchvision-keyed checkpoint."""
    cfg = _cfg(tmp_path, device="cuda", backend="hip", precision="bf16", augment="gpu", model="resnet50",
               synthetic_train_size=100, synthetic_test_size=40, batch_size=16, epochs=2, img_size=64,
               lr=1e-3, ckpt_dir=str(tmp_path / "ck"))
    tr = Trainer(cfg)
    hist = tr.fit()
    out = capsys.readouterr().out.splitlines()
    assert sum(1 for l in out if SERIAL_RE.match(l)) == 2
    assert hist[-1]["train_images"] == 100          # 6 full batches + a native tail batch of 4
    assert all(h["train_loss"] == h["train_loss"] and h["test_loss"] == h["test_loss"] for h in hist)
    sd = torch.load(tmp_path / "best.pth", weights_only=True)
    assert len(sd) == 320 and tuple(sd["conv1.weight"].shape) == (64, 3, 7, 7)
