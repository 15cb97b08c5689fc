"""Inference: top-k prediction with a confidence threshold.

Reference: ``predict_cifar10_image(img_path, topk=3, conf_threshold=0.5)``
(``cifar10_serial_mobilenet_224.py:155-191``): open image -> RGB -> test
transform (Resize 224, ToTensor, ImageNet Normalize) -> eval forward ->
softmax -> topk -> prints the top-k and "Prediction uncertain" below the
threshold -> returns ``[(label, conf), ...]``.

:class:`Predictor` loads the reference's checkpoint format
(``best_mobilenetv2_cifar10_224.pth``, torchvision keys, with or without a
``module.`` prefix) and runs either the PyTorch module (CPU) or, on an MI355X,
the native HIP executor in eval mode (BN from running statistics, no dropout)
with the same GPU resize/normalise kernel used for the test set.
"""
from typing import Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
import torch.nn.functional as F

from .. import CIFAR10_CLASSES, IMAGENET_MEAN, IMAGENET_STD
from ..models import build_model


def _to_uint8_rgb(img) -> np.ndarray:
    from PIL import Image
    if isinstance(img, (str, bytes)) or hasattr(img, "read"):
        img = Image.open(img)
    if isinstance(img, Image.Image):
        img = np.asarray(img.convert("RGB"))
    arr = np.asarray(img)
    if arr.ndim == 2:
        arr = np.stack([arr] * 3, -1)
    return np.ascontiguousarray(arr[..., :3].astype(np.uint8))


def eval_transform(arr: np.ndarray, size: int = 224, mean=IMAGENET_MEAN, std=IMAGENET_STD) -> torch.Tensor:
    """uint8 HWC -> normalised float [1,3,size,size] (Resize((size,size)) + ToTensor + Normalize)."""
    x = torch.from_numpy(np.ascontiguousarray(arr) if arr.flags.writeable else arr.copy())
    x = x.permute(2, 0, 1).float().div(255.0)[None]
    x = F.interpolate(x, size=(size, size), mode="bilinear", align_corners=False)
    m = torch.tensor(mean).view(1, 3, 1, 1)
    s = torch.tensor(std).view(1, 3, 1, 1)
    return (x - m) / s


class Predictor:
    def __init__(self, checkpoint: Optional[str] = None, model: Optional[torch.nn.Module] = None,
                 device: Union[str, torch.device] = "auto", classes: Sequence[str] = CIFAR10_CLASSES,
                 img_size: int = 224, backend: str = "auto", normalize: str = "imagenet",
                 max_batch: int = 16, model_name: str = "mobilenet_v2"):
        dev = torch.device("cuda" if (device == "auto" and torch.cuda.is_available()) else
                           ("cpu" if device == "auto" else device))
        self.device, self.classes, self.img_size = dev, tuple(classes), img_size
        if model is None:
            model = build_model(model_name, num_classes=len(classes))
            if checkpoint:
                from ..engine.checkpoint import load_model_weights
                load_model_weights(model, checkpoint)
        self.model = model.eval().to(dev)
        # The reference's Gradio app normalised with CIFAR statistics although training used
        # ImageNet statistics (GROUP03.pdf p.26); "cifar" reproduces that.
        self.mean, self.std = ((0.4914, 0.4822, 0.4465), (0.2023, 0.1994, 0.2010)) if normalize == "cifar" \
            else (IMAGENET_MEAN, IMAGENET_STD)
        if backend == "auto":
            backend = "hip" if dev.type == "cuda" else "torch"
        self.backend = backend
        self.max_batch = max_batch
        if backend == "hip":   # native eval executor of the model family (BN from running statistics)
            from ..engine.native_step import executor_class
            self.exe = executor_class(self.model)(self.model, max_batch, img_size, dev)
            self.exe.eval_prepare()

    @torch.no_grad()
    def probs(self, images: List) -> torch.Tensor:
        xs = torch.cat([eval_transform(_to_uint8_rgb(im), self.img_size, self.mean, self.std) for im in images])
        if self.backend != "hip":
            logits = self.model(xs.to(self.device))
            return F.softmax(logits.float(), dim=1).cpu()
        out = []
        for s in range(0, xs.shape[0], self.max_batch):
            chunk = xs[s:s + self.max_batch]
            n = chunk.shape[0]
            img = self.exe.img
            img.zero_()
            img[:n, ..., :3] = chunk.permute(0, 2, 3, 1).to(self.device, torch.bfloat16)
            self.exe.forward(train=False)
            out.append(F.softmax(self.exe.logits[:n].float(), dim=1).cpu())
        return torch.cat(out)

    def topk(self, image, k: int = 3) -> List[Tuple[str, float]]:
        p = self.probs([image])[0]
        conf, idx = torch.topk(p, k=min(k, p.numel()))
        return [(self.classes[int(i)], float(c)) for c, i in zip(conf, idx)]

    def label_dict(self, image, k: int = 3) -> Dict[str, float]:
        """Gradio ``Label`` format ``{class: prob}`` (reference app ``predict(img)``)."""
        return {lab: c for lab, c in self.topk(image, k)}


_DEFAULT: Optional[Predictor] = None


def predict_cifar10_image(img_path, topk: int = 3, conf_threshold: float = 0.5,
                          predictor: Optional[Predictor] = None, checkpoint: Optional[str] = None,
                          verbose: bool = True) -> List[Tuple[str, float]]:
    """Reference-compatible helper (same arguments, prints and return value)."""
    global _DEFAULT
    if predictor is None:
        if _DEFAULT is None or checkpoint is not None:
            _DEFAULT = Predictor(checkpoint or "best_mobilenetv2_cifar10_224.pth")
        predictor = _DEFAULT
    res = predictor.topk(img_path, topk)
    if verbose:
        print("Top-{} predictions:".format(topk))
        for label, c in res:
            print(f"  {label}: {c:.3f}")
        best_label, best_conf = res[0]
        if best_conf < conf_threshold:
            print(f"Prediction uncertain (best_conf={best_conf:.3f} < {conf_threshold})")
        else:
            print(f"Predicted: {best_label} confidence: {best_conf:.3f}")
    return res


test_transform = eval_transform  # reference name (cifar10_serial_mobilenet_224.py:42)
inference_transform = eval_transform  # reference :157
