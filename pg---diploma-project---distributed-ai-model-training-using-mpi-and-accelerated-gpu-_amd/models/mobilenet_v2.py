"""MobileNetV2 with torchvision-identical module tree and ``state_dict`` keys.

Reference usage: ``models.mobilenet_v2(pretrained=True)`` followed by the head
swap ``classifier[1] = nn.Linear(1280, 10)``
(``cifar10_serial_mobilenet_224.py:70-73``, ``cifar10_mpi_mobilenet_224.py:137-140``).
torchvision is not available in this environment, so the architecture is
re-declared here; the parameter count (2,236,682 for 10 classes) and the key set
(314 entries) are pinned by tests.

This module is the *semantic* definition (and the CPU / oracle execution path).
The MI355X execution path does not run ``forward`` through autograd: it is
compiled into a static plan by :mod:`pgdist.engine.executor`, which reads the
same parameters.
"""
from typing import List, Optional

import torch
from torch import nn
import torch.nn.functional as F


def _make_divisible(v: float, divisor: int = 8, min_value: Optional[int] = None) -> int:
    if min_value is None:
        min_value = divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < 0.9 * v:
        new_v += divisor
    return new_v


class ConvBNAct(nn.Sequential):
    """conv -> BN -> (ReLU6).  Children are named 0/1/2 like torchvision's
    ``Conv2dNormActivation`` so keys read ``features.0.0.weight`` etc."""

    def __init__(self, cin: int, cout: int, kernel_size: int = 3, stride: int = 1,
                 groups: int = 1, act: bool = True):
        padding = (kernel_size - 1) // 2
        layers = [nn.Conv2d(cin, cout, kernel_size, stride, padding, groups=groups, bias=False),
                  nn.BatchNorm2d(cout)]
        if act:
            layers.append(nn.ReLU6(inplace=True))
        super().__init__(*layers)
        self.out_channels = cout


class InvertedResidual(nn.Module):
    def __init__(self, inp: int, oup: int, stride: int, expand_ratio: int):
        super().__init__()
        assert stride in (1, 2)
        self.stride = stride
        self.expand_ratio = expand_ratio
        hidden = int(round(inp * expand_ratio))
        self.use_res_connect = stride == 1 and inp == oup
        layers: List[nn.Module] = []
        if expand_ratio != 1:
            layers.append(ConvBNAct(inp, hidden, kernel_size=1))
        layers.extend([
            ConvBNAct(hidden, hidden, stride=stride, groups=hidden),
            nn.Conv2d(hidden, oup, 1, 1, 0, bias=False),
            nn.BatchNorm2d(oup),
        ])
        self.conv = nn.Sequential(*layers)
        self.inp, self.oup, self.hidden = inp, oup, hidden

    def forward(self, x):
        if self.use_res_connect:
            return x + self.conv(x)
        return self.conv(x)


# (t, c, n, s) — torchvision's inverted_residual_setting
MOBILENET_V2_SETTING = [
    [1, 16, 1, 1],
    [6, 24, 2, 2],
    [6, 32, 3, 2],
    [6, 64, 4, 2],
    [6, 96, 3, 1],
    [6, 160, 3, 2],
    [6, 320, 1, 1],
]


class MobileNetV2(nn.Module):
    def __init__(self, num_classes: int = 1000, width_mult: float = 1.0,
                 dropout: float = 0.2, round_nearest: int = 8):
        super().__init__()
        input_channel = _make_divisible(32 * width_mult, round_nearest)
        self.last_channel = _make_divisible(1280 * max(1.0, width_mult), round_nearest)
        features: List[nn.Module] = [ConvBNAct(3, input_channel, stride=2)]
        for t, c, n, s in MOBILENET_V2_SETTING:
            out = _make_divisible(c * width_mult, round_nearest)
            for i in range(n):
                features.append(InvertedResidual(input_channel, out, s if i == 0 else 1, t))
                input_channel = out
        features.append(ConvBNAct(input_channel, self.last_channel, kernel_size=1))
        self.features = nn.Sequential(*features)
        self.classifier = nn.Sequential(nn.Dropout(p=dropout),
                                        nn.Linear(self.last_channel, num_classes))
        self.dropout_p = dropout
        self.reset_parameters()

    def reset_parameters(self):
        # torchvision init: kaiming fan_out for convs, BN (1, 0), Linear N(0, 0.01)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out")
                if m.bias is not None:
                    nn.init.zeros_(m.bias)
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0, 0.01)
                nn.init.zeros_(m.bias)

    def replace_head(self, num_classes: int):
        """The reference's head swap: ``classifier[1] = nn.Linear(1280, num_classes)``."""
        lin = nn.Linear(self.last_channel, num_classes)
        self.classifier[1] = lin.to(self.classifier[1].weight.device)
        return self

    def forward(self, x):
        x = self.features(x)
        x = F.adaptive_avg_pool2d(x, (1, 1))
        x = torch.flatten(x, 1)
        return self.classifier(x)


def mobilenet_v2(num_classes: int = 10, pretrained: Optional[str] = None, **kw) -> MobileNetV2:
    """Build MobileNetV2.

    ``pretrained`` is a *path* to a torchvision-format state_dict (there is no
    network access to fetch ImageNet weights).  When a 1000-class checkpoint is
    given and ``num_classes != 1000`` the head is swapped after loading, exactly
    like the reference (load ImageNet weights, then replace ``classifier[1]``).
    """
    if pretrained:
        sd = torch.load(pretrained, map_location="cpu", weights_only=True)
        n_ckpt = sd["classifier.1.weight"].shape[0]
        model = MobileNetV2(num_classes=n_ckpt, **kw)
        model.load_state_dict(sd)
        if n_ckpt != num_classes:
            model.replace_head(num_classes)
        return model
    return MobileNetV2(num_classes=num_classes, **kw)
