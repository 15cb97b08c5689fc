from .mobilenet_v2 import MobileNetV2, InvertedResidual, ConvBNAct, mobilenet_v2, MOBILENET_V2_SETTING
from .resnet import ResNet, resnet50

_REGISTRY = {"mobilenet_v2": mobilenet_v2, "resnet50": resnet50}


def build_model(name: str, num_classes: int = 10, pretrained=None):
    if name not in _REGISTRY:
        raise KeyError(f"unknown model {name!r}; available: {sorted(_REGISTRY)}")
    return _REGISTRY[name](num_classes=num_classes, pretrained=pretrained)


__all__ = ["MobileNetV2", "InvertedResidual", "ConvBNAct", "mobilenet_v2", "ResNet",
           "resnet50", "build_model", "MOBILENET_V2_SETTING"]
