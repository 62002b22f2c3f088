"""Model zoo: every network of the reference stacks plus the BASELINE.json extensions.

``build_model(name)`` accepts the reference's ``--network`` names (LeNet, ResNet18/34/50/101/152 —
pytorch_code/distributed_nn.py:58-63, sync_replicas_master_nn.py:104-109) and the new ones.
"""
from __future__ import annotations

from .lenet import LeNet
from .mlp import MLP, TFConvNet, mlp2, mlp_cpp, mlp_s2, mlp_tf
from .resnet import (BasicBlock, Bottleneck, ResNet, ResNet18, ResNet34, ResNet50, ResNet101, ResNet152,
                     ResNetImageNet, resnet18_imagenet, resnet34_imagenet, resnet50_imagenet,
                     resnet101_imagenet, resnet152_imagenet)

_REGISTRY = {
    "lenet": lambda nc: LeNet(nc),
    "resnet18_cifar": ResNet18, "resnet34_cifar": ResNet34, "resnet50_cifar": ResNet50,
    "resnet101_cifar": ResNet101, "resnet152_cifar": ResNet152,
    "resnet18": resnet18_imagenet, "resnet34": resnet34_imagenet, "resnet50": resnet50_imagenet,
    "resnet101": resnet101_imagenet, "resnet152": resnet152_imagenet,
    "mlp2": mlp2, "mlp": mlp2, "mlp_cpp": mlp_cpp, "mlp_s2": mlp_s2, "mlp_tf": mlp_tf,
    "tfconvnet": lambda nc: TFConvNet(nc),
}

# reference --network spellings (CIFAR-stem ResNets, as in pytorch_code/model_ops/resnet.py)
_ALIASES = {"LeNet": "lenet", "ResNet18": "resnet18_cifar", "ResNet34": "resnet34_cifar",
            "ResNet50": "resnet50_cifar", "ResNet101": "resnet101_cifar", "ResNet152": "resnet152_cifar",
            "MLP": "mlp2", "ResNet50-ImageNet": "resnet50", "GPT2-small": "gpt2_small"}


def build_model(name: str, num_classes: int | None = None, **kw):
    key = _ALIASES.get(name, name).lower()
    if key.startswith("gpt2"):
        from .gpt2 import build_gpt2
        return build_gpt2(key, **kw)
    if key not in _REGISTRY:
        raise ValueError(f"unknown model {name!r}; known: {sorted(_REGISTRY) + ['gpt2_small']}")
    if num_classes is None:
        num_classes = 1000 if key in ("resnet18", "resnet34", "resnet50", "resnet101", "resnet152") else 10
    return _REGISTRY[key](num_classes)


def model_names():
    return sorted(_REGISTRY) + ["gpt2_small", "gpt2_medium"]
