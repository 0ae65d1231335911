"""Backbone registry: ``cirtorch.backbones.__dict__["resnet50"](norm_act=..., config=..., classes=0)``
(reference ``cirtorch/backbones/__init__.py`` / ``scripts/train_globalF.py:257-259``).
Only the ResNet family is on the hot path; VGG / DenseNet / ResNeXt / WiderResNet
are out of scope."""
from .resnet import *  # noqa: F401,F403
from .resnet import ResNet  # noqa: F401
