"""Upstream operator-surface names (the reference keeps an empty
``cirtorch/layers`` package; ``cirtorch/modules/utils.py:1`` still imports
``cirtorch.layers.pooling``)."""
from . import functional, normalization, pooling  # noqa: F401
