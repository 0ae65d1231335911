"""Normalisation modules (reference ``cirtorch/modules/normalizations.py:9-16``)."""

import torch.nn as nn

from . import functional as LF


class L2N(nn.Module):
    def __init__(self, eps=1e-6):
        super().__init__()
        self.eps = eps

    def forward(self, x):
        return LF.l2n(x, eps=self.eps)

    def __repr__(self):
        return "%s(eps=%s)" % (self.__class__.__name__, self.eps)
