"""Pooling modules (reference ``cirtorch/modules/pools.py:10-38``)."""

import torch
import torch.nn as nn
from torch.nn.parameter import Parameter

from . import functional as LF


class MAC(nn.Module):
    def forward(self, x):
        return LF.mac(x)

    def __repr__(self):
        return self.__class__.__name__ + "()"


class SPoC(nn.Module):
    def forward(self, x):
        return LF.spoc(x)

    def __repr__(self):
        return self.__class__.__name__ + "()"


class GeM(nn.Module):
    """Generalized-mean pooling with a learnable scalar p (state key ``p``,
    ``pools.py:34``): (mean_hw clamp(x, eps)^p)^(1/p)."""

    def __init__(self, p=3, eps=1e-6):
        super().__init__()
        self.p = Parameter(torch.ones(1) * p)
        self.eps = eps

    def forward(self, x):
        return LF.gem(x, p=self.p, eps=self.eps)

    def __repr__(self):
        return "%s(p=%.4f, eps=%s)" % (self.__class__.__name__, float(self.p.data[0]), self.eps)
