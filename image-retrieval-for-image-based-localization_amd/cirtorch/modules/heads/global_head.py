"""globalHead (reference ``cirtorch/modules/heads/global_head.py:16-67``).

forward: pool -> L2N -> squeeze -> Linear whiten -> L2N -> permute(1, 0),
returning a D x N tensor (one column per image).  Pooling is one engine
launch reading the NHWC stage map once; L2N / Linear / L2N run as the fused
head tail (``rr_head_l2n_whiten_l2n``).
"""

import torch.nn as nn

from ... import _ops
from ...layers import functional as LF
from ...layers.normalization import L2N
from ...layers.pooling import GeM, MAC, SPoC
from ..abn import ABN
from ..normalizations import NORMALIZATION_LAYERS
from ..pools import POOLING_LAYERS


class globalHead(nn.Module):
    def __init__(self, pooling=None, normal=None, dim=None, norm_act=ABN):
        super().__init__()
        self.dim = dim
        self.whiten = nn.Linear(dim, dim, bias=True)
        if pooling["name"] == "GeMmp":
            self.pool = POOLING_LAYERS[pooling["name"]](**pooling["params"], mp=self.dim)
        else:
            self.pool = POOLING_LAYERS[pooling["name"]](**pooling["params"])
        self.norm = NORMALIZATION_LAYERS[normal["name"]](eps=1e-6)
        self.reset_parameters()

    def reset_parameters(self):
        for _name, mod in self.named_modules():
            if isinstance(mod, nn.Linear):
                nn.init.xavier_normal_(mod.weight, 0.1)
            elif isinstance(mod, ABN):
                nn.init.constant_(mod.weight, 1.0)
            if hasattr(mod, "bias") and isinstance(getattr(mod, "bias"), nn.Parameter) and mod.bias is not None:
                nn.init.constant_(mod.bias, 0.0)

    def pooled(self, x):
        """[N, C, h, w] -> [N, C] float32 (one launch)."""
        from ... import _engine as E
        if isinstance(self.pool, GeM):
            return _ops.global_pool(x, E.RR_POOL_GEM, LF._p_arg(self.pool.p), self.pool.eps)
        if isinstance(self.pool, MAC):
            return _ops.global_pool(x, E.RR_POOL_MAC)
        if isinstance(self.pool, SPoC):
            return _ops.global_pool(x, E.RR_POOL_SPOC)
        return self.pool(x).squeeze(-1).squeeze(-1)

    def forward(self, x, do_whitening=True):
        if not isinstance(self.norm, L2N):
            raise NotImplementedError("only L2N normalisation is supported")
        p = self.pooled(x)
        y = _ops.head_tail(p, self.whiten.weight, self.whiten.bias, whiten=do_whitening, eps=self.norm.eps)
        return y.permute(1, 0)
