"""Functional pooling / normalisation on the GPU engine.

mac / spoc / gem  — cirtorch/modules/pools.py:10-38
l2n               — cirtorch/modules/normalizations.py:9-16
All take NCHW-shaped tensors (NCHW-contiguous or channels_last views, float32
or bfloat16) and return float32 [N, C, 1, 1] like the reference modules.
"""

import torch

from .. import _engine as E
from .. import _ops


def _p_arg(p):
    """GeM exponent for the kernel: a learnable ``pool.p`` Parameter stays in
    device memory and is read by the kernel itself (rr_global_pool_pdev), so
    no forward reads it back to the host (no stream drain, graph-capturable)
    and every update of it — load_state_dict, an optimizer step or an in-place
    ``p.data.fill_`` — is seen by the next launch."""
    if torch.is_tensor(p):
        if p.numel() != 1:
            raise NotImplementedError("per-channel GeM exponents (GeMmp) are out of scope")
        return p
    return float(p)


def mac(x):
    return _ops.global_pool(x, E.RR_POOL_MAC).unsqueeze(-1).unsqueeze(-1)


def spoc(x):
    return _ops.global_pool(x, E.RR_POOL_SPOC).unsqueeze(-1).unsqueeze(-1)


def gem(x, p=3.0, eps=1e-6):
    return _ops.global_pool(x, E.RR_POOL_GEM, _p_arg(p), eps).unsqueeze(-1).unsqueeze(-1)


def l2n(x, eps=1e-6):
    """x / (||x||_2 over dim 1 + eps) for x of shape [N, C] or [N, C, 1, 1]."""
    shape = x.shape
    if x.dim() > 2 and x[0, 0].numel() != 1:
        raise NotImplementedError("L2N over dim 1 of spatial maps: only [N, C(,1,1)] descriptors are supported")
    y = _ops.l2n_rows(x.reshape(shape[0], shape[1]), eps)
    return y.reshape(shape)
