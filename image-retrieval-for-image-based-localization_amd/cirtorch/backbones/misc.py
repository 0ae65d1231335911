"""ResidualBlock (reference ``cirtorch/backbones/misc.py:107-203``): same
submodule names (``convs.conv1/bn1/...``, ``proj_conv``, ``proj_bn``) so
reference / torchvision-converted state dicts load unchanged.

Inside a ResNet the blocks run as part of the backbone's fused engine plan
(resnet.py: fused boundary launches between blocks).  Called on its own, a
block runs its own plan — the same packed weights / folded BN steps, one
``rr_conv2d_fused`` launch per conv, the residual add and post-add activation
in the last conv's epilogue — in the precision of its ResNet (or
``engine_dtype``, default bf16)."""

from collections import OrderedDict

import torch
import torch.nn as nn

from .. import _ops
from ..modules.abn import ABN


class ConvStep:
    """one engine conv: packed weight [c_out][kh*kw*c_in] (PERM32 rows where c_out % 32 == 0),
    folded BN scale / shift, activation"""
    __slots__ = ("w", "kh", "kw", "stride", "pad", "c_out", "scale", "shift", "leaky", "slope", "perm")


def make_step(conv, bn, dtype, cin_pad=None, leaky_override=None):
    st = ConvStep()
    co, ci, kh, kw = conv.weight.shape
    cin_pad = cin_pad or ci
    # engine layout [c_out][(kh*KW + kw)*c_in + ci], 128-B K-steps, rows in the
    # 32-row MFMA-interleaved order so each lane stores 8 consecutive channels
    st.perm = co % 32 == 0
    st.w = _ops.pack_conv_weights(conv.weight, cin_pad, dtype, perm32=st.perm)
    st.kh, st.kw = kh, kw
    st.stride = conv.stride[0]
    st.pad = conv.padding[0]
    st.c_out = co
    st.scale, st.shift = bn.folded()
    st.leaky, st.slope = bn.slope()
    if leaky_override is not None:
        st.leaky = leaky_override
    return st


def run_step(t, st, residual=None, out=None):
    """NHWC t -> NHWC conv + BN (+ residual) + activation (into `out` when given)"""
    return _ops.conv2d_fused(t, st.w, st.kh, st.kw, st.stride, st.pad, st.c_out, st.scale, st.shift,
                             residual=residual, leaky=st.leaky, slope=st.slope, perm32=st.perm, out=out)


class ResidualBlock(nn.Module):
    def __init__(self, in_channels, channels, stride=1, dilation=1, groups=1, norm_act=ABN, dropout=None):
        super().__init__()
        if len(channels) != 2 and len(channels) != 3:
            raise ValueError("channels must contain either two or three values")
        if len(channels) == 2 and groups != 1:
            raise ValueError("groups > 1 are only valid if len(channels) == 3")
        if groups != 1 or dilation != 1:
            raise NotImplementedError("grouped / dilated residual blocks are out of scope")
        self.is_bottleneck = len(channels) == 3
        self.stride = stride
        need_proj_conv = stride != 1 or in_channels != channels[-1]
        if not self.is_bottleneck:
            bn2 = norm_act(channels[1])
            bn2.activation = "identity"
            layers = [
                ("conv1", nn.Conv2d(in_channels, channels[0], 3, stride=stride, padding=dilation, bias=False)),
                ("bn1", norm_act(channels[0])),
                ("conv2", nn.Conv2d(channels[0], channels[1], 3, stride=1, padding=dilation, bias=False)),
                ("bn2", bn2),
            ]
        else:
            bn3 = norm_act(channels[2])
            bn3.activation = "identity"
            layers = [
                ("conv1", nn.Conv2d(in_channels, channels[0], 1, stride=1, padding=0, bias=False)),
                ("bn1", norm_act(channels[0])),
                ("conv2", nn.Conv2d(channels[0], channels[1], 3, stride=stride, padding=dilation, bias=False)),
                ("bn2", norm_act(channels[1])),
                ("conv3", nn.Conv2d(channels[1], channels[2], 1, stride=1, padding=0, bias=False)),
                ("bn3", bn3),
            ]
        # dropout is a training-time op; eval extraction ignores it (reference inserts it at misc.py:176).
        self.convs = nn.Sequential(OrderedDict(layers))
        if need_proj_conv:
            self.proj_conv = nn.Conv2d(in_channels, channels[-1], 1, stride=stride, padding=0, bias=False)
            self.proj_bn = norm_act(channels[-1])
            self.proj_bn.activation = "identity"

    engine_dtype = torch.bfloat16  # set by the owning ResNet (its precision)
    _plan = None

    def engine_plan(self, dtype):
        """(steps, proj) of this block: conv1.. with their BN, the last one carrying the
        post-add activation of bn1 (``misc.py:194-203``); proj with identity activation"""
        c = self.convs
        post_leaky, post_slope = c.bn1.slope()
        if self.is_bottleneck:
            steps = [make_step(c.conv1, c.bn1, dtype), make_step(c.conv2, c.bn2, dtype),
                     make_step(c.conv3, c.bn3, dtype)]
        else:
            steps = [make_step(c.conv1, c.bn1, dtype), make_step(c.conv2, c.bn2, dtype)]
        steps[-1].leaky, steps[-1].slope = post_leaky, post_slope
        proj = make_step(self.proj_conv, self.proj_bn, dtype, leaky_override=False) \
            if hasattr(self, "proj_conv") else None
        return steps, proj

    def _apply(self, fn, *args, **kwargs):
        self._plan = None
        return super()._apply(fn, *args, **kwargs)

    def _load_from_state_dict(self, *args, **kwargs):
        self._plan = None
        return super()._load_from_state_dict(*args, **kwargs)

    def forward(self, x):
        """x: [N, C, H, W] on the GPU -> act(convs(x) + residual), [N, C', H', W'] in x's
        dtype (an NCHW-shaped channels_last view when that is the engine dtype)."""
        dtype = self.engine_dtype
        if self._plan is None or self._plan[0] != dtype:
            self._plan = (dtype, self.engine_plan(dtype))
        steps, proj = self._plan[1]
        t = x.permute(0, 2, 3, 1).to(dtype).contiguous()
        res = t if proj is None else run_step(t, proj)
        y = t
        for st in steps[:-1]:
            y = run_step(y, st)
        out = run_step(y, steps[-1], residual=res).permute(0, 3, 1, 2)
        return out if x.dtype == dtype else out.to(x.dtype)
