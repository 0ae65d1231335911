"""ResidualBlock (reference ``cirtorch/backbones/misc.py:107-203``): same
submodule names (``convs.conv1/bn1/...``, ``proj_conv``, ``proj_bn``) so
reference / torchvision-converted state dicts load unchanged.  Its forward is
executed by the backbone's fused engine plan (see resnet.py)."""

from collections import OrderedDict

import torch.nn as nn

from ..modules.abn import ABN


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

    def forward(self, x):
        raise RuntimeError("ResidualBlock runs inside the fused backbone plan; call the ResNet module")
