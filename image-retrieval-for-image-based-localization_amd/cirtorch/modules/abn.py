"""Activated batch-norm parameter holder (the reference imports ``ABN`` /
``InPlaceABN`` / ``InPlaceABNSync`` from the third-party ``inplace_abn==1.1.0``,
``cirtorch/backbones/resnet.py:6``, ``utils/misc.py:10``).

On this engine BN + activation never run as a separate pass: the backbone
folds (weight, bias, running_mean, running_var, eps) into a per-channel
scale/shift applied in the convolution epilogue, followed by the activation
named here (``leaky_relu`` with ``activation_param`` slope, ``relu`` or
``identity``).  Eval-mode semantics only; Sync-BN statistics are training
machinery and out of scope.
"""

import torch
import torch.nn as nn

SUPPORTED_ACTIVATIONS = ("leaky_relu", "relu", "identity")


class ABN(nn.Module):
    def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True, activation="leaky_relu",
                 activation_param=0.01, **_ignored):
        super().__init__()
        self.num_features = num_features
        self.eps = eps
        self.momentum = momentum
        self.affine = affine
        self.activation = activation
        self.activation_param = activation_param
        if affine:
            self.weight = nn.Parameter(torch.ones(num_features))
            self.bias = nn.Parameter(torch.zeros(num_features))
        else:
            self.register_parameter("weight", None)
            self.register_parameter("bias", None)
        self.register_buffer("running_mean", torch.zeros(num_features))
        self.register_buffer("running_var", torch.ones(num_features))

    def folded(self):
        """(scale, shift) float32 with y = x * scale + shift == eval batch_norm."""
        var = self.running_var.detach().double()
        inv = torch.rsqrt(var + self.eps)
        w = self.weight.detach().double() if self.affine else torch.ones_like(var)
        b = self.bias.detach().double() if self.affine else torch.zeros_like(var)
        scale = w * inv
        shift = b - self.running_mean.detach().double() * scale
        return scale.float().contiguous(), shift.float().contiguous()

    def slope(self):
        if self.activation == "leaky_relu":
            return True, float(self.activation_param)
        if self.activation == "relu":
            return True, 0.0
        if self.activation == "identity":
            return False, 0.0
        raise NotImplementedError("activation %r is not supported by the MI355X engine" % self.activation)

    def forward(self, x):
        raise RuntimeError("ABN runs fused inside the backbone convolution epilogue; "
                           "it has no standalone forward on the MI355X engine")

    def extra_repr(self):
        return "%d, eps=%s, affine=%s, activation=%s[%s]" % (self.num_features, self.eps, self.affine,
                                                          self.activation, self.activation_param)


InPlaceABN = ABN
InPlaceABNSync = ABN
# reference cirtorch/utils/misc.py:48-86: "drop-in replacement for ABN which performs
# inference-mode BN + activation" -- exactly the folded epilogue above
ActivatedAffine = ABN
