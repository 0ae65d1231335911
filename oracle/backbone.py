"""torch-CPU restatement of the reference extractor (TEST INFRASTRUCTURE ONLY).

Follows, op for op:
  * normalize            ``cirtorch/utils/image.py:86-127`` ((x - mean_c) / std_c),
                         applied after padding (``random_augmentation.py:102,174``)
  * pad_packed_images    ``cirtorch/utils/sequence.py:4-67`` (top-left, zero fill)
  * ResNet body          ``cirtorch/backbones/resnet.py:60-66,151-164`` with mod4/mod5
                         restored and ``backbones/misc.py:163-203``
  * BN + activation      inplace_abn 1.1.0 ``ABN`` eval semantics = F.batch_norm with
                         running stats (eps 1e-5) then leaky_relu(0.01) / identity
                         (``utils/misc.py:175-235``, ``global_config.ini:26-28``)
  * globalHead           ``cirtorch/modules/heads/global_head.py:52-67``
                         GeM (``modules/pools.py:30-38``) -> L2N (``normalizations.py:9-16``)
                         -> Linear -> L2N -> permute to D x N
  * multi-scale          ``cirtorch/models/GF_net.py:20-40,74-92``: per-image bilinear
                         resize (align_corners=False), mean over scales, no re-norm.
"""

import numpy as np
import torch
import torch.nn.functional as F

from .weights import NETS, conv_specs, _bn_name

BN_EPS = 1e-5
SLOPE = 0.01


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


class OracleNet:
    """Stateless-ish CPU model: body + global head, fp32 (or fp64 for error studies)."""

    def __init__(self, arch, body_state, head_state, dtype=torch.float32):
        self.arch = arch
        self.bottleneck = NETS[arch][1]
        self.dtype = dtype
        self.sd = {k: _t(v).to(dtype) for k, v in body_state.items()}
        self.hd = {k: _t(v).to(dtype) for k, v in head_state.items()}
        self.specs = {s[0]: s for s in conv_specs(arch)}

    # -- primitives -------------------------------------------------------
    def _conv_bn(self, x, name, act):
        _, _cin, _cout, k, stride, _role = self.specs[name]
        y = F.conv2d(x, self.sd[name + ".weight"], None, stride=stride, padding=k // 2)
        bn = _bn_name(name)
        y = F.batch_norm(y, self.sd[bn + ".running_mean"], self.sd[bn + ".running_var"],
                         self.sd[bn + ".weight"], self.sd[bn + ".bias"], False, 0.0, BN_EPS)
        return F.leaky_relu(y, SLOPE) if act else y

    def _block(self, x, prefix):
        if prefix + ".proj_conv" in self.specs:
            residual = self._conv_bn(x, prefix + ".proj_conv", act=False)
        else:
            residual = x
        if self.bottleneck:
            y = self._conv_bn(x, prefix + ".convs.conv1", True)
            y = self._conv_bn(y, prefix + ".convs.conv2", True)
            y = self._conv_bn(y, prefix + ".convs.conv3", False)
        else:
            y = self._conv_bn(x, prefix + ".convs.conv1", True)
            y = self._conv_bn(y, prefix + ".convs.conv2", False)
        return F.leaky_relu(y + residual, SLOPE)

    # -- body ---------------------------------------------------------------
    def body(self, x):
        """x: N x 3 x H x W normalised -> OrderedDict mod1..mod5 (NCHW)."""
        outs = {}
        y = self._conv_bn(x, "mod1.conv1", True)
        y = F.max_pool2d(y, 3, stride=2, padding=1)
        outs["mod1"] = y
        structure = NETS[self.arch][0]
        for mod_id, num in enumerate(structure):
            for b in range(num):
                y = self._block(y, "mod%d.block%d" % (mod_id + 2, b + 1))
            outs["mod%d" % (mod_id + 2)] = y
        return outs

    # -- head ---------------------------------------------------------------
    def head(self, x, whiten=True):
        """x: N x C x h x w -> D x N (``global_head.py:52-67``)."""
        p = self.hd["pool.p"]
        y = F.avg_pool2d(x.clamp(min=1e-6).pow(p), (x.size(-2), x.size(-1))).pow(1.0 / p)
        y = l2n(y).squeeze(-1).squeeze(-1)
        if whiten:
            y = F.linear(y, self.hd["whiten.weight"], self.hd["whiten.bias"])
            y = l2n(y)
        return y.permute(1, 0)

    # -- full forward -----------------------------------------------------------
    def forward_padded(self, img, normalize=True):
        x = img.to(self.dtype)
        if normalize:
            x = normalize_images(x)
        return self.head(self.body(x)["mod5"])

    def forward(self, images, scales=(1,), normalize=True):
        """images: list of 3 x H_i x W_i float tensors in [0,1) (a PackedSequence).
        Returns D x N (``GF_net.py:63-126``)."""
        if len(scales) > 1:
            preds = []
            for s in scales:
                if s == 1:
                    imgs = images
                else:
                    imgs = [F.interpolate(im.unsqueeze(0), scale_factor=s, mode="bilinear",
                                          align_corners=False).squeeze(0) for im in images]
                preds.append(self.forward(imgs, scales=(1,), normalize=normalize).unsqueeze(0))
            pred = torch.cat(preds, 0).permute(1, 2, 0)
            return F.avg_pool1d(pred, kernel_size=len(scales)).squeeze(-1)
        padded, _ = pad_images(images)
        return self.forward_padded(padded, normalize=normalize)


def l2n(x, eps=1e-6):
    """``cirtorch/modules/normalizations.py:16``: x / (||x||_2 over dim 1 + eps)."""
    return x / (torch.norm(x, p=2, dim=1, keepdim=True) + eps).expand_as(x)


def normalize_images(x, mean=(0.485, 0.456, 0.406), std=(0.229, 0.224, 0.225)):
    """``cirtorch/utils/image.py:86-127``."""
    m = torch.tensor(mean, dtype=x.dtype)[:, None, None]
    s = torch.tensor(std, dtype=x.dtype)[:, None, None]
    return (x - m) / s


def pad_images(images, pad_value=0.0):
    """``cirtorch/utils/sequence.py:4-67`` (3-D case): top-left aligned zero pad."""
    h = max(im.shape[1] for im in images)
    w = max(im.shape[2] for im in images)
    out = images[0].new_full((len(images), images[0].shape[0], h, w), pad_value)
    sizes = []
    for i, im in enumerate(images):
        out[i, :, : im.shape[1], : im.shape[2]] = im
        sizes.append(tuple(im.shape[1:]))
    return out, sizes
