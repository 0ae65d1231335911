"""ResNet body on the MI355X engine.

Module tree, parameter names, registry and ``convert`` follow the reference
``cirtorch/backbones/resnet.py:15-180`` so its state dicts (and torchvision
ones via ``convert``) load unchanged.  ``forward`` follows the *intended*
reference semantics — all five stages (the checked-in reference comments out
mod4/mod5 at ``resnet.py:158-159`` while ``GF_algo._get_level`` needs mod5).

Execution: on first use (and after ``load_state_dict`` / ``.to()`` /
``set_precision``) the module builds an engine plan — per conv a packed
[c_out][kh*kw*c_in] weight in the compute dtype plus the folded BN
scale/shift — and runs the whole body as a chain of librr.so launches:

    image_to_nhwc (normalise + layout) -> stem conv 7x7/2 (+BN+leaky)
    -> maxpool 3x3/2 -> per block: [proj 1x1 (+BN)] , conv1 (+BN+leaky),
       conv2 (+BN+leaky), conv3 (+BN + residual + leaky)

Activations stay NHWC in HBM; the returned stage maps are NCHW-shaped
``channels_last`` views of those buffers (no copies).
"""

import os
import sys
from collections import OrderedDict
from functools import partial

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _ops
from ..modules.abn import ABN
from .misc import ResidualBlock, make_step, run_step

CONV_PARAMS = ["weight"]
BN_PARAMS = ["weight", "bias", "running_mean", "running_var"]

_PRECISIONS = {"bf16": torch.bfloat16, "fp32": torch.float32, "float32": torch.float32, "bfloat16": torch.bfloat16,
               "fp16": torch.float16, "float16": torch.float16}


def try_index(scalar_or_list, i):
    try:
        return scalar_or_list[i]
    except TypeError:
        return scalar_or_list


class ResNet(nn.Module):
    """Standard residual network (reference ``resnet.py:15-164``).

    Extra (engine) argument: ``precision`` in {"bf16", "fp16", "fp32"} — the
    MFMA operand / activation storage type (accumulation is always float32).
    bf16 and fp16 run the fused kernels (stem, direct
    3x3, streaming 1x1, boundary pairs); fp32 is the exact-f32 MFMA parity
    mode."""

    def __init__(self, structure, bottleneck, norm_act=ABN, config=None, classes=0, dilation=1, dropout=None,
                 caffe_mode=False, precision="bf16"):
        super().__init__()
        self.structure = structure
        self.bottleneck = bottleneck
        self.dilation = dilation
        self.dropout = dropout
        self.caffe_mode = caffe_mode
        if len(structure) != 4:
            raise ValueError("Expected a structure with four values")
        if dilation != 1 and len(dilation) != 4:
            raise ValueError("If dilation is not 1 it must contain four values")
        if dilation != 1:
            raise NotImplementedError("dilated ResNets are out of scope for the MI355X engine")
        if caffe_mode:
            raise NotImplementedError("caffe_mode (stem conv bias) is out of scope")
        if classes != 0:
            raise NotImplementedError("the classifier head is out of scope (retrieval uses classes=0)")

        layers = [
            ("conv1", nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)),
            ("bn1", try_index(norm_act, 0)(64)),
            ("pool1", nn.MaxPool2d(3, stride=2, padding=1)),
        ]
        self.mod1 = nn.Sequential(OrderedDict(layers))
        in_channels = 64
        channels = (64, 64, 256) if self.bottleneck else (64, 64)
        for mod_id, num in enumerate(structure):
            blocks = []
            for block_id in range(num):
                stride = 2 if block_id == 0 and mod_id > 0 else 1
                blocks.append(("block%d" % (block_id + 1),
                               ResidualBlock(in_channels, channels, norm_act=try_index(norm_act, mod_id),
                                             stride=stride, dilation=1)))
                in_channels = channels[-1]
            self.add_module("mod%d" % (mod_id + 2), nn.Sequential(OrderedDict(blocks)))
            channels = [c * 2 for c in channels]
        self.out_channels = in_channels
        self.set_precision(precision)

    # ------------------------------------------------------------ reference API
    @staticmethod
    def _stride_dilation(dilation, mod_id, block_id):
        d = try_index(dilation, mod_id)
        s = 2 if d == 1 and block_id == 0 and mod_id > 0 else 1
        return s, d

    def copy_layer(self, inm, outm, name_in, name_out, params):
        for param_name in params:
            outm[name_out + "." + param_name] = inm[name_in + "." + param_name]

    def convert(self, model):
        """torchvision resnet state dict -> this module's keys (``resnet.py:116-149``)."""
        out = dict()
        num_convs = 3 if self.bottleneck else 2
        self.copy_layer(model, out, "conv1", "mod1.conv1", CONV_PARAMS)
        self.copy_layer(model, out, "bn1", "mod1.bn1", BN_PARAMS)
        for mod_id, num in enumerate(self.structure):
            for block_id in range(num):
                for conv_id in range(num_convs):
                    self.copy_layer(model, out, "layer{}.{}.conv{}".format(mod_id + 1, block_id, conv_id + 1),
                                    "mod{}.block{}.convs.conv{}".format(mod_id + 2, block_id + 1, conv_id + 1),
                                    CONV_PARAMS)
                    self.copy_layer(model, out, "layer{}.{}.bn{}".format(mod_id + 1, block_id, conv_id + 1),
                                    "mod{}.block{}.convs.bn{}".format(mod_id + 2, block_id + 1, conv_id + 1),
                                    BN_PARAMS)
                try:
                    self.copy_layer(model, out, "layer{}.{}.downsample.0".format(mod_id + 1, block_id),
                                    "mod{}.block{}.proj_conv".format(mod_id + 2, block_id + 1), CONV_PARAMS)
                    self.copy_layer(model, out, "layer{}.{}.downsample.1".format(mod_id + 1, block_id),
                                    "mod{}.block{}.proj_bn".format(mod_id + 2, block_id + 1), BN_PARAMS)
                except KeyError:
                    pass
        return out

    # ------------------------------------------------------------ engine plan
    def set_precision(self, precision):
        self.engine_dtype = _PRECISIONS[precision]
        for m in self.modules():
            if isinstance(m, ResidualBlock):
                m.engine_dtype = self.engine_dtype  # standalone block calls run in the body's precision
        self._plan = None
        return self

    def refresh_engine(self):
        """Rebuild packed weights (call after modifying parameters in place)."""
        self._plan = None

    def _apply(self, fn, *args, **kwargs):
        self._plan = None
        return super()._apply(fn, *args, **kwargs)

    def _load_from_state_dict(self, *args, **kwargs):
        self._plan = None
        return super()._load_from_state_dict(*args, **kwargs)

    def stem_cin(self):
        return 4 if self.engine_dtype == torch.float32 else 8

    def _step(self, conv, bn, cin_pad=None, leaky_override=None):
        return make_step(conv, bn, self.engine_dtype, cin_pad=cin_pad, leaky_override=leaky_override)

    def _build_plan(self):
        dev = self.mod1.conv1.weight.device
        if dev.type != "cuda":
            raise RuntimeError("the MI355X engine runs on the GPU: call .cuda() on the model first")
        plan = {"stem": self._step(self.mod1.conv1, self.mod1.bn1, cin_pad=self.stem_cin()), "mods": []}
        # bf16 / fp16: conv1 + bn1 + pool1 run as ONE fused kernel (rr_stem_conv_pool)
        plan["stem_fused"] = None
        if self.engine_dtype in (torch.bfloat16, torch.float16) and tuple(self.mod1.conv1.weight.shape) == (64, 3, 7, 7) \
                and hasattr(self.mod1, "pool1") and os.environ.get("RR_STEM_FUSED", "1") != "0":
            plan["stem_fused"] = _ops.pack_stem_weights(self.mod1.conv1.weight, self.engine_dtype)
        for mod_id in range(4):
            mod = getattr(self, "mod%d" % (mod_id + 2))
            blocks = []
            for blk in mod.children():
                blocks.append(blk.engine_plan(self.engine_dtype))
            plan["mods"].append(blocks)
        self._plan = plan
        return plan

    @staticmethod
    def _conv(t, st, residual=None, out=None):
        return run_step(t, st, residual, out)

    def _stem(self, plan, x, mean, std):
        if isinstance(x, (list, tuple)):
            # ragged batch (a PackedSequence of different sizes): the stem reads every
            # image at its own address; the batch map is the max extent, padded with
            # zeros before normalisation (utils/sequence.py:51, random_augmentation.py:102,174)
            live = [t for t in x if t is not None]
            if not live:
                raise ValueError("at least one image of the batch must be non-None")
            h = max(int(t.shape[-2]) for t in live)
            w = max(int(t.shape[-1]) for t in live)
            st = plan["stem"]
            if plan["stem_fused"] is not None:
                return _ops.stem_conv_pool_ragged(x, h, w, plan["stem_fused"], st.scale, st.shift, leaky=st.leaky,
                                                  slope=st.slope, mean=mean, std=std)
            t = _ops.image_to_nhwc_ragged(x, h, w, self.stem_cin(), self.engine_dtype, mean, std)
            return _ops.maxpool2d(self._conv(t, st), 3, 2, 1)
        if x.dtype == torch.uint8 and plan["stem_fused"] is None:
            x = _ops.pixels_to_unit(x)  # pixels -> [0, 1] (to_tensor); the fused stem reads uint8 itself
        if plan["stem_fused"] is not None:
            st = plan["stem"]
            return _ops.stem_conv_pool(x, plan["stem_fused"], st.scale, st.shift, leaky=st.leaky, slope=st.slope,
                                       mean=mean, std=std)
        t = _ops.image_to_nhwc(x, self.stem_cin(), self.engine_dtype, mean, std)
        t = self._conv(t, plan["stem"])
        return _ops.maxpool2d(t, 3, 2, 1)

    def _blocks(self, t, flat, i0, i1, outs, pending=None):
        """blocks flat[i0:i1] on the NHWC map t (the conv1 output of block i0 may come
        precomputed as `pending`); stage maps into outs (when not None)."""
        for i in range(i0, i1):
            mod_id, steps, proj = flat[i]
            nxt = flat[i + 1][1][0] if i + 1 < i1 else None
            pair = self._pairable(steps[-1], nxt)
            fuse_proj = pair and proj is not None and self._proj_fusable(proj)
            res = t if proj is None else (None if fuse_proj else self._conv(t, proj))
            # the whole block (3x3 + boundary pair) in one launch: the 3x3 is not run on its own
            block = pair and self._c3pairable(t, steps, nxt, fuse_proj)
            # the stage's first block: its conv1 (64 -> 64 on the block input) in the same launch
            conv1 = block and fuse_proj and pending is None and self._conv1_fusable(t, steps[0])
            y = t
            for j, st in enumerate(steps[:-2] if block else steps[:-1]):
                if conv1:
                    break
                y = pending if (j == 0 and pending is not None) else self._conv(y, st)
            pending = None
            if block:
                mid, last = steps[-2], steps[-1]
                c1 = steps[0]
                t, pending = _ops.conv3x3_pair(y, mid.w, mid.scale, mid.shift, mid.leaky, mid.slope,
                                               last.w, last.scale, last.shift, res, last.leaky, last.slope,
                                               nxt.w, nxt.scale, nxt.shift, nxt.c_out, nxt.leaky, nxt.slope,
                                               proj=(t, proj.w, proj.scale, proj.shift) if fuse_proj else None,
                                               conv1=(c1.w, c1.scale, c1.shift, c1.leaky, c1.slope) if conv1 else None)
            elif pair:
                last = steps[-1]
                t, pending = _ops.conv1x1_pair(y, last.w, last.scale, last.shift, res, last.leaky, last.slope,
                                               nxt.w, nxt.scale, nxt.shift, nxt.c_out, nxt.leaky, nxt.slope,
                                               proj=(t, proj.w, proj.scale, proj.shift) if fuse_proj else None)
            else:
                t = self._conv(y, steps[-1], residual=res)
            if outs is not None and (i + 1 == len(flat) or flat[i + 1][0] != mod_id):
                outs["mod%d" % (mod_id + 2)] = t
        return t, pending

    def forward(self, x, normalize=None):
        """x: [N, 3, H, W] float32 on the GPU, or uint8 pixels (read as x / 255), or a ragged batch -- a list
        (PackedSequence) of [3, H_i, W_i] images, None allowed, run as the zero-padded max-extent batch
        without building it -- (already normalised unless
        ``normalize=(mean, std)`` is given, which fuses cirtorch/utils/image.py
        ``normalize`` into the first kernel).  Returns OrderedDict mod1..mod5."""
        plan = self._plan or self._build_plan()
        mean, std = normalize if normalize is not None else (None, None)
        outs = OrderedDict()
        flat = [(mod_id, steps, proj) for mod_id, blocks in enumerate(plan["mods"]) for steps, proj in blocks]
        t = self._stem(plan, x, mean, std)
        outs["mod1"] = t
        self._blocks(t, flat, 0, len(flat), outs)
        return OrderedDict((k, v.permute(0, 3, 1, 2)) for k, v in outs.items())

    @staticmethod
    def _proj_fusable(proj):
        """stride-1 1x1 projection 64 -> 256 (first block of the 256-channel stage), identity activation"""
        return (proj.kh == 1 and proj.stride == 1 and proj.pad == 0 and proj.perm and proj.c_out == 256
                and proj.w.shape[1] == 64 and not proj.leaky)

    @staticmethod
    def _c3pairable(t, steps, nxt, fuse_proj):
        """a 256-channel-stage bottleneck (1x1 -> 3x3 64 -> 64 -> 1x1 64 -> 256) whose boundary pairs
        with the next block's conv1: rr_conv3x3_pair runs the 3x3 and the pair as one launch
        (t2 never reaches HBM).  Needs H % 4 == 0 and W % 32 == 0; RR_C3PAIR=0 keeps two launches."""
        if len(steps) != 3 or os.environ.get("RR_C3PAIR", "1") == "0":
            return False
        mid, last = steps[1], steps[2]
        n, h, w, c = t.shape
        return (mid.kh == 3 and mid.kw == 3 and mid.stride == 1 and mid.pad == 1 and mid.perm and mid.c_out == 64
                and tuple(mid.w.shape) == (64, 576) and last.c_out == 256 and last.w.shape[1] == 64
                and nxt.c_out in ((64,) if fuse_proj else (64, 128)) and h % 4 == 0 and w % 32 == 0
                and n * h * w * 64 * 2 < 2 ** 31)

    @staticmethod
    def _conv1_fusable(t, st):
        """the block's conv1 is a 1x1 / stride-1 64 -> 64 PERM32 conv of its 64-channel input.
        Opt-in (RR_C3PAIR_CONV1=1): measured -2 % for that block isolated but neutral in the
        bench step (the extra barrier per tile slows the block by about what conv1's own
        launch cost; profiles/r05_ab/r05cv_*), so conv1 stays its own launch by default."""
        return (os.environ.get("RR_C3PAIR_CONV1", "0") == "1" and st.kh == 1 and st.kw == 1 and st.stride == 1
                and st.pad == 0 and st.perm and st.c_out == 64 and tuple(st.w.shape) == (64, 64) and t.shape[-1] == 64)

    def _pairable(self, last, nxt):
        """conv3 of a bottleneck followed by a stride-1 1x1 conv1 of the next block: one fused
        rr_conv1x1_pair launch (bf16 / fp16) for the 64 -> 256 -> 64/128 boundaries (mod2) and
        the 128 -> 512 -> 128 ones (mod3; RR_PAIR_MID=0 keeps those as two launches)."""
        if nxt is None or self.engine_dtype == torch.float32 or os.environ.get("RR_PAIR_FUSED", "1") == "0":
            return False
        if not (last.kh == 1 and last.stride == 1 and last.perm and nxt.kh == 1 and nxt.stride == 1
                and nxt.pad == 0 and nxt.perm):
            return False
        if last.c_out == 256 and last.w.shape[1] == 64:
            return nxt.w.shape[1] == 256 and nxt.c_out in (64, 128)
        if last.c_out == 512 and last.w.shape[1] == 128 and os.environ.get("RR_PAIR_MID", "1") != "0":
            return nxt.w.shape[1] == 512 and nxt.c_out == 128
        return False


_NETS = {
    "18": {"structure": [2, 2, 2, 2], "bottleneck": False},
    "34": {"structure": [3, 4, 6, 3], "bottleneck": False},
    "50": {"structure": [3, 4, 6, 3], "bottleneck": True},
    "101": {"structure": [3, 4, 23, 3], "bottleneck": True},
    "152": {"structure": [3, 8, 36, 3], "bottleneck": True},
}

__all__ = []
for _name, _params in _NETS.items():
    _net_name = "resnet" + _name
    setattr(sys.modules[__name__], _net_name, partial(ResNet, **_params))
    __all__.append(_net_name)
