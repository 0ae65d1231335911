"""Deterministic random weights in the reference's state-dict layout
(TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

No pretrained checkpoint is reachable offline, so every parity
case uses weights drawn here.  Each tensor gets its own PCG64 stream keyed by
(base seed, crc32(key)), so a tensor's values never depend on which other
tensors exist — the product side regenerates exactly these arrays from this
module's twin in the tests.

Key layout follows the reference:
  backbone  ``cirtorch/backbones/resnet.py:60-66`` (mod1.conv1 / mod1.bn1),
            ``resnet.py:74-100`` + ``backbones/misc.py:163-182``
            (modK.blockB.convs.conv{1,2,3}, convs.bn{1,2,3}, proj_conv, proj_bn)
  head      ``cirtorch/modules/heads/global_head.py:26-34`` (pool.p, whiten.weight, whiten.bias)

Conditioning (SURVEY §7 hard part (v)): He-normal conv weights, BN running
statistics near (0, 1), gamma in [0.5, 1.0] on activated BNs and a small gamma
in [0.15, 0.3] on the identity BNs that feed the residual sum (bn3 / bn2 of a
basic block / proj_bn), so activations stay O(1) through 150 layers and GeM's
clamp(1e-6) does not dominate.  gamma > 0 everywhere (keeps the
inplace_abn |gamma| convention irrelevant).
"""

import zlib

import numpy as np

from .data import SEED_WEIGHTS

NETS = {
    "resnet18": ([2, 2, 2, 2], False),
    "resnet34": ([3, 4, 6, 3], False),
    "resnet50": ([3, 4, 6, 3], True),
    "resnet101": ([3, 4, 23, 3], True),
    "resnet152": ([3, 8, 36, 3], True),
}  # reference ``cirtorch/backbones/resnet.py:167-173``

OUTPUT_DIM = {"resnet18": 512, "resnet34": 512, "resnet50": 2048, "resnet101": 2048, "resnet152": 2048}


def conv_specs(arch):
    """Yield (prefix, cin, cout, k, stride, role) for every conv of the body, in
    forward order.  role in {"stem", "conv1", "conv2", "conv3", "proj"}.
    Stride placement: first block of mod3..mod5 strides on its 3x3 conv
    (``resnet.py:102-106``, ``misc.py:169``) and on the projection (``misc.py:180``)."""
    structure, bottleneck = NETS[arch]
    yield ("mod1.conv1", 3, 64, 7, 2, "stem")
    cin = 64
    chans = (64, 64, 256) if bottleneck else (64, 64)
    for mod_id, num in enumerate(structure):
        for b in range(num):
            stride = 2 if (b == 0 and mod_id > 0) else 1
            p = "mod%d.block%d" % (mod_id + 2, b + 1)
            if bottleneck:
                yield (p + ".convs.conv1", cin, chans[0], 1, 1, "conv1")
                yield (p + ".convs.conv2", chans[0], chans[1], 3, stride, "conv2")
                yield (p + ".convs.conv3", chans[1], chans[2], 1, 1, "conv3")
            else:
                yield (p + ".convs.conv1", cin, chans[0], 3, stride, "conv1")
                yield (p + ".convs.conv2", chans[0], chans[1], 3, 1, "conv2")
            if stride != 1 or cin != chans[-1]:
                yield (p + ".proj_conv", cin, chans[-1], 1, stride, "proj")
            cin = chans[-1]
        chans = tuple(c * 2 for c in chans)


def _bn_name(conv_name):
    if conv_name.endswith("proj_conv"):
        return conv_name[: -len("proj_conv")] + "proj_bn"
    head, _, last = conv_name.rpartition(".")
    return head + "." + last.replace("conv", "bn")


def _stream(seed, key):
    return np.random.Generator(np.random.PCG64([seed & 0xFFFFFFFF, zlib.crc32(key.encode())]))


def backbone_state(arch, seed=SEED_WEIGHTS):
    """Ordered dict name -> float32 ndarray with the reference backbone keys."""
    _, bottleneck = NETS[arch]
    out = {}
    for name, cin, cout, k, _stride, role in conv_specs(arch):
        fan_in = cin * k * k
        w = _stream(seed, name + ".weight").standard_normal((cout, cin, k, k), dtype=np.float32)
        out[name + ".weight"] = (w * np.float32(np.sqrt(2.0 / fan_in))).astype(np.float32)
        bn = _bn_name(name)
        branch_end = (role == "conv3") or (role == "conv2" and not bottleneck)
        g = _stream(seed, bn + ".weight")
        lo, hi = (0.2, 0.4) if branch_end else (0.8, 1.2)
        out[bn + ".weight"] = g.uniform(lo, hi, cout).astype(np.float32)
        out[bn + ".bias"] = _stream(seed, bn + ".bias").uniform(-0.02, 0.02, cout).astype(np.float32)
        out[bn + ".running_mean"] = _stream(seed, bn + ".running_mean").uniform(-0.02, 0.02, cout).astype(np.float32)
        out[bn + ".running_var"] = _stream(seed, bn + ".running_var").uniform(0.8, 1.2, cout).astype(np.float32)
    return out


def head_state(dim, p=3.0, seed=SEED_WEIGHTS):
    """globalHead params (``global_head.py:26-50``): whiten ~ xavier_normal(gain 0.1)
    like ``reset_parameters``, plus a small non-zero bias so the bias path is exercised."""
    std = 0.1 * np.sqrt(2.0 / (dim + dim))
    w = _stream(seed, "whiten.weight").standard_normal((dim, dim), dtype=np.float32) * np.float32(std)
    b = _stream(seed, "whiten.bias").uniform(-0.002, 0.002, dim).astype(np.float32)
    return {"pool.p": np.array([p], dtype=np.float32), "whiten.weight": w.astype(np.float32), "whiten.bias": b}
