"""Deterministic synthetic parameters and images for checking a deployment
against the committed reference fixtures (``tests/golden/*.npz``) without a
checkpoint or a dataset (none is reachable offline).

The fixtures were produced by running the reference modules on parameters
and images drawn with exactly these recipes (numpy PCG64 streams; see
``tests/golden/make_golden.py``), so ``bench.py`` can report the descriptor
cosine of each engine precision against the reference output for the same
inputs.  Nothing here computes a result: it only draws inputs.

  backbone_state(arch)   reference state-dict keys (``backbones/resnet.py:60-100``,
                         ``backbones/misc.py:163-182``): He-normal convs, BN
                         statistics near (0, 1), small gamma on the residual
                         branch ends so activations stay O(1) over 150 layers
  head_state(dim)        globalHead keys (``global_head.py:26-50``)
  structured_images(n, h, w, seed)
                         a random 6 x 8 colour field, bilinearly upsampled,
                         plus pixel noise: images differ in their large-scale
                         statistics, so descriptors are far apart
"""

import zlib

import numpy as np

SEED_WEIGHTS = 0x1A2B0004
_NETS = {"resnet18": ([2, 2, 2, 2], False), "resnet34": ([3, 4, 6, 3], False), "resnet50": ([3, 4, 6, 3], True),
         "resnet101": ([3, 4, 23, 3], True), "resnet152": ([3, 8, 36, 3], True)}


def _stream(seed, key):
    return np.random.Generator(np.random.PCG64([seed & 0xFFFFFFFF, zlib.crc32(key.encode())]))


def _convs(arch):
    structure, bottleneck = _NETS[arch]
    yield "mod1.conv1", 3, 64, 7, "stem"
    cin = 64
    chans = (64, 64, 256) if bottleneck else (64, 64)
    for mod_id, num in enumerate(structure):
        for b in range(num):
            stride = 2 if (b == 0 and mod_id > 0) else 1
            p = "mod%d.block%d" % (mod_id + 2, b + 1)
            if bottleneck:
                yield p + ".convs.conv1", cin, chans[0], 1, "conv1"
                yield p + ".convs.conv2", chans[0], chans[1], 3, "conv2"
                yield p + ".convs.conv3", chans[1], chans[2], 1, "conv3"
            else:
                yield p + ".convs.conv1", cin, chans[0], 3, "conv1"
                yield p + ".convs.conv2", chans[0], chans[1], 3, "conv2"
            if stride != 1 or cin != chans[-1]:
                yield p + ".proj_conv", cin, chans[-1], 1, "proj"
            cin = chans[-1]
        chans = tuple(c * 2 for c in chans)


def backbone_state(arch, seed=SEED_WEIGHTS):
    """name -> float32 ndarray, reference backbone key layout."""
    bottleneck = _NETS[arch][1]
    out = {}
    for name, cin, cout, k, role in _convs(arch):
        w = _stream(seed, name + ".weight").standard_normal((cout, cin, k, k), dtype=np.float32)
        out[name + ".weight"] = (w * np.float32(np.sqrt(2.0 / (cin * k * k)))).astype(np.float32)
        if name.endswith("proj_conv"):
            bn = name[: -len("proj_conv")] + "proj_bn"
        else:
            head, _, last = name.rpartition(".")
            bn = head + "." + last.replace("conv", "bn")
        lo, hi = (0.2, 0.4) if (role == "conv3" or (role == "conv2" and not bottleneck)) else (0.8, 1.2)
        out[bn + ".weight"] = _stream(seed, bn + ".weight").uniform(lo, hi, cout).astype(np.float32)
        out[bn + ".bias"] = _stream(seed, bn + ".bias").uniform(-0.02, 0.02, cout).astype(np.float32)
        out[bn + ".running_mean"] = _stream(seed, bn + ".running_mean").uniform(-0.02, 0.02, cout).astype(np.float32)
        out[bn + ".running_var"] = _stream(seed, bn + ".running_var").uniform(0.8, 1.2, cout).astype(np.float32)
    return out


def head_state(dim, p=3.0, seed=SEED_WEIGHTS):
    std = 0.1 * np.sqrt(2.0 / (dim + dim))
    w = _stream(seed, "whiten.weight").standard_normal((dim, dim), dtype=np.float32) * np.float32(std)
    b = _stream(seed, "whiten.bias").uniform(-0.002, 0.002, dim).astype(np.float32)
    return {"pool.p": np.array([p], dtype=np.float32), "whiten.weight": w.astype(np.float32), "whiten.bias": b}


def _lerp_idx(n_out, n_in):
    pos = np.linspace(0.0, n_in - 1.0, n_out)
    i0 = np.minimum(np.floor(pos).astype(np.int64), n_in - 2)
    return i0, (pos - i0)


def structured_images(n, h, w, seed, grid=(6, 8), noise=0.2):
    """n x 3 x h x w float32 in [0, 1)."""
    r = np.random.Generator(np.random.PCG64(seed))
    g = r.random((n, 3, grid[0], grid[1]))
    iy, fy = _lerp_idx(h, grid[0])
    ix, fx = _lerp_idx(w, grid[1])
    rows = g[:, :, iy, :] * (1 - fy)[None, None, :, None] + g[:, :, iy + 1, :] * fy[None, None, :, None]
    up = rows[:, :, :, ix] * (1 - fx) + rows[:, :, :, ix + 1] * fx
    pix = r.random((n, 3, h, w))
    return np.ascontiguousarray(((1.0 - noise) * up + noise * pix).astype(np.float32))


def load_into(net, arch, head_bias=None, seed=SEED_WEIGHTS):
    """Load backbone_state / head_state (optionally a fixture's centring
    whitening bias) into a cirtorch ImageRetrievalNet built by make_net."""
    import torch
    missing, unexpected = net.body.load_state_dict(
        {k: torch.from_numpy(v) for k, v in backbone_state(arch, seed).items()}, strict=False)
    if unexpected or [m for m in missing if "num_batches" not in m]:
        raise RuntimeError("state dict mismatch: %s %s" % (missing[:3], unexpected[:3]))
    dim = net.ret_head.dim
    hs = head_state(dim, seed=seed)
    if head_bias is not None:
        hs["whiten.bias"] = np.asarray(head_bias, dtype=np.float32)
    net.ret_head.load_state_dict({k: torch.from_numpy(v) for k, v in hs.items()})
    return net
