"""torch-tensor wrappers over the librr.so entry points (device memory and
streams come from PyTorch; all arithmetic is in the HIP kernels).

Shapes follow the engine's layouts: activations NHWC ([N, H, W, C] tensors),
packed conv weights [c_out, k_packed], descriptors row-major [n, D].
"""

import ctypes
import os

import numpy as np
import torch

from . import _engine as E


def _st():
    return E.stream_ptr()


# ---------------------------------------------------------------- extractor ops
def image_to_nhwc(img, c_pad, dtype, mean=None, std=None):
    """img: [N, C<=4, H, W] float32 (GPU) -> [N, H, W, c_pad] `dtype`, normalised
    with (x - mean) / std when mean/std are given (cirtorch/utils/image.py:86-127)."""
    E.require_gpu(img)
    img = img.contiguous().float()
    n, c, h, w = img.shape
    out = torch.empty((n, h, w, c_pad), dtype=dtype, device=img.device)
    do = mean is not None
    m = (ctypes.c_float * 4)(*(list(mean) + [0.0] * (4 - c))[:4]) if do else (ctypes.c_float * 4)()
    s = (ctypes.c_float * 4)(*(list(std) + [1.0] * (4 - c))[:4]) if do else (ctypes.c_float * 4)(1, 1, 1, 1)
    E.check(E.lib().rr_image_to_nhwc(E.ptr(img), n, c, h, w, m, s, int(do), E.ptr(out), c_pad,
                                     E.dtype_code(dtype), _st()), "rr_image_to_nhwc")
    return out


def pack_conv_weights(weight, cin_pad, dtype, perm32=False, k_mult=64):
    """nn.Conv2d weight [c_out, c_in, kh, kw] (GPU) -> engine layout [c_out, k_packed]."""
    E.require_gpu(weight)
    w = weight.detach().float().contiguous()
    co, ci, kh, kw = w.shape
    kp = (kh * kw * cin_pad + k_mult - 1) // k_mult * k_mult
    out = torch.empty((co, kp), dtype=dtype, device=w.device)
    E.check(E.lib().rr_pack_conv_weights(E.ptr(w), co, ci, kh, kw, cin_pad, kp, int(bool(perm32)), E.ptr(out),
                                         E.dtype_code(dtype), _st()), "rr_pack_conv_weights")
    return out


def conv2d_fused(x, w_packed, kh, kw, stride, pad, c_out, scale=None, shift=None, residual=None,
                 leaky=True, slope=0.01, out_dtype=None, dil=1, perm32=False, out=None):
    """x: [N, H, W, C] -> act(conv(x) * scale + shift (+ residual)) as [N, Ho, Wo, c_out].
    perm32: w_packed rows are in the RR_CONV_PERM32 order (pack_conv_weights(perm32=True)).
    out: an optional contiguous [N, Ho, Wo, c_out] destination (e.g. a batch slice)."""
    E.require_gpu(x, w_packed)
    n, h, w, c = x.shape
    ho = (h + 2 * pad - dil * (kh - 1) - 1) // stride + 1
    wo = (w + 2 * pad - dil * (kw - 1) - 1) // stride + 1
    out_dtype = out_dtype or x.dtype
    if out is not None:
        E.require_gpu(out)
        assert tuple(out.shape) == (n, ho, wo, c_out) and out.dtype == out_dtype and out.is_contiguous()
        y = out
    else:
        y = torch.empty((n, ho, wo, c_out), dtype=out_dtype, device=x.device)
    flags = 0
    if scale is not None:
        flags |= E.RR_CONV_AFFINE
    if residual is not None:
        flags |= E.RR_CONV_RESIDUAL
        assert residual.shape == y.shape and residual.dtype == out_dtype and residual.is_contiguous()
    if perm32:
        flags |= E.RR_CONV_PERM32
    d = E.ConvDesc(n=n, h=h, w=w, c_in=c, ho=ho, wo=wo, c_out=c_out, kh=kh, kw=kw, stride=stride, pad=pad,
                   dil=dil, k_packed=w_packed.shape[1], ldy=c_out,
                   act=E.RR_ACT_LEAKY if leaky else E.RR_ACT_IDENTITY, slope=slope, flags=flags)
    E.check(E.lib().rr_conv2d_fused(E.ptr(x), E.ptr(w_packed), E.ptr(scale), E.ptr(shift), E.ptr(residual),
                                    E.ptr(y), ctypes.byref(d), E.dtype_code(x.dtype), E.dtype_code(out_dtype),
                                    _st()), "rr_conv2d_fused")
    return y


def conv1x1_pair(x, w3, scale3, shift3, residual, leaky3, slope3, w1, scale1, shift1, c_out, leaky1, slope1,
                 proj=None):
    """Fused y = act3(conv1x1(x, w3)*scale3 + shift3 + shortcut); z = act1(conv1x1(y, w1)*scale1 + shift1)
    (conv3 of one bottleneck block + conv1 of the next, cirtorch/backbones/misc.py:166-203).
    shortcut = residual, or with residual=None and proj=(xp, wp, scalep, shiftp) the block's 1x1
    projection proj_bn(proj_conv(xp)) computed in the same pass (64 -> 256 boundaries only).
    x: [N, H, W, 64] or [N, H, W, 128] bf16 / fp16, PERM32-packed weights; returns
    (y [N, H, W, 256 | 512], z [N, H, W, c_out])."""
    E.require_gpu(x, w3, residual, w1)
    n, h, w, c = x.shape
    c_mid = w3.shape[0]
    y = torch.empty((n, h, w, c_mid), dtype=x.dtype, device=x.device)
    z = torch.empty((n, h, w, c_out), dtype=x.dtype, device=x.device)
    assert x.is_contiguous()
    if residual is not None:
        assert residual.shape == y.shape and residual.dtype == x.dtype and residual.is_contiguous()
        xp = wp = sp = hp = None
    else:
        xp, wp, sp, hp = proj
        E.require_gpu(xp, wp, sp, hp)
        assert xp.shape == x.shape and xp.dtype == x.dtype and xp.is_contiguous()
    E.check(E.lib().rr_conv1x1_pair(E.ptr(x), n * h * w, c, E.ptr(w3), E.ptr(scale3), E.ptr(shift3), c_mid,
                                    E.ptr(residual), E.ptr(xp), E.ptr(wp), E.ptr(sp), E.ptr(hp),
                                    E.RR_ACT_LEAKY if leaky3 else E.RR_ACT_IDENTITY, float(slope3),
                                    E.ptr(w1), E.ptr(scale1), E.ptr(shift1), c_out,
                                    E.RR_ACT_LEAKY if leaky1 else E.RR_ACT_IDENTITY, float(slope1), E.ptr(y), E.ptr(z),
                                    E.dtype_code(x.dtype), _st()), "rr_conv1x1_pair")
    return y, z


def conv3x3_pair(t1, w33, scale2, shift2, leaky2, slope2, w3, scale3, shift3, residual, leaky3, slope3,
                 w1, scale1, shift1, c_out, leaky1, slope1, proj=None, dynamic=None, conv1=None):
    """One whole bottleneck block of the 256-channel stage plus the next block's conv1 in one
    launch (cirtorch/backbones/misc.py:163-203): t2 = act2(conv3x3(t1, w33)*scale2 + shift2),
    y = act3(conv1x1(t2, w3)*scale3 + shift3 + shortcut), z = act1(conv1x1(y, w1)*scale1 + shift1);
    t2 stays on chip.  shortcut = residual, or with residual=None and proj=(xp, wp, scalep, shiftp)
    the block's projection.  t1: [N, H, W, 64] bf16 / fp16 with H % 4 == 0 and W % 32 == 0, PERM32
    weights; returns (y [N, H, W, 256], z [N, H, W, c_out]), bit-identical to the 3x3 launch
    followed by conv1x1_pair.  dynamic (default: RR_C3PAIR_QUEUE != "0"): per-XCD tile counters
    (a zeroed 8-int array per launch) instead of the static tile walk — same results.
    conv1=(w0, scale0, shift0, leaky0, slope0) (projection form, the stage's first block): t1 is
    the block input x (pass it as proj's xp too) and the block's conv1 runs in the launch."""
    E.require_gpu(t1, w33, w3, residual, w1)
    n, h, w, c = t1.shape
    assert c == 64 and t1.is_contiguous() and tuple(w33.shape) == (64, 576) and tuple(w3.shape) == (256, 64)
    assert tuple(w1.shape) == (c_out, 256)
    y = torch.empty((n, h, w, 256), dtype=t1.dtype, device=t1.device)
    z = torch.empty((n, h, w, c_out), dtype=t1.dtype, device=t1.device)
    if residual is not None:
        assert residual.shape == y.shape and residual.dtype == t1.dtype and residual.is_contiguous()
        xp = wp = sp = hp = None
    else:
        xp, wp, sp, hp = proj
        E.require_gpu(xp, wp, sp, hp)
        assert tuple(xp.shape) == (n, h, w, 64) and xp.dtype == t1.dtype and xp.is_contiguous()
    act = lambda leaky: E.RR_ACT_LEAKY if leaky else E.RR_ACT_IDENTITY
    if dynamic is None:
        dynamic = os.environ.get("RR_C3PAIR_QUEUE", "1") != "0"
    queue = torch.zeros(8, dtype=torch.int32, device=t1.device) if dynamic else None
    w0, s0, h0, leaky0, slope0 = conv1 if conv1 is not None else (None, None, None, False, 0.0)
    if conv1 is not None:
        E.require_gpu(w0, s0, h0)
        assert proj is not None and tuple(w0.shape) == (64, 64)
    E.check(E.lib().rr_conv3x3_pair(E.ptr(t1), n, h, w, E.ptr(w0), E.ptr(s0), E.ptr(h0), act(leaky0), float(slope0),
                                    E.ptr(w33), E.ptr(scale2), E.ptr(shift2), act(leaky2),
                                    float(slope2), E.ptr(w3), E.ptr(scale3), E.ptr(shift3), E.ptr(residual),
                                    E.ptr(xp), E.ptr(wp), E.ptr(sp), E.ptr(hp), act(leaky3), float(slope3),
                                    E.ptr(w1), E.ptr(scale1), E.ptr(shift1), c_out, act(leaky1), float(slope1),
                                    E.ptr(y), E.ptr(z), E.ptr(queue), E.dtype_code(t1.dtype), _st()),
            "rr_conv3x3_pair")
    return y, z


def maxpool2d(x, k=3, stride=2, pad=1):
    E.require_gpu(x)
    n, h, w, c = x.shape
    ho = (h + 2 * pad - k) // stride + 1
    wo = (w + 2 * pad - k) // stride + 1
    y = torch.empty((n, ho, wo, c), dtype=x.dtype, device=x.device)
    E.check(E.lib().rr_maxpool2d(E.ptr(x), n, h, w, c, k, stride, pad, E.ptr(y), ho, wo, E.dtype_code(x.dtype),
                                 _st()), "rr_maxpool2d")
    return y


def pack_stem_weights(weight, dtype=torch.bfloat16):
    """conv1 weight [64, 3, 7, 7] (GPU) -> the fused stem's [64, 448] layout (bf16 or fp16):
    kernel-row K (v1-v3 stems) then space-to-depth K (v4)."""
    E.require_gpu(weight)
    w = weight.detach().float().contiguous()
    co, ci, kh, kw = w.shape
    out = torch.empty((co, 448), dtype=dtype, device=w.device)
    E.check(E.lib().rr_stem_pack_weights(E.ptr(w), co, ci, kh, kw, E.ptr(out), E.dtype_code(dtype), _st()),
            "rr_stem_pack_weights")
    return out


_UNIT_LUT = {}


def pixels_to_unit(x):
    """uint8 pixels -> float32 x / 255 with numpy's IEEE division (torchvision
    ``to_tensor``): a 256-entry table computed on the host, gathered on the
    device (torch's scalar division multiplies by the reciprocal, which differs
    in the last bit for some pixel values)."""
    lut = _UNIT_LUT.get(x.device)
    if lut is None:
        lut = torch.from_numpy(np.arange(256, dtype=np.float32) / np.float32(255.0)).to(x.device)
        _UNIT_LUT[x.device] = lut
    return lut[x.long()]


def stem_conv_pool(img, wpk, scale, shift, leaky=True, slope=0.01, mean=None, std=None):
    """Fused normalise + conv1 7x7/s2/p3 + BN + act + maxpool 3x3/s2/p1
    (cirtorch/backbones/resnet.py:59-66): [N, 3, H, W] float32 -> [N, Hp, Wp, 64] in wpk's dtype
    (bf16 or fp16).  uint8 images are read as pixels (value / 255, torchvision
    ``to_tensor``) by ``rr_stem_conv_pool_u8``: identical output to the float32
    path on ``img.float() / 255``."""
    E.require_gpu(img, wpk, scale, shift)
    u8 = img.dtype == torch.uint8
    img = img.contiguous() if u8 else img.contiguous().float()
    n, c, h, w = img.shape
    if c != 3:
        raise RuntimeError("stem_conv_pool: expected 3-channel images, got %d" % c)
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    hp, wp = (ho - 1) // 2 + 1, (wo - 1) // 2 + 1
    y = torch.empty((n, hp, wp, 64), dtype=wpk.dtype, device=img.device)
    do = mean is not None
    m = (ctypes.c_float * 3)(*mean) if do else (ctypes.c_float * 3)()
    s = (ctypes.c_float * 3)(*std) if do else (ctypes.c_float * 3)(1, 1, 1)
    fn = E.lib().rr_stem_conv_pool_u8 if u8 else E.lib().rr_stem_conv_pool
    E.check(fn(E.ptr(img), n, h, w, m, s, int(do), E.ptr(wpk), E.ptr(scale), E.ptr(shift),
               E.RR_ACT_LEAKY if leaky else E.RR_ACT_IDENTITY, float(slope), E.ptr(y), hp, wp,
               E.dtype_code(wpk.dtype), _st()), "rr_stem_conv_pool")
    return y


def _ragged(images):
    """a ragged batch (list of [C, h_i, w_i] GPU tensors of one dtype, None entries
    allowed) -> the C ABI's host (pointer, extent) arrays + the contiguous tensors
    they point into (kept referenced until the launch is enqueued)."""
    n = len(images)
    ptrs = (ctypes.c_void_p * n)()
    ext = (ctypes.c_int * (2 * n))()
    kept = []
    for i, t in enumerate(images):
        if t is None:
            continue
        E.require_gpu(t)
        t = t.contiguous()
        kept.append(t)
        ptrs[i] = t.data_ptr()
        ext[2 * i], ext[2 * i + 1] = int(t.shape[-2]), int(t.shape[-1])
    return ptrs, ext, kept


def _norm_arrays(mean, std, c):
    do = mean is not None
    m = (ctypes.c_float * 4)(*(list(mean) + [0.0] * (4 - c))[:4]) if do else (ctypes.c_float * 4)()
    s = (ctypes.c_float * 4)(*(list(std) + [1.0] * (4 - c))[:4]) if do else (ctypes.c_float * 4)(1, 1, 1, 1)
    return m, s, int(do)


def image_to_nhwc_ragged(images, h, w, c_pad, dtype, mean=None, std=None):
    """ragged batch of [C, h_i, w_i] float32 or uint8 images (h_i <= h, w_i <= w) ->
    [N, h, w, c_pad] `dtype`: the padded, normalised map (map pixels outside an
    image read 0 before normalisation, utils/sequence.py:51 then utils/image.py:125)
    without a padded copy of the inputs."""
    ref = next(t for t in images if t is not None)
    c = int(ref.shape[0])
    u8 = ref.dtype == torch.uint8
    if not u8 and ref.dtype != torch.float32:
        images = [t.float() if t is not None else None for t in images]
    ptrs, ext, kept = _ragged(images)
    out = torch.empty((len(images), h, w, c_pad), dtype=dtype, device=ref.device)
    m, s, do = _norm_arrays(mean, std, c)
    E.check(E.lib().rr_image_to_nhwc_ragged(ptrs, ext, len(images), c, h, w, int(u8), m, s, do, E.ptr(out), c_pad,
                                            E.dtype_code(dtype), _st()), "rr_image_to_nhwc_ragged")
    return out


def stem_conv_pool_ragged(images, h, w, wpk, scale, shift, leaky=True, slope=0.01, mean=None, std=None):
    """The fused stem (stem_conv_pool) on a ragged batch padded to h x w: equals
    stem_conv_pool on the padded batch bit for bit, with no padded copy."""
    E.require_gpu(wpk, scale, shift)
    ref = next(t for t in images if t is not None)
    if ref.shape[0] != 3:
        raise RuntimeError("stem_conv_pool: expected 3-channel images, got %d" % ref.shape[0])
    u8 = ref.dtype == torch.uint8
    if not u8 and ref.dtype != torch.float32:
        images = [t.float() if t is not None else None for t in images]
    ptrs, ext, kept = _ragged(images)
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    hp, wp = (ho - 1) // 2 + 1, (wo - 1) // 2 + 1
    y = torch.empty((len(images), hp, wp, 64), dtype=wpk.dtype, device=ref.device)
    do = mean is not None
    m = (ctypes.c_float * 3)(*mean) if do else (ctypes.c_float * 3)()
    s = (ctypes.c_float * 3)(*std) if do else (ctypes.c_float * 3)(1, 1, 1)
    E.check(E.lib().rr_stem_conv_pool_ragged(ptrs, ext, len(images), h, w, int(u8), m, s, int(do), E.ptr(wpk),
                                             E.ptr(scale), E.ptr(shift), E.RR_ACT_LEAKY if leaky else E.RR_ACT_IDENTITY,
                                             float(slope), E.ptr(y), hp, wp, E.dtype_code(wpk.dtype), _st()),
            "rr_stem_conv_pool_ragged")
    return y


_ELEM_CT = {1: ctypes.c_uint8, 2: ctypes.c_uint16, 4: ctypes.c_uint32, 8: ctypes.c_uint64}


def pad_images(images, h, w, pad_value=0.0):
    """ragged batch of [C, h_i, w_i] (or [h_i, w_i]) GPU tensors -> one padded
    [N, C, h, w] (or [N, h, w]) tensor, images top-left, pad_value elsewhere:
    one rr_pad_images launch (utils/sequence.py:4-67)."""
    ref = next(t for t in images if t is not None)
    chw = ref.dim() == 3
    c = int(ref.shape[0]) if chw else 1
    shape = (len(images), c, h, w) if chw else (len(images), h, w)
    out = torch.empty(shape, dtype=ref.dtype, device=ref.device)
    esz = out.element_size()
    pv = torch.tensor([pad_value], dtype=ref.dtype).view(_ELEM_TORCH[esz]).item()
    pad = _ELEM_CT[esz](pv & ((1 << (8 * esz)) - 1))
    ptrs, ext, kept = _ragged(images)
    E.check(E.lib().rr_pad_images(ptrs, ext, len(images), c, h, w, esz, ctypes.byref(pad), E.ptr(out), _st()),
            "rr_pad_images")
    return out


_ELEM_TORCH = {1: torch.uint8, 2: torch.int16, 4: torch.int32, 8: torch.int64}


def resize_bilinear(img, scale_factor):
    """img: [C, H, W] (or a same-size batch [N, C, H, W]) float32 -> bilinear
    (align_corners=False) resize by scale_factor, output size floor(H*s) x
    floor(W*s) like nn.functional.interpolate(scale_factor=s)
    (cirtorch/models/GF_net.py:32-35).  Planes are independent, so a batch is
    one launch over N*C planes."""
    E.require_gpu(img)
    img = img.contiguous().float()
    lead = img.shape[:-2]
    h, w = img.shape[-2:]
    c = int(np.prod(lead)) if len(lead) else 1
    ho, wo = int(h * scale_factor), int(w * scale_factor)
    out = torch.empty(tuple(lead) + (ho, wo), dtype=torch.float32, device=img.device)
    E.check(E.lib().rr_resize_bilinear(E.ptr(img), c, h, w, E.ptr(out), ho, wo, 1.0 / scale_factor,
                                       1.0 / scale_factor, _st()), "rr_resize_bilinear")
    return out


# ---------------------------------------------------------------- head ops
def global_pool(x, mode, p=3.0, eps=1e-6):
    """x: [N, C, H, W] (NCHW-contiguous or channels_last view) -> [N, C] float32.
    p: a float, or a one-element GPU tensor (the learnable ``pool.p``) that the
    kernel reads from device memory (rr_global_pool_pdev: no host read-back)."""
    E.require_gpu(x)
    p_dev = None
    if torch.is_tensor(p):
        if p.numel() != 1:
            raise NotImplementedError("per-channel GeM exponents (GeMmp) are out of scope")
        E.require_gpu(p)
        p_dev = p.detach().reshape(1)
        if p_dev.dtype != torch.float32:
            p_dev = p_dev.float()
        p = 1.0
    n, c, h, w = x.shape
    if x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous():
        layout = E.RR_NHWC
    elif x.is_contiguous():
        layout = E.RR_NCHW
    else:
        x = x.contiguous()
        layout = E.RR_NCHW
    if layout == E.RR_NHWC and c % 4:
        x = x.contiguous()
        layout = E.RR_NCHW
    if x.dtype not in (torch.float32, torch.bfloat16, torch.float16):
        x = x.float()
    out = torch.empty((n, c), dtype=torch.float32, device=x.device)
    if p_dev is not None:
        E.check(E.lib().rr_global_pool_pdev(E.ptr(x), n, c, h * w, layout, mode, float(p), E.ptr(p_dev), float(eps),
                                            E.ptr(out), E.dtype_code(x.dtype), _st()), "rr_global_pool_pdev")
    else:
        E.check(E.lib().rr_global_pool(E.ptr(x), n, c, h * w, layout, mode, float(p), float(eps), E.ptr(out),
                                       E.dtype_code(x.dtype), _st()), "rr_global_pool")
    return out


def l2n_rows(x, eps=1e-6):
    E.require_gpu(x)
    x = x.contiguous().float()
    rows = x.shape[0]
    dim = x.numel() // max(rows, 1)
    y = torch.empty_like(x)
    E.check(E.lib().rr_l2n_rows(E.ptr(x), rows, dim, float(eps), E.ptr(y), _st()), "rr_l2n_rows")
    return y


def linear_rows(x, weight, bias=None):
    E.require_gpu(x, weight, bias)
    x = x.contiguous().float()
    weight = weight.contiguous().float()
    bias = bias.contiguous().float() if bias is not None else None
    rows, in_dim = x.shape
    out_dim = weight.shape[0]
    y = torch.empty((rows, out_dim), dtype=torch.float32, device=x.device)
    E.check(E.lib().rr_linear_rows(E.ptr(x), rows, in_dim, E.ptr(weight), E.ptr(bias), out_dim, E.ptr(y), _st()),
            "rr_linear_rows")
    return y


def head_tail(pooled, weight, bias, whiten=True, eps=1e-6):
    """pooled [N, D] -> L2N(W . L2N(pooled) + b) (global_head.py:59-64), [N, D]."""
    E.require_gpu(pooled, weight, bias)
    pooled = pooled.contiguous().float()
    rows, dim = pooled.shape
    y = torch.empty_like(pooled)
    ws = torch.empty(int(E.lib().rr_head_workspace_bytes(rows, dim)) // 4 + 1, dtype=torch.float32,
                     device=pooled.device) if whiten else None
    w = weight.contiguous().float() if whiten else None
    b = bias.contiguous().float() if (whiten and bias is not None) else None
    E.check(E.lib().rr_head_l2n_whiten_l2n(E.ptr(pooled), rows, dim, E.ptr(w), E.ptr(b), int(bool(whiten)),
                                           float(eps), E.ptr(y), E.ptr(ws), _st()), "rr_head_l2n_whiten_l2n")
    return y


def whitenapply_rows(x, m, P, d_out):
    """x [N, D] float32 rows, m [D] / P [>= d_out, D] float64 (GPU) ->
    L2N(P[:d_out] (x - m)) [N, d_out] float32, computed in float64 on the f64
    MFMA (cirtorch/utils/whiten.py:4-12)."""
    E.require_gpu(x, m, P)
    x = x.contiguous().float()
    m = m.contiguous().double().reshape(-1)
    P = P.contiguous().double()
    rows, dim = x.shape
    if dim % 16:
        # the f64 MFMA kernel takes 16-wide K-steps: zero columns of x, m and P
        # add exact zeros to every dot product (any D, like the numpy reference)
        pad = 16 - dim % 16
        x = torch.nn.functional.pad(x, (0, pad))
        m = torch.nn.functional.pad(m, (0, pad))
        P = torch.nn.functional.pad(P, (0, pad))
        dim += pad
    y = torch.empty((rows, d_out), dtype=torch.float32, device=x.device)
    ws = torch.empty(max(1, int(E.lib().rr_whiten_workspace_bytes(rows, d_out))), dtype=torch.uint8, device=x.device)
    E.check(E.lib().rr_whitenapply(E.ptr(x), rows, dim, E.ptr(m), E.ptr(P), int(d_out), E.ptr(y), E.ptr(ws),
                                   ws.numel(), _st()), "rr_whitenapply")
    return y


# ---------------------------------------------------------------- matching
def knn_workspace_bytes(n_db, nq, d, k, cand=0, dtype=torch.float32):
    return int(E.lib().rr_knn_workspace_bytes(int(n_db), int(nq), int(d), int(k), int(cand), E.dtype_code(dtype)))


def knn_topk(db, db_f32, q, q_f32, k, cand=0, idx_offset=0, workspace=None, db_norm_max=None, i8_scales=None):
    """db/q: [n, D] rows in the screening dtype (float32, bfloat16, float16 or int8);
    db_f32/q_f32: the float32 rows used for the exact re-score.
    Returns (scores float64 [Q, k], idx int64 [Q, k]); with db_norm_max (the
    largest database row norm) also int32 [Q] flags: 1 where the screening
    margin could not be certified (rr_knn_topk_checked).  int8 screening is
    certified with i8_scales = (query max|x| [Q] or [1], database max|x| [1])
    (rr_knn_topk_checked_i8); without them every int8 query is flagged."""
    E.require_gpu(db, db_f32, q, q_f32)
    assert db.dtype == q.dtype and db_f32.dtype == torch.float32 and q_f32.dtype == torch.float32
    for t in (db, db_f32, q, q_f32):
        assert t.is_contiguous()
    if i8_scales is not None and (db_norm_max is None or db.dtype != torch.int8):
        raise ValueError("knn_topk: i8_scales apply to the certified int8 search only "
                         "(int8 rows with db_norm_max); they would be ignored here")
    n_db, d = db.shape
    nq = q.shape[0]
    need = knn_workspace_bytes(n_db, nq, d, k, cand, db.dtype)
    if workspace is None or workspace.numel() < need:
        workspace = torch.empty(need, dtype=torch.uint8, device=db.device)
    out_s = torch.empty((nq, k), dtype=torch.float64, device=db.device)
    out_i = torch.empty((nq, k), dtype=torch.int64, device=db.device)
    if db_norm_max is None:
        E.check(E.lib().rr_knn_topk(E.ptr(db), E.ptr(db_f32), n_db, E.ptr(q), E.ptr(q_f32), nq, d, k, int(cand),
                                    int(idx_offset), E.ptr(out_s), E.ptr(out_i), E.ptr(workspace),
                                    workspace.numel(), E.dtype_code(db.dtype), _st()), "rr_knn_topk")
        return out_s, out_i
    unc = torch.empty(nq, dtype=torch.int32, device=db.device)
    if i8_scales is not None:
        qa, da = i8_scales
        assert qa.dtype == torch.float32 and da.dtype == torch.float32 and qa.numel() in (1, nq)
        E.check(E.lib().rr_knn_topk_checked_i8(E.ptr(db), E.ptr(db_f32), n_db, E.ptr(q), E.ptr(q_f32), nq, d, k,
                                               int(cand), int(idx_offset), E.ptr(out_s), E.ptr(out_i),
                                               E.ptr(workspace), workspace.numel(), float(db_norm_max), E.ptr(qa),
                                               int(qa.numel() == nq and nq > 1), E.ptr(da), E.ptr(unc), _st()),
                "rr_knn_topk_checked_i8")
        return out_s, out_i, unc
    E.check(E.lib().rr_knn_topk_checked(E.ptr(db), E.ptr(db_f32), n_db, E.ptr(q), E.ptr(q_f32), nq, d, k, int(cand),
                                        int(idx_offset), E.ptr(out_s), E.ptr(out_i), E.ptr(workspace),
                                        workspace.numel(), E.dtype_code(db.dtype), float(db_norm_max), E.ptr(unc),
                                        _st()), "rr_knn_topk_checked")
    return out_s, out_i, unc


def rank_full(db_f32, q_f32):
    """db_f32 [n, D], q_f32 [Q, D] float32 rows (D % 256 == 0) -> int64 [Q, n]: every
    database row per query by (float64 score desc, index asc) (rr_rank_full)."""
    E.require_gpu(db_f32, q_f32)
    assert db_f32.dtype == torch.float32 and q_f32.dtype == torch.float32
    assert db_f32.is_contiguous() and q_f32.is_contiguous() and db_f32.shape[1] == q_f32.shape[1]
    n, d = db_f32.shape
    nq = q_f32.shape[0]
    ws = torch.empty(int(E.lib().rr_rank_workspace_bytes(n, nq)), dtype=torch.uint8, device=db_f32.device)
    out = torch.empty((nq, n), dtype=torch.int64, device=db_f32.device)
    E.check(E.lib().rr_rank_full(E.ptr(db_f32), n, E.ptr(q_f32), nq, d, E.ptr(out), E.ptr(ws), ws.numel(), _st()),
            "rr_rank_full")
    return out


def topk_merge(scores, idx, k):
    """scores/idx: [R, Q, k_in] per-shard lists -> merged [Q, k]."""
    E.require_gpu(scores, idx)
    r, nq, k_in = scores.shape
    out_s = torch.empty((nq, k), dtype=torch.float64, device=scores.device)
    out_i = torch.empty((nq, k), dtype=torch.int64, device=scores.device)
    E.check(E.lib().rr_topk_merge(E.ptr(scores.contiguous()), E.ptr(idx.contiguous()), r, nq, k_in, k,
                                  E.ptr(out_s), E.ptr(out_i), _st()), "rr_topk_merge")
    return out_s, out_i


def fill_unit_rows(rows, d, seed, row0=0, device=None):
    out = torch.empty((rows, d), dtype=torch.float32, device=device or "cuda")
    E.check(E.lib().rr_fill_unit_rows(E.ptr(out), int(rows), int(d), ctypes.c_ulonglong(seed), int(row0), _st()),
            "rr_fill_unit_rows")
    return out


def cast_bf16(x):
    E.require_gpu(x)
    x = x.contiguous()
    y = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    E.check(E.lib().rr_cast_f32_bf16(E.ptr(x), E.ptr(y), x.numel(), _st()), "rr_cast_f32_bf16")
    return y


def cast_f16(x):
    """float32 -> IEEE fp16 (round to nearest even): the kNN screening copy of an
    fp16 database."""
    E.require_gpu(x)
    x = x.contiguous()
    y = torch.empty(x.shape, dtype=torch.float16, device=x.device)
    E.check(E.lib().rr_cast_f32_f16(E.ptr(x), E.ptr(y), x.numel(), _st()), "rr_cast_f32_f16")
    return y


def quantize_i8(x, per_row=False, with_scale=False):
    """float32 rows -> int8 screening copy: rint(x * 127 / max|x|) clamped to +-127, the
    scale reduced on the device (no host read-back): one scale for the whole tensor (the
    database), or with per_row one per row (queries: a query's screened candidates then
    do not depend on the other queries of its batch).  with_scale: also return the
    float32 max |x| ([1] or [rows]) -- the certificate's quantisation scale."""
    E.require_gpu(x)
    x = x.contiguous()
    y = torch.empty(x.shape, dtype=torch.int8, device=x.device)
    if per_row:
        rows, d = x.shape
        if d % 4:
            raise RuntimeError("quantize_i8: row length must be a multiple of 4")
        amax = torch.empty(rows, dtype=torch.float32, device=x.device)
        E.check(E.lib().rr_quantize_i8_rows(E.ptr(x), rows, d, E.ptr(y), E.ptr(amax), _st()), "rr_quantize_i8_rows")
    else:
        if x.numel() % 4:
            raise RuntimeError("quantize_i8: element count must be a multiple of 4")
        amax = torch.empty(1, dtype=torch.float32, device=x.device)
        E.check(E.lib().rr_quantize_i8(E.ptr(x), x.numel(), E.ptr(y), E.ptr(amax), _st()), "rr_quantize_i8")
    return (y, amax) if with_scale else y


def cast_screen(x, dtype):
    """float32 rows -> the screening dtype's copy (the rows themselves for float32)."""
    if dtype == torch.float32:
        return x
    if dtype == torch.int8:
        return quantize_i8(x)
    if dtype == torch.bfloat16:
        return cast_bf16(x)
    if dtype == torch.float16:
        return cast_f16(x)
    raise RuntimeError("unsupported screening dtype %s" % dtype)


# ---------------------------------------------------------------- local descriptors
def local_head(x, kpts, weight, bias):
    """x: [N, C, H, W] feature map (channels_last view or NHWC-able, f32/bf16), kpts [N, P, 2]
    normalised (x, y) -> normalize(Linear(grid_sample(x, kpts))) as [N, P, E] float32
    (cirtorch/modules/heads/local_head.py:43-71)."""
    E.require_gpu(x, kpts, weight, bias)
    n, c, h, w = x.shape
    xh = x.permute(0, 2, 3, 1)
    if not xh.is_contiguous():
        xh = xh.contiguous()
    if xh.dtype not in (torch.float32, torch.bfloat16, torch.float16):
        xh = xh.float()
    kp = kpts.contiguous().float()
    npts = kp.shape[1]
    wt = weight.contiguous().float()
    b = bias.contiguous().float() if bias is not None else None
    e = wt.shape[0]
    out = torch.empty((n, npts, e), dtype=torch.float32, device=x.device)
    ws = torch.empty(int(E.lib().rr_local_head_workspace_bytes(n * npts, c, e)), dtype=torch.uint8, device=x.device)
    E.check(E.lib().rr_local_head(E.ptr(xh), n, h, w, c, E.dtype_code(xh.dtype), E.ptr(kp), npts, E.ptr(wt), E.ptr(b),
                                  e, E.ptr(out), E.ptr(ws), ws.numel(), _st()), "rr_local_head")
    return out


def mutual_nn(nn12, nn21):
    """int64 top-1 lists of both directions -> match [n1] (-1 where not mutual)."""
    E.require_gpu(nn12, nn21)
    a, b = nn12.contiguous().long(), nn21.contiguous().long()
    out = torch.empty_like(a)
    E.check(E.lib().rr_mutual_nn(E.ptr(a), a.numel(), E.ptr(b), b.numel(), E.ptr(out), _st()), "rr_mutual_nn")
    return out
