"""ctypes binding of librr.so (the C ABI in include/rr.h).

This is the only place the Python host touches native code.  Tensors cross
the boundary as raw device pointers + sizes; the stream is PyTorch's current
HIP stream, so every call is asynchronous and ordered with torch work.

There is deliberately no CPU fallback: if librr.so cannot be loaded, or a
tensor is not on the GPU, the call raises.
"""

import ctypes
import os
import threading

import torch

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("RR_LIB", os.path.join(PKG_DIR, "librr.so"))

RR_F32, RR_BF16, RR_F16, RR_I8 = 0, 1, 2, 3
RR_ACT_IDENTITY, RR_ACT_LEAKY = 0, 1
RR_POOL_GEM, RR_POOL_MAC, RR_POOL_SPOC = 0, 1, 2
RR_CONV_AFFINE, RR_CONV_RESIDUAL, RR_CONV_PERM32 = 1, 2, 4
RR_NHWC, RR_NCHW = 0, 1

_DTYPE_CODE = {torch.float32: RR_F32, torch.bfloat16: RR_BF16, torch.float16: RR_F16,
               torch.int8: RR_I8}  # RR_I8: kNN screening only


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("n", "h", "w", "c_in", "ho", "wo", "c_out", "kh", "kw", "stride",
                                            "pad", "dil", "k_packed", "ldy", "act")] + \
               [("slope", ctypes.c_float), ("flags", ctypes.c_int)]


_vp, _i, _ll, _f, _d, _sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float, ctypes.c_double, ctypes.c_size_t
_SIGS = {
    "rr_version": ([], _i),
    "rr_build_info": ([], ctypes.c_char_p),
    "rr_last_error": ([], ctypes.c_char_p),
    "rr_device_arch": ([ctypes.c_char_p, _i], _i),
    "rr_image_to_nhwc": ([_vp, _i, _i, _i, _i, ctypes.POINTER(_f), ctypes.POINTER(_f), _i, _vp, _i, _i, _vp], _i),
    "rr_conv2d_fused": ([_vp, _vp, _vp, _vp, _vp, _vp, ctypes.POINTER(ConvDesc), _i, _i, _vp], _i),
    "rr_conv1x1_pair": ([_vp, _ll, _i, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _vp, _i, _f, _vp, _vp, _vp, _i, _i, _f,
                         _vp, _vp, _i, _vp], _i),
    "rr_conv3x3_pair": ([_vp, _i, _i, _i, _vp, _vp, _vp, _i, _f, _vp, _vp, _vp, _i, _f, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _f,
                         _vp, _vp, _vp, _i, _i, _f, _vp, _vp, _vp, _i, _vp], _i),
    "rr_pack_conv_weights": ([_vp, _i, _i, _i, _i, _i, _i, _i, _vp, _i, _vp], _i),
    "rr_stem_pack_weights": ([_vp, _i, _i, _i, _i, _vp, _i, _vp], _i),
    "rr_stem_conv_pool": ([_vp, _i, _i, _i, ctypes.POINTER(_f), ctypes.POINTER(_f), _i, _vp, _vp, _vp, _i, _f, _vp,
                           _i, _i, _i, _vp], _i),
    "rr_stem_conv_pool_u8": ([_vp, _i, _i, _i, ctypes.POINTER(_f), ctypes.POINTER(_f), _i, _vp, _vp, _vp, _i, _f,
                              _vp, _i, _i, _i, _vp], _i),
    "rr_image_to_nhwc_ragged": ([_vp, _vp, _i, _i, _i, _i, _i, ctypes.POINTER(_f), ctypes.POINTER(_f), _i, _vp, _i,
                                 _i, _vp], _i),
    "rr_stem_conv_pool_ragged": ([_vp, _vp, _i, _i, _i, _i, ctypes.POINTER(_f), ctypes.POINTER(_f), _i, _vp, _vp, _vp,
                                  _i, _f, _vp, _i, _i, _i, _vp], _i),
    "rr_pad_images": ([_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp], _i),
    "rr_maxpool2d": ([_vp, _i, _i, _i, _i, _i, _i, _i, _vp, _i, _i, _i, _vp], _i),
    "rr_resize_bilinear": ([_vp, _i, _i, _i, _vp, _i, _i, _d, _d, _vp], _i),
    "rr_global_pool": ([_vp, _i, _i, _i, _i, _i, _f, _f, _vp, _i, _vp], _i),
    "rr_global_pool_pdev": ([_vp, _i, _i, _i, _i, _i, _f, _vp, _f, _vp, _i, _vp], _i),
    "rr_l2n_rows": ([_vp, _i, _i, _f, _vp, _vp], _i),
    "rr_linear_rows": ([_vp, _i, _i, _vp, _vp, _i, _vp, _vp], _i),
    "rr_head_workspace_bytes": ([_i, _i], _sz),
    "rr_whiten_workspace_bytes": ([_i, _i], _sz),
    "rr_whitenapply": ([_vp, _i, _i, _vp, _vp, _i, _vp, _vp, _sz, _vp], _i),
    "rr_head_l2n_whiten_l2n": ([_vp, _i, _i, _vp, _vp, _i, _f, _vp, _vp, _vp], _i),
    "rr_knn_workspace_bytes": ([_ll, _i, _i, _i, _i, _i], _sz),
    "rr_knn_topk": ([_vp, _vp, _ll, _vp, _vp, _i, _i, _i, _i, _ll, _vp, _vp, _vp, _sz, _i, _vp], _i),
    "rr_knn_topk_checked": ([_vp, _vp, _ll, _vp, _vp, _i, _i, _i, _i, _ll, _vp, _vp, _vp, _sz, _i, _f, _vp, _vp], _i),
    "rr_topk_merge": ([_vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp], _i),
    "rr_comm_unique_id": ([_vp, _i], _i),
    "rr_comm_init": ([ctypes.POINTER(_vp), _i, _vp, _i, _i], _i),
    "rr_comm_destroy": ([_vp], _i),
    "rr_topk_allgather_workspace_bytes": ([_i, _i, _i], _sz),
    "rr_topk_allgather_merge": ([_vp, _vp, _vp, _i, _i, _vp, _vp, _vp, _sz, _vp], _i),
    "rr_local_head_workspace_bytes": ([_ll, _i, _i], _sz),
    "rr_local_head": ([_vp, _i, _i, _i, _i, _i, _vp, _i, _vp, _vp, _i, _vp, _vp, _sz, _vp], _i),
    "rr_mutual_nn": ([_vp, _i, _vp, _i, _vp, _vp], _i),
    "rr_rank_workspace_bytes": ([_ll, _i], _sz),
    "rr_rank_full": ([_vp, _ll, _vp, _i, _i, _vp, _vp, _sz, _vp], _i),
    "rr_set_tuning": ([_i, _i], _i),
    "rr_fill_unit_rows": ([_vp, _ll, _i, ctypes.c_ulonglong, _ll, _vp], _i),
    "rr_cast_f32_bf16": ([_vp, _vp, _ll, _vp], _i),
    "rr_cast_f32_f16": ([_vp, _vp, _ll, _vp], _i),
    "rr_quantize_i8": ([_vp, _ll, _vp, _vp, _vp], _i),
    "rr_quantize_i8_rows": ([_vp, _i, _i, _vp, _vp, _vp], _i),
    "rr_knn_topk_checked_i8": ([_vp, _vp, _ll, _vp, _vp, _i, _i, _i, _i, _ll, _vp, _vp, _vp, _sz, _f, _vp, _i, _vp,
                                _vp, _vp], _i),
}

_lib = None
_lock = threading.Lock()


def lib():
    """Load librr.so once; raise (never fall back) if it is missing."""
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise RuntimeError("librr.so not found at %s — build it with "
                                       "`python -c 'import __graft_entry__ as g; g.build()'`" % LIB_PATH)
                handle = ctypes.CDLL(LIB_PATH)
                for name, (args, res) in _SIGS.items():
                    fn = getattr(handle, name)
                    fn.argtypes = args
                    fn.restype = res
                _lib = handle
    return _lib


def check(rc, what):
    if rc != 0:
        msg = lib().rr_last_error().decode(errors="replace")
        raise RuntimeError("%s failed (rc=%d): %s" % (what, rc, msg))


def stream_ptr(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def require_gpu(*tensors):
    for t in tensors:
        if t is None:
            continue
        if not t.is_cuda:
            raise RuntimeError("cirtorch (MI355X engine) operates on GPU tensors only; got a %s tensor. "
                               "Move the model and inputs to the GPU (net.cuda()); there is no CPU path." % t.device)


def dtype_code(dt):
    try:
        return _DTYPE_CODE[dt]
    except KeyError:
        raise RuntimeError("unsupported dtype %s (float32, bfloat16; float16 for kNN screening)" % dt)


def device_arch():
    buf = ctypes.create_string_buffer(64)
    check(lib().rr_device_arch(buf, 64), "rr_device_arch")
    return buf.value.decode()
