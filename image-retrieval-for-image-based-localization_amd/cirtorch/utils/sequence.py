"""pad_packed_images / pack_padded_images: surface of the reference
``cirtorch/utils/sequence.py:4-79`` (same arguments, return values and
ValueError cases).

The model itself never calls these: the body consumes a PackedSequence as a
ragged batch (see ``utils/parallel/packed_sequence.py``).  They remain for
callers that want the padded tensor: device entries are padded by ONE
``rr_pad_images`` launch reading every image at its own address (instead of
a fill plus a copy per image); host entries with ``torch.nn.functional.pad``.
"""

import torch
import torch.nn.functional as F

from .parallel import PackedSequence


def _padded_extent(live, snap_size_to):
    h = max(int(t.shape[-2]) for t in live)
    w = max(int(t.shape[-1]) for t in live)
    if snap_size_to:
        h, w = (-(-h // snap_size_to) * snap_size_to, -(-w // snap_size_to) * snap_size_to)
    return h, w


def _check_ranks(live):
    ndim = live[0].dim()
    for t in live:
        if t.dim() not in (2, 3):
            raise ValueError("pad_packed_images takes 2D (H, W) or 3D (C, H, W) tensors")
        if t.dim() != ndim:
            raise ValueError("pad_packed_images: every tensor must have the same number of dimensions")
    if ndim == 3 and len({int(t.shape[0]) for t in live}) > 1:
        raise ValueError("pad_packed_images: 3D tensors must agree on the channel count")
    return ndim


def pad_packed_images(packed_images, pad_value=0., snap_size_to=None):
    """PackedSequence of N tensors ([C,] H_i, W_i) -> (padded [N, [C,] H, W] with every
    tensor at the top-left and pad_value elsewhere, sizes = [(H_i, W_i) or (0, 0)]);
    H, W = the max extents, rounded up to a multiple of snap_size_to when given."""
    entries = list(packed_images)
    live = [t for t in entries if t is not None]
    if not live:
        raise ValueError("pad_packed_images: the sequence holds no tensor (all entries are None)")
    _check_ranks(live)
    h, w = _padded_extent(live, snap_size_to)
    sizes = [(0, 0) if t is None else t.shape[-2:] for t in entries]
    if live[0].is_cuda:
        from .. import _ops
        return _ops.pad_images(entries, h, w, pad_value), sizes
    blank = live[0].new_full(live[0].shape[:-2] + (h, w), pad_value)
    padded = torch.stack([blank if t is None else
                          F.pad(t, (0, w - t.shape[-1], 0, h - t.shape[-2]), value=pad_value) for t in entries])
    return padded, sizes


def pack_padded_images(padded_images, sizes):
    """inverse of pad_packed_images: crop each padded image back to its size."""
    return PackedSequence([img[..., :int(hw[0]), :int(hw[1])].contiguous() for img, hw in zip(padded_images, sizes)])
