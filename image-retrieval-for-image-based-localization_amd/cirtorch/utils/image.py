"""Per-channel image normalisation, ``(x - mean_c) / std_c`` (reference
``cirtorch/utils/image.py:86-127``, called by ``random_augmentation.py:174``).

On the extraction path this never runs: the engine's stem kernel normalises the
pixels it loads (``rr_stem_conv_pool*``, ``rr_image_to_nhwc``).  This is the
standalone utility for callers of the reference's name.  Statistics may be a
scalar, one value per channel ``[C]`` or one per image and channel ``[N, C]``
(the latter for ``[..., N, C, H, W]`` inputs: N is dimension -4);
channels are dimension -3 of ``[..., C, H, W]`` (for the 4-D batches the
reference takes, the same elements and the same two IEEE operations per element
as its ``view(N, C, -1)`` form, so the results are bit-identical)."""

import torch


def _stat(value, data, what):
    """mean / std -> a tensor that broadcasts against ``data`` per channel"""
    if not torch.is_tensor(value) and not isinstance(value, (list, tuple, float, int)):
        raise TypeError("%s should be a tensor, a sequence or a number, got %s" % (what, type(value).__name__))
    t = torch.as_tensor(value, dtype=data.dtype, device=data.device)
    if t.dim() == 0 or t.numel() == 1:
        return t.reshape(())
    channels = data.shape[-3]
    if t.dim() == 1:
        if t.shape[0] != channels:
            raise ValueError("%s has %d values for %d channels (shapes %s, %s)"
                             % (what, t.shape[0], channels, tuple(t.shape), tuple(data.shape)))
        return t.reshape(channels, 1, 1)
    if t.dim() == 2 and data.dim() >= 4 and tuple(t.shape) == tuple(data.shape[-4:-2]):
        return t.reshape(t.shape[0], t.shape[1], 1, 1)
    raise ValueError("%s of shape %s does not match images of shape %s" % (what, tuple(t.shape), tuple(data.shape)))


def normalize(data, mean, std):
    """(data - mean) / std per channel; ``data`` is a [..., C, H, W] tensor."""
    if not torch.is_tensor(data):
        raise TypeError("data should be a tensor, got %s" % type(data).__name__)
    if data.dim() < 3:
        raise ValueError("normalize expects [..., C, H, W] images, got shape %s" % (tuple(data.shape),))
    return torch.sub(data, _stat(mean, data, "mean")).div_(_stat(std, data, "std"))
