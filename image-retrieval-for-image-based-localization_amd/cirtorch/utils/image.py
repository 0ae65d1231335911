"""normalize (reference ``cirtorch/utils/image.py:86-127``).  On the extraction
path normalisation is fused into the first engine kernel (``rr_image_to_nhwc``);
this function is the standalone utility with the reference's semantics."""

import torch


def normalize(data, mean, std):
    shape = data.shape
    if not isinstance(data, torch.Tensor):
        raise TypeError("data should be a tensor. Got {}".format(type(data)))
    mean = torch.as_tensor(mean, device=data.device, dtype=data.dtype)
    std = torch.as_tensor(std, device=data.device, dtype=data.dtype)
    if mean.shape and mean.shape[0] != 1 and mean.shape[0] != data.shape[-3]:
        raise ValueError("mean length and number of channels do not match")
    if std.shape and std.shape[0] != 1 and std.shape[0] != data.shape[-3]:
        raise ValueError("std length and number of channels do not match")
    if mean.shape:
        mean = mean[..., :, None]
    if std.shape:
        std = std[..., :, None]
    out = (data.view(shape[0], shape[1], -1) - mean) / std
    return out.view(shape)
