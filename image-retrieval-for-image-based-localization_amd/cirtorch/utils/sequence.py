"""pad_packed_images / pack_padded_images (reference ``cirtorch/utils/sequence.py:4-79``).
Pure data movement (device copies into one padded batch buffer)."""

from .parallel import PackedSequence


def pad_packed_images(packed_images, pad_value=0.0, snap_size_to=None):
    if packed_images.all_none:
        raise ValueError("at least one image in packed_images should be non-None")
    reference_img = next(img for img in packed_images if img is not None)
    max_size = list(reference_img.shape[-2:])
    ndims = len(reference_img.shape)
    chn = reference_img.shape[0] if ndims == 3 else 0
    for img in packed_images:
        if img is not None:
            if len(img.shape) not in (2, 3):
                raise ValueError("The input sequence must contain 2D or 3D tensors")
            if len(img.shape) != ndims:
                raise ValueError("All tensors in the input sequence must have the same number of dimensions")
            if ndims == 3 and img.shape[0] != chn:
                raise ValueError("3D tensors must all have the same number of channels")
            max_size = [max(s1, s2) for s1, s2 in zip(max_size, img.shape[-2:])]
    if snap_size_to is not None:
        max_size = [(s + snap_size_to - 1) // snap_size_to * snap_size_to for s in max_size]
    shape = [len(packed_images), chn] + max_size if ndims == 3 else [len(packed_images)] + max_size
    same = all(img is not None and list(img.shape[-2:]) == max_size for img in packed_images)
    if same and ndims == 3:
        import torch
        padded = torch.stack(list(packed_images), 0)
        return padded, [img.shape[1:] for img in packed_images]
    padded = reference_img.new_full(shape, pad_value)
    sizes = []
    for i, t in enumerate(packed_images):
        if t is not None:
            if ndims == 3:
                padded[i, :, :t.shape[1], :t.shape[2]] = t
                sizes.append(t.shape[1:])
            else:
                padded[i, :t.shape[0], :t.shape[1]] = t
                sizes.append(t.shape)
        else:
            sizes.append((0, 0))
    return padded, sizes


def pack_padded_images(padded_images, sizes):
    images = []
    for img, size in zip(padded_images, sizes):
        if img.dim() == 2:
            images.append(img[:int(size[0]), :int(size[1])])
        else:
            images.append(img[:, :int(size[0]), :int(size[1])])
    return PackedSequence([img.contiguous() for img in images])
