"""Eval-time image transform of the in-tree loaders: ``ISSTestTransform``
(reference ``cirtorch/datasets/generic/transform.py:81-130``), used by the
query and database loaders of ``scripts/train_globalF.py:642-644,685-687``.

Semantics kept exactly, including the ``window`` quirk: the configs pass
``random_scale = [0.8, 1.2]`` (``global_config.ini:127``) and the reference
computes ``shortest_size * random_scale`` — list repetition in Python — so
``window == [0.8, 1.2]`` and every image whose short side is > 1 px is
rescaled to ``shortest_size`` (then capped so the long side is at most
``longest_max_size``).  Sizes are truncated with ``int(dim * scale)`` and the
resize is PIL ``BILINEAR``, as in the reference.

``__call__`` returns ``dict(img=float32 CHW tensor in [0, 1])`` (torchvision
``to_tensor``).  ``pixels(img, bbx)`` returns the same image as a uint8 CHW
tensor — the engine's stem reads it as x / 255 bit-identically, so a decoded
image crosses PCIe at 1 B per channel (``GF_net.extract_vectors``).
"""

import numpy as np
import torch


class ISSTestTransform:
    def __init__(self, shortest_size=None, longest_max_size=None, random_scale=None):
        self.shortest_size = shortest_size
        self.longest_max_size = longest_max_size
        self.random_scale = random_scale

    def _adjusted_scale(self, in_width, in_height):
        min_size = min(in_width, in_height)
        max_size = max(in_width, in_height)
        window = self.shortest_size * self.random_scale    # list * int: repetition (see module doc)
        scale = 1.0
        if int(min_size) > window[1] or int(min_size) < window[0]:
            scale = self.shortest_size / min_size
        if int(max_size * scale) > self.longest_max_size:
            scale = self.longest_max_size / max_size
        return scale

    def output_size(self, width, height):
        """(width, height) of the transformed image for an input of that size."""
        if not self.shortest_size:
            return width, height
        scale = self._adjusted_scale(width, height)
        return tuple(int(dim * scale) for dim in (width, height))

    def _resized(self, img, bbx):
        from PIL import Image
        if bbx is not None:
            img = img.crop(box=bbx)
        if self.shortest_size:
            out_size = self.output_size(img.size[0], img.size[1])
            img = img.resize(out_size, resample=Image.BILINEAR)
        return img

    def pixels(self, img, bbx=None):
        """PIL RGB image -> uint8 [3, H, W] tensor of the transformed image."""
        a = np.asarray(self._resized(img, bbx).convert("RGB"), dtype=np.uint8)
        return torch.from_numpy(np.ascontiguousarray(a.transpose(2, 0, 1)))

    def __call__(self, img, bbx=None):
        px = self.pixels(img, bbx)
        return dict(img=px.float().div(255))
