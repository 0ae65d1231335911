"""Upstream ``cirtorch.datasets.datahelpers`` names used by ``scripts/test.py:13,196``
(in-tree twin: ``cirtorch/datasets/globalFeatures/misc.py:17-30``)."""

import os


def cid2filename(cid, prefix):
    return os.path.join(prefix, cid[-2:], cid[-4:-2], cid[-6:-4], cid)


def default_loader(path):
    from PIL import Image
    with open(path, "rb") as f:
        return Image.open(f).convert("RGB")


def imresize(img, imsize):
    from PIL import Image
    img.thumbnail((imsize, imsize), Image.LANCZOS)
    return img
