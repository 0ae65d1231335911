"""Seeded synthetic inputs (TEST INFRASTRUCTURE ONLY — see oracle/__init__.py).

All inputs are produced by numpy's PCG64 generator from a fixed seed per role,
so the golden generator (build container) and the tests (GPU box) regenerate
bit-identical arrays instead of storing them.

Roles and shapes follow BASELINE.md §2 "Inputs":
  images  : U[0,1) pixels, NCHW float32 (normalised later, like the reference
            ``cirtorch/utils/image.py:86-127`` called from
            ``datasets/augmentation/random_augmentation.py:174``)
  db / q  : N(0,1) rows, L2-normalised, float32, row-major [n][D]
            (the reference stores D x n columns, ``scripts/test.py:243-248``;
            our [n][D] row-major array is exactly that matrix's transpose view)
"""

import numpy as np

SEED_IMAGES = 0x1A2B0001
SEED_DB = 0x1A2B0002
SEED_QUERIES = 0x1A2B0003
SEED_WEIGHTS = 0x1A2B0004

IMAGENET_MEAN = [0.485, 0.456, 0.406]
IMAGENET_STD = [0.229, 0.224, 0.225]


def rng(seed):
    return np.random.Generator(np.random.PCG64(seed))


def images(n, h, w, seed=SEED_IMAGES):
    """n x 3 x h x w float32 in [0,1)."""
    return rng(seed).random((n, 3, h, w), dtype=np.float32)


def _lerp_matrix_idx(n_out, n_in):
    """Bilinear (align-corners) source indices / weights for 1-D upsampling."""
    pos = np.linspace(0.0, n_in - 1.0, n_out)
    i0 = np.minimum(np.floor(pos).astype(np.int64), n_in - 2)
    return i0, (pos - i0)


def structured_images(n, h, w, seed=SEED_IMAGES, grid=(6, 8), noise=0.2):
    """n x 3 x h x w float32 in [0,1): a random low-resolution colour field,
    bilinearly upsampled (elementwise numpy, bit-reproducible), plus pixel noise.
    Unlike iid noise, images differ in their large-scale statistics, so the
    random-weight extractor yields distinguishable descriptors."""
    r = rng(seed)
    g = r.random((n, 3, grid[0], grid[1]))
    iy, fy = _lerp_matrix_idx(h, grid[0])
    ix, fx = _lerp_matrix_idx(w, grid[1])
    rows = g[:, :, iy, :] * (1 - fy)[None, None, :, None] + g[:, :, iy + 1, :] * fy[None, None, :, None]
    up = rows[:, :, :, ix] * (1 - fx) + rows[:, :, :, ix + 1] * fx
    pix = r.random((n, 3, h, w))
    return np.ascontiguousarray(((1.0 - noise) * up + noise * pix).astype(np.float32))


def unit_rows(n, d, seed):
    """n x d float32 rows ~ N(0,1), each L2-normalised (float64 norm, then cast)."""
    x = rng(seed).standard_normal((n, d), dtype=np.float32)
    nrm = np.sqrt((x.astype(np.float64) ** 2).sum(axis=1, keepdims=True))
    return (x / nrm).astype(np.float32)


def database(n, d=2048, seed=SEED_DB):
    return unit_rows(n, d, seed)


def queries(q, d=2048, seed=SEED_QUERIES):
    return unit_rows(q, d, seed)
