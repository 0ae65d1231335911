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


def map_gnd(nq, ndb, seed):
    """roxford-shaped synthetic ground truth: per query easy / hard / junk lists
    (``ParisOxfordEval.py:116-195`` reads exactly these keys) and a bbx."""
    r = rng(seed)
    gnd = []
    for _ in range(nq):
        perm = r.permutation(ndb)
        ne, nh, nj = r.integers(0, 40), r.integers(0, 30), r.integers(0, 10)
        gnd.append({"easy": perm[:ne], "hard": perm[ne:ne + nh], "junk": perm[ne + nh:ne + nh + nj],
                    "bbx": r.random(4)})
    return gnd


def map_problem(nq=70, ndb=4993, d=256):
    """The G5 mAP problem (tests/golden/map.npz): DB rows, query rows, gnd.
    The positives of each query are pulled towards it so the ranking is
    informative.  Returns (db [ndb][d] f32, q [nq][d] f32, gnd list)."""
    db = unit_rows(ndb, d, seed=501)
    qq = unit_rows(nq, d, seed=502)
    gnd = map_gnd(nq, ndb, seed=503)
    r = rng(504)
    for i, g in enumerate(gnd):
        for j in np.concatenate([g["easy"], g["hard"]])[: r.integers(0, 20)]:
            db[j] = db[j] + 0.3 * qq[i]
    return db, qq, gnd


def local_head_problem(b, c, e, npts, seed):
    """Keypoints (normalised (x, y), some outside [-1, 1]) and localHead Linear
    weights for a [b, c, h, w] map: (kpts [b][npts][2], w [e][c], bias [e])."""
    r = rng(seed)
    kp = (r.random((b, npts, 2)) * 2.2 - 1.1).astype(np.float32)
    w = (r.standard_normal((e, c)) * (1.0 / c) ** 0.5).astype(np.float32)
    bias = (r.standard_normal(e) * 0.05).astype(np.float32)
    return kp, w, bias


def nn_descriptors(n1, n2, d, seed):
    """Two unit-descriptor sets for the mutual-NN matcher: desc2 holds noisy
    copies of part of desc1 (true matches), unrelated rows, and exact duplicate
    rows (distance ties -> np.argmin takes the lower index)."""
    r = rng(seed)
    d1 = r.standard_normal((n1, d)).astype(np.float32)
    d1 /= np.linalg.norm(d1, axis=1, keepdims=True)
    m = min(n1, n2) // 2
    d2 = r.standard_normal((n2, d)).astype(np.float32)
    d2[:m] = d1[r.permutation(n1)[:m]] + 0.05 * r.standard_normal((m, d)).astype(np.float32)
    d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
    d2[m + 1] = d2[m]          # duplicate row in desc2 (tie for the nearest of some desc1 rows)
    d1[-1] = d1[-2]            # duplicate row in desc1
    return d1.astype(np.float32), d2.astype(np.float32)


def transform_images():
    """(w, h, bbx) cases for ISSTestTransform (generic/transform.py:81-130) and
    their uint8 RGB pixels (h x w x 3), deterministic."""
    cases = [(50, 40, None), (200, 100, None), (90, 300, None), (64, 64, None), (120, 80, None),
             (160, 120, (10, 20, 150, 100)), (33, 97, None), (300, 299, (0, 0, 200, 120))]
    r = rng(901)
    return [(w, h, bbx, r.integers(0, 256, (h, w, 3), dtype=np.uint8)) for (w, h, bbx) in cases]
