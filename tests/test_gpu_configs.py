"""BASELINE configs 3, 4 and 5 on the GPU at their workload sizes, pinned by
fixtures the reference produced (tests/golden/make_golden.py):

  config 3  R101-GeM multi-scale x0.5/1/2 at 3x768x1024  (r101ms.npz)
  config 4  roxford-shaped 70 x 4993 ranking + E/M/H mAP (map.npz), and the
            R50 + whitening + post-hoc Lw flow at 768x1024 through the product
  config 5  R152 at 3x768x1024 (fp32 / fp16) + the local head on its stage map
            (r152.npz), mutual-NN matcher vs the reference nn_matcher
            (nnmatch.npz), 10M x 2048 fp16-screened kNN (size-independent
            properties + an exact CPU oracle for two queries)
"""

import numpy as np
import pytest
import torch

from conftest import cosines, golden
from test_gpu_extract import BF16_COS, FP16_COS, FP32_COS, normalized, product_net

pytestmark = pytest.mark.gpu


# ----------------------------------------------------------------------------- config 3
@pytest.mark.parametrize("precision", ["fp32", "fp16", "bf16"])
def test_config3_r101_multiscale_768x1024(cuda, precision):
    """R101 at scales (0.5, 1, 2) of 3x768x1024 (384x512, 768x1024, 1536x2048
    pyramid levels, GF_net.py:20-40,74-92) vs the reference run."""
    from oracle import data
    g = golden("r101ms.npz")
    imgs = data.structured_images(int(g["n"]), *[int(v) for v in g["res"]], seed=int(g["seed"]))
    net = product_net("resnet101", g["head_bias"], precision, cuda)
    bar = {"fp32": FP32_COS, "bf16": BF16_COS, "fp16": FP16_COS}[precision]
    x = normalized(imgs, cuda)
    single = net.extract(x).cpu().numpy()
    ms = net.extract(x, scales=(0.5, 1, 2)).cpu().numpy()
    cs, cm = cosines(single, g["desc_s1"]), cosines(ms, g["desc_s0.5_1_2"])
    print(precision, "r101 768x1024 cos single", cs, "multi-scale", cm)
    assert cs.min() >= bar and cm.min() >= bar
    # mean of unit vectors, not re-normalised (GF_net.py:84-85)
    np.testing.assert_allclose(np.linalg.norm(ms, axis=0), np.linalg.norm(g["desc_s0.5_1_2"], axis=0), rtol=1e-3)


def test_config3_batched_pyramid_equals_per_image(cuda):
    """A same-size batch through the multi-scale path (one batched resize per
    scale) gives the same descriptors as per-image calls."""
    from cirtorch.models.GF_net import make_net
    from cirtorch.models.init import random_init_
    net = make_net("resnet101", precision="fp16", mean=[0.485, 0.456, 0.406], std=[0.229, 0.224, 0.225])
    random_init_(net, seed=2)
    net = net.to(cuda).eval()
    g = torch.Generator(device=cuda).manual_seed(11)
    x = torch.rand((4, 3, 192, 256), generator=g, device=cuda)
    batched = net.extract(x, scales=(0.5, 1, 2))
    single = torch.cat([net.extract(x[i:i + 1], scales=(0.5, 1, 2)) for i in range(4)], dim=1)
    assert cosines(batched.cpu().numpy(), single.cpu().numpy()).min() > 1 - 1e-6


# ----------------------------------------------------------------------------- config 5
@pytest.mark.parametrize("precision", ["fp32", "fp16"])
def test_config5_r152_768x1024_and_local_head(cuda, precision):
    """R152 at 3x768x1024 vs the reference, then the local head (localHead,
    local_head.py:19-71) on the product's mod3 stage map vs the reference
    head applied to the reference mod3 map."""
    from cirtorch.modules.heads.local_head import localHead
    from oracle import data
    g = golden("r152.npz")
    imgs = data.structured_images(int(g["n"]), *[int(v) for v in g["res"]], seed=int(g["seed"]))
    net = product_net("resnet152", g["head_bias"], precision, cuda)
    x = normalized(imgs, cuda)
    got = net.extract(x).cpu().numpy()
    cos = cosines(got, g["desc_s1"])
    print(precision, "r152 768x1024 cos", cos)
    assert cos.min() >= (FP32_COS if precision == "fp32" else FP16_COS)
    with torch.no_grad():
        fm = net.body(x[0][None], normalize=None)[str(g["local_stage"])]
    npts, e, seed = int(g["local_npts"]), int(g["local_e"]), int(g["local_seed"])
    kp, lw, lb = data.local_head_problem(1, fm.shape[1], e, npts, seed)
    head = localHead(fm.shape[1], e).to(cuda)
    head.load_state_dict({"whiten.weight": torch.from_numpy(lw), "whiten.bias": torch.from_numpy(lb)})
    d = head(fm, torch.from_numpy(kp).to(cuda)).cpu().numpy()
    ref = g["local_desc"]
    c = (d * ref).sum(-1) / (np.linalg.norm(d, axis=-1) * np.linalg.norm(ref, axis=-1))
    print(precision, "r152 mod3 local descriptors cos min", c.min())
    assert c.min() >= (1 - 1e-4 if precision == "fp32" else 1 - 2e-3)


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_mutual_nn_vs_reference_nn_matcher(cuda, tag):
    """cirtorch.search.mutual_nn == the reference HPatchesEval.nn_matcher on the
    L2 distance matrix (fixture from the reference function itself), including
    duplicate-row ties (np.argmin -> lower index)."""
    from cirtorch.search import mutual_nn
    from oracle import data
    g = golden("nnmatch.npz")
    n1, n2, d, seed = [int(v) for v in g["shape_" + tag]]
    d1, d2 = data.nn_descriptors(n1, n2, d, seed)
    got = mutual_nn(torch.from_numpy(d1).to(cuda), torch.from_numpy(d2).to(cuda)).cpu().numpy()
    np.testing.assert_array_equal(got, g["match_" + tag])


def _exact_topk_chunked(db, q_np, k, rows_per_chunk=500_000, margin=1e-5):
    """CPU oracle over a GPU-resident database too large to hold in float64:
    per chunk, float32 scores on the host pick every row within `margin` of the
    chunk's k-th best (fp32 dot error for unit 2048-d rows is ~1e-7 << margin),
    then those rows are re-scored exactly in float64 and ordered by (score desc,
    index asc)."""
    n = db.shape[0]
    cand_s, cand_i = [], []
    for r0 in range(0, n, rows_per_chunk):
        chunk = db[r0:r0 + rows_per_chunk].cpu().numpy()
        s32 = q_np @ chunk.T                                  # [Q, rows]
        for j in range(q_np.shape[0]):
            kth = np.partition(s32[j], -k)[-k]
            rows = np.nonzero(s32[j] >= kth - margin)[0]
            s64 = chunk[rows].astype(np.float64) @ q_np[j].astype(np.float64)
            cand_s.append((j, s64))
            cand_i.append((j, rows + r0))
        del chunk, s32
    out_s, out_i = [], []
    for j in range(q_np.shape[0]):
        s = np.concatenate([c for (jj, c) in cand_s if jj == j])
        i = np.concatenate([c for (jj, c) in cand_i if jj == j])
        order = np.lexsort((i, -s))[:k]
        out_s.append(s[order])
        out_i.append(i[order])
    return np.stack(out_s), np.stack(out_i)


def test_config5_knn_10m_fp16(cuda):
    """Config 5 database at full size: 10M x 2048 rows (counter-hash generator,
    82 GB float32 + 41 GB fp16 screening copy on one GPU), 64 queries, k = 100,
    fp16 screening + exact float64 re-score.  Properties: self-retrieval with
    score 1; results sorted; two queries equal to the exact CPU oracle over all
    10M rows; a 4-shard search + merge is bit-identical to the single search."""
    from cirtorch import _ops
    from cirtorch.search import KnnIndex, merge_topk
    n, d, q, k = 10_000_000, 2048, 64, 100
    db = _ops.fill_unit_rows(n, d, seed=0x10D5EED, device=cuda)
    qq = _ops.fill_unit_rows(q, d, seed=0x10E5EED, device=cuda)
    self_rows = [0, 4_999_999, 7_654_321, n - 1]
    qq[:4] = db[self_rows]
    index = KnnIndex(db, "fp16")
    s, i = index.search(qq, k)
    s_np, i_np = s.cpu().numpy(), i.cpu().numpy()
    assert i_np[:4, 0].tolist() == self_rows
    assert np.abs(s_np[:4, 0] - 1.0).max() < 1e-6
    assert (np.diff(s_np, axis=1) <= 0).all()
    ref_s, ref_i = _exact_topk_chunked(db, qq[4:6].cpu().numpy(), k)
    np.testing.assert_array_equal(i_np[4:6], ref_i)
    np.testing.assert_allclose(s_np[4:6], ref_s, rtol=0, atol=1e-12)
    del index
    torch.cuda.empty_cache()
    R, per = 4, n // 4
    ss, ii = [], []
    for r in range(R):
        sh = KnnIndex(db[r * per:(r + 1) * per], "fp16", idx_offset=r * per)
        sh_s, sh_i = sh.search(qq, k)
        ss.append(sh_s)
        ii.append(sh_i)
        del sh
    sm, im = merge_topk(torch.stack(ss), torch.stack(ii), k)
    assert torch.equal(im, i) and torch.equal(sm, s)


# ----------------------------------------------------------------------------- config 4
def test_config4_map_problem_ranked_on_gpu(cuda):
    """The G5 problem (70 queries x 4993 DB, roxford-shaped gnd) ranked on the
    GPU: full ranks equal the exact (float64, ties -> lower index) order, and
    E / M / H mAP, per-query AP and mP@k equal the reference's exactly.  The
    reference's own fp32 np.argsort differs from the exact order only by
    swaps of near-tied neighbours (checked), none of which moves an mAP."""
    from cirtorch.search import rank
    from cirtorch.utils.evaluation.ParisOxfordEval import compute_map, compute_map_and_print
    from oracle import data
    from test_host_round2 import _gnd
    g = golden("map.npz")
    db, qq, gnd = data.map_problem()
    ranks = rank(torch.from_numpy(db.T.copy()).to(cuda), torch.from_numpy(qq.T.copy()).to(cuda))
    r_np = ranks.cpu().numpy()
    s64 = qq.astype(np.float64) @ db.astype(np.float64).T
    exact = np.stack([np.lexsort((np.arange(db.shape[0]), -s64[j])) for j in range(qq.shape[0])], axis=1)
    np.testing.assert_array_equal(r_np, exact)
    diff = np.nonzero(r_np != g["ranks"])
    gaps = np.abs(s64[diff[1], r_np[diff]] - s64[diff[1], g["ranks"][diff]])
    assert gaps.size == 0 or gaps.max() < 1e-6, gaps.max()
    logs = []
    score = compute_map_and_print("roxford5k", ranks, _gnd(g), lambda *a: logs.append(a))
    assert score["mAP"] == float(g["score_mAP"])
    for proto in ("E", "M", "H"):
        assert score["map" + proto] == float(g["map" + proto])
    m, aps, pr, _ = compute_map(ranks, [{"ok": np.concatenate([q["easy"], q["hard"]]), "junk": q["junk"]}
                                        for q in gnd], [1, 5, 10])
    assert m == float(g["old_map"])


def _structured_images_gpu(n, h, w, gen, grid=(6, 8), noise=0.2):
    """GPU analogue of oracle.data.structured_images (test input generator):
    a random low-resolution colour field, bilinearly upsampled, plus noise —
    images that differ in their large-scale statistics, so the extractor's
    descriptors are spread (not near-collinear as for iid noise)."""
    field = torch.rand((n, 3) + grid, generator=gen, device=gen.device)
    up = torch.nn.functional.interpolate(field, size=(h, w), mode="bilinear", align_corners=True)
    return (1.0 - noise) * up + noise * torch.rand((n, 3, h, w), generator=gen, device=gen.device)


def test_config4_r50_whiten_70x4993_768x1024(cuda):
    """Config 4 flow through the product at its shape: R50-GeM + head whitening
    (fp16; reference-layout weights, centred head) on 4993 DB + 70 query images
    at 3x768x1024 (batched extraction), post-hoc Lw learned on the host
    (whitenlearn, scripts/test.py:205) and applied on the GPU (whitenapply,
    :253-254), full GPU ranks, revisited mAP.  Ranks equal the exact float64
    order of the same descriptors and mAP equals the oracle's compute_map on
    them (bit-exact); whitenapply agrees with the reference formula."""
    from cirtorch.search import rank
    from cirtorch.utils.evaluation.ParisOxfordEval import compute_map_and_print
    from cirtorch.utils.whiten import whitenapply, whitenlearn
    from oracle import data, ops
    ndb, nq, B = 4993, 70, 128
    g = golden("r50.npz")
    net = product_net("resnet50", g["head_bias"], "fp16", cuda)
    from cirtorch.models.GF_net import Normalize
    net.augment = Normalize()    # ImageNet mean / std fused into the stem
    gen = torch.Generator(device=cuda).manual_seed(44)
    vecs = torch.empty((2048, ndb + nq), device=cuda)
    for c0 in range(0, ndb + nq, B):
        nb = min(B, ndb + nq - c0)
        vecs[:, c0:c0 + nb] = net.extract(_structured_images_gpu(nb, 768, 1024, gen))
    torch.cuda.synchronize()
    assert torch.isfinite(vecs).all()
    qv, dv = vecs[:, ndb:], vecs[:, :ndb]
    cosmat = (dv[:, :200].t() @ dv[:, :200]).cpu().numpy()
    print("config4 descriptor pairwise cosine range", cosmat[np.triu_indices(200, 1)].min(),
          cosmat[np.triu_indices(200, 1)].max())
    r = data.rng(45)
    qidx = r.integers(0, ndb, 3000)
    pidx = (qidx + r.integers(1, 7, 3000)) % ndb
    X = dv.double().cpu().numpy()
    m, P = whitenlearn(X, qidx, pidx)
    dw = whitenapply(dv, m, P)
    qw = whitenapply(qv, m, P)
    ranks = rank(dw, qw)
    gnd = data.map_gnd(nq, ndb, seed=46)
    score = compute_map_and_print("roxford5k", ranks, gnd, lambda *a: None)
    dn, qn = dw.cpu().numpy().T, qw.cpu().numpy().T
    s64 = qn.astype(np.float64) @ dn.astype(np.float64).T
    exact = np.stack([np.lexsort((np.arange(ndb), -s64[j])) for j in range(nq)], axis=1)
    np.testing.assert_array_equal(ranks.cpu().numpy(), exact)
    ref = ops.compute_map_revisited(exact, gnd)
    for proto in ("E", "M", "H"):
        assert score["map" + proto] == ref["map" + proto]
    # GPU whitenapply (f64 MFMA) vs the reference formula in float64 (whiten.py:4-12)
    ref_w = ops.whitenapply(X[:, :64], m, P)
    got_w = dw[:, :64].double().cpu().numpy()
    cw = cosines(got_w, ref_w)
    print("config4 whitenapply cos min", cw.min(), "max |d|", np.abs(got_w - ref_w).max())
    assert cw.min() >= 1 - 1e-12 and np.abs(got_w - ref_w).max() < 1e-7


# ----------------------------------------------------------------------------- GeM exponent
def test_gem_exponent_read_on_device(cuda):
    """The learnable GeM p is read by the kernel from device memory: two nets
    with different p in one process, an in-place p.data.fill_ and a
    load_state_dict are all seen by the next forward."""
    from cirtorch.modules.heads.global_head import globalHead
    from oracle import ops
    x = torch.rand(2, 64, 5, 7, device=cuda) + 0.05
    heads = []
    for p in (3.0, 2.5):
        h = globalHead(pooling={"name": "GeM", "params": {"p": p, "eps": 1e-6}},
                       normal={"name": "L2N", "params": {}}, dim=64).to(cuda)
        heads.append(h)
    for h, p in zip(heads, (3.0, 2.5)):
        ref = ops.gem(x.cpu(), p).reshape(2, 64)
        torch.testing.assert_close(h.pooled(x).cpu(), ref, rtol=2e-5, atol=1e-6)
    h = heads[0]
    h.pool.p.data.fill_(2.0)
    torch.testing.assert_close(h.pooled(x).cpu(), ops.gem(x.cpu(), 2.0).reshape(2, 64), rtol=2e-5, atol=1e-6)
    sd = h.state_dict()
    sd["pool.p"] = torch.tensor([4.0])
    h.load_state_dict(sd)
    torch.testing.assert_close(h.pooled(x).cpu(), ops.gem(x.cpu(), 4.0).reshape(2, 64), rtol=2e-5, atol=1e-6)
    # graph capture of a forward that reads p on device, replayed after p changes
    from cirtorch.utils.graph import GraphedForward
    gf = GraphedForward(lambda t: h.pooled(t), x)
    h.pool.p.data.fill_(3.0)
    torch.testing.assert_close(gf(x).cpu(), ops.gem(x.cpu(), 3.0).reshape(2, 64), rtol=2e-5, atol=1e-6)
