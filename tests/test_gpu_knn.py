"""kNN parity on the GPU: top-k indices identical to the reference
(np.dot + np.argsort, tests/golden/knn.npz), scores within fp32 rounding of
the reference's, full ranks identical to np.argsort for mAP, shard merge
bit-identical to the single-GPU result."""


import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("precision", ["fp32", "bf16", "fp16", "int8"])
@pytest.mark.parametrize("tag", ["4k", "100k"])
def test_knn_vs_reference_golden(cuda, precision, tag):
    from cirtorch.search import KnnIndex
    from oracle import data
    g = golden("knn.npz")
    n, q, k = (int(v) for v in g["shape_" + tag])
    db = torch.from_numpy(data.database(n)).to(cuda)
    qq = torch.from_numpy(data.queries(q, seed=int(g["qseed_" + tag]))).to(cuda)
    s, i = KnnIndex(db, precision).search(qq, k)
    np.testing.assert_array_equal(i.cpu().numpy(), g["idx_" + tag])
    np.testing.assert_allclose(s.cpu().numpy(), g["score_" + tag], rtol=0, atol=2e-7)


def test_knn_matches_exact_oracle_random_shapes(cuda):
    from cirtorch.search import KnnIndex
    from oracle import data, ops
    for n, q, d, k in ((1, 3, 64, 1), (37, 5, 128, 10), (16384, 3, 256, 64), (40000, 9, 512, 100), (70001, 2, 64, 7)):
        db = data.unit_rows(n, d, seed=n)
        qq = data.unit_rows(q, d, seed=n + 1)
        kk = min(k, n)
        ref_s, ref_i = ops.topk_exact(db, qq, kk)
        for prec in ("fp32", "bf16", "fp16", "int8"):
            s, i = KnnIndex(torch.from_numpy(db).to(cuda), prec).search(torch.from_numpy(qq).to(cuda), kk)
            np.testing.assert_array_equal(i.cpu().numpy(), ref_i, err_msg="%s %s" % (prec, (n, q, d, k)))
            np.testing.assert_allclose(s.cpu().numpy(), ref_s, rtol=0, atol=1e-12)


def test_knn_ties_lower_index_first(cuda):
    """Duplicated rows give exactly equal scores: ties resolve to the lower index."""
    from cirtorch.search import KnnIndex
    from oracle import data, ops
    base = data.unit_rows(50, 128, seed=3)
    db = np.concatenate([base, base, base[:10]], 0)  # rows i, i+50 identical
    qq = data.unit_rows(4, 128, seed=4)
    ref_s, ref_i = ops.topk_exact(db, qq, 20)
    s, i = KnnIndex(torch.from_numpy(db).to(cuda), "fp32").search(torch.from_numpy(qq).to(cuda), 20)
    np.testing.assert_array_equal(i.cpu().numpy(), ref_i)


def test_knn_running_screen_across_chunks(cuda):
    """The chunk select drops keys below a query's running threshold (the best
    K-th screening key of earlier chunks).  Databases that stress it, over
    several 16384-row chunks: blocks duplicated across chunks (ties at the
    threshold, lower index must win), rows whose scores rise chunk after chunk
    (threshold overtaken every chunk), and all-equal rows (every key ties)."""
    from cirtorch.search import KnnIndex
    from oracle import data, ops
    d = 256
    base = data.unit_rows(20000, d, seed=41)
    qq = data.unit_rows(5, d, seed=42)
    dup = np.concatenate([base, base, base[:9000]], 0)                     # 49000 rows, 3 chunks+
    # rising: row i = normalize(q0 * t_i + noise), t_i increasing with i
    t = np.linspace(0.0, 1.0, 50000, dtype=np.float32)[:, None]
    rise = qq[:1] * t + data.unit_rows(50000, d, seed=43)
    rise = (rise / np.linalg.norm(rise, axis=1, keepdims=True)).astype(np.float32)
    same = np.repeat(base[:1], 40000, 0)
    for name, db in (("dup", dup), ("rise", rise), ("same", same)):
        ref_s, ref_i = ops.topk_exact(db, qq, 100)
        for prec in ("fp32", "bf16", "fp16", "int8"):
            s, i = KnnIndex(torch.from_numpy(db).to(cuda), prec).search(torch.from_numpy(qq).to(cuda), 100)
            np.testing.assert_array_equal(i.cpu().numpy(), ref_i, err_msg="%s %s" % (name, prec))
            np.testing.assert_allclose(s.cpu().numpy(), ref_s, rtol=0, atol=1e-12)


def test_knn_k_larger_than_db(cuda):
    from cirtorch.search import KnnIndex
    from oracle import data
    db = data.unit_rows(5, 64, seed=9)
    qq = data.unit_rows(2, 64, seed=10)
    s, i = KnnIndex(torch.from_numpy(db).to(cuda), "fp32").search(torch.from_numpy(qq).to(cuda), 8)
    i = i.cpu().numpy()
    assert (i[:, 5:] == -1).all() and sorted(i[0, :5].tolist()) == list(range(5))


def test_rank_full_equals_argsort(cuda):
    from cirtorch.search import rank
    g = golden("map.npz")
    from oracle import data
    db = data.unit_rows(700, 256, seed=21)
    qq = data.unit_rows(6, 256, seed=22)
    ranks = rank(torch.from_numpy(db.T.copy()), torch.from_numpy(qq.T.copy())).cpu().numpy()
    ref = np.argsort(-np.dot(db.astype(np.float64), qq.astype(np.float64).T), axis=0, kind="stable")
    np.testing.assert_array_equal(ranks, ref)
    assert g["ranks"].shape == (4993, 70)


def test_topk_merge_equals_single_shard(cuda):
    from cirtorch.search import KnnIndex, merge_topk
    from oracle import data
    n, q, d, k, R = 30000, 6, 256, 50, 4
    db = torch.from_numpy(data.unit_rows(n, d, seed=31)).to(cuda)
    qq = torch.from_numpy(data.unit_rows(q, d, seed=32)).to(cuda)
    s1, i1 = KnnIndex(db, "bf16").search(qq, k)
    per = (n + R - 1) // R
    ss, ii = [], []
    for r in range(R):
        sl = db[r * per:(r + 1) * per]
        s, i = KnnIndex(sl, "bf16", idx_offset=r * per).search(qq, k)
        ss.append(s)
        ii.append(i)
    sm, im = merge_topk(torch.stack(ss), torch.stack(ii), k)
    assert torch.equal(im, i1) and torch.equal(sm, s1)


def test_fp16_screening_copy_and_limits(cuda):
    """The fp16 screening copy is IEEE binary16 round-to-nearest-even (== torch
    .half()); the engine's fp16 score GEMM needs d >= 64 (the C ABI refuses
    less), KnnIndex zero-pads other widths (D = 32, 16, 100, 300) and returns
    the exact results."""
    from cirtorch import _engine as E
    from cirtorch import _ops
    from cirtorch.search import KnnIndex
    from oracle import data, ops
    x = torch.randn(1003, 64, device=cuda) * 3.0
    assert torch.equal(_ops.cast_f16(x), x.half())
    db = torch.from_numpy(data.unit_rows(100, 32, seed=5)).to(cuda)
    with pytest.raises(RuntimeError, match="d >= 64"):
        _ops.knn_topk(db.half(), db, db[:2].half(), db[:2], 3)
    assert E.lib().rr_last_error()
    for d in (32, 16, 100, 300):
        dbn = data.unit_rows(700, d, seed=d)
        qn = data.unit_rows(3, d, seed=d + 1)
        ref_s, ref_i = ops.topk_exact(dbn, qn, 9)
        for prec in ("fp16", "bf16", "fp32"):
            s, i = KnnIndex(torch.from_numpy(dbn).to(cuda), prec).search(torch.from_numpy(qn).to(cuda), 9)
            np.testing.assert_array_equal(i.cpu().numpy(), ref_i, err_msg="%d %s" % (d, prec))
            np.testing.assert_allclose(s.cpu().numpy(), ref_s, rtol=0, atol=1e-12)


@pytest.mark.parametrize("prec", ["bf16", "int8"])
def test_knn_full_size_1m_bench_shape(cuda, prec):
    """BASELINE config size (1M x 2048 database, 128 queries, k = 100, bf16 or
    int8 screening, the uncertified screen) through size-independent properties: a query that is a database
    row retrieves itself first with score 1; two queries checked against the
    CPU oracle over the whole database (chunked exact float64 top-k); a
    4-shard search + merge is bit-identical to the single search."""
    from cirtorch import _ops
    from cirtorch.search import KnnIndex, merge_topk
    from oracle import ops
    n, d, q, k = 1_000_000, 2048, 128, 100
    db = _ops.fill_unit_rows(n, d, seed=0xDB5EED, device=cuda)
    qq = _ops.fill_unit_rows(q, d, seed=0x0E5EED, device=cuda)
    self_rows = [5, 77777, 500000, n - 1]
    qq[:4] = db[self_rows]
    index = KnnIndex(db, prec)
    s, i = index.search(qq, k, verify=False)   # the raw screen; the certified mode: next test
    i_np, s_np = i.cpu().numpy(), s.cpu().numpy()
    assert i_np[:4, 0].tolist() == self_rows
    assert np.abs(s_np[:4, 0] - 1.0).max() < 1e-6
    assert (np.diff(s_np, axis=1) <= 0).all()                      # sorted best first
    # exact oracle for two queries over all 1M rows (chunked)
    db_np, q_np = db.cpu().numpy(), qq[4:6].cpu().numpy()
    cs, ci = [], []
    for r0 in range(0, n, 125_000):
        s_c, i_c = ops.topk_exact(db_np[r0:r0 + 125_000], q_np, k)
        cs.append(s_c)
        ci.append(i_c + r0)
    cs, ci = np.concatenate(cs, 1), np.concatenate(ci, 1)
    for j in range(2):
        order = np.lexsort((ci[j], -cs[j]))[:k]
        np.testing.assert_array_equal(i_np[4 + j], ci[j][order])
        np.testing.assert_allclose(s_np[4 + j], cs[j][order], rtol=0, atol=1e-12)
    # 4 shards + merge == single
    R, per = 4, n // 4
    ss, ii = [], []
    for r in range(R):
        sh_s, sh_i = KnnIndex(db[r * per:(r + 1) * per], prec, idx_offset=r * per).search(qq, k, verify=False)
        ss.append(sh_s)
        ii.append(sh_i)
    sm, im = merge_topk(torch.stack(ss), torch.stack(ii), k)
    assert torch.equal(im, i) and torch.equal(sm, s)


def _exact_topk_1m(db, q_np, k, chunk=125_000):
    """the exact (float64 score desc, index asc) top-k of a few queries over a
    device database, chunk by chunk on the host (oracle ops.topk_exact)"""
    from oracle import ops
    cs, ci = [], []
    for r0 in range(0, db.shape[0], chunk):
        s_c, i_c = ops.topk_exact(db[r0:r0 + chunk].cpu().numpy(), q_np, k)
        cs.append(s_c)
        ci.append(i_c + r0)
    cs, ci = np.concatenate(cs, 1), np.concatenate(ci, 1)
    out_s, out_i = [], []
    for j in range(q_np.shape[0]):
        order = np.lexsort((ci[j], -cs[j]))[:k]
        out_s.append(cs[j][order])
        out_i.append(ci[j][order])
    return np.stack(out_s), np.stack(out_i)


def test_knn_headline_fp16_deferred_q1024(cuda):
    """The bench's headline search mode at its own shape (bench.py run_steps / match):
    1M x 2048 database, Q = 1024 queries per search, k = 100, fp16 screening with the
    deferred certificate, the next batch's search queued before the previous one is
    resolved.  Six queries sit on planted 2048-d near-duplicate clusters (600 rows, noise
    of norm 0.05: scores within ~1e-4 of each other, under the fp16 error bound ~1e-3), so
    the certificate must fire at D = 2048 and the repair run (requeried > 0).  Checks:
    every query bit-identical (indices and float64 scores) to an fp32-screened
    verify=True search; the planted queries + 6 random ones + 2 self-retrievals equal
    the chunked exact host oracle over all 1M rows; the flagged set covers the planted
    queries.  Reference: scripts/test.py:247-248 (np.dot + np.argsort)."""
    from cirtorch import _ops
    from cirtorch.search import KnnIndex
    n, d, q, k = 1_000_000, 2048, 1024, 100
    db = _ops.fill_unit_rows(n, d, seed=0xDB5EED, device=cuda)
    qa = _ops.fill_unit_rows(q, d, seed=0x0E5EED, device=cuda)
    qb = _ops.fill_unit_rows(q, d, seed=0x0E5EEE, device=cuda)
    gen = torch.Generator(device=cuda).manual_seed(77)
    planted = [3, 200, 511, 512, 800, 1023]          # queries of batch a with a cluster
    for c, j in enumerate(planted):
        # noise of norm 0.05 (0.05 / sqrt(d) per element): cosine ~0.9988, the 600 scores
        # within ~1e-4 of each other, far inside the fp16 screening bound
        rows = qa[j] + (0.05 / d ** 0.5) * torch.randn((600, d), generator=gen, device=cuda)
        r0 = 1000 + c * 160_000                      # one cluster per region of the database
        db[r0:r0 + 600] = rows / rows.norm(dim=1, keepdim=True)
    self_rows = [7, 999_999]
    qa[[40, 41]] = db[self_rows]
    index = KnnIndex(db, "fp16")
    # the bench's order: search a, search b, resolve a, resolve b
    sa, ia, pa = index.search(qa, k, verify="deferred")
    sb, ib, pb = index.search(qb, k, verify="deferred")
    na, nb = pa.resolve(), pb.resolve()
    assert na >= len(planted), na                    # the certificate fired at D = 2048
    assert nb <= 16, nb        # random queries certify, bar a rare near-tie at the k-th score
    _, _, unc = index.search_checked(qa, k)
    flagged = set(torch.nonzero(unc).flatten().tolist())
    assert set(planted) <= flagged, (planted, sorted(flagged))
    # every query == the fp32-screened certified search, bit for bit
    ref = KnnIndex(db, "fp32")
    for (s, i, qq) in ((sa, ia, qa), (sb, ib, qb)):
        s32, i32 = ref.search(qq, k, verify=True)
        assert torch.equal(i, i32) and torch.equal(s, s32)
    del ref
    torch.cuda.empty_cache()
    # 14 queries against the exact host oracle over all 1M rows
    pick = planted + [0, 1, 2, 300, 600, 900] + [40, 41]
    ref_s, ref_i = _exact_topk_1m(db, qa[pick].cpu().numpy(), k)
    np.testing.assert_array_equal(ia[pick].cpu().numpy(), ref_i)
    np.testing.assert_allclose(sa[pick].cpu().numpy(), ref_s, rtol=0, atol=1e-12)
    assert ia[40, 0].item() == self_rows[0] and ia[41, 0].item() == self_rows[1]
    # the planted clusters are what the planted queries retrieve
    for c, j in enumerate(planted):
        r0 = 1000 + c * 160_000
        assert ((ia[j] >= r0) & (ia[j] < r0 + 600)).all()


def _fused_vs_slab(cuda, db, qq, k, prec):
    """search with the screening-epilogue pipeline (default) and with every chunk
    through the score slab (RR_TUNE_KNN_FUSED = 0)"""
    from cirtorch import _engine as E
    from cirtorch.search import KnnIndex
    index = KnnIndex(torch.from_numpy(db).to(cuda), prec)
    q = torch.from_numpy(qq).to(cuda)
    s1, i1 = index.search(q, k, verify=False)
    E.check(E.lib().rr_set_tuning(9, 0), "rr_set_tuning")
    try:
        s0, i0 = index.search(q, k, verify=False)
    finally:
        E.lib().rr_set_tuning(9, 1)
    return (s1.cpu().numpy(), i1.cpu().numpy()), (s0.cpu().numpy(), i0.cpu().numpy())


@pytest.mark.parametrize("prec", ["bf16", "fp16", "fp32", "int8"])
def test_knn_fused_screen_stress(cuda, prec):
    """Databases past the 4-chunk prefix (65536 rows), so the screening GEMM
    epilogue runs: (a) scores rising row after row — every screened chunk
    overflows its slot and is rebuilt by the fix-up kernel; (b) blocks of the
    prefix duplicated in screened chunks — equal keys across the two paths,
    the lower index must win; (c) all rows equal — every key ties; (d) 600
    noisy copies of one query planted in one chunk — a single overflowing
    slot (score std 2e-3: above the 16-bit screening resolution at d = 128).
    Every query of every database, through the certified search
    (verify=True: the certificate of the screening dtype, uncertified queries
    re-searched), equals the exact oracle.  The unverified fused and all-slab
    pipelines equal each other and, for the 16/32-bit screens, the oracle;
    unverified int8 is the UNCERTIFIED mode: its recall on the
    planted cluster, below int8's resolution, is only bounded here."""
    from cirtorch.search import KnnIndex
    from oracle import data, ops
    d = 128
    base = data.unit_rows(40000, d, seed=61)
    qq = data.unit_rows(4, d, seed=62)
    t = np.linspace(0.0, 1.0, 180000, dtype=np.float32)[:, None]
    rise = qq[:1] * t + data.unit_rows(180000, d, seed=63)
    rise = (rise / np.linalg.norm(rise, axis=1, keepdims=True)).astype(np.float32)
    dup = np.concatenate([base, base, base, base[:30000]], 0)                     # 150k rows
    same = np.repeat(base[:1], 150000, 0)
    plant = data.unit_rows(170000, d, seed=64)
    plant[140000:140600] = qq[2] + 0.3 * data.unit_rows(600, d, seed=65)   # scores ~0.96 +- 0.02
    plant[140000:140600] /= np.linalg.norm(plant[140000:140600], axis=1, keepdims=True)
    for name, db in (("rise", rise), ("dup", dup), ("same", same), ("plant", plant)):
        ref_s, ref_i = ops.topk_exact(db, qq, 100)
        index = KnnIndex(torch.from_numpy(db).to(cuda), prec)
        sv, iv = index.search(torch.from_numpy(qq).to(cuda), 100, verify=True)
        np.testing.assert_array_equal(iv.cpu().numpy(), ref_i, err_msg="%s %s verified" % (name, prec))
        np.testing.assert_allclose(sv.cpu().numpy(), ref_s, rtol=0, atol=1e-12)
        (s1, i1), (s0, i0) = _fused_vs_slab(cuda, db, qq, 100, prec)
        np.testing.assert_array_equal(i1, i0, err_msg="%s %s fused vs slab" % (name, prec))
        assert np.array_equal(s1, s0)
        if prec == "int8":
            recall = np.mean([len(set(i1[j]) & set(ref_i[j])) / 100.0 for j in range(len(qq))])
            assert recall >= 0.95, (name, recall)
            continue
        np.testing.assert_array_equal(i1, ref_i, err_msg="%s %s fused" % (name, prec))
        np.testing.assert_allclose(s1, ref_s, rtol=0, atol=1e-12)


def test_knn_int8_query_scale_per_row(cuda):
    """int8 queries carry one scale per row (rr_quantize_i8_rows): a query's
    screening copy, and so its top-k, is the same alone and inside a batch of
    queries with very different norms (the whole-tensor scale made a
    query's candidates depend on its batch)."""
    from cirtorch import _ops
    from cirtorch.search import KnnIndex
    from oracle import data
    db = torch.from_numpy(data.unit_rows(90000, 256, seed=81)).to(cuda)
    q = torch.from_numpy(data.unit_rows(6, 256, seed=82)).to(cuda)
    batch = q * torch.tensor([1.0, 40.0, 0.01, 3.0, 1.0, 0.5], device=cuda)[:, None]
    index = KnnIndex(db, "int8")
    s_all, i_all = index.search(batch, 50)
    for j in range(6):
        s1, i1 = index.search(batch[j:j + 1].contiguous(), 50)
        assert torch.equal(i1[0], i_all[j]) and torch.equal(s1[0], s_all[j])
    y, a = _ops.quantize_i8(batch, per_row=True, with_scale=True)
    ref = np.clip(np.rint(batch.cpu().numpy() * (np.float32(127) / batch.abs().amax(1, keepdim=True).cpu().numpy())),
                  -127, 127)
    np.testing.assert_array_equal(y.cpu().numpy(), ref.astype(np.int8))
    np.testing.assert_array_equal(a.cpu().numpy(), batch.abs().amax(1).cpu().numpy())


def test_knn_int8_certificate(cuda):
    """The int8 certificate (rr_knn_topk_checked_i8, quantisation-residual bound):
    queries whose top-k stand well clear of the rest (10 planted near-copies at
    score ~0.9 among random rows at ~0 +- 0.09) certify and are exact without a
    re-search; a query whose top-k sits in a 300-row cluster 1e-3 wide (gaps <<
    the ~0.03 bound at d = 128) does not certify, and verify=True re-searches it
    exactly."""
    from cirtorch.search import KnnIndex
    from oracle import data, ops
    d, k = 128, 10
    qq = data.unit_rows(3, d, seed=83)
    db = data.unit_rows(120000, d, seed=84)
    for j in range(2):
        rows = qq[j] + 0.45 * data.unit_rows(k, d, seed=85 + j)
        db[1000 + 5000 * j:1000 + 5000 * j + k] = rows / np.linalg.norm(rows, axis=1, keepdims=True)
    rows = qq[2] + 0.02 * data.unit_rows(300, d, seed=87)
    db[90000:90300] = rows / np.linalg.norm(rows, axis=1, keepdims=True)
    ref_s, ref_i = ops.topk_exact(db, qq, k)
    index = KnnIndex(torch.from_numpy(db).to(cuda), "int8")
    q = torch.from_numpy(qq).to(cuda)
    s, i, unc = index.search_checked(q, k)
    unc = unc.cpu().numpy()
    assert unc[0] == 0 and unc[1] == 0 and unc[2] == 1, unc
    np.testing.assert_array_equal(i.cpu().numpy()[:2], ref_i[:2])
    np.testing.assert_allclose(s.cpu().numpy()[:2], ref_s[:2], rtol=0, atol=1e-12)
    sv, iv = index.search(q, k, verify=True)
    np.testing.assert_array_equal(iv.cpu().numpy(), ref_i)


@pytest.mark.parametrize("prec", ["fp16", "int8"])
def test_knn_deferred_certificate(cuda, prec):
    """verify="deferred": the search returns at once with the certificate copied
    to pinned memory; resolve() waits for it, re-searches the flagged queries in
    place and returns their count -- the tight-cluster query is flagged (and
    only it, for fp16), and after resolve every query equals the exact oracle."""
    from cirtorch.search import KnnIndex
    from oracle import data, ops
    d = 128
    qq = data.unit_rows(4, d, seed=62)
    db = data.unit_rows(170000, d, seed=64)
    db[140000:140600] = qq[2] + 0.01 * data.unit_rows(600, d, seed=65)
    db[140000:140600] /= np.linalg.norm(db[140000:140600], axis=1, keepdims=True)
    ref_s, ref_i = ops.topk_exact(db, qq, 100)
    index = KnnIndex(torch.from_numpy(db).to(cuda), prec)
    s, i, pend = index.search(torch.from_numpy(qq).to(cuda), 100, verify="deferred")
    n = pend.resolve()
    assert n == (1 if prec == "fp16" else 4) or (prec == "int8" and n >= 1)
    assert pend.resolve() == n            # idempotent
    np.testing.assert_array_equal(i.cpu().numpy(), ref_i)
    np.testing.assert_allclose(s.cpu().numpy(), ref_s, rtol=0, atol=1e-12)


def test_knn_fused_graph_replay(cuda):
    """The screening pipeline (reset, prefix, fused GEMM, fix-up) captured in a
    hipGraph and replayed equals eager launches."""
    from cirtorch.search import KnnIndex
    from cirtorch.utils.graph import GraphedForward
    from oracle import data, ops
    db = torch.from_numpy(data.unit_rows(200000, 256, seed=71)).to(cuda)
    q1 = torch.from_numpy(data.unit_rows(300, 256, seed=72)).to(cuda)
    q2 = torch.from_numpy(data.unit_rows(300, 256, seed=73)).to(cuda)
    index = KnnIndex(db, "bf16")
    g = GraphedForward(lambda q: index.search(q, 50, verify=False), q1)
    for q in (q1, q2, q1):
        s, i = g(q)
        es, ei = index.search(q, 50, verify=False)
        assert torch.equal(i, ei) and torch.equal(s, es)
    ref_s, ref_i = ops.topk_exact(db.cpu().numpy(), q2.cpu().numpy(), 50)
    np.testing.assert_array_equal(index.search(q2, 50, verify=False)[1].cpu().numpy(), ref_i)


@pytest.mark.parametrize("prec", ["bf16", "fp16", "fp32", "int8"])
def test_knn_verify_tight_cluster(cuda, prec):
    """600 near-copies of a query (scores within ~1e-4 of each other, tighter
    than the bf16 / fp16 screening error) straddle the candidate cut: the
    screening certificate flags that query (rr_knn_topk_checked), and
    search(verify=True) re-searches it with float32 screening / more
    candidates — the result equals the exact oracle.  Queries away from the
    cluster certify."""
    from cirtorch import _ops
    from cirtorch.search import KnnIndex
    from oracle import data, ops
    d = 128
    qq = data.unit_rows(4, d, seed=62)
    db = data.unit_rows(170000, d, seed=64)
    db[140000:140600] = qq[2] + 0.01 * data.unit_rows(600, d, seed=65)
    db[140000:140600] /= np.linalg.norm(db[140000:140600], axis=1, keepdims=True)
    ref_s, ref_i = ops.topk_exact(db, qq, 100)
    index = KnnIndex(torch.from_numpy(db).to(cuda), prec)
    q = torch.from_numpy(qq).to(cuda)
    s, i = index.search(q, 100, verify=True)
    np.testing.assert_array_equal(i.cpu().numpy(), ref_i)
    np.testing.assert_allclose(s.cpu().numpy(), ref_s, rtol=0, atol=1e-12)
    _, _, unc = index.search_checked(q, 100)
    unc = unc.cpu().numpy()
    if prec == "int8":   # the int8 residual bound (~0.03 at d = 128) is far above these gaps
        assert unc[2] == 1
        return
    assert unc[0] == 0 and unc[1] == 0 and unc[3] == 0
    if prec != "fp32":
        assert unc[2] == 1


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("nq", [1, 37, 128])
def test_knn_half_width_gemm_equals_tiled(cuda, prec, nq):
    """<= 128 queries: the score GEMM on k_gemm8h (256 database rows x 128
    queries, 8-phase staggered, 3-stage ring) vs the tiled engine
    (rr_set_tuning(RR_TUNE_GEMM8, 1 | 8)): identical top-k indices and exact
    float64 scores, over the prefix slab and the fused screen (n = 300k rows,
    a ragged last database tile)."""
    from cirtorch import _engine as E
    from cirtorch import _ops
    from cirtorch.search import KnnIndex
    db = _ops.fill_unit_rows(300_001, 2048, seed=0x5EED8, device=cuda)
    q = _ops.fill_unit_rows(nq, 2048, seed=0x5EED9 + nq, device=cuda)
    out = {}
    try:
        for v in (1, 9):
            E.check(E.lib().rr_set_tuning(8, v), "rr_set_tuning")
            out[v] = KnnIndex(db, prec).search(q, 100, verify=False)
    finally:
        E.lib().rr_set_tuning(8, 1)
    assert torch.equal(out[1][1], out[9][1])
    assert torch.equal(out[1][0], out[9][0])


def test_int8_quantization_and_score_gemm(cuda):
    """rr_quantize_i8 == rint(x * 127 / max|x|) clipped (numpy); the int8 score GEMM's
    prefix slab and screened epilogue both rank like the exact int32 dot products:
    Q = 1024 queries (k_gemm8 int8) and Q = 100 (k_gemm8s int8) equal the exact
    float64 oracle on 300k rows (top-100)."""
    from cirtorch import _ops
    from cirtorch.search import KnnIndex
    from oracle import ops
    x = torch.randn(4097 * 4, device=cuda) * 0.3
    q = _ops.quantize_i8(x).cpu().numpy()
    xn = x.cpu().numpy()
    ref = np.clip(np.rint(xn * (np.float32(127.0) / np.abs(xn).max())), -127, 127).astype(np.int8)
    assert np.abs(q.astype(np.int32) - ref).max() <= 1 and (q == ref).mean() > 0.9999
    db = _ops.fill_unit_rows(300_001, 2048, seed=0x5EEDA, device=cuda)
    index = KnnIndex(db, "int8")
    db_np = db.cpu().numpy()
    for nq in (100, 1024):
        qq = _ops.fill_unit_rows(nq, 2048, seed=0x5EEDB + nq, device=cuda)
        s, i = index.search(qq, 100, verify=False)
        ref_s, ref_i = ops.topk_exact(db_np, qq[:6].cpu().numpy(), 100)
        np.testing.assert_array_equal(i[:6].cpu().numpy(), ref_i)
        np.testing.assert_allclose(s[:6].cpu().numpy(), ref_s, rtol=0, atol=1e-12)
        s2, i2 = KnnIndex(db, "bf16").search(qq, 100, verify=False)
        assert torch.equal(i, i2) and torch.equal(s, s2)


@pytest.mark.parametrize("prec", ["fp16", "bf16", "fp32"])
def test_knn_rescore_cut_changes_nothing(cuda, prec):
    """The certified re-score cut (rr_knn.hip rescore_cut, on in the checked search):
    candidates whose screening key is more than twice the error bound below the k-th
    key are not re-scored; the top-k (indices and float64 scores) equal the uncut
    search bit for bit, on random rows and on a database with a planted cluster."""
    from cirtorch import _ops
    from cirtorch.search import KnnIndex
    from oracle import data, ops
    db = _ops.fill_unit_rows(300_000, 512, seed=0xC0FE, device=cuda)
    q = _ops.fill_unit_rows(200, 512, seed=0xC0FF, device=cuda)
    index = KnnIndex(db, prec)
    s0, i0 = index.search(q, 100, verify=False)         # unchecked: every candidate re-scored
    s1, i1, unc = index.search_checked(q, 100)          # checked: the cut
    assert torch.equal(i0, i1) and torch.equal(s0, s1)
    assert int(unc.sum()) == 0
    d = 128
    qq = data.unit_rows(4, d, seed=62)
    pl = data.unit_rows(170000, d, seed=64)
    pl[140000:140600] = qq[2] + 0.3 * data.unit_rows(600, d, seed=65)
    pl[140000:140600] /= np.linalg.norm(pl[140000:140600], axis=1, keepdims=True)
    ix = KnnIndex(torch.from_numpy(pl).to(cuda), prec)
    sv, iv = ix.search(torch.from_numpy(qq).to(cuda), 100, verify=True)
    ref_s, ref_i = ops.topk_exact(pl, qq, 100)
    np.testing.assert_array_equal(iv.cpu().numpy(), ref_i)
    np.testing.assert_allclose(sv.cpu().numpy(), ref_s, rtol=0, atol=1e-12)
