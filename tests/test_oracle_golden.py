"""The CPU oracle against the golden vectors produced by the reference modules
(tests/golden/make_golden.py).  CPU only — this is what pins the oracle that
every GPU parity test compares against."""

import numpy as np
import pytest
import torch

from conftest import cosines, golden
from oracle import backbone as obb, data, ops, weights


def test_ops_gem_mac_spoc_l2n():
    g = golden("ops.npz")
    x = torch.from_numpy(g["x"])
    for p in (3.0, 2.5):
        np.testing.assert_allclose(ops.gem(x, p).numpy(), g["gem_p%g" % p], rtol=1e-6, atol=0)
    np.testing.assert_array_equal(ops.mac(x).numpy(), g["mac"])
    np.testing.assert_allclose(ops.spoc(x).numpy(), g["spoc"], rtol=1e-6)
    np.testing.assert_allclose(ops.l2n(torch.from_numpy(g["l2n_x"])).numpy(), g["l2n"], rtol=1e-6)


def test_ops_head():
    g = golden("ops.npz")
    hs = {k: torch.from_numpy(v) for k, v in weights.head_state(512).items()}
    x = torch.from_numpy(g["head_x"])
    np.testing.assert_allclose(ops.head(x, hs["pool.p"], hs["whiten.weight"], hs["whiten.bias"]).numpy(),
                               g["head"], rtol=1e-6, atol=1e-8)
    np.testing.assert_allclose(ops.head(x, hs["pool.p"], hs["whiten.weight"], hs["whiten.bias"], whiten=False).numpy(),
                               g["head_nowhiten"], rtol=1e-6, atol=1e-8)


def _net(arch, g):
    hs = weights.head_state(weights.OUTPUT_DIM[arch])
    hs["whiten.bias"] = g["head_bias"]
    return obb.OracleNet(arch, weights.backbone_state(arch), hs)


def test_resnet18_single_and_multiscale():
    g = golden("r18.npz")
    net = _net("resnet18", g)
    imgs = [torch.from_numpy(im) for im in data.structured_images(int(g["n"]), *[int(v) for v in g["res"]],
                                                                   seed=int(g["seed"]))]
    assert cosines(net.forward(imgs).numpy(), g["desc_s1"]).min() > 1 - 1e-6
    assert cosines(net.forward(imgs, scales=(0.5, 1, 2)).numpy(), g["desc_s0.5_1_2"]).min() > 1 - 1e-6


def test_resnet18_stage_checksums():
    g = golden("r18.npz")
    net = _net("resnet18", g)
    imgs = data.structured_images(int(g["n"]), *[int(v) for v in g["res"]], seed=int(g["seed"]))
    outs = net.body(obb.normalize_images(torch.from_numpy(imgs[:1])))
    for k in ("mod1", "mod2", "mod3", "mod4", "mod5"):
        np.testing.assert_allclose(outs[k][0].double().sum(dim=(1, 2)).numpy(), g["chk_" + k], rtol=1e-5,
                                   atol=1e-4 * np.abs(g["chk_" + k]).max())


def test_resnet18_mixed_sizes():
    g = golden("r18.npz")
    net = _net("resnet18", g)
    mixed = [tuple(int(v) for v in hw) for hw in g["mixed_sizes"]]
    imgs = [obb.normalize_images(torch.from_numpy(data.structured_images(1, h, w, seed=int(g["seed"]) + 1 + i)[0]))
            for i, (h, w) in enumerate(mixed)]
    assert cosines(net.forward(imgs, normalize=False).numpy(), g["desc_mixed"]).min() > 1 - 1e-6


@pytest.mark.slow
def test_resnet50_768x1024():
    g = golden("r50.npz")
    net = _net("resnet50", g)
    imgs = [torch.from_numpy(im) for im in data.structured_images(int(g["n"]), *[int(v) for v in g["res"]],
                                                                   seed=int(g["seed"]))]
    assert cosines(net.forward(imgs).numpy(), g["desc_s1"]).min() > 1 - 1e-6


def test_resnet101_and_r50_multiscale():
    for f, arch, scales in (("r101.npz", "resnet101", (1,)), ("r50ms.npz", "resnet50", (0.5, 1, 2))):
        g = golden(f)
        net = _net(arch, g)
        imgs = [torch.from_numpy(im) for im in data.structured_images(int(g["n"]), *[int(v) for v in g["res"]],
                                                                       seed=int(g["seed"]))]
        key = "desc_s" + "_".join("%g" % s for s in scales)
        assert cosines(net.forward(imgs, scales=scales).numpy(), g[key]).min() > 1 - 1e-6


def test_knn_reference_rank_and_exact_topk():
    g = golden("knn.npz")
    for tag in ("4k", "100k"):
        n, q, k = (int(v) for v in g["shape_" + tag])
        db = data.database(n)
        qq = data.queries(q, seed=int(g["qseed_" + tag]))
        scores, ranks = ops.rank_reference(db, qq)
        np.testing.assert_array_equal(ranks[:k].T, g["idx_" + tag])
        s64, i64 = ops.topk_exact(db, qq, k)
        np.testing.assert_array_equal(i64, g["idx_" + tag])
        np.testing.assert_allclose(s64, g["score_" + tag], rtol=0, atol=2e-7)


def _gnd(g):
    out = []
    offs = {k: np.concatenate([[0], np.cumsum(g["gnd_%s_len" % k])]) for k in ("easy", "hard", "junk")}
    for i in range(len(g["gnd_easy_len"])):
        out.append({k: g["gnd_" + k][offs[k][i]:offs[k][i + 1]] for k in ("easy", "hard", "junk")})
    return out


def test_map_restatement_equals_reference():
    g = golden("map.npz")
    gnd = _gnd(g)
    res = ops.compute_map_revisited(g["ranks"].astype(np.int64), gnd)
    for proto in ("E", "M", "H"):
        assert res["map" + proto] == pytest.approx(float(g["map" + proto]), abs=1e-12)
        np.testing.assert_allclose(res["mpr" + proto], g["pr" + proto], atol=1e-12)
    assert (res["mapM"] + res["mapH"]) / 2 * 100 == pytest.approx(float(g["score_mAP"]), abs=1e-10)
    old = ops.compute_map(g["ranks"].astype(np.int64),
                          [{"ok": np.concatenate([q["easy"], q["hard"]]), "junk": q["junk"]} for q in gnd], [1, 5, 10])
    assert old[0] == pytest.approx(float(g["old_map"]), abs=1e-12)


def test_whiten_restatement():
    g = golden("whiten.npz")
    X = data.unit_rows(600, 64, seed=601).T.astype(np.float64)
    np.testing.assert_allclose(ops.whitenapply(X, g["m"], g["P"]), g["Y"], rtol=1e-9, atol=1e-12)
    m, P = ops.whitenlearn(X, g["qidxs"], g["pidxs"])
    np.testing.assert_allclose(m, g["m"], rtol=1e-12)
    # eigenvectors are defined up to sign: compare |P| row-wise
    np.testing.assert_allclose(np.abs(P), np.abs(g["P"]), rtol=1e-6, atol=1e-8)


def test_local_head_restatement():
    """oracle.local_head == the reference localHead (local_head.py:43-71) on the G7 fixtures."""
    import torch
    g = golden("local.npz")
    for tag in ("a", "b"):
        got = ops.local_head(torch.from_numpy(g["x_" + tag]), torch.from_numpy(g["kpts_" + tag]),
                             torch.from_numpy(g["w_" + tag]), torch.from_numpy(g["b_" + tag])).numpy()
        np.testing.assert_allclose(got, g["desc_" + tag], rtol=0, atol=1e-6)
    assert (ops.nn_matcher(g["desc_b"][0], g["nn_d2"]) == g["nn_match"]).all()
