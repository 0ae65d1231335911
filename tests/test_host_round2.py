"""CPU checks of host-side code against fixtures produced by the reference
itself (tests/golden/make_golden.py): the vectorised mAP evaluation
(map.npz), ISSTestTransform (transform.npz), the mutual-NN matcher oracle
(nnmatch.npz), plus host logic of the search wrappers (no GPU compute)."""

import numpy as np
import pytest
import torch

from conftest import golden


def _gnd(g):
    out = []
    offs = {k: np.concatenate([[0], np.cumsum(g["gnd_%s_len" % k])]) for k in ("easy", "hard", "junk")}
    for i in range(len(g["gnd_easy_len"])):
        out.append({k: g["gnd_" + k][offs[k][i]:offs[k][i + 1]] for k in ("easy", "hard", "junk")})
    return out


@pytest.mark.parametrize("as_tensor", [False, True])
def test_vectorised_map_bit_identical_to_reference(as_tensor):
    """ParisOxfordEval.py:41-195 outputs (reference run) reproduced exactly:
    E/M/H mAP, per-query AP (NaN for empty queries), mP@k, old protocol."""
    from cirtorch.utils.evaluation.ParisOxfordEval import compute_map, compute_map_and_print
    g = golden("map.npz")
    gnd = _gnd(g)
    ranks = g["ranks"].astype(np.int64)
    r = torch.from_numpy(ranks) if as_tensor else ranks
    logs = []
    score = compute_map_and_print("roxford5k", r, gnd, lambda *a: logs.append(a))
    assert score["mAP"] == float(g["score_mAP"])
    for proto, okk, jk in (("E", ["easy"], ["junk", "hard"]), ("M", ["easy", "hard"], ["junk"]),
                           ("H", ["hard"], ["junk", "easy"])):
        g2 = [{"ok": np.concatenate([q[k] for k in okk]), "junk": np.concatenate([q[k] for k in jk])} for q in gnd]
        m, aps, pr, _ = compute_map(r, g2, [1, 5, 10])
        assert m == float(g["map" + proto]), proto
        np.testing.assert_array_equal(aps, g["aps" + proto])
        np.testing.assert_array_equal(pr, g["pr" + proto])
    old = compute_map(r, [{"ok": np.concatenate([q["easy"], q["hard"]]), "junk": q["junk"]} for q in gnd], [1, 5, 10])
    assert old[0] == float(g["old_map"])
    np.testing.assert_array_equal(old[1], g["old_aps"])
    np.testing.assert_array_equal(old[3], g["old_prs"])
    assert len(logs) == 4


def test_map_partial_ranks_and_no_junk():
    """Positives absent from a truncated ranked list are skipped (np.isin over
    the list); queries without a junk key use no junk."""
    from cirtorch.utils.evaluation.ParisOxfordEval import compute_map
    from oracle import ops
    r = np.random.default_rng(3)
    full = np.stack([r.permutation(50) for _ in range(4)], axis=1)
    gnd = [{"ok": np.array([3, 7, 11])}, {"ok": np.array([0, 49]), "junk": np.array([5])},
           {"ok": np.array([], dtype=np.int64)}, {"ok": np.array([1, 2, 3, 4]), "junk": np.array([9, 8])}]
    ref = ops.compute_map(full, gnd, [1, 5])
    got = compute_map(full, gnd, [1, 5])
    assert got[0] == ref[0]
    np.testing.assert_array_equal(got[1], ref[1])


@pytest.mark.parametrize("cfg", [0, 1, 2])
def test_iss_test_transform_matches_reference(cfg):
    """ISSTestTransform (generic/transform.py:81-130, window quirk :100-104):
    output size and pixels identical to the reference run."""
    from PIL import Image
    from cirtorch.datasets.generic import ISSTestTransform
    from oracle import data
    g = golden("transform.npz")
    short, longest = [int(v) for v in g["cfg_%d" % cfg]]
    tf = ISSTestTransform(shortest_size=short, longest_max_size=longest, random_scale=[0.8, 1.2])
    for ii, (w, h, bbx, pix) in enumerate(data.transform_images()):
        ref = g["out_%d_%d" % (cfg, ii)]
        img = Image.fromarray(pix, mode="RGB")
        out = tf(img, bbx=bbx)["img"]
        assert tuple(out.shape) == ref.shape, (cfg, ii, out.shape, ref.shape)
        np.testing.assert_array_equal(out.numpy(), ref.astype(np.float32) / np.float32(255.0))
        assert torch.equal(tf.pixels(img, bbx), torch.from_numpy(ref))
        cw, ch = (bbx[2] - bbx[0], bbx[3] - bbx[1]) if bbx else (w, h)
        assert tf.output_size(cw, ch) == (ref.shape[2], ref.shape[1])


def test_iss_test_transform_window_quirk():
    """shortest_size * [0.8, 1.2] is list repetition: every short side > 1 px
    is rescaled to shortest_size (then capped by longest_max_size)."""
    from cirtorch.datasets.generic import ISSTestTransform
    tf = ISSTestTransform(shortest_size=800, longest_max_size=1024, random_scale=[0.8, 1.2])
    assert tf.output_size(1024, 768) == (1024, 768)       # 800/768 then capped at 1024/1024
    assert tf.output_size(600, 400) == (1024, 682)
    assert tf.output_size(900, 800) == (900, 800)
    with pytest.raises(TypeError):
        ISSTestTransform(shortest_size=800, longest_max_size=1024, random_scale=None).output_size(10, 10)


def test_nn_matcher_oracle_equals_reference():
    """The mutual-NN restatement vs the reference HPatchesEval.nn_matcher output
    (generated with a test-only cv2 stand-in, make_golden.py gen_nn_match)."""
    from oracle import data, ops
    g = golden("nnmatch.npz")
    for tag in ("a", "b", "c"):
        n1, n2, d, seed = [int(v) for v in g["shape_" + tag]]
        d1, d2 = data.nn_descriptors(n1, n2, d, seed)
        np.testing.assert_array_equal(ops.nn_matcher(d1, d2), g["match_" + tag])


def test_init_network_defaults_to_fp16():
    from cirtorch.models.GF_net import init_network
    net = init_network({"architecture": "resnet18", "pooling": "gem"})
    assert net.body.engine_dtype == torch.float16
    net = init_network({"architecture": "resnet18", "pooling": "gem", "precision": "bf16"})
    assert net.body.engine_dtype == torch.bfloat16


def test_empty_shard_search_contributes_sentinels():
    """A rank whose DB shard is empty returns (-inf, -1) lists instead of failing
    before the all-gather (which would hang the other ranks)."""
    from cirtorch.search import KnnIndex, shard_range
    assert shard_range(3, 3, 4) == (3, 0)
    idx = KnnIndex(torch.empty((0, 64)), "bf16", idx_offset=3)
    s, i = idx.search(torch.rand(5, 64), 7)
    assert s.shape == (5, 7) and torch.isinf(s).all() and (s < 0).all() and (i == -1).all()


def test_synthetic_generators_match_fixture_recipes():
    """cirtorch.utils.synthetic (used by bench.py's parity fields) draws exactly
    the parameters / images the fixtures were generated from."""
    from cirtorch.utils import synthetic
    from oracle import data, weights
    for arch in ("resnet18", "resnet50", "resnet152"):
        a, b = synthetic.backbone_state(arch), weights.backbone_state(arch)
        assert list(a) == list(b)
        for k in a:
            assert np.array_equal(a[k], b[k]), (arch, k)
    for dim in (512, 2048):
        a, b = synthetic.head_state(dim), weights.head_state(dim)
        assert all(np.array_equal(a[k], b[k]) for k in b)
    assert np.array_equal(synthetic.structured_images(2, 64, 96, seed=2001), data.structured_images(2, 64, 96, seed=2001))
