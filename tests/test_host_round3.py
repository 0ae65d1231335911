"""CPU checks of the round-3 host surface: snapshot I/O (reference
``cirtorch/utils/snapshot.py:6-75``), ``norm_act_from_config``
(``utils/misc.py:175-235``), ``modules.utils.OUTPUT_DIM``
(``modules/utils.py:61-79``), the model built the way
``scripts/train_globalF.py:make_model`` builds it (``:240-356``), and mAP over
kNN ranks padded with -1 (k > N).  No GPU compute."""

import configparser

import numpy as np
import pytest
import torch

BODY_INI = """
[body]
arch = resnet50
normalization_mode = syncbn+bn
activation = leaky_relu
activation_slope = 0.01
gn_groups = 16
"""


def _body_section(mode="syncbn+bn", activation="leaky_relu", slope="0.01"):
    cp = configparser.ConfigParser()
    cp.read_string(BODY_INI)
    cp["body"]["normalization_mode"] = mode
    cp["body"]["activation"] = activation
    cp["body"]["activation_slope"] = slope
    return cp


def _make_model(cp, arch="resnet18"):
    """make_model's construction sequence (train_globalF.py:252-259,331-354) on our modules"""
    from cirtorch import backbones as models
    from cirtorch.algos.GF_algo import globalFeatureAlgo
    from cirtorch.models.GF_net import ImageRetrievalNet, Normalize
    from cirtorch.modules.heads.global_head import globalHead
    from cirtorch.modules.utils import OUTPUT_DIM
    from cirtorch.utils.misc import norm_act_from_config
    norm_act_static, _ = norm_act_from_config(cp["body"])
    body = models.__dict__[arch](norm_act=norm_act_static, config=cp["body"])
    output_dim = OUTPUT_DIM[arch]
    algo = globalFeatureAlgo(loss=None, min_level=2, fpn_levels=1)
    head = globalHead(pooling={"name": "GeM", "params": {"p": 3, "eps": 1e-6}},
                      normal={"name": "L2N", "params": {}}, dim=output_dim)
    return ImageRetrievalNet(body, algo, head, augment=Normalize()), ["body"], output_dim


def test_output_dim_table():
    from cirtorch.modules.utils import OUTPUT_DIM
    from cirtorch.models.GF_net import OUTPUT_DIM as net_dims
    assert OUTPUT_DIM["resnet18"] == 512 and OUTPUT_DIM["resnet50"] == 2048 and OUTPUT_DIM["resnet152"] == 2048
    assert OUTPUT_DIM["densenet264"] == 2688  # the live (second) reference table
    assert net_dims is OUTPUT_DIM


@pytest.mark.parametrize("mode", ["bn", "syncbn", "syncbn+bn", "off"])
@pytest.mark.parametrize("activation,slope", [("leaky_relu", "0.01"), ("relu", "0.0"), ("identity", "0.0")])
def test_norm_act_from_config_modes(mode, activation, slope):
    from cirtorch.modules.abn import ABN
    from cirtorch.utils.misc import norm_act_from_config
    static, dynamic = norm_act_from_config(_body_section(mode, activation, slope)["body"])
    for fn in (static, dynamic):
        m = fn(64)
        assert isinstance(m, ABN)
        assert m.activation == activation and m.activation_param == float(slope)
    # plain mappings work too (no configparser getfloat)
    s2, _ = norm_act_from_config({"normalization_mode": mode, "activation": activation, "activation_slope": slope})
    assert s2(8).activation_param == float(slope)


def test_norm_act_from_config_errors():
    from cirtorch.utils.misc import norm_act_from_config
    with pytest.raises(NotImplementedError):
        norm_act_from_config(_body_section("gn")["body"])
    with pytest.raises(ValueError, match="Unrecognized normalization_mode"):
        norm_act_from_config(_body_section("nope")["body"])
    with pytest.raises(NotImplementedError):
        norm_act_from_config(_body_section("bn", "elu", "1.0")["body"])


def _randomise(module, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in module.parameters():
            p.copy_(torch.randn(p.shape, generator=g))
        for name, b in module.named_buffers():
            if name.endswith("running_var"):
                b.copy_(torch.rand(b.shape, generator=g) + 0.5)
            elif name.endswith("running_mean"):
                b.copy_(torch.randn(b.shape, generator=g) * 0.1)


def test_make_model_snapshot_round_trip(tmp_path):
    """save_snapshot -> resume_from_snapshot(model, path, ["body", "ret_head"]) restores every
    tensor; the snapshot keeps config text and training meta (snapshot.py:6-17,41-51)."""
    from cirtorch.utils.snapshot import resume_from_snapshot, save_snapshot
    cp = _body_section()
    src, modules, dim = _make_model(cp)
    assert dim == 512 and modules == ["body"]
    assert src.body.mod2.block1.convs.bn1.activation == "leaky_relu"
    _randomise(src, 1)
    path = str(tmp_path / "model_last.pth.tar")
    save_snapshot(path, cp, 7, 0.5, 0.6, 1234, body=src.body.state_dict(), ret_head=src.ret_head.state_dict())
    dst, _, _ = _make_model(cp)
    _randomise(dst, 2)
    snap = resume_from_snapshot(dst, path, ["body", "ret_head"])
    assert snap["training_meta"] == {"epoch": 7, "last_score": 0.5, "best_score": 0.6, "global_step": 1234}
    assert "normalization_mode = syncbn+bn" in snap["config"]
    for (k, a), (k2, b) in zip(src.state_dict().items(), dst.state_dict().items()):
        assert k == k2 and torch.equal(a, b), k
    with pytest.raises(KeyError, match="does not contain a state_dict for module 'mod9'"):
        resume_from_snapshot(dst, path, ["mod9"])


def test_upstream_checkpoint_format_and_shape_tolerance(tmp_path):
    """upstream {'meta', 'state_dict'} (flat whole-network keys, scripts/test.py:95-106) splits by
    module prefix; entries whose shape differs are dropped, not raised (snapshot.py:54-75)."""
    from cirtorch.utils.snapshot import pre_train_from_snapshots, resume_from_snapshot
    cp = _body_section()
    src, _, _ = _make_model(cp)
    _randomise(src, 3)
    sd = dict(src.state_dict())
    sd["ret_head.whiten.weight"] = torch.zeros(3, 3)  # wrong shape: ignored
    path = str(tmp_path / "upstream.pth")
    torch.save({"meta": {"architecture": "resnet18", "pooling": "gem"}, "state_dict": sd}, path)
    dst, _, _ = _make_model(cp)
    _randomise(dst, 4)
    before = dst.ret_head.whiten.weight.detach().clone()
    resume_from_snapshot(dst, path, ["body", "ret_head"])
    assert torch.equal(dst.body.mod1.conv1.weight, src.body.mod1.conv1.weight)
    assert torch.equal(dst.ret_head.pool.p, src.ret_head.pool.p)
    assert torch.equal(dst.ret_head.whiten.weight, before)
    dst2, _, _ = _make_model(cp)
    pre_train_from_snapshots(dst2, ["body:" + path], ["body", "ret_head"])
    assert torch.equal(dst2.body.mod5.block2.convs.conv2.weight, src.body.mod5.block2.convs.conv2.weight)
    with pytest.raises(ValueError):
        pre_train_from_snapshots(dst2, ["fpn:" + path], ["body"])


class NotAllowed:
    """an arbitrary class instance inside a checkpoint"""


def test_snapshot_loader_refuses_pickled_objects(tmp_path):
    """the loader never unpickles arbitrary objects (weights_only=True)"""
    from cirtorch.utils.snapshot import resume_from_snapshot
    path = str(tmp_path / "evil.pth")
    torch.save({"state_dict": {"body": {}}, "x": NotAllowed()}, path)
    cp = _body_section()
    dst, _, _ = _make_model(cp)
    with pytest.raises(Exception):
        resume_from_snapshot(dst, path, ["body"])


@pytest.mark.parametrize("as_tensor", [False, True])
def test_map_ignores_minus_one_padding(as_tensor):
    """kNN ranks with k > N carry -1 in unfilled slots: mAP equals the mAP of the
    unpadded list (no wrap-around into the last column, no scatter of -1)."""
    from cirtorch.utils.evaluation.ParisOxfordEval import compute_map
    r = np.random.default_rng(5)
    n, q = 20, 6
    full = np.stack([r.permutation(n) for _ in range(q)], axis=1)
    padded = np.concatenate([full, -np.ones((7, q), dtype=np.int64)], axis=0)
    gnd = [{"ok": r.choice(n, 3, replace=False), "junk": r.choice(n, 2, replace=False)} for _ in range(q)]
    for g in gnd:
        g["junk"] = np.setdiff1d(g["junk"], g["ok"])
    g2 = [dict(g, ok=np.append(g["ok"], n - 1)) for g in gnd]  # the last column must not be hit by -1
    for gg in (gnd, g2):
        ref = compute_map(full, gg, [1, 5])
        got = compute_map(torch.from_numpy(padded) if as_tensor else padded, gg, [1, 5])
        assert got[0] == ref[0]
        np.testing.assert_array_equal(got[1], ref[1])
        np.testing.assert_array_equal(got[3], ref[3])


def test_process_decoder_ring_matches_thread_loader(tmp_path):
    """extract_vectors' process decoder (cirtorch/utils/decode_procs.py): every
    file decodes into its shared-memory slot with the same bytes as the thread
    path's PIL loader (GF_net._load_pil: RGB, bbx crop, thumbnail); an image
    larger than a slot comes back pickled; released slots are reused."""
    import numpy as np
    from PIL import Image
    from cirtorch.models.GF_net import _load_pil
    from cirtorch.utils.decode_procs import ProcDecoder
    r = np.random.default_rng(0)
    paths = []
    for i, (h, w) in enumerate([(40, 52), (61, 33), (90, 120), (12, 8)]):
        a = (r.random((h, w, 3)) * 255).astype(np.uint8)
        p = str(tmp_path / ("%d.%s" % (i, "png" if i % 2 else "jpg")))
        Image.fromarray(a).save(p)
        paths.append(p)
    d = ProcDecoder(2, 3, slot_bytes=64 * 64 * 3)
    try:
        for bbx, imsize in [(None, None), ((2, 3, 30, 11), None), (None, 24)]:
            pend = [d.submit(p, imsize, bbx) for p in paths[:3]]
            outs = [q.result() for q in pend]
            for p, t in zip(paths, outs):
                ref = np.asarray(_load_pil(p, imsize, bbx), dtype=np.uint8)
                assert t.shape == ref.shape and (t.numpy() == ref).all(), (p, bbx, imsize)
            # hand the ring views back (an event that has completed: a CPU stand-in)
            class Done:
                def query(self):
                    return True
            d.release(outs, Done())
        big = d.submit(paths[2], None, None).result()      # 90 x 120 x 3 > one slot
        assert not d.owns(big) and big.shape == (90, 120, 3)
        # several files per task (extract_vectors submits groups of 4)
        outs = [q.result() for q in d.submit_group([(p, None, None) for p in (paths[0], paths[1], paths[3])])]
        for p, t in zip((paths[0], paths[1], paths[3]), outs):
            assert (t.numpy() == np.asarray(_load_pil(p, None, None), dtype=np.uint8)).all(), p
    finally:
        d.close()


def test_pinned_block_pool_free_list():
    """extract_vectors' pinned block pool: a request takes the smallest free block
    that holds it (by identity, never by tensor comparison), hands out a view of the
    requested shape, and takes back only its own views once their event completes."""
    from cirtorch.models.GF_net import _PinnedBlocks

    class Done:
        def query(self):
            return True

    pool = _PinnedBlocks()
    pool.free = [torch.zeros(100, dtype=torch.uint8), torch.zeros(50, dtype=torch.uint8),
                 torch.zeros(80, dtype=torch.uint8)]
    v = pool.acquire((2, 20))
    assert v.shape == (2, 20) and sorted(b.numel() for b in pool.free) == [80, 100]
    pool.release([v, torch.zeros(3, dtype=torch.uint8)], Done())   # a foreign tensor is ignored
    pool._reclaim()
    assert sorted(b.numel() for b in pool.free) == [50, 80, 100]
