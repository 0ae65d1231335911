"""Generate the golden fixtures in tests/golden/*.npz by running the REFERENCE
modules themselves (build container only — /root/reference never travels).

    python tests/golden/make_golden.py            # writes tests/golden/*.npz

What is imported from the reference, unmodified (``PYTHONPATH=/root/reference``):
  cirtorch.modules.pools (GeM/MAC/SPoC), cirtorch.modules.normalizations (L2N),
  cirtorch.modules.heads.global_head.globalHead, cirtorch.backbones (ResNet),
  cirtorch.algos.GF_algo.globalFeatureAlgo, cirtorch.models.GF_net.ImageRetrievalNet,
  cirtorch.utils.parallel.PackedSequence, cirtorch.utils.image.normalize,
  cirtorch.utils.whiten, cirtorch.utils.evaluation.ParisOxfordEval.

Third-party dependency absent from the image: ``inplace_abn==1.1.0``
(reference ``requirements.txt:9``).  Its only role on this path is the eval-mode
ABN arithmetic, whose published algorithm is F.batch_norm(running stats,
weight, bias, eps=1e-5) followed by the configured activation.  We register
that restatement as the module ``inplace_abn`` for the duration of this script
(SURVEY §8c recipe); gamma > 0 in all weights, so the in-place variant's
|gamma| convention cannot differ.  Two reference defects on the path are
worked around exactly as SURVEY §0.3 records: ResNet.forward stops at mod3
(``resnet.py:158-159``) so a wrapper appends mod4/mod5, and
ImageRetrievalNet's broken augment call is bypassed with augment=None.

No reference source is copied: fixtures hold only inputs/outputs (and seeds).
"""

import os
import sys
import types
from functools import partial

sys.dont_write_bytecode = True  # never write __pycache__ into /root/reference
REF = os.environ.get("RR_REFERENCE", "/root/reference")
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, REF)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from oracle import backbone as obb, data, ops, weights  # noqa: E402


def _install_inplace_abn_restatement():
    mod = types.ModuleType("inplace_abn")

    class ABN(nn.Module):
        def __init__(self, num_features, eps=1e-5, momentum=0.1, affine=True,
                     activation="leaky_relu", activation_param=0.01):
            super().__init__()
            self.num_features, self.eps, self.momentum = num_features, eps, momentum
            self.affine, self.activation, self.activation_param = affine, activation, activation_param
            self.weight = nn.Parameter(torch.ones(num_features))
            self.bias = nn.Parameter(torch.zeros(num_features))
            self.register_buffer("running_mean", torch.zeros(num_features))
            self.register_buffer("running_var", torch.ones(num_features))

        def forward(self, x):
            x = F.batch_norm(x, self.running_mean, self.running_var, self.weight, self.bias,
                             self.training, self.momentum, self.eps)
            if self.activation == "relu":
                return F.relu(x)
            if self.activation == "leaky_relu":
                return F.leaky_relu(x, negative_slope=self.activation_param)
            if self.activation == "elu":
                return F.elu(x, alpha=self.activation_param)
            if self.activation == "identity":
                return x
            raise RuntimeError(self.activation)

    mod.ABN = ABN
    mod.InPlaceABN = ABN
    mod.InPlaceABNSync = ABN
    mod.active_group = lambda *a, **k: None
    mod.set_active_group = lambda *a, **k: None
    sys.modules["inplace_abn"] = mod
    return ABN


ABN = _install_inplace_abn_restatement()

from cirtorch.modules import pools as R_pools  # noqa: E402
from cirtorch.modules import normalizations as R_norms  # noqa: E402
from cirtorch.modules.heads.global_head import globalHead  # noqa: E402
import cirtorch.backbones as R_backbones  # noqa: E402
from cirtorch.algos.GF_algo import globalFeatureAlgo  # noqa: E402
from cirtorch.models.GF_net import ImageRetrievalNet  # noqa: E402
from cirtorch.utils.parallel import PackedSequence  # noqa: E402
from cirtorch.utils.image import normalize as R_normalize  # noqa: E402
from cirtorch.utils import whiten as R_whiten  # noqa: E402
from cirtorch.utils.evaluation import ParisOxfordEval as R_eval  # noqa: E402

torch.set_num_threads(os.cpu_count() or 8)
MEAN, STD = data.IMAGENET_MEAN, data.IMAGENET_STD


class _Body5(nn.Module):
    """Appends mod4/mod5 to the reference forward (resnet.py:158-159)."""

    def __init__(self, body):
        super().__init__()
        self.body = body

    def forward(self, x):
        outs = self.body(x)
        outs["mod4"] = self.body.mod4(outs["mod3"])
        outs["mod5"] = self.body.mod5(outs["mod4"])
        return outs


def reference_net(arch, head_bias=None):
    body = R_backbones.__dict__[arch](norm_act=partial(ABN, activation="leaky_relu", activation_param=0.01),
                                      config=None, classes=0)
    sd = {k: torch.from_numpy(v) for k, v in weights.backbone_state(arch).items()}
    missing, unexpected = body.load_state_dict(sd, strict=False)
    assert not unexpected, unexpected
    assert all(("num_batches" in m) for m in missing), missing
    dim = weights.OUTPUT_DIM[arch]
    head = globalHead(pooling={"name": "GeM", "params": {"p": 3, "eps": 1e-6}},
                      normal={"name": "L2N", "params": {}}, dim=dim)
    hs = weights.head_state(dim)
    if head_bias is not None:
        hs["whiten.bias"] = head_bias
    head.load_state_dict({k: torch.from_numpy(v) for k, v in hs.items()})
    algo = globalFeatureAlgo(loss=None, min_level=0, fpn_levels=1)
    net = ImageRetrievalNet(_Body5(body), algo, head, augment=None).eval()
    return net, body


def centering_bias(arch, res=224, n=16, seed=7):
    """Whitening bias b = -W mu, mu = mean un-whitened descriptor of n calibration
    images (reference head with do_whitening=False).  Makes descriptors of
    different images far apart, so 1-1e-4 cosine parity is not vacuous."""
    net, _ = reference_net(arch)
    x = R_normalize(torch.from_numpy(data.structured_images(n, res, res, seed=seed)), MEAN, STD)
    with torch.no_grad():
        feats = net.body(x)["mod5"]
        pre = net.ret_head(feats, do_whitening=False)  # D x n
    mu = pre.double().mean(1)
    w = torch.from_numpy(weights.head_state(weights.OUTPUT_DIM[arch])["whiten.weight"]).double()
    return (-(w @ mu)).float().numpy()


def run_ref(net, imgs_np, scales=(1,)):
    imgs = [R_normalize(torch.from_numpy(im).unsqueeze(0), MEAN, STD).squeeze(0) for im in imgs_np]
    with torch.no_grad():
        _, pred = net(img=PackedSequence(imgs), scales=list(scales), do_prediction=True)
    return pred["ret_pred"].numpy()


def check_close(name, ref, mine, tol):
    cos = (ref * mine).sum(0) / (np.linalg.norm(ref, axis=0) * np.linalg.norm(mine, axis=0))
    err = np.abs(ref - mine).max()
    print("  %-28s max|d|=%.3g min cos=%.9f" % (name, err, cos.min()))
    assert err < tol, (name, err)


# ----------------------------------------------------------------------------- G3
def gen_ops():
    r = data.rng(101)
    x = (r.standard_normal((2, 64, 5, 7)).astype(np.float32) * 0.5 + 0.2).astype(np.float32)
    xt = torch.from_numpy(x)
    out = {"x": x}
    for p in (3.0, 2.5):
        out["gem_p%g" % p] = R_pools.GeM(p=p, eps=1e-6)(xt).detach().numpy()
    out["mac"] = R_pools.MAC()(xt).numpy()
    out["spoc"] = R_pools.SPoC()(xt).numpy()
    v = r.standard_normal((3, 300)).astype(np.float32)
    out["l2n_x"] = v
    out["l2n"] = R_norms.L2N(eps=1e-6)(torch.from_numpy(v)).numpy()
    # full globalHead on a small map, D=512 weights from the oracle generator
    hx = np.abs(r.standard_normal((2, 512, 3, 4)).astype(np.float32))
    head = globalHead(pooling={"name": "GeM", "params": {"p": 3, "eps": 1e-6}},
                      normal={"name": "L2N", "params": {}}, dim=512)
    head.load_state_dict({k: torch.from_numpy(v) for k, v in weights.head_state(512).items()})
    with torch.no_grad():
        out["head_x"] = hx
        out["head"] = head(torch.from_numpy(hx)).numpy()
        out["head_nowhiten"] = head(torch.from_numpy(hx), do_whitening=False).numpy()
    # oracle restatement check
    check_close("gem p3", out["gem_p3"].reshape(2, -1).T, ops.gem(xt, 3.0).numpy().reshape(2, -1).T, 1e-6)
    hs = {k: torch.from_numpy(v) for k, v in weights.head_state(512).items()}
    check_close("head", out["head"], ops.head(torch.from_numpy(hx), hs["pool.p"], hs["whiten.weight"],
                                              hs["whiten.bias"]).numpy(), 1e-6)
    np.savez_compressed(os.path.join(HERE, "ops.npz"), **out)


# ----------------------------------------------------------------------------- G1 / G2
def gen_net(arch, res, n, seed, scales_list, fname, mixed=None, local=None):
    bias = centering_bias(arch)
    net, body = reference_net(arch, head_bias=bias)
    imgs = data.structured_images(n, res[0], res[1], seed=seed)
    out = {"head_bias": bias, "seed": np.int64(seed), "res": np.array(res), "n": np.int64(n)}
    onet = obb.OracleNet(arch, weights.backbone_state(arch),
                         dict(weights.head_state(weights.OUTPUT_DIM[arch]), **{"whiten.bias": bias}))
    for scales in scales_list:
        key = "desc_s" + "_".join("%g" % s for s in scales)
        ref = run_ref(net, list(imgs), scales)
        out[key] = ref
        mine = onet.forward([torch.from_numpy(im) for im in imgs], scales=scales).numpy()
        check_close(arch + " " + key, ref, mine, 1e-4)
    # per-stage channel checksums of image 0 (single scale)
    x = R_normalize(torch.from_numpy(imgs[:1]), MEAN, STD)
    with torch.no_grad():
        stages = _Body5(body)(x)
    for k in ("mod1", "mod2", "mod3", "mod4", "mod5"):
        out["chk_" + k] = stages[k][0].double().sum(dim=(1, 2)).numpy()
    if local is not None:
        # config 5: the reference localHead (local_head.py:19-71) on the stage map
        # the local-feature config selects (local_config.ini:61 inputs = ["mod3"];
        # its FPN is out of scope), keypoints / weights regenerated from the seed
        from cirtorch.modules.heads.local_head import localHead as R_localHead
        stage, npts, e, lseed = local
        fm = stages[stage]
        kp, lw, lb = data.local_head_problem(fm.shape[0], fm.shape[1], e, npts, lseed)
        head = R_localHead(fm.shape[1], e)
        head.load_state_dict({"whiten.weight": torch.from_numpy(lw), "whiten.bias": torch.from_numpy(lb)})
        with torch.no_grad():
            ref = head(fm, torch.from_numpy(kp)).numpy()
        mine = ops.local_head(fm, torch.from_numpy(kp), torch.from_numpy(lw), torch.from_numpy(lb)).numpy()
        assert np.abs(ref - mine).max() < 1e-5, np.abs(ref - mine).max()
        out.update({"local_stage": np.array(stage), "local_npts": np.int64(npts), "local_e": np.int64(e),
                    "local_seed": np.int64(lseed), "local_desc": ref})
    if mixed is not None:
        mimgs = [data.structured_images(1, h, w, seed=seed + 1 + i)[0] for i, (h, w) in enumerate(mixed)]
        ref = run_ref(net, mimgs)
        out["mixed_sizes"] = np.array(mixed)
        out["desc_mixed"] = ref
        # oracle: normalise each image, then zero-pad (augment=None path)
        nimgs = [obb.normalize_images(torch.from_numpy(im)) for im in mimgs]
        mine = onet.forward(nimgs, normalize=False).numpy()
        check_close(arch + " mixed", ref, mine, 1e-4)
    np.savez_compressed(os.path.join(HERE, fname), **out)


def gen_mixed(arch, sizes, seed, fname):
    """A ragged batch (PackedSequence of different sizes) through the reference, in
    both orders the reference code has: (a) augment=None on pre-normalised images:
    ImageRetrievalNet pads the normalised images with zeros (GF_net.py:99 ->
    sequence.py:4-67); (b) the in-tree augment order, pad first then normalise
    (random_augmentation.py:102 then :174): the reference pad_packed_images on the
    raw images, the reference normalize on the padded batch, then the net."""
    from cirtorch.utils.sequence import pad_packed_images as R_pad
    bias = centering_bias(arch)
    net, _ = reference_net(arch, head_bias=bias)
    imgs = [data.structured_images(1, h, w, seed=seed + i)[0] for i, (h, w) in enumerate(sizes)]
    onet = obb.OracleNet(arch, weights.backbone_state(arch),
                         dict(weights.head_state(weights.OUTPUT_DIM[arch]), **{"whiten.bias": bias}))
    out = {"head_bias": bias, "seed": np.int64(seed), "mixed_sizes": np.array(sizes)}
    out["desc_mixed"] = run_ref(net, imgs)
    nimgs = [obb.normalize_images(torch.from_numpy(im)) for im in imgs]
    check_close(arch + " mixed (normalise, pad)", out["desc_mixed"],
                onet.forward(nimgs, normalize=False).numpy(), 1e-4)
    padded, _ = R_pad(PackedSequence([torch.from_numpy(im) for im in imgs]))
    padded = R_normalize(padded, MEAN, STD)
    with torch.no_grad():
        _, pred = net(img=PackedSequence(list(padded)), scales=[1], do_prediction=True)
    out["desc_mixed_padnorm"] = pred["ret_pred"].numpy()
    check_close(arch + " mixed (pad, normalise)", out["desc_mixed_padnorm"],
                onet.forward([torch.from_numpy(im) for im in imgs], normalize=True).numpy(), 1e-4)
    np.savez_compressed(os.path.join(HERE, fname), **out)


# ----------------------------------------------------------------------------- G10
def gen_testpy():
    """scripts/test.py:84-259 replayed (tests/testpy_replay.py) with the oracle
    extractor (torch-CPU restatement, decoded by the same PIL calls) and the
    reference's own whitenlearn / whitenapply / compute_map_and_print.  The upstream
    multi-scale power mean of extract_vectors (msp) is not in /root/reference
    (parity unpinned for that rule: restated as oracle.ops.extract_ms_upstream).
    Two cases: (A) meta whitening=False -> msp = pool.p = 3; (B) whitening=True
    (head Linear with the centering bias) -> msp = 1.  Each is also run with a
    float64 oracle; the stored ranks are required to be the same in both, so a
    float32 engine cannot differ from them by rounding alone."""
    import tempfile
    import types as _types
    from PIL import Image
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import testpy_replay as T
    out = {}
    with tempfile.TemporaryDirectory() as root:
        hashes = T.make_dataset(root)
        names = sorted(hashes)
        out["file_names"] = np.array(names)
        out["file_sha1"] = np.array([hashes[k] for k in names])
        bias = centering_bias(T.ARCH)
        out["head_bias"] = bias
        for tag, whitening in (("A", False), ("B", True)):
            ck = os.path.join(root, "ck_%s.pth" % tag)
            T.checkpoint(ck, whitening, bias if whitening else None)
            runs = {}
            for dt in (torch.float32, torch.float64):
                def load_net(state, dt=dt):
                    meta = state["meta"]
                    sd = state["state_dict"]
                    bs = {k[5:]: v.numpy() for k, v in sd.items() if k.startswith("body.")}
                    hs = {k[9:]: v.numpy() for k, v in sd.items() if k.startswith("ret_head.")}
                    net = obb.OracleNet(meta["architecture"], bs, hs, dtype=dt)
                    return (net, meta["whitening"]), meta, float(hs["pool.p"].reshape(-1)[0])

                def extract(netw, images, size, bbxs, ms, msp, dt=dt):
                    net, whiten = netw
                    cols = []
                    for i, p in enumerate(images):
                        with open(p, "rb") as f:
                            img = Image.open(f).convert("RGB")
                        if bbxs is not None:
                            img = img.crop(bbxs[i])
                        img.thumbnail((size, size), Image.LANCZOS)
                        x = torch.from_numpy(np.asarray(img, dtype=np.float32).transpose(2, 0, 1).copy() / 255.0)
                        x = obb.normalize_images(x.to(dt), T.MEAN, T.STD)
                        cols.append(ops.extract_ms_upstream(net, x, ms, msp, whiten))
                    return torch.stack(cols, 1)

                api = _types.SimpleNamespace(
                    load_net=load_net, extract_vectors=extract,
                    whitenlearn=lambda X, q, p_: R_whiten.whitenlearn(X, q, p_),
                    whitenapply=lambda X, m, P: R_whiten.whitenapply(X, m, P),
                    compute_map=lambda ds, ranks, gnd: R_eval.compute_map_and_print(ds, ranks, gnd, lambda *a: None),
                    cid2filename=lambda cid, prefix: os.path.join(prefix, cid[-2:], cid[-4:-2], cid[-6:-4], cid),
                    configdataset=_oracle_configdataset,
                    to_numpy=lambda v: v.float().numpy())
                with torch.no_grad():
                    runs[dt] = T.run(api, root, ck)
            r32, r64 = runs[torch.float32], runs[torch.float64]
            for key in ("ranks", "ranks_lw"):
                same = (r32[key] == r64[key]).all()
                diff = np.argwhere(r32[key] != r64[key])
                print("  testpy %s %s: float32 == float64 oracle ranks: %s (%d entries differ: %s)"
                      % (tag, key, same, len(diff), diff[:10].tolist()))
                out["%s_%s_stable" % (tag, key)] = np.bool_(same)
            print("  testpy %s: msp %g, mAP %.4f, + whiten %.4f" % (tag, r32["msp"], r32["map"]["mAP"],
                                                                   r32["map_lw"]["mAP"]))
            out.update({tag + "_ranks": r32["ranks"].astype(np.int32), tag + "_ranks_lw": r32["ranks_lw"].astype(np.int32),
                        tag + "_map": np.float64(r32["map"]["mAP"]), tag + "_map_lw": np.float64(r32["map_lw"]["mAP"]),
                        tag + "_vecs": r32["vecs"], tag + "_qvecs": r32["qvecs"], tag + "_msp": np.float64(r32["msp"])})
    np.savez_compressed(os.path.join(HERE, "testpy.npz"), **out)


def _oracle_configdataset(dataset, dir_main):
    """upstream configdataset (the gnd pickle is this script's own file)"""
    import pickle
    with open(os.path.join(dir_main, dataset, "gnd_%s.pkl" % dataset), "rb") as f:
        cfg = pickle.load(f)
    cfg["n"], cfg["nq"] = len(cfg["imlist"]), len(cfg["qimlist"])
    d = os.path.join(dir_main, dataset, "jpg")
    cfg["im_fname"] = lambda c, i: os.path.join(d, c["imlist"][i] + ".jpg")
    cfg["qim_fname"] = lambda c, i: os.path.join(d, c["qimlist"][i] + ".jpg")
    return cfg


# ----------------------------------------------------------------------------- G4
def gen_knn():
    out = {}
    # query seeds chosen so that the reference fp32 order equals the exact fp64
    # order over the top-k; the default seed has two near-tie
    # flips (|d score| ~ 2e-8) at 100k, where the reference order is unspecified.
    for (n, q, k, tag, qseed) in ((100000, 70, 100, "100k", 77), (4096, 16, 32, "4k", 78)):
        db = data.database(n)
        qq = data.queries(q, seed=qseed)
        out["qseed_" + tag] = np.int64(qseed)
        scores = np.dot(db, qq.T)                      # == np.dot(vecs.T, qvecs) (test.py:247)
        ranks = np.argsort(-scores, axis=0)            # test.py:248
        s64, i64 = ops.topk_exact(db, qq, k)
        top = ranks[:k].T
        assert (top == i64).all(), "fp32 reference order != fp64 order; pick another seed"
        out["idx_" + tag] = top.astype(np.int32)
        out["score_" + tag] = np.take_along_axis(scores, ranks[:k], axis=0).T.astype(np.float32)
        out["shape_" + tag] = np.array([n, q, k])
        gaps = np.diff(-s64, axis=1)
        print("  knn %s: min adjacent fp64 gap in top-%d = %.3g" % (tag, k, gaps.min()))
    np.savez_compressed(os.path.join(HERE, "knn.npz"), **out)


# ----------------------------------------------------------------------------- G5
def gen_map():
    db, qq, gnd = data.map_problem()
    ranks = np.argsort(-np.dot(db, qq.T), axis=0)
    logs = []
    score = R_eval.compute_map_and_print("roxford5k", ranks, gnd, lambda *a: logs.append(a))
    old = R_eval.compute_map(ranks, [{"ok": np.concatenate([g["easy"], g["hard"]]), "junk": g["junk"]}
                                     for g in gnd], [1, 5, 10])
    mine = ops.compute_map_revisited(ranks, gnd)
    assert abs((mine["mapM"] + mine["mapH"]) / 2 * 100 - score["mAP"]) < 1e-12
    out = {"ranks": ranks.astype(np.int32), "score_mAP": np.float64(score["mAP"]),
           "old_map": np.float64(old[0]), "old_aps": old[1], "old_pr": old[2], "old_prs": old[3]}
    for key in ("easy", "hard", "junk"):
        out["gnd_" + key] = np.concatenate([g[key] for g in gnd]).astype(np.int64)
        out["gnd_" + key + "_len"] = np.array([len(g[key]) for g in gnd], dtype=np.int64)
    # E/M/H mAP and mP@k as the reference logs them
    for a in logs:
        print("  ", a[0] % tuple(a[1:]))
    for proto, okk, jk in (("E", ["easy"], ["junk", "hard"]), ("M", ["easy", "hard"], ["junk"]),
                           ("H", ["hard"], ["junk", "easy"])):
        g2 = [{"ok": np.concatenate([g[k] for k in okk]), "junk": np.concatenate([g[k] for k in jk])} for g in gnd]
        m, aps, pr, prs = R_eval.compute_map(ranks, g2, [1, 5, 10])
        out["map" + proto], out["aps" + proto], out["pr" + proto] = np.float64(m), aps, pr
    np.savez_compressed(os.path.join(HERE, "map.npz"), **out)


# ----------------------------------------------------------------------------- G6
def gen_whiten():
    d, n = 64, 600
    X = data.unit_rows(n, d, seed=601).T.astype(np.float64)  # D x N
    r = data.rng(602)
    qidxs = r.integers(0, n, 200)
    pidxs = (qidxs + r.integers(1, 5, 200)) % n
    m, P = R_whiten.whitenlearn(X, qidxs, pidxs)
    Y = R_whiten.whitenapply(X, m, P)
    Y32 = R_whiten.whitenapply(X.astype(np.float32), m.astype(np.float32), P.astype(np.float32), dimensions=32)
    np.savez_compressed(os.path.join(HERE, "whiten.npz"), qidxs=qidxs, pidxs=pidxs, m=m, P=P, Y=Y,
                        Y32=Y32, m32=m.astype(np.float32), P32=P.astype(np.float32))


# ----------------------------------------------------------------------------- G7
def gen_local():
    """localHead (config 5 head, local_head.py:19-71) on a random NCHW map and
    keypoints, reference module run unmodified."""
    from cirtorch.modules.heads.local_head import localHead as R_localHead
    r = data.rng(701)
    out = {}
    for tag, (b, c, h, w, n, e) in (("a", (2, 64, 13, 17, 50, 32)), ("b", (1, 128, 16, 24, 300, 128))):
        x = r.standard_normal((b, c, h, w)).astype(np.float32)
        kp = (r.random((b, n, 2)) * 2.2 - 1.1).astype(np.float32)   # some keypoints outside [-1, 1]
        head = R_localHead(c, e)
        sd = {"whiten.weight": (r.standard_normal((e, c)) * (1.0 / c) ** 0.5).astype(np.float32),
              "whiten.bias": (r.standard_normal(e) * 0.05).astype(np.float32)}
        head.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()})
        with torch.no_grad():
            ref = head(torch.from_numpy(x), torch.from_numpy(kp)).numpy()
        mine = ops.local_head(torch.from_numpy(x), torch.from_numpy(kp), torch.from_numpy(sd["whiten.weight"]),
                              torch.from_numpy(sd["whiten.bias"])).numpy()
        assert np.abs(ref - mine).max() < 1e-6, np.abs(ref - mine).max()
        out.update({"x_" + tag: x, "kpts_" + tag: kp, "w_" + tag: sd["whiten.weight"], "b_" + tag: sd["whiten.bias"],
                    "desc_" + tag: ref})
    # mutual NN between two descriptor sets of set b (oracle restatement of HPatchesEval.nn_matcher)
    d1 = out["desc_b"][0]
    d2 = (d1[::-1] + 0.05 * r.standard_normal(d1.shape)).astype(np.float32)
    d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
    out["nn_d2"] = d2
    out["nn_match"] = ops.nn_matcher(d1, d2)
    np.savez_compressed(os.path.join(HERE, "local.npz"), **out)


# ----------------------------------------------------------------------------- G8
def gen_nn_match():
    """The reference mutual-NN matcher itself (HPatchesEval.py:23-43).  That
    module imports cv2 at the top (for RANSAC homographies, not used by
    get_desc_dist / nn_matcher); cv2 is absent, so a test-only empty ``cv2``
    module is registered while it is imported (same recipe as inplace_abn)."""
    had = "cv2" in sys.modules
    if not had:
        sys.modules["cv2"] = types.ModuleType("cv2")
    try:
        from cirtorch.utils.evaluation import HPatchesEval as R_hp
    finally:
        if not had:
            del sys.modules["cv2"]
    out = {}
    for tag, (n1, n2, d, seed) in (("a", (300, 260, 128, 801)), ("b", (2048, 1900, 128, 802)), ("c", (7, 9, 16, 803))):
        d1, d2 = data.nn_descriptors(n1, n2, d, seed)
        dist = R_hp.get_desc_dist({"descriptors": d1}, {"descriptors": d2})
        match = R_hp.nn_matcher(dist)
        assert (match == ops.nn_matcher(d1, d2)).all()
        out["shape_" + tag] = np.array([n1, n2, d, seed])
        out["match_" + tag] = match.astype(np.int64)
        print("  nn %s: %d mutual of %d" % (tag, (match >= 0).sum(), n1))
    np.savez_compressed(os.path.join(HERE, "nnmatch.npz"), **out)


# ----------------------------------------------------------------------------- G9
def gen_transform():
    """ISSTestTransform (cirtorch/datasets/generic/transform.py:81-130) run
    unmodified on synthetic PIL images.  The module imports torchvision only for
    ``functional.to_tensor`` (absent here): a test-only stand-in with the
    published to_tensor of an RGB PIL image (HWC uint8 -> CHW float32 / 255) is
    registered while it is loaded.  The file is loaded directly so the dataset
    package __init__ (PIL-less dataset.py, samplers) is not imported."""
    import importlib.util
    from PIL import Image
    tv = types.ModuleType("torchvision")
    tvt = types.ModuleType("torchvision.transforms")
    tvf = types.ModuleType("torchvision.transforms.functional")

    def to_tensor(pic):
        a = np.asarray(pic, dtype=np.uint8)
        return torch.from_numpy(a.transpose(2, 0, 1).copy()).float().div(255)

    tvf.to_tensor = to_tensor
    tvt.functional = tvf
    tv.transforms = tvt
    saved = {k: sys.modules.get(k) for k in ("torchvision", "torchvision.transforms", "torchvision.transforms.functional")}
    sys.modules.update({"torchvision": tv, "torchvision.transforms": tvt, "torchvision.transforms.functional": tvf})
    try:
        spec = importlib.util.spec_from_file_location(
            "ref_generic_transform", os.path.join(REF, "cirtorch", "datasets", "generic", "transform.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    out = {}
    cfgs = [(64, 96, [0.8, 1.2]), (80, 80, [0.8, 1.2]), (48, 200, [0.8, 1.2])]
    for ci, (short, longest, rs) in enumerate(cfgs):
        tf = mod.ISSTestTransform(shortest_size=short, longest_max_size=longest, random_scale=rs)
        for ii, (w, h, bbx, pix) in enumerate(data.transform_images()):
            img = Image.fromarray(pix, mode="RGB")
            t = tf(img, bbx=bbx)["img"]
            u8 = np.rint(t.numpy() * 255.0).astype(np.uint8)
            assert np.array_equal(u8.astype(np.float32) / np.float32(255.0), t.numpy())
            out["out_%d_%d" % (ci, ii)] = u8
        out["cfg_%d" % ci] = np.array([short, longest])
    np.savez_compressed(os.path.join(HERE, "transform.npz"), **out)


GENERATORS = {
    "ops": lambda: gen_ops(),
    "r18": lambda: gen_net("resnet18", (224, 224), 8, 1001, [(1,), (0.5, 1, 2)], "r18.npz",
                           mixed=[(200, 240), (224, 192), (160, 160)]),
    "r50": lambda: gen_net("resnet50", (768, 1024), 2, 2001, [(1,)], "r50.npz"),
    "r50ms": lambda: gen_net("resnet50", (384, 512), 1, 2101, [(0.5, 1, 2)], "r50ms.npz"),
    "r101": lambda: gen_net("resnet101", (256, 320), 2, 2201, [(1,)], "r101.npz"),
    # config 3: R101 multi-scale x0.5/1/2 at the 768x1024 workload size
    "r101ms": lambda: gen_net("resnet101", (768, 1024), 1, 2301, [(1,), (0.5, 1, 2)], "r101ms.npz"),
    # config 5: R152 at 768x1024 + the local head on mod3
    "r152": lambda: gen_net("resnet152", (768, 1024), 1, 2401, [(1,)], "r152.npz", local=("mod3", 512, 128, 2402)),
    # a2: a ragged R50 batch at 768x1024 / 640x960 / 700x1000 (both pad orders)
    "r50mixed": lambda: gen_mixed("resnet50", [(768, 1024), (640, 960), (700, 1000)], 2501, "r50mixed.npz"),
    # the scripts/test.py call sequence on a synthetic roxford5k + Lw dataset
    "testpy": lambda: gen_testpy(),
    "knn": lambda: gen_knn(),
    "map": lambda: gen_map(),
    "whiten": lambda: gen_whiten(),
    "local": lambda: gen_local(),
    "nnmatch": lambda: gen_nn_match(),
    "transform": lambda: gen_transform(),
}


if __name__ == "__main__":
    names = sys.argv[1:] or list(GENERATORS)
    for name in names:
        print("golden", name)
        GENERATORS[name]()
    print("done")
