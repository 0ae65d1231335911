"""Replay of the upstream evaluation driver ``scripts/test.py:84-259`` as one
call sequence, on a small synthetic dataset written to disk in the upstream
formats (test infrastructure: used by tests/test_gpu_round4.py with the
product, and by tests/golden/make_golden.py with the oracle + the reference's
own whiten / evaluation modules).

The sequence (scripts/test.py line numbers):
  * ``torch.load`` of a ``{meta, state_dict}`` checkpoint -> net_params from
    the meta -> ``init_network`` -> ``load_state_dict``          (:89-106)
  * ``msp = net.pool.p`` for multi-scale GeM without whitening, else 1  (:135-142)
  * ``transform = Compose([ToTensor(), Normalize(meta mean, std)])`` (:149-156)
  * Lw: the ``<whitening>-whiten.pkl`` db, ``cid2filename`` images,
    ``extract_vectors(..., ms, msp)``, ``whitenlearn(wvecs, qidxs, pidxs)`` (:190-206)
  * ``configdataset`` -> ``extract_vectors`` of the database and of the
    queries with their ``bbx`` crops                              (:226-238)
  * ``np.dot`` / ``np.argsort`` -> ``compute_map_and_print``       (:247-249)
  * ``whitenapply`` of both -> rank again -> ``compute_map_and_print`` (:251-259)

Files are generated from a seed (numpy + PIL JPEG, quality 90); their sha1s
are stored in the golden so a different encoder cannot pass silently.
"""

import hashlib
import os
import pickle

import numpy as np

DATASET = "roxford5k"
WHITEN = "retrieval-SfM-120k"
ARCH = "resnet18"
IMAGE_SIZE = 160          # longest side after thumbnail (scripts/test.py --image-size)
WHITEN_SIZE = 96          # whitening images are decoded at this size
MS = [1, 1 / 2 ** 0.5, 2 ** 0.5]
N_DB, N_Q, N_W, N_PAIRS = 40, 8, 640, 1600
MEAN, STD = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]


def _cid(i):
    return hashlib.md5(b"cid%d" % i).hexdigest()


def _field_image(r, h, w):
    """a structured random image (smooth colour field + noise), uint8 HWC"""
    gh, gw = 3 + int(r.integers(0, 4)), 4 + int(r.integers(0, 4))
    field = r.random((gh, gw, 3))
    ys = np.linspace(0, gh - 1, h)
    xs = np.linspace(0, gw - 1, w)
    y0 = np.clip(ys.astype(int), 0, gh - 2)
    x0 = np.clip(xs.astype(int), 0, gw - 2)
    fy, fx = (ys - y0)[:, None, None], (xs - x0)[None, :, None]
    f = (field[y0][:, x0] * (1 - fy) * (1 - fx) + field[y0 + 1][:, x0] * fy * (1 - fx)
         + field[y0][:, x0 + 1] * (1 - fy) * fx + field[y0 + 1][:, x0 + 1] * fy * fx)
    return (np.clip(0.75 * f + 0.25 * r.random((h, w, 3)), 0, 1) * 255).astype(np.uint8)


def make_dataset(root, seed=4242):
    """write <root>/test/roxford5k/{jpg/*.jpg, gnd_roxford5k.pkl} and
    <root>/train/retrieval-SfM-120k/{ims/.., retrieval-SfM-120k-whiten.pkl};
    returns {relative path: sha1} of every image file"""
    from PIL import Image
    r = np.random.default_rng(seed)
    hashes = {}

    def save(path, arr):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        Image.fromarray(arr).save(path, format="JPEG", quality=90)
        hashes[os.path.relpath(path, root)] = hashlib.sha1(open(path, "rb").read()).hexdigest()

    droot = os.path.join(root, "test", DATASET)
    imlist = ["db%03d" % i for i in range(N_DB)]
    qimlist = ["q%02d" % i for i in range(N_Q)]
    for name in imlist + qimlist:
        h, w = int(r.integers(120, 200)), int(r.integers(150, 260))
        save(os.path.join(droot, "jpg", name + ".jpg"), _field_image(r, h, w))
    gnd = []
    for qi in range(N_Q):
        perm = r.permutation(N_DB)
        w_, h_ = 150, 120
        x0, y0 = int(r.integers(0, 40)), int(r.integers(0, 30))
        gnd.append({"bbx": [float(x0), float(y0), float(x0 + int(r.integers(70, w_ - x0 + 1))),
                            float(y0 + int(r.integers(60, h_ - y0 + 1)))],
                    "easy": perm[:6].tolist(), "hard": perm[6:10].tolist(), "junk": perm[10:12].tolist()})
    with open(os.path.join(droot, "gnd_%s.pkl" % DATASET), "wb") as f:
        pickle.dump({"imlist": imlist, "qimlist": qimlist, "gnd": gnd}, f)

    wroot = os.path.join(root, "train", WHITEN)
    cids = [_cid(i) for i in range(N_W)]
    from_cid = lambda cid: os.path.join(wroot, "ims", cid[-2:], cid[-4:-2], cid[-6:-4], cid)  # noqa: E731
    for cid in cids:
        h, w = int(r.integers(60, 100)), int(r.integers(70, 120))
        save(from_cid(cid), _field_image(r, h, w))
    qidxs = r.integers(0, N_W, N_PAIRS)
    pidxs = (qidxs + r.integers(1, 5, N_PAIRS)) % N_W
    with open(os.path.join(wroot, "%s-whiten.pkl" % WHITEN), "wb") as f:
        pickle.dump({"cids": cids, "qidxs": qidxs.tolist(), "pidxs": pidxs.tolist()}, f)
    return hashes


def checkpoint(path, whitening, head_bias=None):
    """the {meta, state_dict} file of scripts/test.py:89-106, random weights from the
    oracle's generator in the engine's module layout"""
    import torch
    from oracle import weights
    sd = {"body." + k: torch.from_numpy(v) for k, v in weights.backbone_state(ARCH).items()}
    hs = weights.head_state(weights.OUTPUT_DIM[ARCH])
    if head_bias is not None:
        hs["whiten.bias"] = head_bias
    sd.update({"ret_head." + k: torch.from_numpy(v) for k, v in hs.items()})
    meta = {"architecture": ARCH, "pooling": "gem", "local_whitening": False, "regional": False,
            "whitening": whitening, "mean": MEAN, "std": STD}
    torch.save({"meta": meta, "state_dict": sd}, path)


def run(api, root, ckpt):
    """scripts/test.py:84-259 through `api` (a namespace: load_net(state) -> net,
    extract_vectors, whitenlearn, whitenapply, compute_map, to_numpy) ->
    {ranks, map, ranks_lw, map_lw, vecs, qvecs, msp}"""
    import torch
    state = torch.load(ckpt, map_location="cpu", weights_only=True)
    net, meta, p = api.load_net(state)
    ms = list(MS)
    msp = p if (len(ms) > 1 and meta["pooling"] == "gem" and not meta.get("regional", False)
                and not meta.get("whitening", False)) else 1
    # Lw from the whitening db (:190-206)
    wroot = os.path.join(root, "train", WHITEN)
    with open(os.path.join(wroot, "%s-whiten.pkl" % WHITEN), "rb") as f:
        db = pickle.load(f)
    wimages = [api.cid2filename(db["cids"][i], os.path.join(wroot, "ims")) for i in range(len(db["cids"]))]
    wvecs = api.to_numpy(api.extract_vectors(net, wimages, WHITEN_SIZE, None, ms, msp))
    m, P = api.whitenlearn(wvecs, db["qidxs"], db["pidxs"])
    # the test dataset (:226-238)
    cfg = api.configdataset(DATASET, os.path.join(root, "test"))
    images = [cfg["im_fname"](cfg, i) for i in range(cfg["n"])]
    qimages = [cfg["qim_fname"](cfg, i) for i in range(cfg["nq"])]
    bbxs = [tuple(cfg["gnd"][i]["bbx"]) for i in range(cfg["nq"])]
    vecs = api.to_numpy(api.extract_vectors(net, images, IMAGE_SIZE, None, ms, msp))
    qvecs = api.to_numpy(api.extract_vectors(net, qimages, IMAGE_SIZE, bbxs, ms, msp))
    # rank + mAP, then with Lw (:247-259)
    scores = np.dot(vecs.T, qvecs)
    ranks = np.argsort(-scores, axis=0)
    map0 = api.compute_map(DATASET, ranks, cfg["gnd"])
    vecs_lw = api.whitenapply(vecs, m, P)
    qvecs_lw = api.whitenapply(qvecs, m, P)
    ranks_lw = np.argsort(-np.dot(vecs_lw.T, qvecs_lw), axis=0)
    map_lw = api.compute_map(DATASET + " + whiten", ranks_lw, cfg["gnd"])
    return {"ranks": ranks, "map": map0, "ranks_lw": ranks_lw, "map_lw": map_lw, "vecs": vecs, "qvecs": qvecs,
            "msp": msp}
