"""End-to-end pipelines on the GPU engine:
* the upstream ``extract_vectors`` front end on real image files (PIL decode,
  longest side -> image_size, ToTensor + Normalize semantics, ms/msp rule);
* config 4's flow: extract DB + query descriptors, GPU full ranks, mAP with the
  reference protocol — ranks identical to ``np.argsort`` on the same vectors,
  mAP equal to the oracle's on the oracle's descriptors within 1e-3."""

import os

import numpy as np
import pytest
import torch

from conftest import cosines

pytestmark = pytest.mark.gpu

MEAN, STD = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]


def _product_and_oracle(arch, cuda):
    from cirtorch.models.GF_net import make_net
    from oracle import backbone as obb, weights
    bs = weights.backbone_state(arch)
    hs = weights.head_state(weights.OUTPUT_DIM[arch])
    net = make_net(arch, precision="fp32", mean=MEAN, std=STD)
    net.body.load_state_dict({k: torch.from_numpy(v) for k, v in bs.items()}, strict=False)
    net.ret_head.load_state_dict({k: torch.from_numpy(v) for k, v in hs.items()})
    return net.to(cuda).eval(), obb.OracleNet(arch, bs, hs)


def test_extract_vectors_from_image_files(cuda, tmp_path):
    from PIL import Image
    from cirtorch.models.GF_net import extract_vectors, _load_pil, _to_tensor
    from oracle import data, backbone as obb
    net, onet = _product_and_oracle("resnet18", cuda)
    paths = []
    imgs = data.structured_images(3, 150, 200, seed=41)
    for i, im in enumerate(imgs):
        arr = (np.clip(im.transpose(1, 2, 0), 0, 1) * 255).astype(np.uint8)
        p = os.path.join(str(tmp_path), "im%d.png" % i)
        Image.fromarray(arr).save(p)
        paths.append(p)
    bbxs = [None, (10, 20, 120, 140), None]
    # msp = p only applies to un-whitened GeM nets upstream (scripts/test.py:136-137); whitened -> msp = 1
    for ms, msp in (([1], 1), ([1, 0.5], 1.0)):
        vecs = extract_vectors(net, paths, 96, ms=ms, msp=msp, bbxs=[b if b else (0, 0, 200, 150) for b in bbxs])
        assert vecs.shape == (512, 3)
        # oracle on the same decoded tensors
        for i, p in enumerate(paths):
            x = _to_tensor(_load_pil(p, 96, bbxs[i] if bbxs[i] else (0, 0, 200, 150)))
            xn = obb.normalize_images(x)
            if ms == [1]:
                ref = onet.forward([xn], normalize=False)[:, 0]
            else:
                acc = 0
                for s in ms:
                    xs = xn if s == 1 else torch.nn.functional.interpolate(
                        xn[None], scale_factor=s, mode="bilinear", align_corners=False)[0]
                    acc = acc + onet.forward([xs], normalize=False)[:, 0].double() ** msp
                ref = (acc / len(ms)) ** (1.0 / msp)
                ref = ref / ref.norm()
            assert cosines(vecs[:, i:i + 1].numpy(), ref[:, None].numpy())[0] > 1 - 1e-4


def test_config4_rank_and_map(cuda):
    """roxford-shaped flow on a small synthetic set: descriptors from the
    engine, ranks on the GPU, mAP with the revisited protocol."""
    from cirtorch.search import rank
    from cirtorch.utils.evaluation.ParisOxfordEval import compute_map_and_print
    from oracle import data, ops, backbone as obb
    net, onet = _product_and_oracle("resnet18", cuda)
    ndb, nq = 60, 6
    db_imgs = data.structured_images(ndb, 64, 80, seed=51)
    q_imgs = db_imgs[:nq] * 0.9 + 0.05          # queries = perturbed copies of the first DB images
    to_dev = [torch.from_numpy(im).to(cuda) for im in db_imgs]
    vecs = net.extract(to_dev).cpu()              # D x ndb
    qvecs = net.extract([torch.from_numpy(im).to(cuda) for im in q_imgs]).cpu()
    ref_vecs = onet.forward([torch.from_numpy(im) for im in db_imgs]).numpy()
    ref_q = onet.forward([torch.from_numpy(im) for im in q_imgs]).numpy()
    assert cosines(vecs.numpy(), ref_vecs).min() > 1 - 1e-4
    # GPU full ranks == np.argsort on the same vectors (exact fp64 order; stable ties)
    ranks = rank(vecs, qvecs).cpu().numpy()
    ref_ranks = np.argsort(-np.dot(vecs.double().numpy().T, qvecs.double().numpy()), axis=0, kind="stable")
    np.testing.assert_array_equal(ranks, ref_ranks)
    # mAP vs the oracle pipeline (reference descriptors + numpy rank)
    r = data.rng(52)
    gnd = [{"easy": np.array([i]), "hard": r.choice(np.arange(nq, ndb), 2, replace=False),
            "junk": np.array([], dtype=np.int64)} for i in range(nq)]
    got = compute_map_and_print("roxford5k", ranks, gnd, lambda *a: None)
    _, oranks = ops.rank_reference(ref_vecs.T.copy(), ref_q.T.copy())
    ref = ops.compute_map_revisited(oranks, gnd)
    assert abs(got["mAP"] - 100 * (ref["mapM"] + ref["mapH"]) / 2) < 1e-3 * 100


def test_extract_vectors_uint8_files_equal_float_tensors(cuda, tmp_path):
    """Image files go to the GPU as uint8 pixels (fused stem reads x / 255):
    bit-identical to extract_vectors on the float32 to_tensor images (bf16 net,
    fused stem) and to the fp32 net's float path."""
    from PIL import Image
    from cirtorch.models.GF_net import extract_vectors, make_net, _load_pil, _to_tensor
    from cirtorch.models.init import random_init_
    from oracle import data
    paths = []
    for i, im in enumerate(data.structured_images(2, 150, 200, seed=61)):
        arr = (np.clip(im.transpose(1, 2, 0), 0, 1) * 255).astype(np.uint8)
        p = os.path.join(str(tmp_path), "u%d.png" % i)
        Image.fromarray(arr).save(p)
        paths.append(p)
    for prec in ("bf16", "fp32"):
        net = make_net("resnet18", precision=prec, mean=MEAN, std=STD)
        random_init_(net, seed=4)
        net = net.to(cuda).eval()
        a = extract_vectors(net, paths, 128)
        b = extract_vectors(net, [_to_tensor(_load_pil(p, 128)) for p in paths], 128)
        assert torch.equal(a, b), prec


def _write_pngs(tmp_path, n_distinct, h, w, copies, seed):
    from PIL import Image
    from oracle import data
    paths = []
    for i, im in enumerate(data.structured_images(n_distinct, h, w, seed=seed)):
        arr = (np.clip(im.transpose(1, 2, 0), 0, 1) * 255).astype(np.uint8)
        p = os.path.join(str(tmp_path), "b%d.png" % i)
        Image.fromarray(arr).save(p, compress_level=1)
        paths.append(p)
    return [paths[i % n_distinct] for i in range(n_distinct * copies)]


@pytest.mark.parametrize("prec", ["fp16", "fp32"])
def test_extract_vectors_batched_equals_batch1(cuda, tmp_path, prec):
    """extract_vectors groups same-size images into chains (pinned uint8
    pixels, copy stream double-buffered against the extractor); every column
    equals the batch-1 extraction of that image (one call per file) up to the
    kernel variant the chain size selects (fp32: one kernel family, identical)."""
    from cirtorch.models.GF_net import extract_vectors, make_net
    from cirtorch.models.init import random_init_
    net = make_net("resnet50", precision=prec, mean=MEAN, std=STD)
    random_init_(net, seed=6)
    net = net.to(cuda).eval()
    paths = _write_pngs(tmp_path, 6, 240, 320, 4, seed=71)          # 24 same-size files
    other = tmp_path / "other"
    other.mkdir()
    paths.insert(5, _write_pngs(other, 1, 200, 300, 1, seed=72)[0])    # one image of another size
    vecs = extract_vectors(net, paths, None, batch=8, workers=4)
    one = torch.cat([extract_vectors(net, [p], None) for p in paths[:9]], dim=1)
    d = (vecs[:, :9] - one).abs().max().item()
    print(prec, "batched vs batch-1 max |d|", d)
    assert cosines(vecs[:, :9].numpy(), one.numpy()).min() > 1 - 1e-6
    if prec == "fp32":
        assert d < 1e-6
    # the same file appears several times: identical columns
    assert torch.equal(vecs[:, 0], vecs[:, 6 + 1])


def test_extract_vectors_iss_test_transform(cuda, tmp_path):
    """test_transform=ISSTestTransform: the in-tree loaders' resize rule (shortest
    side -> shortest_size, longest capped) feeds the engine as uint8 pixels;
    equal to extracting the transform's float output."""
    from PIL import Image
    from cirtorch.datasets.generic import ISSTestTransform
    from cirtorch.models.GF_net import extract_vectors, make_net
    from cirtorch.models.init import random_init_
    net = make_net("resnet18", precision="fp16", mean=MEAN, std=STD)
    random_init_(net, seed=8)
    net = net.to(cuda).eval()
    paths = _write_pngs(tmp_path, 3, 150, 210, 1, seed=81)
    tf = ISSTestTransform(shortest_size=96, longest_max_size=128, random_scale=[0.8, 1.2])
    bbxs = [None, (5, 10, 180, 140), None]
    a = extract_vectors(net, paths, None, bbxs=bbxs, test_transform=tf)
    imgs = []
    for p, b in zip(paths, bbxs):
        with open(p, "rb") as f:
            imgs.append(tf(Image.open(f).convert("RGB"), bbx=b)["img"])
    b_ = extract_vectors(net, imgs, None)
    assert torch.equal(a, b_)
    assert tuple(imgs[0].shape[1:]) == tf.output_size(210, 150)[::-1] == (91, 128)
    assert tuple(imgs[1].shape[1:]) == tf.output_size(175, 130)[::-1]


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_backbone_mod3_boundary_fusion_bit_identical(cuda, prec, monkeypatch):
    """ResNet-50 body with the 128/512 boundaries fused (k_pair_mid, default)
    vs the same body with them as two launches (RR_PAIR_MID=0): every stage
    output bit-identical (same MFMA K-step order and roundings)."""
    from cirtorch.backbones import resnet
    from cirtorch.models.init import random_init_
    body = resnet.resnet50(precision=prec)
    random_init_(body, 3)
    body = body.to(cuda).eval()
    x = torch.rand(2, 3, 256, 512, generator=torch.Generator().manual_seed(4)).to(cuda)
    with torch.no_grad():
        fused = body(x)
        monkeypatch.setenv("RR_PAIR_MID", "0")
        plain = body(x)
    for k in fused:
        assert torch.equal(fused[k], plain[k]), k
