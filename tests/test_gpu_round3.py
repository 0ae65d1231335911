"""GPU checks of the round-3 surface through librr.so: a ResidualBlock called on
its own (reference ``cirtorch/backbones/misc.py:184-203``), a model built the
``make_model`` way (``scripts/train_globalF.py:240-356``) extracting the same
descriptors after a snapshot round trip (``utils/snapshot.py:41-75``), and the
multi-scale forward's loss dict (``models/GF_net.py:89-92``)."""

import pytest
import torch
import torch.nn.functional as F

from test_host_round3 import _body_section, _make_model

pytestmark = pytest.mark.gpu


def _block_reference(blk, x):
    """float64 restatement of ResidualBlock.forward (misc.py:163-203) with eval BN"""
    def bn(m, t):
        inv = torch.rsqrt(m.running_var.double() + m.eps)
        s = m.weight.double() * inv
        return t * s[None, :, None, None] + (m.bias.double() - m.running_mean.double() * s)[None, :, None, None]

    def act(m, t):
        return F.leaky_relu(t, m.activation_param) if m.activation == "leaky_relu" else t

    c = blk.convs
    names = ["1", "2", "3"] if blk.is_bottleneck else ["1", "2"]
    y = x
    for i, k in enumerate(names):
        conv, b = getattr(c, "conv" + k), getattr(c, "bn" + k)
        y = bn(b, F.conv2d(y, conv.weight.double(), stride=conv.stride, padding=conv.padding))
        if i + 1 < len(names):
            y = act(b, y)
    res = bn(blk.proj_bn, F.conv2d(x, blk.proj_conv.weight.double(), stride=blk.proj_conv.stride)) \
        if hasattr(blk, "proj_conv") else x
    return act(c.bn1, y + res)


@pytest.mark.parametrize("precision", ["fp32", "bf16", "fp16"])
@pytest.mark.parametrize("arch,mod,block", [("resnet50", 3, 1), ("resnet50", 2, 2), ("resnet18", 4, 1)])
def test_residual_block_standalone(cuda, precision, arch, mod, block):
    from cirtorch.backbones import resnet
    from cirtorch.models.init import random_init_
    body = resnet.__dict__[arch](precision=precision)
    random_init_(body, 3)
    blk = getattr(getattr(body, "mod%d" % mod), "block%d" % block)
    cin = blk.convs.conv1.in_channels
    g = torch.Generator().manual_seed(11)
    x = torch.randn(2, cin, 24, 32, generator=g)
    body = body.to(cuda).eval()
    dt = body.engine_dtype
    xq = x.to(dt).float()  # the engine's operand rounding of the input
    ref = _block_reference(blk.cpu(), xq.double())
    blk.to(cuda)
    got = blk(x.to(cuda))
    assert got.dtype == torch.float32 and got.shape == ref.shape
    err = (got.cpu().double() - ref).abs().max().item()
    scale = ref.abs().max().item()
    tol = {"fp32": 2e-5, "bf16": 3e-2, "fp16": 5e-3}[precision]
    assert err <= tol * scale, (err, scale)
    # in the engine dtype the block returns an NCHW-shaped view of its NHWC buffer
    got16 = blk(x.to(cuda).to(dt))
    assert got16.dtype == dt and got16.shape == ref.shape


def test_block_chain_equals_body_stage(cuda):
    """fp32: the stage map of the fused body equals its blocks called one by one"""
    from cirtorch.backbones import resnet
    from cirtorch.models.init import random_init_
    body = resnet.resnet50(precision="fp32")
    random_init_(body, 5)
    body = body.to(cuda).eval()
    x = torch.rand(2, 3, 128, 160, device=cuda)
    with torch.no_grad():
        outs = body(x)
        t = outs["mod3"].float()
        for blk in body.mod4.children():
            t = blk(t)
    assert torch.equal(t, outs["mod4"].float())


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_make_model_snapshot_descriptors(cuda, tmp_path, precision):
    """the make_model-built net extracts the same descriptors after
    save_snapshot -> resume_from_snapshot into a fresh net (engine plans rebuilt)"""
    from cirtorch.models.init import random_init_
    from cirtorch.utils.snapshot import resume_from_snapshot, save_snapshot
    cp = _body_section()
    src, _, _ = _make_model(cp, "resnet50")
    random_init_(src, 7)
    src.body.set_precision(precision)
    path = str(tmp_path / "snap.pth")
    save_snapshot(path, cp, 1, 0.0, 0.0, 10, body=src.body.state_dict(), ret_head=src.ret_head.state_dict())
    src = src.to(cuda).eval()
    imgs = torch.rand(2, 3, 224, 288, device=cuda)
    ref = src.extract(imgs)
    dst, _, _ = _make_model(cp, "resnet50")
    random_init_(dst, 8)
    dst.body.set_precision(precision)
    dst = dst.to(cuda).eval()
    before = dst.extract(imgs)
    resume_from_snapshot(dst, path, ["body", "ret_head"])
    dst = dst.to(cuda)
    got = dst.extract(imgs)
    assert not torch.equal(before, ref)
    assert torch.equal(got, ref)


def test_multiscale_forward_returns_loss_dict(cuda):
    from cirtorch.models.GF_net import make_net
    from cirtorch.models.init import random_init_
    from cirtorch.utils.parallel import PackedSequence
    net = random_init_(make_net("resnet18", precision="bf16"), 1).to(cuda).eval()
    imgs = torch.rand(2, 3, 96, 128, device=cuda)
    with torch.no_grad():
        for img in (imgs, PackedSequence(list(imgs))):
            loss, pred = net(img=img, scales=[0.5, 1])
            assert list(loss.keys()) == ["ret_loss"] and loss["ret_loss"] is None
            assert pred["ret_pred"].shape == (512, 2)


def test_fp16_overflow_falls_back_to_bf16(cuda):
    """a checkpoint whose activations leave fp16 range (stem BN gamma x 1e6): the fp16
    descriptors would be inf / NaN; extract_vectors returns the bf16 ones instead"""
    from cirtorch.models.GF_net import extract_vectors, make_net
    from cirtorch.models.init import random_init_
    net = random_init_(make_net("resnet18", precision="fp16", mean=[0.485, 0.456, 0.406],
                                std=[0.229, 0.224, 0.225]), 2)
    with torch.no_grad():
        net.body.mod1.bn1.weight.mul_(1e6)
    net.body.refresh_engine()
    net = net.to(cuda).eval()
    imgs = [torch.randint(0, 256, (3, 96, 128), dtype=torch.uint8) for _ in range(3)]
    with torch.no_grad():
        raw = net.extract(torch.stack(imgs).to(cuda))
    assert not torch.isfinite(raw).all()  # the fp16 chain overflowed
    with pytest.warns(UserWarning, match="overflowed fp16"):
        got = extract_vectors(net, imgs, None, batch=2)
    assert net.body.engine_dtype == torch.float16
    net.body.set_precision("bf16")
    ref = extract_vectors(net, imgs, None, batch=2)
    assert torch.isfinite(got).all() and torch.equal(got, ref)


@pytest.mark.parametrize("layout", ["nchw", "nhwc"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_pool_propagates_nan_like_torch(cuda, layout, dtype):
    """GeM / MAC / SPoC keep a NaN activation (torch.clamp(min=eps) and max keep it,
    pools.py:10-38): only the channel holding it is NaN, the others match torch"""
    from cirtorch.layers import functional as LF
    g = torch.Generator().manual_seed(3)
    x = torch.rand(2, 64, 5, 7, generator=g).to(dtype)
    x[1, 9, 2, 3] = float("nan")
    x[0, 17, 4, 6] = float("nan")
    xd = x.to(cuda)
    if layout == "nhwc":
        xd = xd.contiguous(memory_format=torch.channels_last)
    xf = x.double()
    refs = {"gem": xf.clamp(min=1e-6).pow(3).mean(dim=(2, 3)).pow(1.0 / 3),
            "mac": xf.amax(dim=(2, 3)), "spoc": xf.mean(dim=(2, 3))}
    for name, fn in (("gem", LF.gem), ("mac", LF.mac), ("spoc", LF.spoc)):
        got = fn(xd).reshape(2, 64).cpu().double()
        ref = refs[name]
        assert torch.equal(torch.isnan(got), torch.isnan(ref)), name
        ok = ~torch.isnan(ref)
        assert torch.allclose(got[ok], ref[ok], rtol=1e-5, atol=1e-6), name


def test_extract_vectors_device_tensors(cuda):
    """same-size GPU tensors are stacked on the device (no pinned host staging)"""
    from cirtorch.models.GF_net import extract_vectors, make_net
    from cirtorch.models.init import random_init_
    net = random_init_(make_net("resnet18", precision="bf16"), 4).to(cuda).eval()
    imgs = [torch.rand(3, 64, 96) for _ in range(3)]
    host = extract_vectors(net, imgs, None, batch=4)
    dev = extract_vectors(net, [t.to(cuda) for t in imgs], None, batch=4)
    assert torch.equal(host, dev)



def test_extract_vectors_process_decoder_equals_threads_and_batch1(cuda, tmp_path, monkeypatch):
    """A file list long enough for the process decoder (>= 2 x batch: spawned
    workers, page-locked shared-memory ring, grouped tasks, early short chains)
    gives the same bits as decode threads and as one image at a time; mixed sizes,
    bbx crops, JPEG and PNG."""
    import numpy as np
    from PIL import Image
    from cirtorch.models.GF_net import extract_vectors, make_net
    from cirtorch.models.init import random_init_
    net = random_init_(make_net("resnet18", precision="bf16"), 6).to(cuda).eval()
    r = np.random.default_rng(8)
    paths, bbxs = [], []
    for i in range(22):
        h, w = [(96, 128), (128, 96), (80, 112)][i % 3]
        a = (r.random((h, w, 3)) * 255).astype(np.uint8)
        p = str(tmp_path / ("f%02d.%s" % (i, "jpg" if i % 2 else "png")))
        Image.fromarray(a).save(p)
        paths.append(p)
        bbxs.append((3, 5, w - 7, h - 2) if i % 5 == 0 else None)
    procs = extract_vectors(net, paths, None, bbxs=bbxs, batch=4)
    monkeypatch.setenv("RR_DECODE_PROCS", "0")
    threads = extract_vectors(net, paths, None, bbxs=bbxs, batch=4)
    assert torch.equal(procs, threads)
    for i in (0, 7, 21):
        one = extract_vectors(net, [paths[i]], None, bbxs=[bbxs[i]], batch=4)
        assert torch.equal(procs[:, i:i + 1], one), i


def _unit_rows(n, d, seed, dup_every=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, d, generator=g)
    if dup_every:
        x[dup_every::dup_every] = x[0]  # exact duplicates: equal float64 scores -> index order
    return x / x.norm(dim=1, keepdim=True)


@pytest.mark.parametrize("n,nq,d", [(20000, 7, 2048), (9000, 17, 512), (4099, 3, 256)])
def test_rank_full_vs_numpy(cuda, n, nq, d):
    """rr_rank_full (any N) == np.argsort of the float64 scores with ties to the lower
    index (scripts/test.py:247-248 order, exact scores), incl. exact duplicate rows"""
    import numpy as np
    from cirtorch.search import rank
    db = _unit_rows(n, d, 1, dup_every=997)
    q = _unit_rows(nq, d, 2)
    got = rank(db.t().to(cuda), q.t().to(cuda), method="full").cpu().numpy()
    s = db.double().numpy() @ q.double().numpy().T               # [n, nq]
    for j in range(nq):
        ref = np.lexsort((np.arange(n), -s[:, j]))
        np.testing.assert_array_equal(got[:, j], ref)


def test_rank_full_equals_knn_pipeline(cuda):
    """the float64 score of rr_rank_full is rr_knn_topk's re-score: at N = 8192 the two
    full rankings are identical, and the first k of a 30000-row ranking equal top-k"""
    from cirtorch.search import knn, rank
    db = _unit_rows(8192, 2048, 3, dup_every=1001).t().to(cuda)
    q = _unit_rows(9, 2048, 4).t().to(cuda)
    assert torch.equal(rank(db, q, method="full"), rank(db, q, method="knn"))
    db2 = _unit_rows(30000, 2048, 5, dup_every=4999).t().to(cuda)
    r = rank(db2, q)
    top, _ = knn(db2, q, 100)
    assert torch.equal(r[:100], top)


@pytest.mark.parametrize("precision", ["bf16", "fp16"])
def test_batch_invariant_descriptors(cuda, precision):
    """image 0 of an 8-image chain gets the same bits as the image alone, although
    the kernel a layer runs on depends on the batch (CU cap 16: the mod4 / mod5 3x3s
    take k_gemm8 at 8 images and the direct kernel at 1) -- extract_vectors' batched
    drop-in path returns what batch 1 returns"""
    from cirtorch import _engine as E
    from cirtorch.models.GF_net import make_net
    from cirtorch.models.init import random_init_
    mean, std = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]
    net = random_init_(make_net("resnet50", precision=precision, mean=mean, std=std), 6).to(cuda).eval()
    g = torch.Generator().manual_seed(2)
    x = torch.randint(0, 256, (8, 3, 768, 1024), generator=g, dtype=torch.uint8).to(cuda)
    try:
        E.check(E.lib().rr_set_tuning(7, 16), "rr_set_tuning")
        with torch.no_grad():
            many = net.extract(x)
            one = net.extract(x[3:4].clone())
    finally:
        E.lib().rr_set_tuning(7, 0)
    assert torch.equal(many[:, 3:4], one)


@pytest.mark.parametrize("nq", [77, 300])
@pytest.mark.parametrize("cap", [9, 64])
def test_search_with_capped_grid_equals_full_grid(cuda, nq, cap):
    """The persistent score GEMMs (k_gemm8s at <= 128 queries, k_gemm8 above) on a
    capped grid (RR_TUNE_GRID_CUS, as bench.py --search-cus sets around the step's
    search) give the same ranks and scores as on the whole chip."""
    from cirtorch import _engine as E
    from cirtorch.search import KnnIndex
    db = _unit_rows(200_000, 2048, seed=31).to(cuda)
    q = _unit_rows(nq, 2048, seed=32).to(cuda)
    idx = KnnIndex(db, "bf16")
    s0, i0 = idx.search(q, 50, verify=False)
    E.check(E.lib().rr_set_tuning(7, cap), "rr_set_tuning")
    try:
        s1, i1 = idx.search(q, 50, verify=False)
    finally:
        E.lib().rr_set_tuning(7, 0)
    assert torch.equal(i0, i1) and torch.equal(s0, s1)
