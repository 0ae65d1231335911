"""The fused 256-channel-stage block (rr_conv3x3_pair: conv2 3x3 + conv3 + shortcut of block i and
conv1 of block i + 1, cirtorch/backbones/misc.py:163-203, in one launch with t2 kept on chip) vs
the two unfused launches (the 3x3 kernel, then rr_conv1x1_pair): y and z bit-identical — same
MFMA K-step order and the same 16-bit rounding of t2 — for the dynamic (per-XCD tile queue) and
the static tile walk, and vs a float64 restatement.  GPU only."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _case(cuda, dt, n, h, w, c_out, proj, seed):
    from cirtorch import _ops as ops
    rnd = lambda t: t.to(dt).float()  # noqa: E731
    g = torch.Generator().manual_seed(seed)
    t1 = rnd(torch.randn(n, 64, h, w, generator=g))
    xin = rnd(torch.randn(n, 64, h, w, generator=g))
    w33 = rnd(torch.randn(64, 64, 3, 3, generator=g) * (2.0 / 576) ** 0.5)
    w3 = rnd(torch.randn(256, 64, 1, 1, generator=g) * (2.0 / 64) ** 0.5)
    wpj = rnd(torch.randn(256, 64, 1, 1, generator=g) * (2.0 / 64) ** 0.5)
    w1 = rnd(torch.randn(c_out, 256, 1, 1, generator=g) * (2.0 / 256) ** 0.5)
    aff = lambda c: (torch.rand(c, generator=g) + 0.5, torch.randn(c, generator=g) * 0.1)  # noqa: E731
    (s2, h2), (s3, h3), (sp, hp), (s1, h1) = aff(64), aff(256), aff(256), aff(c_out)
    res = rnd(torch.randn(n, 256, h, w, generator=g))

    def nhwc(t):
        return t.permute(0, 2, 3, 1).contiguous().to(dt).to(cuda)

    dev = lambda *ts: [t.to(cuda) for t in ts]  # noqa: E731
    s2d, h2d, s3d, h3d, spd, hpd, s1d, h1d = dev(s2, h2, s3, h3, sp, hp, s1, h1)
    w33p = ops.pack_conv_weights(w33.to(cuda), 64, dt, perm32=True)
    w3p = ops.pack_conv_weights(w3.to(cuda), 64, dt, perm32=True)
    wpp = ops.pack_conv_weights(wpj.to(cuda), 64, dt, perm32=True)
    w1p = ops.pack_conv_weights(w1.to(cuda), 256, dt, perm32=True)
    t1e, xe, re = nhwc(t1), nhwc(xin), nhwc(res)
    pj = (xe, wpp, spd, hpd) if proj else None
    r = None if proj else re
    y, z = ops.conv3x3_pair(t1e, w33p, s2d, h2d, True, 0.01, w3p, s3d, h3d, r, True, 0.01,
                            w1p, s1d, h1d, c_out, True, 0.01, proj=pj, dynamic=True)
    # the static tile walk: same bits
    ys, zs = ops.conv3x3_pair(t1e, w33p, s2d, h2d, True, 0.01, w3p, s3d, h3d, r, True, 0.01,
                              w1p, s1d, h1d, c_out, True, 0.01, proj=pj, dynamic=False)
    assert torch.equal(y, ys) and torch.equal(z, zs)
    # the unfused launches
    t2 = ops.conv2d_fused(t1e, w33p, 3, 3, 1, 1, 64, s2d, h2d, leaky=True, slope=0.01, perm32=True)
    y2, z2 = ops.conv1x1_pair(t2, w3p, s3d, h3d, r, True, 0.01, w1p, s1d, h1d, c_out, True, 0.01, proj=pj)

    def col(v):
        return v.double()[None, :, None, None]

    # float64 restatement (16-bit roundings of t2 and y where the engine stores them)
    t2r = rnd(F.leaky_relu(F.conv2d(t1.double(), w33.double(), padding=1) * col(s2) + col(h2), 0.01).float())
    short = F.conv2d(xin.double(), wpj.double()) * col(sp) + col(hp) if proj else res.double()
    yr = F.leaky_relu(F.conv2d(t2r.double(), w3.double()) * col(s3) + col(h3) + short, 0.01)
    zr = F.leaky_relu(F.conv2d(rnd(yr.float()).double(), w1.double()) * col(s1) + col(h1), 0.01)
    return y, z, y2, z2, yr, zr


CASES = [
    # n, h, w, c_out, projection
    (2, 16, 64, 64, False),      # 16 tiles: 2 blocks of 8 per XCD slot, one tile each
    (3, 20, 96, 128, False),     # 45 tiles over 40 blocks: some blocks take two
    (2, 12, 32, 64, True),       # projection shortcut (first block of the stage)
    (16, 48, 128, 64, False),    # 768 tiles over the whole chip, three per block
    (5, 36, 160, 128, False),    # 225 tiles, image borders inside the XCD ranges
    (9, 28, 64, 64, True),
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_conv3x3_pair_bit_identical(cuda, dt, case):
    n, h, w, c_out, proj = case
    y, z, y2, z2, yr, zr = _case(cuda, dt, n, h, w, c_out, proj, 7 * h + w + c_out)
    assert torch.equal(y, y2), (y.float() - y2.float()).abs().max().item()
    assert torch.equal(z, z2), (z.float() - z2.float()).abs().max().item()
    gy = y.float().permute(0, 3, 1, 2).cpu().double()
    gz = z.float().permute(0, 3, 1, 2).cpu().double()
    assert (gy - yr).abs().max().item() <= 8e-3 * yr.abs().max().item()
    assert (gz - zr).abs().max().item() <= 1.6e-2 * zr.abs().max().item()


def test_conv3x3_pair_rejects_shapes(cuda):
    """tiles are 4 x 32 pixels: other extents are refused (the caller keeps two launches)"""
    from cirtorch import _ops as ops
    dt = torch.bfloat16
    z64 = lambda *s: torch.zeros(*s, dtype=dt, device=cuda)  # noqa: E731
    f = lambda c: torch.ones(c, device=cuda)  # noqa: E731
    for h, w in ((18, 64), (16, 48)):
        with pytest.raises(RuntimeError):
            ops.conv3x3_pair(z64(1, h, w, 64), z64(64, 576), f(64), f(64), True, 0.01, z64(256, 64), f(256), f(256),
                             z64(1, h, w, 256), True, 0.01, z64(64, 256), f(64), f(64), 64, True, 0.01)
    with pytest.raises(RuntimeError):  # projection form with c_out 128
        ops.conv3x3_pair(z64(1, 16, 32, 64), z64(64, 576), f(64), f(64), True, 0.01, z64(256, 64), f(256), f(256),
                         None, True, 0.01, z64(128, 256), f(128), f(128), 128, True, 0.01,
                         proj=(z64(1, 16, 32, 64), z64(256, 64), f(256), f(256)))


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_backbone_block_fusion_bit_identical(cuda, prec, monkeypatch):
    """ResNet-50 body with the 256-channel stage's blocks fused (rr_conv3x3_pair, default) vs the
    same body with the 3x3 as its own launch (RR_C3PAIR=0): every stage output bit-identical."""
    from cirtorch.backbones import resnet
    from cirtorch.models.init import random_init_
    body = resnet.resnet50(precision=prec)
    random_init_(body, 5)
    body = body.to(cuda).eval()
    x = torch.rand(2, 3, 256, 512, generator=torch.Generator().manual_seed(6)).to(cuda)
    calls = []
    from cirtorch import _ops
    orig = _ops.conv3x3_pair
    monkeypatch.setattr(_ops, "conv3x3_pair", lambda *a, **k: calls.append(1) or orig(*a, **k))
    with torch.no_grad():
        monkeypatch.setenv("RR_C3PAIR_CONV1", "1")  # block 1's conv1 in the launch too (opt-in)
        fused = body(x)
        assert len(calls) == 3  # every block of the stage
        monkeypatch.setenv("RR_C3PAIR_CONV1", "0")  # block 1's conv1 as its own launch (default)
        part = body(x)
        monkeypatch.setenv("RR_C3PAIR", "0")
        plain = body(x)
        assert len(calls) == 6
    for k in fused:
        assert torch.equal(fused[k], plain[k]), k
        assert torch.equal(part[k], plain[k]), k


def test_conv3x3_pair_dynamic_queue_under_contention(cuda):
    """The per-XCD tile queue hands tiles to whichever blocks run first: with another stream's
    long kernels holding part of the chip (as the bench step's search does), the blocks take
    different tile sets, and y / z stay bit-identical to the static walk."""
    from cirtorch import _ops as ops
    dt = torch.float16
    n, h, w = 24, 48, 128
    g = torch.Generator(device=cuda).manual_seed(11)
    rn = lambda *s, sc=0.5: (torch.randn(*s, generator=g, device=cuda) * sc).to(dt)  # noqa: E731
    t1, res = rn(n, h, w, 64), rn(n, h, w, 256)
    w33 = ops.pack_conv_weights(torch.randn(64, 64, 3, 3, generator=g, device=cuda) * 0.06, 64, dt, perm32=True)
    w3, w1 = rn(256, 64, sc=0.1), rn(128, 256, sc=0.05)
    one = lambda c: torch.ones(c, device=cuda)  # noqa: E731
    zero = lambda c: torch.zeros(c, device=cuda)  # noqa: E731

    def run(dyn):
        return ops.conv3x3_pair(t1, w33, one(64), zero(64), True, 0.01, w3, one(256), zero(256), res, True, 0.01,
                                w1, one(128), zero(128), 128, True, 0.01, dynamic=dyn)

    ys, zs = run(False)
    a = torch.randn(4096, 4096, device=cuda, dtype=dt)
    side = torch.cuda.Stream(device=cuda)
    for _ in range(3):
        side.wait_stream(torch.cuda.current_stream(cuda))
        with torch.cuda.stream(side):
            for _ in range(4):
                a = (a @ a).clamp_(-1, 1)  # long kernels on a second stream
        y, z = run(True)
        torch.cuda.synchronize()
        assert torch.equal(y, ys) and torch.equal(z, zs)


@pytest.mark.parametrize("c_out,proj", [(64, True), (64, False), (128, False)])
def test_conv3x3_pair_bench_shape(cuda, c_out, proj):
    """The bench's mod2 map (192 x 256 pixels, 8 images: 3072 tiles, ~12 per block, both tile
    walks): y / z bit-identical to the unfused launches at full spatial size."""
    from cirtorch import _ops as ops
    dt = torch.float16
    n, h, w = 8, 192, 256
    g = torch.Generator(device=cuda).manual_seed(c_out + proj)
    rn = lambda *s, sc=0.5: (torch.randn(*s, generator=g, device=cuda) * sc).to(dt)  # noqa: E731
    t1, xin, res = rn(n, h, w, 64), rn(n, h, w, 64), rn(n, h, w, 256)
    w33 = ops.pack_conv_weights(torch.randn(64, 64, 3, 3, generator=g, device=cuda) * 0.06, 64, dt, perm32=True)
    w3, wp, w1 = rn(256, 64, sc=0.1), rn(256, 64, sc=0.1), rn(c_out, 256, sc=0.05)
    aff = lambda c: (torch.rand(c, generator=g, device=cuda) + 0.5, torch.randn(c, generator=g, device=cuda) * 0.1)  # noqa: E731
    (s2, h2), (s3, h3), (sp, hp), (s1, h1) = aff(64), aff(256), aff(256), aff(c_out)
    pj = (xin, wp, sp, hp) if proj else None
    r = None if proj else res
    t2 = ops.conv2d_fused(t1, w33, 3, 3, 1, 1, 64, s2, h2, leaky=True, slope=0.01, perm32=True)
    y2, z2 = ops.conv1x1_pair(t2, w3, s3, h3, r, True, 0.01, w1, s1, h1, c_out, True, 0.01, proj=pj)
    for dyn in (True, False):
        y, z = ops.conv3x3_pair(t1, w33, s2, h2, True, 0.01, w3, s3, h3, r, True, 0.01, w1, s1, h1, c_out, True, 0.01,
                                proj=pj, dynamic=dyn)
        assert torch.equal(y, y2) and torch.equal(z, z2), dyn


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("shape", [(2, 12, 32), (9, 28, 64), (4, 192, 256)])
def test_conv3x3_pair_with_conv1(cuda, dt, shape):
    """The stage's first block with its conv1 (1x1 64 -> 64 + bn1 + act on the block input) in
    the same launch: y / z bit-identical to conv1 as its own launch followed by the fused block
    (t1's zero padding restored outside the image), both tile walks."""
    from cirtorch import _ops as ops
    n, h, w = shape
    g = torch.Generator(device=cuda).manual_seed(h + w)
    rn = lambda *s, sc=0.5: (torch.randn(*s, generator=g, device=cuda) * sc).to(dt)  # noqa: E731
    x = rn(n, h, w, 64)
    w0 = ops.pack_conv_weights(torch.randn(64, 64, 1, 1, generator=g, device=cuda) * 0.15, 64, dt, perm32=True)
    w33 = ops.pack_conv_weights(torch.randn(64, 64, 3, 3, generator=g, device=cuda) * 0.06, 64, dt, perm32=True)
    w3, wp, w1 = rn(256, 64, sc=0.1), rn(256, 64, sc=0.1), rn(64, 256, sc=0.05)
    aff = lambda c: (torch.rand(c, generator=g, device=cuda) + 0.5, torch.randn(c, generator=g, device=cuda) * 0.1)  # noqa: E731
    (s0, h0), (s2, h2), (s3, h3), (sp, hp), (s1, h1) = aff(64), aff(64), aff(256), aff(256), aff(64)
    pj = (x, wp, sp, hp)
    t1 = ops.conv2d_fused(x, w0, 1, 1, 1, 0, 64, s0, h0, leaky=True, slope=0.01, perm32=True)
    y2, z2 = ops.conv3x3_pair(t1, w33, s2, h2, True, 0.01, w3, s3, h3, None, True, 0.01, w1, s1, h1, 64, True, 0.01,
                              proj=pj)
    for dyn in (True, False):
        y, z = ops.conv3x3_pair(x, w33, s2, h2, True, 0.01, w3, s3, h3, None, True, 0.01, w1, s1, h1, 64, True, 0.01,
                                proj=pj, dynamic=dyn, conv1=(w0, s0, h0, True, 0.01))
        assert torch.equal(y, y2), (dyn, (y.float() - y2.float()).abs().max().item())
        assert torch.equal(z, z2), (dyn, (z.float() - z2.float()).abs().max().item())
