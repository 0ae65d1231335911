"""Op-level parity of the HIP kernels (through the C ABI) against the CPU oracle
and the reference golden vectors.  GPU only."""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import cosines, golden

pytestmark = pytest.mark.gpu


def _ops():
    from cirtorch import _ops
    return _ops


def _bf16_round(t):
    return t.to(torch.bfloat16).to(torch.float32)


CONV_CASES = [
    # n, cin, h, w, cout, k, stride, pad, residual, leaky
    (2, 64, 17, 19, 64, 1, 1, 0, True, True),
    (2, 64, 16, 20, 256, 1, 1, 0, False, False),
    (1, 128, 15, 13, 96, 1, 2, 0, False, False),
    (2, 64, 14, 18, 64, 3, 1, 1, False, True),
    (1, 128, 16, 16, 128, 3, 2, 1, False, True),
    (1, 256, 7, 9, 512, 3, 1, 1, True, True),
    (2, 3, 40, 36, 64, 7, 2, 3, False, True),   # stem, input channels padded
]


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("perm", [False, True])
def test_conv_fused(cuda, case, prec, perm):
    _check_conv(cuda, case, prec, perm)


TILE_CASES = CONV_CASES + [
    (2, 256, 20, 24, 256, 1, 1, 0, True, True),    # one channel tile, one K-step (A-stationary 256x64)
    (2, 64, 21, 23, 64, 3, 1, 1, False, True),     # 64 channels, 9 K-steps
    (2, 128, 18, 20, 64, 1, 1, 0, False, True),    # 64 channels, 2 K-steps
]


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("case", TILE_CASES)
@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_conv_tile_configs(cuda, cfg, case, prec):
    """Every forced tile configuration of the GEMM engine (rr_set_tuning) is
    exact on every conv shape — the automatic choice may pick any of them."""
    from cirtorch import _engine as E
    E.check(E.lib().rr_set_tuning(0, cfg), "rr_set_tuning")
    try:
        _check_conv(cuda, case, prec, True)
    finally:
        E.lib().rr_set_tuning(0, 0)


@pytest.mark.parametrize("cfg", [1, 2, 5])
@pytest.mark.parametrize("case", TILE_CASES)
def test_conv_tile_configs_3stage(cuda, cfg, case):
    """3-stage LDS ring (one barrier per K-step, refill issued after it) on the
    4-wave tiles: exact on every conv shape."""
    from cirtorch import _engine as E
    E.check(E.lib().rr_set_tuning(0, cfg), "rr_set_tuning")
    E.check(E.lib().rr_set_tuning(1, 3), "rr_set_tuning")
    try:
        _check_conv(cuda, case, "bf16", True)
    finally:
        E.lib().rr_set_tuning(0, 0)
        E.lib().rr_set_tuning(1, 2)


STREAM_CASES = [
    # HBM-bound bf16 1x1 shapes of the bottleneck blocks (rr_stream.hip), P >= 4096, ragged P
    (2, 64, 47, 51, 64, 1, 1, 0, False, True),
    (2, 64, 41, 59, 256, 1, 1, 0, True, True),
    (2, 64, 41, 59, 256, 1, 1, 0, False, False),
    (2, 256, 39, 53, 64, 1, 1, 0, False, True),
    (2, 256, 39, 53, 128, 1, 1, 0, False, True),
    (1, 128, 63, 71, 512, 1, 1, 0, True, True),
    (1, 512, 63, 67, 128, 1, 1, 0, False, True),
    (1, 256, 65, 67, 1024, 1, 1, 0, True, True),
    (2, 256, 83, 101, 512, 1, 2, 0, False, False),   # strided projection
    (1, 512, 64, 67, 2048, 1, 1, 0, True, True),     # mod5 conv3: 16 slices of 128 channels
    (1, 512, 65, 67, 256, 1, 1, 0, False, True),     # mod4 conv1: 2 slices of 128 channels
    (2, 512, 130, 70, 1024, 1, 2, 0, False, True),   # mod4 projection (stride 2): 8 slices
]


@pytest.mark.parametrize("case", STREAM_CASES)
@pytest.mark.parametrize("mode,prec", [(1, "bf16"), (0, "bf16"), (1, "fp16")])
def test_conv_stream1x1(cuda, case, mode, prec):
    """The weight-stationary streaming 1x1 kernel (mode 1) and the tiled engine
    (mode 0) on the same shapes."""
    from cirtorch import _engine as E
    E.check(E.lib().rr_set_tuning(5, mode), "rr_set_tuning")
    E.check(E.lib().rr_set_tuning(14, 0), "rr_set_tuning")  # the streaming kernel, not k_wres1x1
    try:
        _check_conv(cuda, case, prec, True)
    finally:
        E.lib().rr_set_tuning(5, 1)
        E.lib().rr_set_tuning(14, 2)


XCD_CASES = [
    # chip-filling streaming 1x1s whose grid is a multiple of 8 x slices (XCD map on)
    (4, 256, 48, 64, 1024, 1, 1, 0, True, True),    # mod4 conv3: 4 slices of 256 channels
    (2, 128, 96, 128, 512, 1, 1, 0, True, True),    # mod3 conv3: 2 slices
    (2, 512, 48, 64, 2048, 1, 1, 0, True, True),    # mod5 conv3 shape: 16 slices of 128
]


@pytest.mark.parametrize("case", XCD_CASES)
def test_stream1x1_xcd_map(cuda, case):
    """RR_TUNE_STREAM_XCD: the channel-slice blocks of one strip on one XCD is a
    pure block-to-work remapping: exact vs float64, bit-identical to the plain order."""
    from cirtorch import _engine as E
    outs = []
    E.check(E.lib().rr_set_tuning(14, 0), "rr_set_tuning")  # the streaming kernel, not k_wres1x1
    try:
        for xcd in (1, 0):
            E.check(E.lib().rr_set_tuning(12, xcd), "rr_set_tuning")
            outs.append(_check_conv(cuda, case, "bf16", True))
    finally:
        E.lib().rr_set_tuning(12, 1)
        E.lib().rr_set_tuning(14, 2)
    assert torch.equal(outs[0], outs[1])


WRES_CASES = [
    # residual conv3 shapes of mod4 / mod5 that k_wres1x1 takes (RR_TUNE_WRES = 1)
    (1, 256, 65, 67, 1024, 1, 1, 0, True, True),    # 4355 pixels: partial last tile, 2 slices
    (1, 512, 64, 67, 2048, 1, 1, 0, True, True),    # 8 slices of 256 channels
    (4, 256, 48, 64, 1024, 1, 1, 0, True, True),    # chip-filling grid: XCD map on
    (2, 512, 48, 64, 2048, 1, 1, 0, True, False),   # identity activation
    # RR_TUNE_WRES = 2: the non-residual K = 256 / 512 1x1s, strided or not
    (1, 512, 65, 67, 256, 1, 1, 0, False, True),    # mod4 block-1 conv1: one slice
    (2, 512, 130, 70, 1024, 1, 2, 0, False, True),  # mod4 projection (stride 2), ragged last tile
    (2, 256, 83, 101, 512, 1, 2, 0, False, False),  # mod3 projection (stride 2, odd map)
    (1, 256, 64, 70, 1024, 1, 1, 0, False, True),
    (1, 128, 63, 71, 512, 1, 1, 0, True, True),     # mod3 last-block conv3 (K = 128): one 512-channel slice
    (4, 128, 48, 64, 512, 1, 1, 0, True, False),
]


@pytest.mark.parametrize("case", WRES_CASES)
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_wres1x1(cuda, case, prec):
    """Weight-stationary residual 1x1 (weights in VGPRs, tiles by LDS-DMA):
    exact vs float64 and bit-identical to the streaming 1x1 (same K order)."""
    from cirtorch import _engine as E
    outs = []
    try:
        for on in (2, 0):
            E.check(E.lib().rr_set_tuning(14, on), "rr_set_tuning")
            outs.append(_check_conv(cuda, case, prec, True))
        # RR_TUNE_WRES_RING = 0: the non-residual forms two tiles ahead instead of 5 / 3
        E.check(E.lib().rr_set_tuning(14, 2), "rr_set_tuning")
        E.check(E.lib().rr_set_tuning(16, 0), "rr_set_tuning")
        outs.append(_check_conv(cuda, case, prec, True))
    finally:
        E.lib().rr_set_tuning(14, 2)
        E.lib().rr_set_tuning(16, 1)
    assert torch.equal(outs[0], outs[1])
    assert torch.equal(outs[0], outs[2])


C3W64_CASES = [
    (2, 64, 48, 64, 64, 3, 1, 1, False, True),     # 24 tiles: fewer than the grid's blocks
    (3, 64, 64, 96, 64, 3, 1, 1, False, False),
    (16, 64, 48, 128, 64, 3, 1, 1, False, True),   # 384 tiles over 256 blocks
]


@pytest.mark.parametrize("case", C3W64_CASES)
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_c3w64_bit_identical(cuda, case, prec):
    """mod2 3x3 with the weights in VGPRs (RR_TUNE_CONV3X3 = 9): exact vs float64 and
    bit-identical to the A-stationary direct kernel (same (tap, half-step) order)."""
    from cirtorch import _engine as E
    outs = []
    try:
        for mode in (9, 4):
            E.check(E.lib().rr_set_tuning(6, mode), "rr_set_tuning")
            outs.append(_check_conv(cuda, case, prec, True))
    finally:
        E.lib().rr_set_tuning(6, 1)
    assert torch.equal(outs[0], outs[1])


CONV3_CASES = [
    # bf16 stride-1 3x3 shapes the direct LDS-patch kernel (rr_conv3.hip) takes
    (2, 64, 16, 64, 64, 3, 1, 1, False, True),     # c_in = c_out = 64: weights resident in LDS
    (2, 64, 8, 32, 128, 3, 1, 1, False, False),    # one input chunk, weight ring
    (1, 128, 16, 64, 128, 3, 1, 1, False, True),   # two chunks
    (1, 256, 8, 32, 256, 3, 1, 1, False, True),    # two channel tiles
    (1, 512, 12, 32, 512, 3, 1, 1, False, True),   # 8 chunks, height only 4-divisible
    (2, 256, 12, 64, 256, 3, 1, 1, False, True),   # 256-channel tiles (mode 8)
]


@pytest.mark.parametrize("case", CONV3_CASES)
@pytest.mark.parametrize("mode,prec", [(1, "bf16"), (2, "bf16"), (3, "bf16"), (4, "bf16"), (6, "bf16"), (7, "bf16"),
                                       (8, "bf16"), (9, "bf16"), (0, "bf16"), (1, "fp16"), (8, "fp16"), (9, "fp16"),
                                       (0, "fp16")])
def test_conv3x3_direct(cuda, case, mode, prec):
    """Direct 3x3 kernel (modes 1-4, 6: auto / 8x32 / 4x32 tiles / A-stationary wave layouts) and the
    implicit-GEMM fallback (mode 0) against the float64 reference."""
    from cirtorch import _engine as E
    E.check(E.lib().rr_set_tuning(6, mode), "rr_set_tuning")
    try:
        _check_conv(cuda, case, prec, True)
    finally:
        E.lib().rr_set_tuning(6, 1)


@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_conv3x3_pipelined_schedule_bit_identical(cuda, prec):
    """RR_TUNE_CONV3_PIPE: the software-pipelined A-stationary tile loop issues
    the same MFMAs in the same accumulation order as the compiler-scheduled one,
    so the outputs are bit-identical (and both match the float64 reference)."""
    from cirtorch import _engine as E
    case = (3, 64, 24, 96, 64, 3, 1, 1, False, True)
    outs = []
    try:
        for pipe in (0, 1):
            E.check(E.lib().rr_set_tuning(10, pipe), "rr_set_tuning")
            outs.append(_check_conv(cuda, case, prec, True))
    finally:
        E.lib().rr_set_tuning(10, 1)
    assert torch.equal(outs[0], outs[1])


CONV3S_CASES = [
    # (case, grid cap): the staggered persistent direct 3x3 (rr_conv3s.hip); a CU cap
    # gives small problems several tiles per block and ragged XCD ranges
    ((3, 64, 48, 96, 64, 3, 1, 1, False, True), 8),      # mod2 form: 27 tiles of 16 x 32 over 8 blocks
    ((2, 64, 32, 64, 64, 3, 1, 1, False, False), 8),     # identity activation, 2 tiles per block
    ((3, 128, 24, 96, 128, 3, 1, 1, False, True), 8),    # mod3 form: 2 chunks, 27 tiles of 8 x 32
    ((3, 64, 24, 96, 128, 3, 1, 1, False, True), 8),     # one chunk: patch buffers alternate per tile
    ((4, 256, 16, 64, 128, 3, 1, 1, False, True), 8),    # 4 chunks
    ((5, 128, 16, 32, 128, 3, 1, 1, False, True), 16),   # 10 tiles < 2 per block: falls back to k_conv3x3
    ((8, 64, 192, 256, 64, 3, 1, 1, False, True), 0),    # mod2 at 768x1024, whole chip
    ((16, 128, 96, 128, 128, 3, 1, 1, False, True), 0),  # mod3 at 768x1024, whole chip
]


@pytest.mark.parametrize("case,cap", CONV3S_CASES)
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_conv3s_staggered(cuda, case, cap, prec):
    """Staggered two-wave-group direct 3x3 (RR_TUNE_CONV3S) vs float64; the
    c_out = 128 form accumulates in k_conv3x3's (chunk, tap, half-step) order,
    so it is also bit-identical to it."""
    from cirtorch import _engine as E
    outs = []
    try:
        E.check(E.lib().rr_set_tuning(7, cap), "rr_set_tuning")
        # 2: both forms (the c_in = c_out = 64 one is opt-in), 1: default, 0: k_conv3x3
        for on in (2, 1, 0):
            E.check(E.lib().rr_set_tuning(13, on), "rr_set_tuning")
            outs.append(_check_conv(cuda, case, prec, True))
    finally:
        E.lib().rr_set_tuning(13, 1)
        E.lib().rr_set_tuning(7, 0)
    # the c_out = 128 form accumulates in k_conv3x3's (chunk, tap, half-step) order
    if case[4] == 128:
        assert torch.equal(outs[0], outs[2]) and torch.equal(outs[1], outs[2])


def _check_conv(cuda, case, prec, perm):
    n, cin, h, w, cout, k, s, p, use_res, leaky = case
    g = torch.Generator().manual_seed(hash(case) & 0xFFFF)
    x = torch.randn(n, cin, h, w, generator=g)
    wt = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    scale = torch.rand(cout, generator=g) + 0.5
    shift = torch.randn(cout, generator=g) * 0.1
    dtype = {"fp32": torch.float32, "bf16": torch.bfloat16, "fp16": torch.float16}[prec]
    if prec == "bf16":
        x, wt = _bf16_round(x), _bf16_round(wt)
    if prec == "fp16":
        x, wt = x.half().float(), wt.half().float()
    ref = F.conv2d(x.double(), wt.double(), stride=s, padding=p) * scale.double()[None, :, None, None] \
        + shift.double()[None, :, None, None]
    res = None
    if use_res:
        res = torch.randn(ref.shape, generator=g)
        if prec == "bf16":
            res = _bf16_round(res)
        if prec == "fp16":
            res = res.half().float()
        ref = ref + res.double()
    if leaky:
        ref = F.leaky_relu(ref, 0.01)
    # engine layout
    cpad = cin if cin >= 8 else (4 if prec == "fp32" else 8)
    perm = perm and cout % 32 == 0
    xe = F.pad(x.permute(0, 2, 3, 1), (0, cpad - cin)).contiguous().to(dtype).to(cuda)
    wp = _ops().pack_conv_weights(wt.to(cuda), cpad, dtype, perm32=perm)
    # host check of the packed layout (k = (kh*KW + kw)*cin_pad + ci; perm32 row order)
    ref_w = F.pad(wt.permute(0, 2, 3, 1), (0, cpad - cin)).reshape(cout, -1)
    ref_w = F.pad(ref_w, (0, wp.shape[1] - ref_w.shape[1])).to(dtype)
    if perm:
        rows = torch.arange(cout)
        chan = (rows & ~31) | (((rows & 15) >> 2) << 3) | (((rows >> 4) & 1) << 2) | (rows & 3)
        ref_w = ref_w[chan]
    assert torch.equal(wp.cpu(), ref_w)
    re = res.permute(0, 2, 3, 1).contiguous().to(dtype).to(cuda) if use_res else None
    y = _ops().conv2d_fused(xe, wp, k, k, s, p, cout, scale.to(cuda), shift.to(cuda), residual=re, leaky=leaky,
                            perm32=perm)
    got = y.float().permute(0, 3, 1, 2).cpu().double()
    assert got.shape == ref.shape
    err = (got - ref).abs().max().item()
    scale_ref = ref.abs().max().item()
    # fp32: exact-f32 MFMA chain (K <= 2304): ~1e-6 relative; bf16 output rounding: 2^-8 relative
    # fp16 output rounding: 2^-11 relative
    tol = 2e-5 * scale_ref if prec == "fp32" else (8e-3 if prec == "bf16" else 2e-3) * scale_ref
    assert err <= tol, (err, scale_ref)
    return y


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float16])
def test_maxpool(cuda, dtype):
    x = torch.randn(2, 21, 19, 64).to(dtype)
    y = _ops().maxpool2d(x.to(cuda), 3, 2, 1).cpu()
    ref = F.max_pool2d(x.float().permute(0, 3, 1, 2), 3, 2, 1).permute(0, 2, 3, 1).to(dtype)
    assert torch.equal(y, ref)


@pytest.mark.parametrize("dtype,cpad", [(torch.float32, 4), (torch.bfloat16, 8), (torch.float16, 8)])
def test_image_to_nhwc(cuda, dtype, cpad):
    """normalise (cirtorch/utils/image.py:125) + NCHW->NHWC + zero channel pad."""
    x = torch.rand(2, 3, 13, 17)
    mean, std = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]
    y = _ops().image_to_nhwc(x.to(cuda), cpad, dtype, mean, std).cpu()
    ref = ((x - torch.tensor(mean)[:, None, None]) / torch.tensor(std)[:, None, None]).permute(0, 2, 3, 1)
    assert y.shape == (2, 13, 17, cpad)
    assert torch.equal(y[..., :3], ref.to(dtype))
    assert y[..., 3:].abs().sum() == 0


def test_resize_bilinear(cuda):
    x = torch.rand(3, 37, 50)
    for s in (0.5, 2.0, 1 / 2 ** 0.5):
        got = _ops().resize_bilinear(x.to(cuda), s).cpu()
        ref = F.interpolate(x[None], scale_factor=s, mode="bilinear", align_corners=False)[0]
        assert got.shape == ref.shape
        assert (got - ref).abs().max() < 1e-5


def test_pool_ops_vs_reference_golden(cuda):
    from cirtorch.layers import functional as LF
    g = golden("ops.npz")
    x = torch.from_numpy(g["x"]).to(cuda)
    for p in (3.0, 2.5):
        got = LF.gem(x, p=p).cpu().numpy()
        np.testing.assert_allclose(got, g["gem_p%g" % p], rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(LF.mac(x).cpu().numpy(), g["mac"], rtol=0, atol=0)
    np.testing.assert_allclose(LF.spoc(x).cpu().numpy(), g["spoc"], rtol=2e-6, atol=1e-7)
    # NHWC (channels_last) input gives the same result
    xc = x.contiguous(memory_format=torch.channels_last)
    np.testing.assert_allclose(LF.gem(xc, p=3.0).cpu().numpy(), g["gem_p3"], rtol=2e-6, atol=1e-7)
    np.testing.assert_allclose(LF.l2n(torch.from_numpy(g["l2n_x"]).to(cuda)).cpu().numpy(), g["l2n"],
                               rtol=2e-6, atol=1e-7)


def test_global_head_vs_reference_golden(cuda):
    from cirtorch.modules.heads.global_head import globalHead
    from oracle import weights
    g = golden("ops.npz")
    head = globalHead(pooling={"name": "GeM", "params": {"p": 3, "eps": 1e-6}},
                      normal={"name": "L2N", "params": {}}, dim=512)
    head.load_state_dict({k: torch.from_numpy(v) for k, v in weights.head_state(512).items()})
    head = head.to(cuda)
    x = torch.from_numpy(g["head_x"]).to(cuda)
    np.testing.assert_allclose(head(x).cpu().numpy(), g["head"], rtol=1e-5, atol=2e-7)
    np.testing.assert_allclose(head(x, do_whitening=False).cpu().numpy(), g["head_nowhiten"], rtol=1e-5, atol=2e-7)


def test_whitenapply_vs_reference_golden(cuda):
    from cirtorch.utils.whiten import whitenapply
    from oracle import data
    g = golden("whiten.npz")
    X = data.unit_rows(600, 64, seed=601).T.astype(np.float32)
    Y = whitenapply(X, g["m32"], g["P32"], dimensions=32)
    np.testing.assert_allclose(Y, g["Y32"], rtol=1e-4, atol=2e-6)
    Yf = whitenapply(X, g["m"].astype(np.float32), g["P"].astype(np.float32))
    assert cosines(Yf, g["Y"]).min() > 1 - 1e-5
    # float64 (m, P) as whitenlearn returns them: the reference arithmetic is
    # float64 (whiten.py:4-12), and so is rr_whitenapply's (f64 MFMA) -> only
    # the final float32 rounding separates the two
    Y64 = whitenapply(X, g["m"], g["P"])
    np.testing.assert_allclose(Y64, g["Y"], rtol=0, atol=1e-7)


@pytest.mark.parametrize("shape", [(2, 61, 83), (1, 96, 128), (1, 40, 300)])
@pytest.mark.parametrize("norm", [True, False])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_stem_conv_pool(cuda, dt, shape, norm):
    """Fused normalise + conv1 7x7/s2/p3 + BN + leaky + maxpool 3x3/s2/p1
    (cirtorch/backbones/resnet.py:59-66) against an fp64 restatement on the
    same bf16-rounded operands, and against the unfused engine path."""
    rnd = lambda t: t.to(dt).float()  # noqa: E731
    n, h, w = shape
    g = torch.Generator().manual_seed(h * 1000 + w)
    x = torch.rand(n, 3, h, w, generator=g)
    wt = rnd(torch.randn(64, 3, 7, 7, generator=g) * 0.1)
    scale = torch.rand(64, generator=g) + 0.5
    shift = torch.randn(64, generator=g) * 0.1
    mean, std = ([0.485, 0.456, 0.406], [0.229, 0.224, 0.225]) if norm else (None, None)
    ops = _ops()
    wpk = ops.pack_stem_weights(wt.to(cuda), dt)
    got = ops.stem_conv_pool(x.to(cuda), wpk, scale.to(cuda), shift.to(cuda), leaky=True, slope=0.01,
                             mean=mean, std=std).float().cpu()
    xn = x if not norm else (x - torch.tensor(mean)[:, None, None]) / torch.tensor(std)[:, None, None]
    xn = rnd(xn)
    ref = F.conv2d(xn.double(), wt.double(), stride=2, padding=3) * scale.double()[None, :, None, None] \
        + shift.double()[None, :, None, None]
    ref = rnd(F.leaky_relu(ref, 0.01).float())
    ref = F.max_pool2d(ref, 3, 2, 1).permute(0, 2, 3, 1)
    assert got.shape == ref.shape
    err = (got - ref).abs().max().item()
    assert err <= 8e-3 * ref.abs().max().item(), err
    # unfused engine path on the same inputs
    xe = ops.image_to_nhwc(x.to(cuda), 8, dt, mean, std)
    wp = ops.pack_conv_weights(wt.to(cuda), 8, dt, perm32=True)
    y = ops.conv2d_fused(xe, wp, 7, 7, 2, 3, 64, scale.to(cuda), shift.to(cuda), leaky=True, perm32=True)
    un = ops.maxpool2d(y, 3, 2, 1).float().cpu()
    assert (got - un).abs().max().item() <= 8e-3 * ref.abs().max().item()
    # most values are bit-identical (only fp32 summation order differs)
    assert (got == un).float().mean().item() > 0.95


# odd stem maps take the v1 kernel in every mode; even ones (2, 64, 84), (1, 100, 472),
# (3, 200, 132) the v2 / v3 tiles (partial wave strips, several tiles both ways)
@pytest.mark.parametrize("shape", [(2, 61, 83), (1, 96, 470), (3, 200, 130), (2, 64, 84), (1, 100, 472),
                                   (3, 200, 132)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_stem_pool_before_epilogue_bit_identical(cuda, dt, shape):
    """RR_TUNE_STEM: the v2 / v3 stems pool the raw conv and applies BN + leaky +
    rounding to the pooled pixels only (exact: the epilogue is non-decreasing
    once negative-scale rows are negated).  Positive- and zero-scale channels
    are bit-identical to the v1 kernel; negative-scale channels differ only
    where the MFMA sum of the negated products is not the exact negation of
    the original sum (1 ulp of the f32 accumulator: measured 2 of 180k fp16
    outputs, 1 output ulp), fp32 and uint8 inputs."""
    n, h, w = shape
    g = torch.Generator().manual_seed(h + 7 * w)
    x = torch.rand(n, 3, h, w, generator=g)
    wt = torch.randn(64, 3, 7, 7, generator=g) * 0.1
    scale = torch.rand(64, generator=g) + 0.5
    scale[::3] *= -1.0
    scale[5] = 0.0
    shift = torch.randn(64, generator=g) * 0.1
    mean, std = [0.485, 0.456, 0.406], [0.229, 0.224, 0.225]
    ops = _ops()
    from cirtorch import _engine as E
    wpk = ops.pack_stem_weights(wt.to(cuda), dt)
    xu = (x * 255).to(torch.uint8)
    outs = {}
    try:
        for mode in (0, 1, 2, 3, 4, 6):
            E.check(E.lib().rr_set_tuning(11, mode), "rr_set_tuning")
            outs[mode] = [ops.stem_conv_pool(inp.to(cuda), wpk, scale.to(cuda), shift.to(cuda), leaky=True,
                                             slope=0.01, mean=mean, std=std).float().cpu() for inp in (x, xu)]
    finally:
        E.lib().rr_set_tuning(11, 2)
    neg = scale < 0
    ulp = 2.0 ** -7 if dt == torch.bfloat16 else 2.0 ** -10
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a[..., ~neg], b[..., ~neg])
        d = (a[..., neg] - b[..., neg]).abs()
        assert (d > 0).float().mean().item() < 1e-3
        assert (d <= ulp * a[..., neg].abs().clamp_min(1.0)).all()
    # v3 (swapped MFMA operands, lane-local pooling, byte table for uint8) == v2
    for b, c in zip(outs[1], outs[2]):
        assert torch.equal(b, c), (b - c).abs().max().item()
    # v3's patch fill in 2 / 5 parts (the default: 3); mode 6: v3 with the interior fast fill
    for m in (3, 4, 6):
        for b, c in zip(outs[2], outs[m]):
            assert torch.equal(b, c), (m, (b - c).abs().max().item())


@pytest.mark.parametrize("c_out", [64, 128])
@pytest.mark.parametrize("shape", [(2, 23, 37), (1, 64, 96)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_conv1x1_pair(cuda, dt, c_out, shape):
    """Fused bottleneck boundary (rr_conv1x1_pair): conv3 (64->256) + BN +
    residual + leaky of block i and conv1 (256->c_out) + BN + leaky of block
    i+1 (cirtorch/backbones/misc.py:166-203) vs a float64 restatement, and vs
    the two separate engine launches (same bf16 roundings, so bit-identical
    up to fp32 summation order)."""
    rnd = lambda t: t.to(dt).float()  # noqa: E731
    n, h, w = shape
    g = torch.Generator().manual_seed(c_out * 7 + h)
    ops = _ops()
    x = rnd(torch.randn(n, 64, h, w, generator=g))
    w3 = rnd(torch.randn(256, 64, 1, 1, generator=g) * (2.0 / 64) ** 0.5)
    w1 = rnd(torch.randn(c_out, 256, 1, 1, generator=g) * (2.0 / 256) ** 0.5)
    s3, h3 = torch.rand(256, generator=g) + 0.5, torch.randn(256, generator=g) * 0.1
    s1, h1 = torch.rand(c_out, generator=g) + 0.5, torch.randn(c_out, generator=g) * 0.1
    res = rnd(torch.randn(n, 256, h, w, generator=g))
    yr = F.leaky_relu(F.conv2d(x.double(), w3.double()) * s3.double()[None, :, None, None]
                      + h3.double()[None, :, None, None] + res.double(), 0.01)
    yb = rnd(yr.float()).double()
    zr = F.leaky_relu(F.conv2d(yb, w1.double()) * s1.double()[None, :, None, None] + h1.double()[None, :, None, None],
                      0.01)
    bf = dt
    xe = x.permute(0, 2, 3, 1).contiguous().to(bf).to(cuda)
    re = res.permute(0, 2, 3, 1).contiguous().to(bf).to(cuda)
    w3p = ops.pack_conv_weights(w3.to(cuda), 64, bf, perm32=True)
    w1p = ops.pack_conv_weights(w1.to(cuda), 256, bf, perm32=True)
    c = [t.to(cuda) for t in (s3, h3, s1, h1)]
    y, z = ops.conv1x1_pair(xe, w3p, c[0], c[1], re, True, 0.01, w1p, c[2], c[3], c_out, True, 0.01)
    gy = y.float().permute(0, 3, 1, 2).cpu().double()
    gz = z.float().permute(0, 3, 1, 2).cpu().double()
    assert (gy - yr).abs().max().item() <= 8e-3 * yr.abs().max().item()
    assert (gz - zr).abs().max().item() <= 1.6e-2 * zr.abs().max().item()
    # the unfused engine path on the same inputs
    y2 = ops.conv2d_fused(xe, w3p, 1, 1, 1, 0, 256, c[0], c[1], residual=re, leaky=True, perm32=True)
    z2 = ops.conv2d_fused(y2, w1p, 1, 1, 1, 0, c_out, c[2], c[3], leaky=True, perm32=True)
    assert torch.equal(y.cpu(), y2.cpu())
    assert (z.float() == z2.float()).float().mean().item() > 0.99


def _mod3_pair_case(dt, n, h, w, seed, cuda, ref=True):
    rnd = lambda t: t.to(dt).float()  # noqa: E731
    g = torch.Generator().manual_seed(seed)
    ops = _ops()
    x = rnd(torch.randn(n, 128, h, w, generator=g))
    w3 = rnd(torch.randn(512, 128, 1, 1, generator=g) * (2.0 / 128) ** 0.5)
    w1 = rnd(torch.randn(128, 512, 1, 1, generator=g) * (2.0 / 512) ** 0.5)
    s3, h3 = torch.rand(512, generator=g) + 0.5, torch.randn(512, generator=g) * 0.1
    s1, h1 = torch.rand(128, generator=g) + 0.5, torch.randn(128, generator=g) * 0.1
    res = rnd(torch.randn(n, 512, h, w, generator=g))
    xe = x.permute(0, 2, 3, 1).contiguous().to(dt).to(cuda)
    re = res.permute(0, 2, 3, 1).contiguous().to(dt).to(cuda)
    w3p = ops.pack_conv_weights(w3.to(cuda), 128, dt, perm32=True)
    w1p = ops.pack_conv_weights(w1.to(cuda), 512, dt, perm32=True)
    c = [t.to(cuda) for t in (s3, h3, s1, h1)]
    y, z = ops.conv1x1_pair(xe, w3p, c[0], c[1], re, True, 0.01, w1p, c[2], c[3], 128, True, 0.01)
    if ref:
        yr = F.leaky_relu(F.conv2d(x.double(), w3.double()) * s3.double()[None, :, None, None]
                          + h3.double()[None, :, None, None] + res.double(), 0.01)
        zr = F.leaky_relu(F.conv2d(rnd(yr.float()).double(), w1.double()) * s1.double()[None, :, None, None]
                          + h1.double()[None, :, None, None], 0.01)
        gy = y.float().permute(0, 3, 1, 2).cpu().double()
        gz = z.float().permute(0, 3, 1, 2).cpu().double()
        assert (gy - yr).abs().max().item() <= 8e-3 * yr.abs().max().item()
        assert (gz - zr).abs().max().item() <= 1.6e-2 * zr.abs().max().item()
    # the two unfused launches on the same inputs
    y2 = ops.conv2d_fused(xe, w3p, 1, 1, 1, 0, 512, c[0], c[1], residual=re, leaky=True, perm32=True)
    z2 = ops.conv2d_fused(y2, w1p, 1, 1, 1, 0, 128, c[2], c[3], leaky=True, perm32=True)
    return y, z, y2, z2


@pytest.mark.parametrize("shape", [(2, 23, 37), (1, 37, 113), (4, 48, 64)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_conv1x1_pair_mod3(cuda, dt, shape):
    """The 128 -> 512 -> 128 boundary (k_pair_mid: weights in VGPRs, LDS-DMA
    tiles of 64 pixels, partial last tile) vs a float64 restatement and vs the
    two unfused launches: y bit-identical, z bit-identical where the unfused
    conv1 is the streaming kernel (same K-step order), else >= 99 %."""
    n, h, w = shape
    y, z, y2, z2 = _mod3_pair_case(dt, n, h, w, 11 * h + w, cuda)
    assert torch.equal(y.cpu(), y2.cpu())
    if n * h * w >= 4096:
        assert torch.equal(z.cpu(), z2.cpu())
    else:
        assert (z.float() == z2.float()).float().mean().item() > 0.99


def test_conv1x1_pair_mod3_pixel_chunks(cuda):
    """More than 2^20 pixels: the C-ABI runs the boundary in 2^20-pixel chunks
    (32-bit buffer offsets); every chunk bit-identical to the unfused launches."""
    y, z, y2, z2 = _mod3_pair_case(torch.bfloat16, 1, 1031, 1029, 5, cuda, ref=False)
    assert y.shape[1] * y.shape[2] > (1 << 20)
    assert torch.equal(y, y2)
    assert torch.equal(z, z2)


@pytest.mark.parametrize("shape", [(1, 3, 7), (2, 23, 37), (3, 96, 128), (1, 1031, 1029)])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_conv1x1_pair_mod3_ring_equals_64px_kernel(cuda, dt, shape):
    """RR_TUNE_PAIR_MID: the 128/512 boundary on 32-pixel tiles with the 4-slot residual
    ring (default, k_pair_mid_ring) vs the 64-pixel one-ahead kernel (k_pair_mid): y and z
    bit for bit -- fewer pixels than one tile, a partial last tile, several tiles per block,
    more than 2^20 pixels (two chunk launches)."""
    from cirtorch import _engine as E
    n, h, w = shape
    try:
        E.check(E.lib().rr_set_tuning(15, 0), "rr_set_tuning")
        y0, z0, _, _ = _mod3_pair_case(dt, n, h, w, 3 * h + w, cuda, ref=False)
        E.check(E.lib().rr_set_tuning(15, 1), "rr_set_tuning")
        y1, z1, _, _ = _mod3_pair_case(dt, n, h, w, 3 * h + w, cuda, ref=False)
    finally:
        E.lib().rr_set_tuning(15, 1)
    assert torch.equal(y0, y1)
    assert torch.equal(z0, z1)


@pytest.mark.parametrize("c_out", [64, 128])
@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_conv1x1_pair_projection(cuda, dt, c_out):
    """First block of the stage: the shortcut is proj_bn(proj_conv(x_in))
    (cirtorch/backbones/misc.py:179-182), computed inside the fused launch."""
    rnd = lambda t: t.to(dt).float()  # noqa: E731
    n, h, w = 2, 19, 29
    g = torch.Generator().manual_seed(c_out + 3)
    ops = _ops()
    x = rnd(torch.randn(n, 64, h, w, generator=g))
    xin = rnd(torch.randn(n, 64, h, w, generator=g))
    w3 = rnd(torch.randn(256, 64, 1, 1, generator=g) * (2.0 / 64) ** 0.5)
    wpj = rnd(torch.randn(256, 64, 1, 1, generator=g) * (2.0 / 64) ** 0.5)
    w1 = rnd(torch.randn(c_out, 256, 1, 1, generator=g) * (2.0 / 256) ** 0.5)
    s3, h3 = torch.rand(256, generator=g) + 0.5, torch.randn(256, generator=g) * 0.1
    sp, hp = torch.rand(256, generator=g) + 0.5, torch.randn(256, generator=g) * 0.1
    s1, h1 = torch.rand(c_out, generator=g) + 0.5, torch.randn(c_out, generator=g) * 0.1

    def col(v):
        return v.double()[None, :, None, None]

    def nhwc(t):
        return t.permute(0, 2, 3, 1).contiguous().to(dt).to(cuda)

    short = F.conv2d(xin.double(), wpj.double()) * col(sp) + col(hp)
    yr = F.leaky_relu(F.conv2d(x.double(), w3.double()) * col(s3) + col(h3) + short, 0.01)
    zr = F.leaky_relu(F.conv2d(rnd(yr.float()).double(), w1.double()) * col(s1) + col(h1), 0.01)
    bf = dt
    w3p = ops.pack_conv_weights(w3.to(cuda), 64, bf, perm32=True)
    wpp = ops.pack_conv_weights(wpj.to(cuda), 64, bf, perm32=True)
    w1p = ops.pack_conv_weights(w1.to(cuda), 256, bf, perm32=True)
    y, z = ops.conv1x1_pair(nhwc(x), w3p, s3.to(cuda), h3.to(cuda), None, True, 0.01, w1p, s1.to(cuda), h1.to(cuda),
                            c_out, True, 0.01, proj=(nhwc(xin), wpp, sp.to(cuda), hp.to(cuda)))
    gy = y.float().permute(0, 3, 1, 2).cpu().double()
    gz = z.float().permute(0, 3, 1, 2).cpu().double()
    assert (gy - yr).abs().max().item() <= 8e-3 * yr.abs().max().item()
    assert (gz - zr).abs().max().item() <= 1.6e-2 * zr.abs().max().item()


FP16_CASES = [
    # the LDS-DMA engine in fp16 (natural-order weights): 1x1, strided 1x1, 3x3
    # s1/s2, the 7x7/s2 stem shape on 8 padded channels, residual + leaky
    (2, 64, 17, 23, 256, 1, 1, 0, True, True),
    (2, 256, 18, 22, 512, 1, 2, 0, False, False),
    (2, 64, 16, 32, 64, 3, 1, 1, False, True),
    (1, 128, 19, 21, 128, 3, 2, 1, False, True),
    (1, 3, 45, 61, 64, 7, 2, 3, False, True),
    (1, 512, 9, 11, 2048, 1, 1, 0, True, True),
]


@pytest.mark.parametrize("case", FP16_CASES)
def test_conv_fp16_generic_engine(cuda, case):
    _check_conv(cuda, case, "fp16", False)


def test_conv_fp16_splits_large_batches(cuda):
    """> 2 GiB of fp16 input: the launch is split into image groups (31-bit
    buffer offsets); each group must equal the same images run alone."""
    g = torch.Generator(device="cpu").manual_seed(3)
    n, h, w, c = 9, 256, 256, 2048                        # 9 x 256 MiB = 2.25 GiB
    x = torch.empty(n, h, w, c, dtype=torch.float16, device=cuda)
    for i in range(n):
        x[i] = (torch.randn(h, w, c, generator=g) * 0.5).half().to(cuda)
    wt = torch.randn(64, c, 1, 1, generator=g) * c ** -0.5
    wp = _ops().pack_conv_weights(wt.to(cuda), c, torch.float16)
    y = _ops().conv2d_fused(x, wp, 1, 1, 1, 0, 64, leaky=False)
    for i in (0, 7, 8):
        yi = _ops().conv2d_fused(x[i:i + 1].contiguous(), wp, 1, 1, 1, 0, 64, leaky=False)
        assert torch.equal(y[i:i + 1], yi)
    del x


GEMM8_CASES = [
    # 16-bit 1x1 / tap-uniform 3x3 shapes with an even number of 64-deep K-steps (ragged P, c_out)
    (2, 128, 17, 19, 256, 1, 1, 0, True, True),     # K = 128: 2 K-steps (one loop iteration)
    (1, 256, 23, 29, 512, 1, 1, 0, False, True),    # two channel tiles
    (1, 1024, 21, 25, 256, 1, 1, 0, False, True),   # mod4 conv1 shape, 16 K-steps
    (1, 512, 19, 21, 320, 1, 1, 0, True, False),    # partial channel tile (OOB weight rows)
    (1, 256, 19, 23, 256, 3, 2, 1, False, True),    # strided 3x3, tap-uniform im2col, 36 K-steps
    (1, 128, 14, 18, 128, 3, 1, 1, True, True),     # halo taps at every border, 18 K-steps
]


@pytest.mark.parametrize("case", GEMM8_CASES)
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
@pytest.mark.parametrize("perm", [True, False])
def test_gemm8_forced_vs_float64(cuda, case, prec, perm):
    """The 8-phase staggered 256x256 GEMM (rr_set_tuning(RR_TUNE_GEMM8, 2):
    forced wherever structurally legal) against the float64 reference."""
    from cirtorch import _engine as E
    E.check(E.lib().rr_set_tuning(8, 2), "rr_set_tuning")
    E.check(E.lib().rr_set_tuning(6, 0), "rr_set_tuning")   # no direct 3x3 kernel
    E.check(E.lib().rr_set_tuning(5, 0), "rr_set_tuning")   # no streaming 1x1 kernel
    try:
        _check_conv(cuda, case, prec, perm)
    finally:
        E.lib().rr_set_tuning(8, 1)
        E.lib().rr_set_tuning(6, 1)
        E.lib().rr_set_tuning(5, 1)


@pytest.mark.parametrize("shape", [(128, 48, 64, 1024, 256, 1, 1), (128, 24, 32, 2048, 512, 1, 1),
                                   (128, 48, 64, 256, 256, 3, 2), (128, 24, 32, 512, 512, 3, 2)])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_gemm8_bit_identical_to_tiled_engine(cuda, shape, prec):
    """R50 128-image shapes (mod4 / mod5 conv1, strided 3x3): the 8-phase
    kernel uses the same operand layout and K order as the 2-stage tiled
    engine, so the outputs are bit-identical."""
    from cirtorch import _engine as E
    n, h, w, cin, cout, k, s = shape
    g = torch.Generator(device=cuda).manual_seed(9)
    dt = torch.bfloat16 if prec == "bf16" else torch.float16
    x = torch.randn((n, h, w, cin), generator=g, device=cuda).to(dt)
    wt = torch.randn((cout, cin, k, k), generator=g, device=cuda) * (2.0 / (cin * k * k)) ** 0.5
    wp = _ops().pack_conv_weights(wt, cin, dt, perm32=True)
    sc = torch.rand(cout, generator=g, device=cuda) + 0.5
    sh = torch.randn(cout, generator=g, device=cuda) * 0.1
    p = 1 if k == 3 else 0
    E.check(E.lib().rr_set_tuning(6, 0), "rr_set_tuning")
    E.check(E.lib().rr_set_tuning(5, 0), "rr_set_tuning")
    E.check(E.lib().rr_set_tuning(8, 2), "rr_set_tuning")
    try:
        a = _ops().conv2d_fused(x, wp, k, k, s, p, cout, sc, sh, leaky=True, perm32=True)
        E.check(E.lib().rr_set_tuning(8, 0), "rr_set_tuning")
        b = _ops().conv2d_fused(x, wp, k, k, s, p, cout, sc, sh, leaky=True, perm32=True)
    finally:
        E.lib().rr_set_tuning(8, 1)
        E.lib().rr_set_tuning(6, 1)
        E.lib().rr_set_tuning(5, 1)
    assert torch.equal(a, b)


@pytest.mark.parametrize("shape", [(128, 24, 32, 512, 2048), (64, 48, 64, 256, 1024), (3, 17, 29, 512, 512)])
@pytest.mark.parametrize("leaky", [True, False])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_gemm8_residual_epilogue_bit_identical(cuda, shape, leaky, prec):
    """Residual 1x1s (mod5 / mod4 conv3 shapes, a ragged one) through k_gemm8's
    branch-free buffer-op epilogue (scale / shift via LDS, residual prefetched,
    act = max(v, slope v)) vs the tiled engine: bit-identical."""
    from cirtorch import _engine as E
    n, h, w, cin, cout = shape
    g = torch.Generator(device=cuda).manual_seed(13)
    dt = torch.bfloat16 if prec == "bf16" else torch.float16
    x = torch.randn((n, h, w, cin), generator=g, device=cuda).to(dt)
    wt = torch.randn((cout, cin, 1, 1), generator=g, device=cuda) * (2.0 / cin) ** 0.5
    wp = _ops().pack_conv_weights(wt, cin, dt, perm32=True)
    sc = torch.rand(cout, generator=g, device=cuda) + 0.5
    sc[::7] *= -1.0
    sh = torch.randn(cout, generator=g, device=cuda) * 0.1
    res = torch.randn((n, h, w, cout), generator=g, device=cuda).to(dt)
    E.check(E.lib().rr_set_tuning(6, 0), "rr_set_tuning")
    E.check(E.lib().rr_set_tuning(5, 0), "rr_set_tuning")
    try:
        E.check(E.lib().rr_set_tuning(8, 2), "rr_set_tuning")
        a = _ops().conv2d_fused(x, wp, 1, 1, 1, 0, cout, sc, sh, residual=res, leaky=leaky, perm32=True)
        E.check(E.lib().rr_set_tuning(8, 0), "rr_set_tuning")
        b = _ops().conv2d_fused(x, wp, 1, 1, 1, 0, cout, sc, sh, residual=res, leaky=leaky, perm32=True)
    finally:
        E.lib().rr_set_tuning(8, 1)
        E.lib().rr_set_tuning(6, 1)
        E.lib().rr_set_tuning(5, 1)
    assert torch.equal(a, b)


@pytest.mark.parametrize("cap", [0, 9, 37])
@pytest.mark.parametrize("resid", [True, False])
@pytest.mark.parametrize("shape", [(16, 48, 64, 1024, 256, 1, 1), (16, 24, 32, 512, 2048, 1, 1),
                                   (16, 48, 64, 256, 256, 3, 1), (5, 19, 29, 512, 256, 1, 1)])
def test_gemm8_persistent_equals_one_block_per_tile(cuda, shape, cap, resid):
    """Persistent k_gemm8 blocks (each walks its XCD's tile range, the next tile's
    prologue DMA overlapping the epilogue) vs one block per tile (RR_TUNE_GEMM8 | 4):
    bit-identical, also with grid caps that give the XCDs unequal block counts, a
    residual epilogue, and ragged pixel tiles between full ones (the counted wait
    after a full tile's 16 epilogue stores vs the full drain after a partial one)."""
    from cirtorch import _engine as E
    n, h, w, cin, cout, k, s = shape
    g = torch.Generator(device=cuda).manual_seed(11)
    x = torch.randn((n, h, w, cin), generator=g, device=cuda).to(torch.bfloat16)
    wt = torch.randn((cout, cin, k, k), generator=g, device=cuda) * (2.0 / (cin * k * k)) ** 0.5
    wp = _ops().pack_conv_weights(wt, cin, torch.bfloat16, perm32=True)
    sc = torch.rand(cout, generator=g, device=cuda) + 0.5
    sh = torch.randn(cout, generator=g, device=cuda) * 0.1
    p = 1 if k == 3 else 0
    if resid and k != 1:
        pytest.skip("residual epilogues are 1x1s")
    res = torch.randn((n, h, w, cout), generator=g, device=cuda).to(torch.bfloat16) if resid else None
    E.check(E.lib().rr_set_tuning(6, 0), "rr_set_tuning")
    E.check(E.lib().rr_set_tuning(5, 0), "rr_set_tuning")
    try:
        E.check(E.lib().rr_set_tuning(8, 2 | 4), "rr_set_tuning")
        ref = _ops().conv2d_fused(x, wp, k, k, s, p, cout, sc, sh, residual=res, leaky=True, perm32=True)
        E.check(E.lib().rr_set_tuning(8, 2), "rr_set_tuning")
        E.check(E.lib().rr_set_tuning(7, cap), "rr_set_tuning")
        got = _ops().conv2d_fused(x, wp, k, k, s, p, cout, sc, sh, residual=res, leaky=True, perm32=True)
    finally:
        E.lib().rr_set_tuning(7, 0)
        E.lib().rr_set_tuning(8, 1)
        E.lib().rr_set_tuning(6, 1)
        E.lib().rr_set_tuning(5, 1)
    assert torch.equal(got, ref)



@pytest.mark.parametrize("shape", [(8, 128, 128, 128, 128, 3, 1), (32, 128, 128, 128, 128, 3, 2),
                                   (11, 100, 124, 128, 128, 3, 1)])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_gemm8a_bit_identical_to_tiled_engine(cuda, shape, prec):
    """128-channel 3x3 convs (mod3 shapes at >= 512 tiles, stride 1 and 2, a
    ragged last pixel tile) on k_gemm8a (128 channels x 256 pixels, 8-phase,
    3-stage ring) vs the tiled engine (RR_TUNE_GEMM8 | 16): same operand
    layout and K order, bit-identical; and against float64 within the 16-bit
    tolerance."""
    from cirtorch import _engine as E
    n, h, w, cin, cout, k, s = shape
    g = torch.Generator(device=cuda).manual_seed(17)
    dt = torch.bfloat16 if prec == "bf16" else torch.float16
    x = torch.randn((n, h, w, cin), generator=g, device=cuda).to(dt)
    wt = torch.randn((cout, cin, k, k), generator=g, device=cuda) * (2.0 / (cin * k * k)) ** 0.5
    wp = _ops().pack_conv_weights(wt, cin, dt, perm32=True)
    sc = torch.rand(cout, generator=g, device=cuda) + 0.5
    sh = torch.randn(cout, generator=g, device=cuda) * 0.1
    E.check(E.lib().rr_set_tuning(6, 0), "rr_set_tuning")
    E.check(E.lib().rr_set_tuning(5, 0), "rr_set_tuning")
    try:
        a = _ops().conv2d_fused(x, wp, k, k, s, 1, cout, sc, sh, leaky=True, perm32=True)
        E.check(E.lib().rr_set_tuning(8, 1 | 128), "rr_set_tuning")  # one block per tile
        c = _ops().conv2d_fused(x, wp, k, k, s, 1, cout, sc, sh, leaky=True, perm32=True)
        E.check(E.lib().rr_set_tuning(8, 1 | 16), "rr_set_tuning")
        b = _ops().conv2d_fused(x, wp, k, k, s, 1, cout, sc, sh, leaky=True, perm32=True)
        # a grid capped below the 8 XCDs (RR_TUNE_GRID_CUS = 4): one block per tile then
        # (the persistent grid left XCDs 4..7's tile ranges unwritten)
        E.check(E.lib().rr_set_tuning(8, 1), "rr_set_tuning")
        E.check(E.lib().rr_set_tuning(7, 4), "rr_set_tuning")
        d = _ops().conv2d_fused(x, wp, k, k, s, 1, cout, sc, sh, leaky=True, perm32=True)
    finally:
        E.lib().rr_set_tuning(7, 0)
        E.lib().rr_set_tuning(8, 1)
        E.lib().rr_set_tuning(6, 1)
        E.lib().rr_set_tuning(5, 1)
    assert torch.equal(a, b)
    assert torch.equal(a, c)
    assert torch.equal(a, d)
    ref = F.conv2d(x[:1].cpu().permute(0, 3, 1, 2).double(), wt.to(dt).cpu().double(), stride=s, padding=1)
    ref = ref * sc.cpu().double()[None, :, None, None] + sh.cpu().double()[None, :, None, None]
    ref = F.leaky_relu(ref, 0.01).permute(0, 2, 3, 1)
    err = (a[:1].cpu().double() - ref).abs().max().item()
    assert err <= 2e-2 * ref.abs().max().item(), err


@pytest.mark.parametrize("case", [
    (2, 256, 12, 64, 256, 3, 1, 1, False, True),   # mod4 3x3 form: direct 256-channel tiles / k_gemm8 / k_igemm
    (1, 512, 12, 32, 512, 3, 1, 1, False, True),   # mod5 form, 8 input chunks
    (3, 128, 16, 64, 128, 3, 1, 1, False, True),   # mod3 form: k_c3s / k_conv3x3 / k_gemm8a / k_igemm
    (2, 256, 19, 23, 256, 3, 2, 1, False, True),   # strided 3x3: k_gemm8 / k_igemm
    (2, 128, 18, 34, 128, 3, 2, 1, False, True),   # strided mod3 form: k_gemm8a / k_igemm
])
@pytest.mark.parametrize("prec", ["bf16", "fp16"])
def test_every_3x3_path_same_bits(cuda, case, prec):
    """All 3x3 kernels accumulate in the (input chunk, tap, 32-channel half) order,
    so whichever the dispatcher picks for a layer (it depends on the batch size)
    the output bits are the same: direct kernels, the 8-phase GEMMs and the tiled
    engine on tap-uniform im2col."""
    from cirtorch import _engine as E
    L = E.lib()
    outs = {}
    # (RR_TUNE_CONV3X3, RR_TUNE_GEMM8, RR_TUNE_GRID_CUS): a CU cap of 8 makes the
    # 8-phase kernels eligible on these small problems
    paths = {"direct": (1, 0, 0), "gemm8": (0, 2, 8), "gemm8a": (0, 1 | 4, 8), "tiled": (0, 0, 0)}
    try:
        for name, (c3, g8, cap) in paths.items():
            E.check(L.rr_set_tuning(6, c3), "rr_set_tuning")
            E.check(L.rr_set_tuning(8, g8), "rr_set_tuning")
            E.check(L.rr_set_tuning(7, cap), "rr_set_tuning")
            outs[name] = _check_conv(cuda, case, prec, True)
    finally:
        L.rr_set_tuning(6, 1)
        L.rr_set_tuning(8, 1)
        L.rr_set_tuning(7, 0)
    ref = outs.pop("tiled")
    for name, o in outs.items():
        assert torch.equal(o, ref), name
