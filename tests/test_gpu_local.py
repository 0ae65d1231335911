"""Local-descriptor head on the GPU: rr_local_head vs
the reference localHead golden (tests/golden/local.npz, produced by the
reference module), and the mutual-NN matcher vs the HPatchesEval restatement."""

import numpy as np
import pytest
import torch

from conftest import golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("tag", ["a", "b"])
@pytest.mark.parametrize("layout", ["nchw", "channels_last"])
def test_local_head_vs_reference_golden(cuda, tag, layout):
    from cirtorch.modules.heads.local_head import localHead
    g = golden("local.npz")
    x = torch.from_numpy(g["x_" + tag]).to(cuda)
    if layout == "channels_last":
        x = x.contiguous(memory_format=torch.channels_last)
    e, c = g["w_" + tag].shape
    head = localHead(c, e).to(cuda)
    head.load_state_dict({"whiten.weight": torch.from_numpy(g["w_" + tag]),
                          "whiten.bias": torch.from_numpy(g["b_" + tag])})
    got = head(x, torch.from_numpy(g["kpts_" + tag]).to(cuda)).cpu().numpy()
    np.testing.assert_allclose(got, g["desc_" + tag], rtol=0, atol=2e-6)


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_local_head_16bit_map(cuda, dt):
    """bf16 / fp16 stage map (the engine's extractor output dtypes): descriptors within input rounding."""
    from cirtorch import _ops
    g = golden("local.npz")
    x = torch.from_numpy(g["x_b"])
    xb = x.to(dt)
    ref = torch.from_numpy(g["desc_b"])
    from oracle import ops
    ref_b = ops.local_head(xb.float(), torch.from_numpy(g["kpts_b"]), torch.from_numpy(g["w_b"]),
                           torch.from_numpy(g["b_b"]))
    got = _ops.local_head(xb.to(cuda).contiguous(memory_format=torch.channels_last),
                          torch.from_numpy(g["kpts_b"]).to(cuda), torch.from_numpy(g["w_b"]).to(cuda),
                          torch.from_numpy(g["b_b"]).to(cuda)).cpu()
    assert (got - ref_b).abs().max().item() < 2e-6
    cos = (got * ref).sum(-1) / (got.norm(dim=-1) * ref.norm(dim=-1))
    assert cos.min().item() > 0.999


def test_mutual_nn_vs_restatement(cuda):
    from cirtorch.search import mutual_nn
    g = golden("local.npz")
    d1 = torch.from_numpy(g["desc_b"][0]).to(cuda)
    d2 = torch.from_numpy(g["nn_d2"]).to(cuda)
    got = mutual_nn(d1, d2).cpu().numpy()
    assert (got == g["nn_match"]).all()
    assert (got >= 0).sum() > 0
