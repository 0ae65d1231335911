"""HIP-graph replay (cirtorch.utils.graph.GraphedForward) of the extractor and
of the kNN search: replay is bit-identical to the eager launches on the same
inputs, re-reads new inputs, and rejects a shape it was not captured for."""

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _net(arch, precision, cuda):
    from cirtorch.models.GF_net import make_net
    from cirtorch.models.init import random_init_
    net = make_net(arch, precision=precision)
    random_init_(net, seed=0)
    return net.to(cuda).eval()


@pytest.mark.parametrize("arch,precision", [("resnet50", "bf16"), ("resnet18", "fp32")])
def test_graphed_extract_equals_eager(cuda, arch, precision):
    from cirtorch.utils.graph import GraphedForward
    net = _net(arch, precision, cuda)
    g0 = torch.Generator(device="cpu").manual_seed(5)
    x1 = torch.rand(2, 3, 192, 256, generator=g0).to(cuda)
    x2 = torch.rand(2, 3, 192, 256, generator=g0).to(cuda)
    e1 = net.extract(x1).clone()
    e2 = net.extract(x2).clone()
    g = GraphedForward(lambda t: net.extract(t), x1)
    assert torch.equal(g(x1), e1)
    assert torch.equal(g(x2), e2)
    assert torch.equal(g(x1), e1)
    with pytest.raises(ValueError):
        g(torch.rand(1, 3, 192, 256, device=cuda))


def test_graphed_search_equals_eager(cuda):
    from cirtorch.search import KnnIndex
    from cirtorch.utils.graph import GraphedForward
    from oracle import data, ops
    db = torch.from_numpy(data.unit_rows(20000, 256, seed=41)).to(cuda)
    q1 = torch.from_numpy(data.unit_rows(8, 256, seed=42)).to(cuda)
    q2 = torch.from_numpy(data.unit_rows(8, 256, seed=43)).to(cuda)
    index = KnnIndex(db, "bf16")
    g = GraphedForward(lambda q: index.search(q, 20, verify=False), q1)
    for q in (q1, q2):
        s, i = g(q)
        es, ei = index.search(q, 20, verify=False)
        assert torch.equal(i, ei) and torch.equal(s, es)
        ref_s, ref_i = ops.topk_exact(db.cpu().numpy(), q.cpu().numpy(), 20)
        np.testing.assert_array_equal(i.cpu().numpy(), ref_i)
