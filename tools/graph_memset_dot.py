"""Developer probe: one kNN search with the tau reset done by
hipMemsetAsync (RR_KNN_TAU_MEMSET=1) captured into a torch CUDAGraph, in
variants of the capture order of tests/test_gpu_graph.py, each compared with
the eager search after 3 replays.

    RR_KNN_TAU_MEMSET=1 python tools/graph_memset_dot.py [variant ...]
"""

import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def run(variant):
    from cirtorch.search import KnnIndex
    from oracle import data
    dev = torch.device("cuda:0")
    db = torch.from_numpy(data.unit_rows(20000, 256, seed=41)).to(dev)
    q1 = torch.from_numpy(data.unit_rows(8, 256, seed=42)).to(dev)
    index = KnnIndex(db, "bf16")
    if "eager_first" in variant:
        index.search(q1, 20)
        torch.cuda.synchronize()
    static_q = q1.clone()
    warm = torch.cuda.current_stream(dev) if "warm_main" in variant else torch.cuda.Stream(dev)
    warm.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(warm):
        for _ in range(0 if "nowarm" in variant else 2):
            index.search(static_q, 20)
    torch.cuda.current_stream(dev).wait_stream(warm)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        s, i = index.search(static_q, 20)
    torch.cuda.synchronize()
    res = []
    for r in range(3):
        if "copy" in variant:
            static_q.copy_(q1)
        g.replay()
        torch.cuda.synchronize()
        es, ei = index.search(q1, 20)
        torch.cuda.synchronize()
        res.append((i != ei).any(dim=1).nonzero().flatten().tolist())
    ws = {hex(k): hex(v.data_ptr()) for k, v in index._ws.items()}
    print("%-32s rows differing from eager per replay: %s  workspaces %s" % (variant, res, ws), flush=True)


def main():
    variants = sys.argv[1:] or ["test_order+copy", "test_order", "eager_first+copy", "warm_main+copy", "nowarm+copy"]
    for v in variants:
        run(v)


if __name__ == "__main__":
    main()
