"""Workload for the HBM-traffic counter passes of the kNN search (the bench's
match kernels): a 1M x 2048 database (fp16 screening copy by default), ITERS certified searches of Q
queries (top-100) between two marker kernels, so tools/pmc_parse.py picks
exactly the searches' dispatches out of the rocprofv3 counter CSV.

    rocprofv3 --pmc FETCH_SIZE -d DIR -o run --output-format csv -- python3 tools/pmc_knn.py --q 1024
    rocprofv3 --pmc WRITE_SIZE -d DIR -o run --output-format csv -- python3 tools/pmc_knn.py --q 1024
    python3 tools/pmc_parse.py DIR_FETCH DIR_WRITE --iters 3 --batch 1024 > profiles/<round>_pmc_knn_q1024.json

Developer tool (not part of the product path)."""

import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--q", type=int, default=1024)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--precision", default="fp16")
    args = ap.parse_args()
    from cirtorch import _ops
    from cirtorch.search import KnnIndex
    db = _ops.fill_unit_rows(args.n, 2048, seed=0xDB5EED)
    q = _ops.fill_unit_rows(args.q, 2048, seed=0x0E5EED)
    index = KnnIndex(db, args.precision)
    marker = torch.zeros(64, device="cuda")
    for _ in range(2):
        index.search(q, 100, verify="deferred")[2].resolve()
    torch.cuda.synchronize()
    _ops.l2n_rows(marker.view(1, 64))          # marker: search dispatches follow
    pends = [index.search(q, 100, verify="deferred")[2] for _ in range(args.iters)]   # the bench's search
    _ops.l2n_rows(marker.view(1, 64))          # marker: end
    torch.cuda.synchronize()
    assert sum(p.resolve() for p in pends) == 0
    print("done", args.iters, "searches of", args.q, "queries vs", args.n)


if __name__ == "__main__":
    main()
