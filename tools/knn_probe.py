"""Time one search of Q queries (default 128, the bench step) against an N x 2048
database (default 1M) for rocprofv3 kernel traces.  Developer tool."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "image-retrieval-for-image-based-localization_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--q", type=int, default=128)
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--tune", default="", help="rr_set_tuning pairs key=value[,key=value]")
    ap.add_argument("--screen", default="fp16", help="screening dtype (int8 / fp16 / bf16 / fp32)")
    ap.add_argument("--no-verify", dest="verify", action="store_false",
                    help="unverified search (default: the bench's certified search, certificate resolved)")
    args = ap.parse_args()
    from cirtorch import _ops
    from cirtorch import _engine as E
    for kv in filter(None, args.tune.split(",")):
        k_, v_ = kv.split("=")
        E.check(E.lib().rr_set_tuning(int(k_), int(v_)), "rr_set_tuning")
    from cirtorch.search import KnnIndex
    db = _ops.fill_unit_rows(args.n, 2048, seed=0xDB5EED)
    q = _ops.fill_unit_rows(args.q, 2048, seed=0x0E5EED)
    idx = KnnIndex(db, args.screen)
    def one():
        if args.verify:
            return idx.search(q, 100, verify="deferred")[2]
        idx.search(q, 100, verify=False)
        return None
    p = one()
    if p is not None:
        p.resolve()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    pends = [one() for _ in range(args.reps)]
    b.record()
    nre = sum(p.resolve() for p in pends if p is not None)
    torch.cuda.synchronize()
    print("search Q=%d N=%d screen=%s verify=%s tune=%s: %.3f ms (re-searched %d)"
          % (args.q, args.n, args.screen, args.verify, args.tune, a.elapsed_time(b) / args.reps, nre))


if __name__ == "__main__":
    main()
