"""Sum the FETCH_SIZE / WRITE_SIZE counters (rocprofv3 --pmc, csv) of the
extractor-body dispatches between the two k_l2n_rows markers written by
tools/pmc_body.py, per forward, with the gfx950 correction of
MI355X_MICROARCH.md §HBM (FETCH_SIZE counts half the bytes of a wide
coalesced read: x2; WRITE_SIZE exact for 16-B stores; both in KiB).

    python3 tools/pmc_parse.py FETCH_DIR WRITE_DIR --iters 3 --batch 32
"""

import argparse
import csv
import sys
import glob
import json
import os


def load(d, counter):
    path = sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True))
    if not path:
        raise SystemExit("no counter_collection.csv under %s" % d)
    rows = list(csv.DictReader(open(path[0])))
    rows = [r for r in rows if r.get("Counter_Name") == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    marks = [i for i, r in enumerate(rows) if "k_l2n_rows" in r["Kernel_Name"]]
    if len(marks) < 2:
        raise SystemExit("markers not found in %s" % path[0])
    body = rows[marks[-2] + 1:marks[-1]]
    per_kernel = {}
    for r in body:
        name = r["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0].replace("void ", "")
        per_kernel.setdefault(name, [0.0, 0])
        per_kernel[name][0] += float(r["Counter_Value"])
        per_kernel[name][1] += 1
    return sum(float(r["Counter_Value"]) for r in body), len(body), per_kernel


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_dir")
    ap.add_argument("write_dir")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--config", default="{}", help="JSON config of the workload (bench.py matches on it)")
    args = ap.parse_args()
    f_kib, nf, fk = load(args.fetch_dir, "FETCH_SIZE")
    w_kib, nw, wk = load(args.write_dir, "WRITE_SIZE")
    read_b = 2.0 * f_kib * 1024 / args.iters      # gfx950: FETCH_SIZE reads half of a wide stream
    write_b = w_kib * 1024 / args.iters
    out = {"hbm_read_bytes_per_forward": read_b, "hbm_write_bytes_per_forward": write_b,
           "hbm_bytes_per_forward": read_b + write_b, "batch": args.batch,
           "hbm_bytes_per_image": (read_b + write_b) / args.batch,
           "dispatches_per_forward": nf / args.iters,
           "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over tools/pmc_body.py; "
                     "body dispatches between two marker kernels; read = 2 x FETCH_SIZE (gfx950 half-count of "
                     "wide reads), write = WRITE_SIZE; KiB -> bytes",
           "per_kernel_read_bytes": {k: 2.0 * v[0] * 1024 / args.iters for k, v in fk.items()},
           "per_kernel_write_bytes": {k: v[0] * 1024 / args.iters for k, v in wk.items()}}
    # the kernel sources the counters were collected on (bench.py attaches the
    # traffic to its roofline only while the digest still matches)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from bench import kernel_source_digest
    cfg = json.loads(args.config)
    cfg["source_digest"] = kernel_source_digest()
    cfg["source_commit"] = os.environ.get("RR_SOURCE_COMMIT", "?")
    out["config"] = cfg
    if "screen" in cfg:  # a kNN search workload
        out["hbm_bytes_per_search"] = out["hbm_bytes_per_forward"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
