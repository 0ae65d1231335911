"""Per-kernel MFMA busy fraction of the extractor body from one rocprofv3 pass
with SQ_VALU_MFMA_BUSY_CYCLES and GRBM_GUI_ACTIVE (tools/pmc_round.sh):
busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs)
(MFMA busy cycles summed over the SIMDs, over the dispatch's shader cycles).

    python3 tools/pmc_mfma.py DIR --iters 3
"""

import argparse
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("d")
    ap.add_argument("--iters", type=int, default=3)
    args = ap.parse_args()
    path = sorted(glob.glob(os.path.join(args.d, "**", "*counter_collection.csv"), recursive=True))[0]
    rows = list(csv.DictReader(open(path)))
    by = {}
    for r in rows:
        by.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"]})[r["Counter_Name"]] = float(r["Counter_Value"])
    ids = sorted(by)
    marks = [i for i in ids if "k_l2n_rows" in by[i]["name"]]
    body = [i for i in ids if marks[-2] < i < marks[-1]]
    agg = {}
    for i in body:
        name = by[i]["name"].replace("(anonymous namespace)", "anon").split("(")[0].replace("void ", "")
        a = agg.setdefault(name, [0.0, 0.0, 0])
        a[0] += by[i].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        a[1] += by[i].get("GRBM_GUI_ACTIVE", 0.0)
        a[2] += 1
    out = {"method": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE over tools/pmc_body.py (R50 bf16, "
                     "128-image forwards); busy = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)",
           "per_kernel": {}}
    tb, tg = 0.0, 0.0
    for k, (b, g, n) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        out["per_kernel"][k] = {"calls_per_forward": n / args.iters,
                                "mfma_busy": b / (g / 8.0 * 1024.0) if g else None}
        tb += b
        tg += g
    out["body_mfma_busy"] = tb / (tg / 8.0 * 1024.0) if tg else None
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
