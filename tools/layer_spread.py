"""Per-layer dispatch times of the extractor body from a rocprofv3 kernel trace of bench.py
(run_kernel_trace.csv), split by whether the step's kNN search was running beside the launch.

A kernel name is shared by several layers (k_gemm8's short-K 1x1 serves K = 512 .. 2048 at three
map sizes, k_pair_mid's boundary is two chunk launches of 2^20 and 0.57 x 2^20 pixels), so the
min / avg / max of a NAME mixes layers of different sizes.  This groups dispatches by their
position in the forward (the launch sequence of one forward is fixed; a forward starts at the
headline dtype's stem kernel) and reports, per position, the median time of forwards with no
other-stream kernel overlapping the launch ("alone") and of forwards where one did ("beside the
search").  Developer tool.

    python3 tools/layer_spread.py run_kernel_trace.csv [--dtype fp16] [--md]
"""
import argparse
import csv
import re
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from prof_summary import is_body  # noqa: E402


def short(name):
    """kernel + template arguments, from a demangled (void rr::k_x<...>(...)) or mangled name"""
    m = re.search(r"(k_[A-Za-z0-9_]+?)(I[A-Za-z0-9_]*?)EEv", name)          # mangled
    if name.startswith("_Z") and m:
        return m.group(1) + "<" + m.group(2)[1:].replace("DF16_", "f16,")[:28] + ">"
    m = re.search(r"(k_[A-Za-z0-9_]+)(<[^()]*>)?", name)                     # demangled
    return (m.group(1) + (m.group(2) or "")[:40]) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--dtype", default="fp16")
    ap.add_argument("--md", action="store_true")
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.trace)))
    for r in rows:
        r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    rows.sort(key=lambda r: r["s"])
    stems = [i for i, r in enumerate(rows) if "k_stem_pool" in r["Kernel_Name"] and is_body(r["Kernel_Name"], args.dtype)]
    if not stems:
        sys.exit("no %s stem dispatch in the trace" % args.dtype)
    stream = rows[stems[0]]["Stream_Id"]
    others = [r for r in rows if r["Stream_Id"] != stream]
    forwards = []
    for a, b in zip(stems, stems[1:] + [len(rows)]):
        fw = [r for r in rows[a:b] if r["Stream_Id"] == stream and is_body(r["Kernel_Name"], args.dtype)]
        forwards.append(fw)
    # the modal forward length is the model's launch count; other lengths are other models / precisions
    lens = statistics.multimode(len(f) for f in forwards)
    n_l = max(lens)
    forwards = [f for f in forwards if len(f) == n_l]

    def contended(r):
        return any(o["s"] < r["e"] and o["e"] > r["s"] for o in others)

    table = []
    for pos in range(n_l):
        name = short(forwards[0][pos]["Kernel_Name"])
        alone, beside = [], []
        for f in forwards:
            r = f[pos]
            if short(r["Kernel_Name"]) != name:
                continue
            (beside if contended(r) else alone).append((r["e"] - r["s"]) / 1e3)
        table.append((pos, name, alone, beside))
    hdr = "| # | kernel | n alone | median alone us | n beside | median beside us | beside / alone |"
    print(hdr)
    print("|---|---|---|---|---|---|---|")
    tot_a = tot_b = 0.0
    for pos, name, alone, beside in table:
        ma = statistics.median(alone) if alone else float("nan")
        mb = statistics.median(beside) if beside else float("nan")
        if alone:
            tot_a += ma
            tot_b += mb if beside else ma
        print("| %d | `%s` | %d | %.1f | %d | %.1f | %.2f |" % (pos, name, len(alone), ma, len(beside), mb,
                                                             mb / ma if alone and beside else float("nan")))
    print("\nforwards analysed: %d (%d launches each); sum of per-layer medians alone %.1f us, with the "
          "contended launches at their beside-median %.1f us" % (len(forwards), n_l, tot_a, tot_b))


if __name__ == "__main__":
    main()
