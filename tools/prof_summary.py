"""Markdown summary of a rocprofv3 --kernel-trace --stats run of bench.py:
top kernels, and the extractor-body family (the bench's dominant kernel
family) per forward, to set beside the bench's HIP-event body time.

    python3 tools/prof_summary.py <run_kernel_stats.csv> <bench.json> --forwards F
F = forwards in the profiled run: (steps + warmup + max(3, steps // 2)) x batch / extract_batch.
"""

import argparse
import csv
import json

BODY = ("k_stem_pool", "k_conv3x3", "k_stream1x1", "k_stream_pair", "k_igemm<unsigned short, unsigned short",
        "k_gemm8<unsigned short, unsigned short", "k_pair_mid", "k_gemm8a<", "k_c3s_w", "k_wres1x1", "k_c3w64")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("bench")
    ap.add_argument("--forwards", type=int, required=True)
    ap.add_argument("--top", type=int, default=25)
    args = ap.parse_args()
    rows = list(csv.DictReader(open(args.stats)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    b = json.loads(open(args.bench).read().strip().splitlines()[-1])
    print("| %% | total us | calls | avg us | kernel |\n|---|---|---|---|---|")
    for r in rows[:args.top]:
        print("| %.2f | %.1f | %s | %.1f | `%s` |" % (100 * float(r["TotalDurationNs"]) / tot,
                                                    float(r["TotalDurationNs"]) / 1e3, r["Calls"],
                                                    float(r["AverageNs"]) / 1e3, r["Name"][:120]))
    # the bf16 headline forwards only (the fp16 e2e line's kernels carry mangled DF16_ names)
    body = [r for r in rows if any(k in r["Name"] for k in BODY) and "DF16_" not in r["Name"]]
    body_us = sum(float(r["TotalDurationNs"]) for r in body) / 1e3 / args.forwards
    eb = b["config"].get("extract_batch", b["config"]["global_batch"])
    per_fwd_bench = b["roofline"]["achieved"] and (b["roofline_layers"]["measured_ms"] * 1e3 *
                                                   eb / b["config"]["global_batch"])
    print()
    print("Extractor-body kernel family (%s): %.1f us of kernel time per %d-image forward "
          "(sum of rocprof durations / %d forwards); bench HIP-event body time per forward: %.1f us "
          "(includes launch gaps)." % (", ".join(BODY), body_us, eb, args.forwards, per_fwd_bench))
    print()
    print("| body kernel | avg us | calls in run | us per forward |\n|---|---|---|---|")
    for r in body:
        name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        print("| `%s` | %.1f | %s | %.1f |" % (name, float(r["AverageNs"]) / 1e3, r["Calls"],
                                            float(r["TotalDurationNs"]) / 1e3 / args.forwards))


if __name__ == "__main__":
    main()
