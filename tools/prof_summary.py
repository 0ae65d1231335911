"""Markdown summary of a rocprofv3 --kernel-trace --stats run of bench.py:
top kernels, and the extractor-body family (the bench's dominant kernel
family) per forward, to set beside the bench's HIP-event body time.

    python3 tools/prof_summary.py <run_kernel_stats.csv> <bench.json> [--forwards F] [--dtype fp16|bf16]
F = forwards of the headline dtype in the profiled run (default: the calls of its stem kernel, one
per forward); dtype default = the bench line's.  fp16 kernels carry mangled DF16_ names.
"""

import argparse
import csv
import json

BODY = ("k_stem_pool", "k_conv3x3", "k_stream1x1", "k_stream_pair", "k_igemm", "k_gemm8", "k_pair_mid", "k_gemm8a",
        "k_c3s_w", "k_wres1x1", "k_c3w64", "k_c3pair")


def is_body(name, dtype):
    """an extractor-body conv kernel of the given 16-bit dtype (not the kNN score GEMMs: float output,
    int8 operands, k_gemm8s)"""
    if not any(k in name for k in BODY):
        return False
    if "k_gemm8s" in name or "float," in name or "float>" in name or "signed char" in name:
        return False
    if ("k_gemm8I" in name or "k_igemmI" in name) and "DF16_f" in name:
        return False
    return ("DF16_" in name) == (dtype == "fp16")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats")
    ap.add_argument("bench")
    ap.add_argument("--forwards", type=int, default=0)
    ap.add_argument("--dtype", default="")
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
    dtype = args.dtype or b.get("dtype", "bf16")
    body = [r for r in rows if is_body(r["Name"], dtype)]
    if not args.forwards:
        args.forwards = max(int(r["Calls"]) for r in body if "k_stem_pool" in r["Name"])
    body_us = sum(float(r["TotalDurationNs"]) for r in body) / 1e3 / args.forwards
    eb = b["config"].get("extract_batch", b["config"]["global_batch"])
    per_fwd_bench = b["roofline"]["achieved"] and (b["roofline_layers"]["measured_ms"] * 1e3 *
                                                   eb / b["config"]["global_batch"])
    print()
    print("Extractor-body kernel family (%s; %s): %.1f us of kernel time per %d-image forward "
          "(sum of rocprof durations / %d forwards); bench HIP-event body time per forward: %.1f us "
          "(includes launch gaps)." % (", ".join(BODY), dtype, body_us, eb, args.forwards, per_fwd_bench))
    print()
    print("| body kernel | avg us | calls in run | us per forward |\n|---|---|---|---|")
    for r in body:
        name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "")
        print("| `%s` | %.1f | %s | %.1f |" % (name, float(r["AverageNs"]) / 1e3, r["Calls"],
                                            float(r["TotalDurationNs"]) / 1e3 / args.forwards))


if __name__ == "__main__":
    main()
