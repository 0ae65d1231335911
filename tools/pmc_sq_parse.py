"""Average SQ / TA / GRBM counters per dispatch of the kernels whose name contains KEY over the
counter passes of tools/g8_pmc.sh (skipping the first SKIP dispatches), with the wave-cycle
breakdown and the MFMA busy fraction.  Developer tool.
    python3 tools/pmc_sq_parse.py <dir with p1 p2 p3> [KEY] [SKIP]"""
import collections
import csv
import os
import sys


def main():
    d = sys.argv[1]
    key = sys.argv[2] if len(sys.argv) > 2 else "k_gemm8"
    skip = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in sorted(os.listdir(d)):
        f = os.path.join(d, p, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            if key in r["Kernel_Name"]:
                agg[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    res = {}
    for c, per in agg.items():
        vals = [per[k] for k in sorted(per)][skip:]
        res[c] = sum(vals) / max(1, len(vals))
    for c in sorted(res):
        print("%-28s %.5g" % (c, res[c]))
    w = res.get("SQ_WAVE_CYCLES")
    if w:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM",
                  "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_WAIT_INST_LDS"):
            if c in res:
                print("%-22s %.3f of wave cycles" % (c, res[c] / w))
    g = res.get("GRBM_GUI_ACTIVE")
    if g and "SQ_VALU_MFMA_BUSY_CYCLES" in res:
        print("MFMA busy %.3f (busy cycles / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)); kernel ~%.1f us at 2.1 GHz"
              % (res["SQ_VALU_MFMA_BUSY_CYCLES"] / (g / 8 * 1024), g / 8 / 2.1e3))


if __name__ == "__main__":
    main()
