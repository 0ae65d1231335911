"""Average the counters of the last N dispatches of one kernel name pattern
over rocprofv3 --pmc CSV passes.  Developer tool.
    python3 tools/pmc_summary.py <dir with p1/ p2/ ...> <kernel substring> [N]"""
import collections
import csv
import glob
import os
import sys


def main():
    d, pat = sys.argv[1], sys.argv[2]
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    vals = collections.OrderedDict()
    for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
        disp = collections.OrderedDict()
        for r in csv.DictReader(open(f)):
            if pat in r["Kernel_Name"]:
                disp.setdefault(r["Dispatch_Id"], []).append(r)
        last = list(disp.values())[-n:]
        acc = collections.defaultdict(float)
        for dd in last:
            for r in dd:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
        for k, v in acc.items():
            vals[k] = v / max(1, len(last))
    for k, v in vals.items():
        print("%-28s %14.4g" % (k, v))


if __name__ == "__main__":
    main()
