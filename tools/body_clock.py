"""Clock the chip held per kernel, from one rocprofv3 run with both --pmc GRBM_GUI_ACTIVE and
--kernel-trace: clock = (GRBM_GUI_ACTIVE summed over the 8 XCDs / 8) / dispatch duration, per
dispatch, then the median per kernel name (the top kernels by time).  Counter collection
serialises the dispatches, so this is the clock of each kernel running alone.  Developer tool.

    rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d DIR -o run --output-format csv -- python3 tools/pmc_body.py ...
    python3 tools/body_clock.py DIR [TOP]
"""
import collections
import csv
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from layer_spread import short  # noqa: E402


def main():
    d = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 14
    gui = collections.defaultdict(float)
    for r in csv.DictReader(open(os.path.join(d, "run_counter_collection.csv"))):
        if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
            gui[int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    per = collections.defaultdict(list)
    tot = collections.defaultdict(float)
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        i = int(r["Dispatch_Id"])
        ns = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        if i in gui and ns > 20000:  # launches of 20 us and more
            name = short(r["Kernel_Name"])
            per[name].append(gui[i] / 8.0 / ns)
            tot[name] += ns
    print("| kernel | dispatches | time ms | median GHz | min | max |")
    print("|---|---|---|---|---|---|")
    for name in sorted(tot, key=lambda n: -tot[n])[:top]:
        v = per[name]
        print("| `%s` | %d | %.2f | %.2f | %.2f | %.2f |" % (name, len(v), tot[name] / 1e6, statistics.median(v), min(v),
                                                       max(v)))


if __name__ == "__main__":
    main()
