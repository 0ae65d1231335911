"""Side-by-side per-layer table of a tools/lib_layers_ab.sh run: python tools/ab_table.py <dir> <rounds>"""
import sys

d, R = sys.argv[1], int(sys.argv[2])


def parse(path):
    out = {}
    for line in open(path):
        t = line.split()
        if len(t) >= 6 and t[-1].isdigit():   # name  shape...  us  TFLOP/s  GFLOP  calls
            try:
                out.setdefault(t[0], float(t[-4]))
            except ValueError:
                pass
    return out


runs = {(s, r): parse("%s/%s_%d.txt" % (d, s, r)) for s in "AB" for r in range(1, R + 1)}
names = list(runs[("A", 1)].keys())
print("%-18s" % "layer" + "".join("%10s" % ("%s%d" % (s, r)) for r in range(1, R + 1) for s in "AB"))
for n in names:
    print("%-18s" % n + "".join("%10.1f" % runs[(s, r)].get(n, float("nan")) for r in range(1, R + 1) for s in "AB"))
