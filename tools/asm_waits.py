"""List the `s_waitcnt vmcnt` instructions between each kernel's first and last MFMA
(developer check, CPU only): a compiler-inserted vmcnt wait inside a tile loop is
counted against the kernel's own LDS-DMA and stores, which the compiler cannot
see, and stalls the loop on them.  Intended waits are the kernels' explicit
`s_waitcnt vmcnt(N)` + `s_barrier` pairs and the rare-path atomics' vmcnt(0).

    python3 tools/asm_waits.py [file.hip ...]      (default: every csrc/*.hip)
"""

import collections
import glob
import os
import re
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "image-retrieval-for-image-based-localization_amd", "csrc")


def waits(asm):
    out = {}
    for m in re.finditer(r"^(_Z\S+):", asm, re.M):
        end = asm.find(".Lfunc_end", m.end())
        body = [l.strip() for l in asm[m.end():end].split("\n")]
        body = [l for l in body if l and not l.startswith((";", "."))]
        idx = [k for k, l in enumerate(body) if l.startswith("v_mfma")]
        if not idx:
            continue
        seg = body[idx[0]:idx[-1] + 1]
        out[m.group(1)] = (len(idx), collections.Counter(l for l in seg if l.startswith("s_waitcnt") and "vmcnt" in l))
    return out


def main():
    files = sys.argv[1:] or sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    for f in files:
        with tempfile.NamedTemporaryFile(suffix=".s") as t:
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                            "-S", f, "-o", t.name], check=True, cwd=CSRC, stderr=subprocess.DEVNULL)
            for name, (n, c) in waits(open(t.name).read()).items():
                print("%-70s mfma %4d  vmcnt waits %3d  %s" % (name[:70], n, sum(c.values()), dict(c.most_common(4))))


if __name__ == "__main__":
    main()
