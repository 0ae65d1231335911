"""Wait-state audit of the LDS-DMA issue sequences in librr's device code.

Every LDS-DMA (`buffer_load_dwordx4 ... offen lds`) is issued from inline asm, whose text hipcc
does not pad for hazards.  Two hazards concern it (cdna_hip_programming.md §5.7 item 2):
  * M0 written by `s_mov_b32 m0, ...` -> the LDS-DMA that reads it: 1 wait state;
  * an SGPR written by a VALU instruction (v_readfirstlane / v_readlane / a VALU with an SGPR
    destination) -> the LDS-DMA reading it as its buffer descriptor: 5 wait states.
The issue sequence carries only the first (`s_nop 0`); the descriptors are produced by
make_rsrc, which ends in a wait-state fence tied to the descriptor registers.  This audit
disassembles the gfx950 code objects of csrc/build/*.o and walks back from every LDS-DMA in
program order: it fails if a VALU SGPR write to the descriptor lies within 5 wait states, if
fewer than 1 wait state separates the M0 write from the DMA, or if any instruction other than
`s_mov_b32` names M0 (an M0 reader the save / restore would have to protect).
Walking back in program order is exact within a basic block; the issue sequences are
straight-line asm statements, so the states inside them never cross a branch.

    python3 tools/dma_audit.py [csrc/build]          (exit 1 on a finding)
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(REPO, "image-retrieval-for-image-based-localization_amd", "csrc", "build")


def disassemble(obj, tmp):
    fb = os.path.join(tmp, "fb.bin")
    co = os.path.join(tmp, "g.co")
    if subprocess.run([LLVM + "/llvm-objcopy", "--dump-section", ".hip_fatbin=" + fb, obj],
                      capture_output=True).returncode:
        return []  # no device code in this object
    subprocess.run([LLVM + "/clang-offload-bundler", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                    "--input=" + fb, "--output=" + co, "--unbundle"], check=True, capture_output=True)
    out = subprocess.run([LLVM + "/llvm-objdump", "-d", co], check=True, capture_output=True, text=True).stdout
    return out.splitlines()


def sgprs(tok):
    """SGPR indices named by an operand token: s5, s[48:51]"""
    m = re.fullmatch(r"s(\d+)", tok)
    if m:
        return {int(m.group(1))}
    m = re.fullmatch(r"s\[(\d+):(\d+)\]", tok)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    return set()


def states(ins):
    m = re.match(r"s_nop\s+(0x[0-9a-f]+|\d+)", ins)
    return int(m.group(1), 0) + 1 if m else 1


def audit(lines):
    findings, n_dma = [], 0
    fn, body = None, []
    funcs = []
    for ln in lines:
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", ln)
        if m:
            if fn:
                funcs.append((fn, body))
            fn, body = m.group(1), []
            continue
        ins = ln.split("//")[0].strip()
        if fn and ins:
            body.append(ins)
    if fn:
        funcs.append((fn, body))
    for fn, body in funcs:
        for i, ins in enumerate(body):
            ops = [o.strip() for o in re.split(r"[ ,]+", ins)]
            if "m0" in ops[1:] and not ins.startswith("s_mov_b32"):
                findings.append((fn, i, "M0 named by %r" % ins))
            if not (ins.startswith("buffer_load_dwordx4") and ins.endswith("lds")):
                continue
            n_dma += 1
            desc = sgprs(ops[2])
            st, j, m0_gap = 0, i - 1, None
            while j >= 0 and st < 5:
                prev = body[j]
                pops = [o.strip() for o in re.split(r"[ ,]+", prev)]
                if prev.startswith("s_mov_b32") and len(pops) > 1 and pops[1] == "m0" and m0_gap is None:
                    m0_gap = st
                if prev.startswith("v_") and len(pops) > 1 and (sgprs(pops[1]) & desc):
                    findings.append((fn, i, "VALU SGPR write %r %d state(s) before %r" % (prev, st, ins)))
                st += states(prev)
                j -= 1
            if m0_gap is not None and m0_gap < 1:
                findings.append((fn, i, "M0 write directly before %r" % ins))
    return findings, n_dma


def main():
    build = sys.argv[1] if len(sys.argv) > 1 else BUILD
    objs = sorted(glob.glob(os.path.join(build, "rr_*.o")))
    objs = [o for o in objs if not o.endswith("rr_build.o")]
    total, bad = 0, []
    with tempfile.TemporaryDirectory() as tmp:
        for o in objs:
            f, n = audit(disassemble(o, tmp))
            total += n
            bad += [(os.path.basename(o),) + x for x in f]
            print("%-18s %6d LDS-DMA, %d finding(s)" % (os.path.basename(o), n, len(f)))
    for b in bad[:40]:
        print("  %s %s @%d: %s" % b)
    print("LDS-DMA audited: %d, findings: %d" % (total, len(bad)))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
