"""tools/dma_audit.py: the LDS-DMA wait-state audit (the issue sequences carry one wait state
after the M0 write; the descriptor's 5 states after a VALU SGPR write come from the fence in
the rsrc makers).  Synthetic disassembly checks that each hazard is found, and the audit of the
in-tree build objects (when present) is clean.  CPU only."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import dma_audit  # noqa: E402

HEAD = ["0000000000001000 <_ZN2rr6k_testEv>:"]


def dis(*ins):
    return HEAD + ["\t%s // 000000001000: 00000000" % i for i in ins]


def test_clean_sequence_passes():
    f, n = dma_audit.audit(dis("v_readfirstlane_b32 s48, v1", "s_nop 4", "s_mov_b32 s92, m0", "s_mov_b32 m0, s90",
                               "s_nop 0", "buffer_load_dwordx4 v3, s[48:51], 0 offen lds", "s_mov_b32 m0, s92"))
    assert n == 1 and f == []


def test_fresh_descriptor_is_found():
    f, n = dma_audit.audit(dis("v_readfirstlane_b32 s49, v1", "s_mov_b32 m0, s90", "s_nop 0",
                               "buffer_load_dwordx4 v3, s[48:51], 0 offen lds"))
    assert n == 1 and len(f) == 1 and "VALU SGPR write" in f[0][2]


def test_unrelated_sgpr_write_is_not_a_finding():
    f, _ = dma_audit.audit(dis("v_readfirstlane_b32 s90, v1", "s_mov_b32 m0, s90", "s_nop 0",
                               "buffer_load_dwordx4 v3, s[48:51], 0 offen lds"))
    assert f == []


def test_m0_write_directly_before_dma_is_found():
    f, _ = dma_audit.audit(dis("s_mov_b32 m0, s90", "buffer_load_dwordx4 v3, s[48:51], 0 offen lds"))
    assert any("M0 write directly" in x[2] for x in f)


def test_other_m0_reader_is_found():
    f, _ = dma_audit.audit(dis("s_movrels_b32 s1, s2", "v_movrels_b32 v1, m0"))
    assert any("M0 named" in x[2] for x in f)


def test_build_objects_are_clean():
    build = dma_audit.BUILD
    if not os.path.exists(os.path.join(build, "rr_gemm.o")):
        pytest.skip("no in-tree build objects")
    import glob
    import subprocess
    if not os.path.exists(dma_audit.LLVM + "/llvm-objdump"):
        pytest.skip("no llvm-objdump")
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "dma_audit.py")], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:]
    assert "findings: 0" in r.stdout and glob.glob(os.path.join(build, "rr_*.o"))
