#!/bin/bash
# SQ / TA counter passes over tools/g8_pmc_work.py (k_gemm8 on a square GEMM), one rocprofv3 run per pass.
#   bash tools/g8_pmc.sh <outdir> [P C K]
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/$1"; shift
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
i=0
for C in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC" \
         "SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "TA_TA_BUSY_sum SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/p$i" -o run --output-format csv -- python3 "$ROOT/tools/g8_pmc_work.py" "$@" > "$OUT/p$i.log" 2>&1 || echo "pass $i failed"
done
echo g8 pmc done
