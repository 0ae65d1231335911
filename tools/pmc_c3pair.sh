#!/bin/bash
# SQ counter passes (one rocprofv3 run per pass) over tools/c3pair_pmc.py:  bash tools/pmc_c3pair.sh <form> <outdir>
set -e
FORM=$1; OUT=$2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for PASS in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA" \
            "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PASS -d "$ROOT/$OUT/p$i" -o run --output-format csv -- \
    python3 "$ROOT/tools/c3pair_pmc.py" "$FORM" > "$ROOT/$OUT/p$i.log" 2>&1
done
