#!/bin/bash
# LDS / MFMA counters of the lab k_gemm8 schedule in several diagnostic modes (one rocprofv3 run per
# mode and pass).   bash tools/lab/g8lab_pmc.sh <outdir> "<modes>" [P C K]
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/$1"; MODES=$2; shift 2
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for M in $MODES; do
  i=0; mkdir -p "$OUT/m$M"
  for C in "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $C -d "$OUT/m$M/p$i" -o run --output-format csv -- python3 "$ROOT/tools/lab/g8lab_pmc_work.py" $M "$@" > "$OUT/m$M/p$i.log" 2>&1 || { echo "mode $M pass $i failed"; exit 1; }
  done
done
echo g8lab pmc done
