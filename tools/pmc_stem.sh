#!/bin/bash
# Counter passes over tools/stem_probe.py (one rocprofv3 run per pass).
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/$1"; TUNE=${2:-}; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for PASS in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $PASS -d "$OUT/p$i" -o run --output-format csv -- \
    python3 "$ROOT/tools/stem_probe.py" --tune "$TUNE" > "$OUT/p$i.log" 2>&1
done
