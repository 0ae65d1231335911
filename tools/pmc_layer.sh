#!/bin/bash
# Counter passes (one rocprofv3 run per pass) over tools/layer_probe.py.
#   bash tools/pmc_layer.sh <layer> <outdir> [tune]
set -e
LAYER=$1; OUT=$2; TUNE=${3:-}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$ROOT/$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for PASS in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES" \
            "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR" \
            "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $PASS -d "$ROOT/$OUT/p$i" -o run --output-format csv -- \
    python3 "$ROOT/tools/layer_probe.py" --layer "$LAYER" --reps 10 --tune "$TUNE" > "$ROOT/$OUT/p$i.log" 2>&1
done
