#!/bin/bash
# Counter passes of one round (each in its own rocprofv3 run: FETCH_SIZE uses
# 3 TCC slots, WRITE_SIZE 2 — never together), HBM bytes of the extractor body
# (128-image forwards) and of the kNN search (Q = 128 and 1024), plus the
# MFMA busy cycles of the body.
#   bash tools/pmc_round.sh <outdir> [precision (default fp16)] [kNN screen (default fp16)]
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/$1"
PREC=${2:-fp16}
SCREEN=${3:-fp16}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C -d "$OUT/body_$C" -o run --output-format csv -- \
    python3 "$ROOT/tools/pmc_body.py" --batch 128 --precision $PREC > "$OUT/body_$C.log" 2>&1
  for Q in 128 1024; do
    timeout -s KILL 240 rocprofv3 --pmc $C -d "$OUT/knn${Q}_$C" -o run --output-format csv -- \
      python3 "$ROOT/tools/pmc_knn.py" --q $Q --precision $SCREEN > "$OUT/knn${Q}_$C.log" 2>&1
  done
done
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d "$OUT/body_mfma" -o run \
  --output-format csv -- python3 "$ROOT/tools/pmc_body.py" --batch 128 --precision $PREC > "$OUT/body_mfma.log" 2>&1
python3 "$ROOT/tools/pmc_parse.py" "$OUT/body_FETCH_SIZE" "$OUT/body_WRITE_SIZE" --iters 3 --batch 128 \
  --config "{\"arch\": \"resnet50\", \"precision\": \"$PREC\", \"image\": [3, 768, 1024], \"batch\": 128}" > "$OUT/traffic_body.json"
for Q in 128 1024; do
  python3 "$ROOT/tools/pmc_parse.py" "$OUT/knn${Q}_FETCH_SIZE" "$OUT/knn${Q}_WRITE_SIZE" --iters 3 --batch $Q \
    --config "{\"db_rows\": 1000000, \"dim\": 2048, \"k\": 100, \"screen\": \"$SCREEN\", \"q\": $Q}" \
    > "$OUT/traffic_knn$Q.json"
done
python3 "$ROOT/tools/pmc_mfma.py" "$OUT/body_mfma" --iters 3 > "$OUT/mfma_body.json"
echo "pmc done"
