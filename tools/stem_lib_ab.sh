#!/bin/bash
# Stem A/B of two librr builds: bash tools/stem_lib_ab.sh <tag> <libB> [rounds] [pytest -k expr]
# the stem tests with libB, then tools/stem_ab.py (mode 2, float + uint8 pixels) alternating A / B
set -e
TAG=$1; LIBB=$2; R=${3:-3}; KEXPR=${4:-stem}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
RR_LIB=$ROOT/$LIBB timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_round4.py tests/test_gpu_extract.py \
  -k "$KEXPR" -x -q --timeout 300 --timeout-method thread > "$OUT/test_B.log" 2>&1 || { tail -30 "$OUT/test_B.log"; exit 1; }
tail -1 "$OUT/test_B.log"
for r in $(seq 1 $R); do
  timeout -k 10 200 python -u tools/stem_ab.py --modes 2 --rounds 1 > "$OUT/stemA_$r.json" 2>&1
  RR_LIB="$ROOT/$LIBB" timeout -k 10 200 python -u tools/stem_ab.py --modes 2 --rounds 1 > "$OUT/stemB_$r.json" 2>&1
  echo "round $r A: $(tail -1 $OUT/stemA_$r.json | cut -c1-200)"
  echo "round $r B: $(tail -1 $OUT/stemB_$r.json | cut -c1-200)"
done
