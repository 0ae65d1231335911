#!/bin/bash
# A/B of two librr builds on one box: bash tools/lib_layers_ab.sh <tag> <libB> [rounds]
# layer_bench (128 images, fp16) and the fused stem (tools/stem_ab.py) alternating the default librr.so and <libB>.
set -e
TAG=$1; LIBB=$2; R=${3:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
for r in $(seq 1 $R); do
  timeout -k 10 300 python -u tools/layer_bench.py --batch 128 --precision fp16 > "$OUT/A_$r.txt" 2>&1
  RR_LIB="$ROOT/$LIBB" timeout -k 10 300 python -u tools/layer_bench.py --batch 128 --precision fp16 > "$OUT/B_$r.txt" 2>&1
  timeout -k 10 200 python -u tools/stem_ab.py --modes 2 --rounds 1 > "$OUT/stemA_$r.json" 2>&1
  RR_LIB="$ROOT/$LIBB" timeout -k 10 200 python -u tools/stem_ab.py --modes 2 --rounds 1 > "$OUT/stemB_$r.json" 2>&1
done
echo ab done
