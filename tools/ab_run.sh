#!/bin/bash
# One-call A/B of a variant librr: bash tools/ab_run.sh <tag> <libB> <pytest -k expr for the variant> [rounds]
# GEMM / kernel tests with libB, then tools/lib_layers_ab.sh (layers + stem) alternating A and B.
set -e
TAG=$1; LIBB=$2; KEXPR=$3; R=${4:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/$TAG"; mkdir -p "$OUT"; cd "$ROOT"
RR_LIB=$ROOT/$LIBB timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "$KEXPR" -x -q --timeout 300 \
  --timeout-method thread > "$OUT/ktest_B.log" 2>&1 || { tail -30 "$OUT/ktest_B.log"; exit 1; }
tail -2 "$OUT/ktest_B.log"
bash tools/lib_layers_ab.sh "$TAG" "$LIBB" "$R"
python3 tools/ab_table.py "$OUT" "$R"
