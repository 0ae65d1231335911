#!/bin/bash
# One GPU-box session: gpu tests, bench line, rocprofv3 kernel stats.
#   bash tools/gpu_round.sh <tag> <steps...>   steps: tests bench prof layers
# Each GPU step runs under its own time limit; the script stops at the first failure.
set -e
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
for STEP in "$@"; do
  case $STEP in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1
      tail -3 "$OUT/pytest_gpu.log" ;;
    bench)
      timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
      cat "$OUT/bench.json" ;;
    benchq)
      timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/benchq.json" 2> "$OUT/benchq.err"
      cat "$OUT/benchq.json" ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run \
        --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-extras --latency 0 --pcie-steps 0 \
        > "$OUT/prof_bench.json" 2> "$OUT/prof.err")
      cat "$OUT/prof_bench.json" ;;
    pmc)
      bash "$ROOT/tools/pmc_round.sh" "gpurun_out/$TAG/pmc" ;;
    layers)
      timeout -k 10 300 python -u tools/layer_bench.py --batch 32 > "$OUT/layers_b32.txt" 2>&1
      cat "$OUT/layers_b32.txt" ;;
    layers4)
      timeout -k 10 300 python -u tools/layer_bench.py --batch 4 > "$OUT/layers_b4.txt" 2>&1
      cat "$OUT/layers_b4.txt" ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
done
