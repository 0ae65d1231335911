#!/bin/bash
# GPU step runner: bash tools/gpu_steps.sh <tag> <step...>
#   steps: ktest:<pytest -k expr>  pytest:<files>  layers:<tune>  bench  benchq:<tune>  tests  prof  pmc
#          knnprof:<Q>:<screen>  stem
# Each GPU step has its own time limit; the first failure ends the script.
set -e
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$ROOT"
i=0
for STEP in "$@"; do
  i=$((i+1))
  case $STEP in
    ktest:*)
      EXPR=${STEP#ktest:}
      timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -k "$EXPR" -x -q --timeout 120 --timeout-method thread \
        > "$OUT/ktest_$i.log" 2>&1 || { tail -30 "$OUT/ktest_$i.log"; exit 1; }
      tail -2 "$OUT/ktest_$i.log" ;;
    pytest:*)
      FILES=${STEP#pytest:}
      timeout -k 10 900 python -u -m pytest $FILES -x -q --timeout 300 --timeout-method thread \
        > "$OUT/pytest_$i.log" 2>&1 || { tail -30 "$OUT/pytest_$i.log"; exit 1; }
      tail -2 "$OUT/pytest_$i.log" ;;
    layers:*)
      TUNE=${STEP#layers:}
      timeout -k 10 300 python -u tools/layer_bench.py --batch 128 --precision fp16 --tune "$TUNE" > "$OUT/layers_$i.txt" 2>&1 || { tail -20 "$OUT/layers_$i.txt"; exit 1; }
      echo "== layers tune=$TUNE"; grep -v amdgpu.ids "$OUT/layers_$i.txt" ;;
    bench)
      timeout -k 10 600 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
      tail -c 3000 "$OUT/bench.json" ;;
    benchq:*)
      TUNE=${STEP#benchq:}
      timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --latency 0 --pcie-steps 0 --local-kpts 0 --fp16-steps 0 --tune "$TUNE" > "$OUT/benchq_$i.json" 2> "$OUT/benchq_$i.err" || { tail -20 "$OUT/benchq_$i.err"; exit 1; }
      python3 -c "
import json
d=json.loads(open('$OUT/benchq_$i.json').read().strip().splitlines()[-1]); print('tune=%-12s' % '$TUNE', '%.1f img/s' % d['value'], '%.3f ms' % d['ms_per_step'], 'knn %.3f ms' % (d.get('knn') or {}).get('ms_per_batch', 0), 'extract %.1f img/s' % d['extract_images_per_sec'], 'body %.3f ms' % d['roofline_layers']['measured_ms'])" ;;
    benchargs:*)
      BARGS=${STEP#benchargs:}
      timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --latency 0 --pcie-steps 0 --local-kpts 0 --fp16-steps 0 $BARGS > "$OUT/benchargs_$i.json" 2> "$OUT/benchargs_$i.err" || { tail -20 "$OUT/benchargs_$i.err"; exit 1; }
      python3 -c "
import json
d=json.loads(open('$OUT/benchargs_$i.json').read().strip().splitlines()[-1]); print('args=%-30s' % '$BARGS', '%.1f img/s' % d['value'], '%.3f ms' % d['ms_per_step'], 'knn %.3f ms' % (d.get('knn') or {}).get('ms_per_batch', 0), 'extract %.1f img/s' % d['extract_images_per_sec'], 'body %.3f ms' % d['roofline_layers']['measured_ms'])" ;;
    benchenv:*)
      ENVV=${STEP#benchenv:}
      env $ENVV timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --latency 0 --pcie-steps 0 --local-kpts 0 --fp16-steps 0 > "$OUT/benchenv_$i.json" 2> "$OUT/benchenv_$i.err" || { tail -20 "$OUT/benchenv_$i.err"; exit 1; }
      python3 -c "
import json
d=json.loads(open('$OUT/benchenv_$i.json').read().strip().splitlines()[-1]); print('env=%-24s' % '$ENVV', '%.1f img/s' % d['value'], '%.3f ms' % d['ms_per_step'], 'knn %.3f ms' % (d.get('knn') or {}).get('ms_per_batch', 0), 'extract %.1f img/s' % d['extract_images_per_sec'], 'body %.3f ms' % d['roofline_layers']['measured_ms'])" ;;
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
      tail -3 "$OUT/pytest_gpu.log" ;;
    prof)
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run \
        --output-format csv -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-extras --latency 0 --pcie-steps 0 --fp16-steps 0 \
        > "$OUT/prof_bench.json" 2> "$OUT/prof.err") || { tail -20 "$OUT/prof.err"; exit 1; }
      tail -c 1500 "$OUT/prof_bench.json" ;;
    knnprof:*)
      QS=${STEP#knnprof:}; Q=${QS%%:*}; SCR=${QS#*:}
      (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/knnprof_${Q}_$SCR" -o run \
        --output-format csv -- python3 "$ROOT/tools/knn_probe.py" --q $Q --screen $SCR > "$OUT/knnprof_${Q}_$SCR.txt" 2>&1) \
        || { tail -20 "$OUT/knnprof_${Q}_$SCR.txt"; exit 1; }
      grep search "$OUT/knnprof_${Q}_$SCR.txt" ;;
    knnenv:*)
      QE=${STEP#knnenv:}; Q=${QE%%:*}; ENVV=${QE#*:}
      env $ENVV timeout -k 10 300 python -u tools/knn_probe.py --q $Q --screen int8 --reps 20 > "$OUT/knnenv_$i.txt" 2>&1 \
        || { tail -20 "$OUT/knnenv_$i.txt"; exit 1; }
      echo "env=$ENVV $(grep search "$OUT/knnenv_$i.txt")" ;;
    stem)
      timeout -k 10 200 python -u tools/stem_ab.py > "$OUT/stem_ab.json" 2>&1 || { tail -20 "$OUT/stem_ab.json"; exit 1; }
      tail -c 600 "$OUT/stem_ab.json" ;;
    pmc)
      timeout -k 10 900 bash "$ROOT/tools/pmc_round.sh" "gpurun_out/$TAG/pmc" > "$OUT/pmc.log" 2>&1 || { tail -20 "$OUT/pmc.log"; exit 1; }
      tail -2 "$OUT/pmc.log" ;;
    *) echo "unknown step $STEP"; exit 2 ;;
  esac
done
