# same-box A/B of the extraction stream priority: bash tools/prio_ab.sh [reps]
set -e
mkdir -p gpurun_out/ab
for i in $(seq 1 ${1:-2}); do
  for P in 0 1; do
    RR_BENCH_PRIO=$P timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --latency 0 --pcie-steps 0 --local-kpts 0 > gpurun_out/ab/p.json 2> gpurun_out/ab/p.err
    python3 -c "
import json
d=json.loads(open('gpurun_out/ab/p.json').read().strip().splitlines()[-1]); print('prio=$P', '%.1f img/s' % d['value'], '%.3f ms' % d['ms_per_step'], 'extract %.1f img/s' % d['extract_images_per_sec'], 'body %.3f ms' % d['roofline_layers']['measured_ms'])"
  done
done
