# bench A/B in one box session: bash tools/bench_ab.sh "<tuneA>" "<tuneB>" [reps]
set -e
mkdir -p gpurun_out/ab
R=${3:-2}
for i in $(seq 1 $R); do
  for T in "$1" "$2"; do
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --latency 0 --pcie-steps 0 --local-kpts 0 --tune "$T" > gpurun_out/ab/b.json 2> gpurun_out/ab/b.err
    python3 -c "
import json
d=json.loads(open('gpurun_out/ab/b.json').read().strip().splitlines()[-1]); print('tune=%-12s' % '$T', '%.1f img/s' % d['value'], '%.3f ms' % d['ms_per_step'], 'knn %.3f ms' % d.get('knn', {}).get('ms_per_batch', 0), 'extract %.1f img/s' % d['extract_images_per_sec'], 'body %.3f ms' % d['roofline_layers']['measured_ms'])"
  done
done
