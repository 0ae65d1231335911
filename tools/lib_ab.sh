# same-box bench A/B of two builds of librr.so: bash tools/lib_ab.sh <libA> <libB> [reps]
set -e
mkdir -p gpurun_out/libab
R=${3:-2}
for i in $(seq 1 $R); do
  for L in "$1" "$2"; do
    RR_LIB=$(realpath "$L") timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --latency 0 --pcie-steps 0 --local-kpts 0 > gpurun_out/libab/b.json 2> gpurun_out/libab/b.err
    python3 -c "
import json
d=json.loads(open('gpurun_out/libab/b.json').read().strip().splitlines()[-1]); print('lib=%-40s' % '$L', '%.1f img/s' % d['value'], '%.3f ms' % d['ms_per_step'], 'knn %.3f ms' % (d.get('knn') or {}).get('ms_per_batch', 0), 'extract %.1f img/s' % d['extract_images_per_sec'], 'body %.3f ms' % d['roofline_layers']['measured_ms'])"
  done
done
