set -e
mkdir -p gpurun_out/qb
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread > gpurun_out/qb/pytest.log 2>&1 || { tail -40 gpurun_out/qb/pytest.log; exit 1; }
tail -2 gpurun_out/qb/pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --latency 0 --pcie-steps 0 > gpurun_out/qb/bench.json 2> gpurun_out/qb/bench.err
python3 -c "
import json
d=json.loads(open('gpurun_out/qb/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('knn', {}).get('ms_per_batch'))"
