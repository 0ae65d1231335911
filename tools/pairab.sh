set -e
mkdir -p gpurun_out/pairab
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_pipeline.py -x -v --timeout 200 --timeout-method thread -k "pair or boundary" > gpurun_out/pairab/pytest.log 2>&1 || { tail -40 gpurun_out/pairab/pytest.log; exit 1; }
tail -3 gpurun_out/pairab/pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --latency 0 --pcie-steps 0 > gpurun_out/pairab/bench_fused.json 2> gpurun_out/pairab/bench_fused.err
RR_PAIR_MID=0 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --latency 0 --pcie-steps 0 > gpurun_out/pairab/bench_plain.json 2> gpurun_out/pairab/bench_plain.err
python3 -c "
import json
for f in ('fused','plain'):
    d=json.loads(open('gpurun_out/pairab/bench_%s.json'%f).read().strip().splitlines()[-1]); print(f, d['value'], d['ms_per_step'])"
