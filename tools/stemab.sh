set -e
mkdir -p gpurun_out/stemab
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_pipeline.py -x -v --timeout 200 --timeout-method thread -k "stem or uint8 or extract" > gpurun_out/stemab/pytest.log 2>&1 || { tail -40 gpurun_out/stemab/pytest.log; exit 1; }
tail -3 gpurun_out/stemab/pytest.log
timeout -k 10 120 python -u tools/stem_probe.py > gpurun_out/stemab/probe.txt 2>&1
cat gpurun_out/stemab/probe.txt
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras --latency 0 --pcie-steps 0 > gpurun_out/stemab/bench.json 2> gpurun_out/stemab/bench.err
python3 -c "
import json
d=json.loads(open('gpurun_out/stemab/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('roofline'))"
for T in "" "0=7" "4=0" "0=7,4=0"; do
  timeout -k 10 120 python -u tools/knn_probe.py --tune "$T" 2>&1 | grep search
done
