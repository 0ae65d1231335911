set -e
mkdir -p gpurun_out/stemab
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "stem" > gpurun_out/stemab/pytest2.log 2>&1 || { tail -40 gpurun_out/stemab/pytest2.log; exit 1; }
tail -2 gpurun_out/stemab/pytest2.log
for T in 11=0 11=1; do timeout -k 10 120 python -u tools/stem_probe.py --tune $T 2>&1 | grep stem; done
