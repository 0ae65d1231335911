# stem v1/v2/v3 parity tests + isolated timing (32 x 3x768x1024), float and uint8 pixels
set -e
mkdir -p gpurun_out/stemab3
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "stem" > gpurun_out/stemab3/pytest.log 2>&1 || { tail -40 gpurun_out/stemab3/pytest.log; exit 1; }
tail -2 gpurun_out/stemab3/pytest.log
for T in 11=1 11=2 11=3 11=4 11=2; do for U in "" --u8; do timeout -k 10 120 python -u tools/stem_probe.py --tune $T $U 2>&1 | grep stem; done; done
