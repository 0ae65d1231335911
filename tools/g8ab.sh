# k_gemm8 epilogue: kernel parity tests + per-layer A/B (streaming vs 8-phase GEMM for the residual 1x1s)
set -e
mkdir -p gpurun_out/g8ab
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "gemm8 or conv" > gpurun_out/g8ab/pytest.log 2>&1 || { tail -40 gpurun_out/g8ab/pytest.log; exit 1; }
tail -2 gpurun_out/g8ab/pytest.log
for T in 5=1 5=2 5=3; do timeout -k 10 300 python -u tools/layer_bench.py --batch 128 --reps 10 --tune $T > gpurun_out/g8ab/l_$T.txt 2>&1; echo "== $T"; grep -E "c1 |c3 |proj|c2 |TOTAL" gpurun_out/g8ab/l_$T.txt | grep -E "mod4|mod5|TOTAL"; done
