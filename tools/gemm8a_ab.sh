# k_gemm8a (128-channel 8-phase conv GEMM): parity tests + per-layer A/B (RR_TUNE_GEMM8 | 16 = off)
set -e
mkdir -p gpurun_out/g8a
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "gemm8a or gemm8 or conv" > gpurun_out/g8a/pytest.log 2>&1 || { tail -40 gpurun_out/g8a/pytest.log; exit 1; }
tail -1 gpurun_out/g8a/pytest.log
for T in 8=1 8=17; do timeout -k 10 300 python -u tools/layer_bench.py --batch 128 --reps 10 --tune $T > gpurun_out/g8a/l_$T.txt 2>&1; echo "== $T"; grep -E "mod3.b1.c2|mod3.b2.c2|TOTAL" gpurun_out/g8a/l_$T.txt; done
