# k_gemm8h (half-width 8-phase score GEMM, <= 128 queries): kNN parity tests + Q = 128 search A/B
set -e
mkdir -p gpurun_out/g8h
timeout -k 10 400 python -u -m pytest tests/test_gpu_knn.py tests/test_gpu_distributed.py tests/test_gpu_graph.py -x -q --timeout 200 --timeout-method thread > gpurun_out/g8h/pytest.log 2>&1 || { tail -40 gpurun_out/g8h/pytest.log; exit 1; }
tail -1 gpurun_out/g8h/pytest.log
for T in 8=1 8=9 8=1 8=9; do timeout -k 10 120 python -u tools/knn_probe.py --q 128 --tune $T 2>&1 | grep search; done
timeout -k 10 120 python -u tools/knn_probe.py --q 64 --tune 8=1 2>&1 | grep search
timeout -k 10 120 python -u tools/knn_probe.py --q 64 --tune 8=9 2>&1 | grep search
