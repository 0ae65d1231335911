set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_knn.py tests/test_gpu_distributed.py -x -q --timeout 200 --timeout-method thread > gpurun_out/knn_tests.log 2>&1 || { tail -30 gpurun_out/knn_tests.log; exit 1; }
tail -1 gpurun_out/knn_tests.log
for T in 0=0 0=0; do RR_LIB=$(realpath librr_base.so) timeout -k 10 120 python -u tools/knn_probe.py --q 128 2>&1 | grep search; timeout -k 10 120 python -u tools/knn_probe.py --q 128 2>&1 | grep search; done
bash tools/lib_ab.sh librr_base.so image-retrieval-for-image-based-localization_amd/librr.so 2
