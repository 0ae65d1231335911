# Q = 128 search vs 1M x 2048: score-GEMM tile configs (RR_TUNE_GEMM_CONFIG [, stages]) A/B
set -e
for T in 0=0 0=7 0=1 0=1,1=3 0=3 0=7 0=1; do timeout -k 10 120 python -u tools/knn_probe.py --q 128 --tune $T 2>&1 | grep search; done
