set -e
mkdir -p gpurun_out/lb
for T in 5=1 5=2 5=3 5=1; do timeout -k 10 300 python -u tools/layer_bench.py --batch 128 --reps 10 --tune $T > gpurun_out/lb/l_$T.txt 2>&1; grep -E "mod5.b1.c3|mod4.b1.c3|TOTAL" gpurun_out/lb/l_$T.txt; done
