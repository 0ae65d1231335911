set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "conv3x3" > gpurun_out/c3ab/pytest.log 2>&1 || { tail -30 gpurun_out/c3ab/pytest.log; exit 1; }
tail -2 gpurun_out/c3ab/pytest.log
for P in 0 1; do
  timeout -k 10 300 python -u tools/layer_bench.py --batch 128 --tune 10=$P > gpurun_out/c3ab/layers_p$P.txt 2>&1
done
grep -i "c2\|3x3" gpurun_out/c3ab/layers_p0.txt | head -20
grep -i "c2\|3x3" gpurun_out/c3ab/layers_p1.txt | head -20
