# PMC passes over the staggered direct 3x3 kernels (tools/pmc_layer.sh per layer)
set -e
bash tools/pmc_layer.sh mod3.b2.c2 gpurun_out/pmc_c3s/m3new ""
bash tools/pmc_layer.sh mod2.b1.c2 gpurun_out/pmc_c3s/m2new ""
bash tools/pmc_layer.sh mod2.b1.c2 gpurun_out/pmc_c3s/m2v1 "13=2"
bash tools/pmc_layer.sh mod4.b2.c2 gpurun_out/pmc_c3s/m4g8 ""
for d in m3new m2new m2v1; do echo "== $d"; python3 tools/pmc_summary.py gpurun_out/pmc_c3s/$d k_c3s 10; done
echo "== m4 gemm8"; python3 tools/pmc_summary.py gpurun_out/pmc_c3s/m4g8 k_gemm8 10
