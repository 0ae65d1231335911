set -e
for L in mod2.b2.c2 mod3.b2.c2 mod3.b1.c2 stem; do
  timeout -k 10 400 bash tools/pmc_layer.sh $L gpurun_out/r02c/$L
done
echo done
