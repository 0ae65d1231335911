mkdir -p gpurun_out/r02j
for c in 0 1 2 3 4 5 7 8; do
  timeout -k 10 200 python -u tools/layer_bench.py --batch 128 --reps 8 --tune "0=$c" > gpurun_out/r02j/cfg$c.txt 2>&1 || exit 1
  echo "cfg $c: $(grep -E 'mod3.b1.c2|mod3.b1.proj|mod4.b1.c1 ' gpurun_out/r02j/cfg$c.txt | awk '{print $1, $4, $5}' | tr '\n' ' ')"
done
