# same-box per-layer A/B of librr.so builds: bash tools/lib_layers_ab.sh <out_dir> <lib>...  (R50, 128 images)
set -e
OUT=$1; shift
mkdir -p "$OUT"
i=0
for L in "$@"; do
  i=$((i+1))
  RR_LIB=$(realpath "$L") timeout -k 10 300 python -u tools/layer_bench.py --batch 128 > "$OUT/layers_$i.txt" 2>&1 || { tail -20 "$OUT/layers_$i.txt"; exit 1; }
  echo "== $L"; grep -E "c2 |TOTAL" "$OUT/layers_$i.txt"
done
