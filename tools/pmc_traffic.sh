#!/bin/bash
# HBM traffic of the extractor body from PMC counters: one rocprofv3 pass per
# counter (FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2: never in one pass).
#   bash tools/pmc_traffic.sh <outdir> [batch]
set -e
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$ROOT/$1"; B=${2:-32}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- \
  python3 "$ROOT/tools/pmc_body.py" --batch $B > "$OUT/fetch.log" 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- \
  python3 "$ROOT/tools/pmc_body.py" --batch $B > "$OUT/write.log" 2>&1
python3 "$ROOT/tools/pmc_parse.py" "$OUT/fetch" "$OUT/write" --iters 3 --batch $B > "$OUT/traffic.json" || true
ls -R "$OUT" | head -20
