#!/bin/bash
# Bench several libdgn builds back to back on one GPU box, two rounds, interleaved:
#   gpurun -- bash tools/ab_multi.sh <tag> lib1.so lib2.so ...
set -eo pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
  for lib in "$@"; do
    name=$(basename "$lib" .so)
    DGN_LIB=$lib timeout -k 10 180 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > "$OUT/${name}_$r.json" 2>> "$OUT/err.log"
    python -c "import json; r=json.load(open('$OUT/${name}_$r.json')); print('$name', r['value'], r['kernel_ms_per_step']['betti_vr'])"
  done
done
