#!/bin/bash
# Graph-only bench (count + scan + emit) for several libdgn builds back to back, two rounds:
#   gpurun -- bash tools/ab_graph.sh <tag> lib1.so lib2.so ...   [extra bench args via BENCH_ARGS]
set -eo pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for r in 1 2; do
  for lib in "$@"; do
    name=$(basename "$lib" .so)
    DGN_LIB=$lib timeout -k 10 180 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-betti --no-alt-rbf $BENCH_ARGS \
        > "$OUT/${name}_$r.json" 2>> "$OUT/err.log"
    python -c "import json; r=json.load(open('$OUT/${name}_$r.json')); k=r['kernel_ms_per_step']; print('$name', {n: k[n] for n in k if not n.startswith('betti')})"
  done
done
