#!/bin/bash
# A/B of two builds of libdgn on one GPU box (same device, back to back):
#   gpurun -- bash tools/ab_betti.sh <tag> <libA.so> <libB.so> [diagA.so diagB.so]
# Each arm: graph+Betti bench (3 steps, no CPU baseline) and, if given, the phase diagnostics.
set -eo pipefail
TAG=${1:-ab}; A=$2; B=$3; DA=${4:-}; DB=${5:-}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for arm in A B A B; do
  lib=$A; [ $arm = B ] && lib=$B
  DGN_LIB=$lib timeout -k 10 180 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side --no-alt-rbf > "$OUT/bench_$arm.json" 2>> "$OUT/err.log"
  python -c "import json,sys; r=json.load(open('$OUT/bench_$arm.json')); print('$arm', r['value'], r['kernel_ms_per_step']['betti_vr'])"
done
if [ -n "$DA" ]; then
  DGN_LIB=$DA timeout -k 10 120 python -u tools/diag_phases.py fcc 4 1024 5.0 > "$OUT/diag_A.json" 2>> "$OUT/err.log"
  DGN_LIB=$DB timeout -k 10 120 python -u tools/diag_phases.py fcc 4 1024 5.0 > "$OUT/diag_B.json" 2>> "$OUT/err.log"
  echo diag ok
fi
