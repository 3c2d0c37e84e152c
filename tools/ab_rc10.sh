#!/bin/bash
# A/B of libdgn builds at the reference's default 10 A cutoff (wide kernel): 32 FCC-256 structures
#   gpurun -- bash tools/ab_rc10.sh <tag> lib1.so lib2.so ...
set -eo pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
  for lib in "$@"; do
    name=$(basename "$lib" .so)
    DGN_LIB=$lib timeout -k 10 200 python -u tools/betti_rc10.py 32 2 > "$OUT/${name}_$r.log" 2>&1
    echo "$name $(grep 'rep 1' "$OUT/${name}_$r.log")"
  done
done
