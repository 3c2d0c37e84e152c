#!/bin/bash
# round 3: waves per SIMD of the one-image count kernel (8 = default, 7, 6), count pass alone
set -eo pipefail
OUT=gpurun_out/r03_cwaves
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2 3; do
  for lib in libdgn libdgn_c7 libdgn_c6; do
    DGN_LIB=defect-gnn-cpp_amd/lib/$lib.so timeout -k 10 120 python -u tools/count_probe.py 30 >> "$OUT/probe.txt" 2>> "$OUT/err.log"
  done
done
cat "$OUT/probe.txt"
