#!/bin/bash
# round 3: one-image count with scalar candidate masks (two compares per half): graph / fused /
# Betti parity tests, then the count pass alone vs the previous build (libdgn_base.so), twice
set -eo pipefail
OUT=gpurun_out/r03_cmask
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_fused.py tests/test_gpu_betti.py tests/test_gpu_edges.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for r in 1 2; do
  for lib in libdgn_base libdgn; do
    DGN_LIB=defect-gnn-cpp_amd/lib/$lib.so timeout -k 10 120 python -u tools/count_probe.py 20 >> "$OUT/probe.txt" 2>> "$OUT/err.log"
  done
done
cat "$OUT/probe.txt"
