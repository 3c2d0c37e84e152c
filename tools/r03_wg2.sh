#!/bin/bash
# WG kernel phase split (diagnostics build) at 10 A, and waves-per-workgroup A/B (4 / 8 / 16)
set -eo pipefail
OUT=gpurun_out/r03_wg2
mkdir -p "$OUT"
export TMPDIR=/tmp
DGN_WIDE_WG=1 timeout -k 10 180 python -u tools/diag_wide.py 16 > "$OUT/diag_wg.json" 2>&1
cat "$OUT/diag_wg.json"
DGN_WIDE_WG=0 timeout -k 10 180 python -u tools/diag_wide.py 16 > "$OUT/diag_wave.json" 2>&1
cat "$OUT/diag_wave.json"
for v in wg4 wg16; do
  DGN_WIDE_WG=1 DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_$v.so timeout -k 10 240 python -u tools/betti_rc10.py 32 2 > "$OUT/rc10_$v.log" 2>&1
  echo "$v $(grep 'rep 1' "$OUT/rc10_$v.log")"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_fused.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_graph.log" 2>&1 || { tail -30 "$OUT/pytest_graph.log"; exit 1; }
tail -2 "$OUT/pytest_graph.log"
timeout -k 10 120 python -u tools/side_graph.py 20 > "$OUT/side_graph.log" 2>&1
cat "$OUT/side_graph.log"
