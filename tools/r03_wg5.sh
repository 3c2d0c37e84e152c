#!/bin/bash
# WG kernel v3 (LDS-only barriers in the pivot search, edge units from the LDS adjacency)
set -eo pipefail
OUT=gpurun_out/r03_wg5
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_gpu_betti_wide.py -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_wide.log" 2>&1 || { tail -40 "$OUT/pytest_wide.log"; exit 1; }
tail -3 "$OUT/pytest_wide.log"
DGN_WIDE_WG=1 timeout -k 10 240 python -u tools/betti_rc10.py 32 2 > "$OUT/rc10_wg.log" 2>&1
cat "$OUT/rc10_wg.log"
DGN_WIDE_WG=1 timeout -k 10 180 python -u tools/diag_wide.py 16 > "$OUT/diag_wg.json" 2>&1
cat "$OUT/diag_wg.json"
