#!/bin/bash
# round-3 session 2: workgroup-per-complex wide kernel (betti_wg.hip) -- wide parity tests, then the
# 10 A timing with the workgroup kernel, the one-wave kernel and the 32-bit-key variant (A/B)
set -eo pipefail
OUT=gpurun_out/r03_wg1
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_gpu_betti_wide.py -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_wide.log" 2>&1 || { tail -40 "$OUT/pytest_wide.log"; exit 1; }
tail -3 "$OUT/pytest_wide.log"
DGN_WIDE_WG=1 timeout -k 10 240 python -u tools/betti_rc10.py 32 2 > "$OUT/rc10_wg.log" 2>&1
cat "$OUT/rc10_wg.log"
DGN_WIDE_WG=0 timeout -k 10 240 python -u tools/betti_rc10.py 32 2 > "$OUT/rc10_wave.log" 2>&1
cat "$OUT/rc10_wave.log"
timeout -k 10 120 python -u tools/side_graph.py 20 > "$OUT/side_graph.log" 2>&1
cat "$OUT/side_graph.log"
DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_fastkey.so timeout -k 10 300 python -u -m pytest tests/test_gpu_betti_wide.py -m gpu -x -q --timeout 200 --timeout-method thread -k "workgroup or rc10 or fcc" > "$OUT/pytest_fastkey.log" 2>&1 || { tail -30 "$OUT/pytest_fastkey.log"; exit 1; }
tail -2 "$OUT/pytest_fastkey.log"
DGN_WIDE_WG=1 DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_fastkey.so timeout -k 10 240 python -u tools/betti_rc10.py 32 2 > "$OUT/rc10_fastkey.log" 2>&1
cat "$OUT/rc10_fastkey.log"
