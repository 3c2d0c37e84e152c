#!/bin/bash
# round-3 call: full GPU suite on the wave-uniform-dequeue build, Betti A/B vs round 2, emit store
# variants (fused), wide-kernel diagnostics at 10 A, then the hang repro (last)
set -eo pipefail
OUT=gpurun_out/r03_call6
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
tail -3 "$OUT/pytest_gpu.log"
bash tools/ab_betti.sh r03_ab_deq defect-gnn-cpp_amd/lib/libdgn_base.so defect-gnn-cpp_amd/lib/libdgn.so
EXP_TAG=r03_stream2 VARIANTS="libdgn libdgn_plain libdgn_direct_plain" bash tools/r03_graph_exp.sh
DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_diag.so timeout -k 10 200 python -u tools/diag_wide.py 4 > "$OUT/diag_wide.json" 2>&1
cat "$OUT/diag_wide.json"
bash tools/hang_repro.sh gpurun_out/hang_fixed repro
