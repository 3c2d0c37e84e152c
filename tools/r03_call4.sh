#!/bin/bash
# round-3 call: Betti parity tests on the current build, A/B vs the round-2 build, then the
# hang-repro variants (last: a hang ends the script)
set -eo pipefail
OUT=gpurun_out/r03_call4
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_betti.py tests/test_gpu_betti_envelope.py tests/test_gpu_fused.py -x -v --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
tail -4 "$OUT/tests.log"
bash tools/ab_betti.sh r03_ab_walk defect-gnn-cpp_amd/lib/libdgn_base.so defect-gnn-cpp_amd/lib/libdgn.so
bash tools/r03_graph_exp.sh
bash tools/hang_repro.sh gpurun_out/hang repro_uni repro
