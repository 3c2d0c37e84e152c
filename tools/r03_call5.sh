#!/bin/bash
# round-3 call: RBF stream variants (split emit: rows launch + RBF launch), Betti A/B and tests of
# the current build, then the hang repro with the EXEC check (last)
set -eo pipefail
OUT=gpurun_out/r03_call5
mkdir -p "$OUT"
export TMPDIR=/tmp
EXP_TAG=r03_stream VARIANTS="libdgn_split libdgn_split_plain libdgn_split_direct libdgn_split_direct_plain libdgn libdgn_direct" bash tools/r03_graph_exp.sh
bash tools/ab_betti.sh r03_ab_pv2 defect-gnn-cpp_amd/lib/libdgn_base.so defect-gnn-cpp_amd/lib/libdgn.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_betti.py tests/test_gpu_betti_envelope.py tests/test_gpu_betti_wide.py -x -v --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
tail -3 "$OUT/tests.log"
bash tools/hang_repro.sh gpurun_out/hang_exec repro_exec
