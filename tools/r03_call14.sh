#!/bin/bash
# round-3 call: triangle min-cofacet table replaced by a clearing bitset + on-the-fly minimal
# cofacets -- Betti GPU tests, then A/B vs HEAD
set -eo pipefail
OUT=gpurun_out/r03_call14
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_betti.py tests/test_gpu_betti_envelope.py tests/test_gpu_betti_wide.py -m gpu -x -v --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
bash tools/ab_betti.sh r03_ab_clr defect-gnn-cpp_amd/lib/libdgn_base.so defect-gnn-cpp_amd/lib/libdgn.so
