#!/bin/bash
# narrow-kernel A/B: apparent owners from the LDS matrix (DGN_APP_LDS) vs the scratch table;
# Betti parity with the variant first
set -eo pipefail
OUT=gpurun_out/r03_app
mkdir -p "$OUT"
export TMPDIR=/tmp
DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_applds.so timeout -k 10 400 python -u -m pytest tests/test_gpu_betti.py tests/test_gpu_betti_envelope.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
bash tools/ab_betti.sh r03_app_ab defect-gnn-cpp_amd/lib/libdgn.so defect-gnn-cpp_amd/lib/libdgn_applds.so
