#!/bin/bash
# one-wave wide kernel: wavefront-scope fences instead of workgroup barriers in the reduction's
# hot loop (-DDGN_WIDE_WAVE_FENCE): wide + envelope parity with the variant, then 10 A A/B
set -eo pipefail
OUT=gpurun_out/r03_wfence
mkdir -p "$OUT"
export TMPDIR=/tmp
V=defect-gnn-cpp_amd/lib/libdgn_wfence.so
DGN_LIB=$V timeout -k 10 500 python -u -m pytest tests/test_gpu_betti_wide.py tests/test_gpu_betti_envelope.py -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
bash tools/ab_rc10.sh r03_wfence_ab defect-gnn-cpp_amd/lib/libdgn.so $V
