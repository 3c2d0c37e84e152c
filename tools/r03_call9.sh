#!/bin/bash
# round-3 call: NP = 44 main tier (20 waves per CU) + NP = 48 mid tier -- GPU suite, A/B vs HEAD
set -eo pipefail
OUT=gpurun_out/r03_call9
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
bash tools/ab_betti.sh r03_ab_t44 defect-gnn-cpp_amd/lib/libdgn_base.so defect-gnn-cpp_amd/lib/libdgn.so
