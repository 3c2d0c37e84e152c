#!/bin/bash
# One GPU-box session: parity tests, the default bench, the Betti phase diagnostics and the
# 10 A (wide kernel) timing. Build here first (make all diag), then:
#   gpurun --timeout 900 -- bash tools/gpu_check.sh <tag> [tests|notests]
# Every GPU step has its own time limit; the script stops at the first failing step.
set -eo pipefail
TAG=${1:-check}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ "${2:-tests}" = "tests" ]; then
  timeout -k 10 480 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  tail -3 "$OUT/pytest_gpu.log"
fi
timeout -k 10 240 python -u bench.py --steps 5 --warmup 1 > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
if [ -f defect-gnn-cpp_amd/lib/libdgn_diag.so ]; then
  DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_diag.so timeout -k 10 120 python -u tools/diag_phases.py fcc 4 1024 5.0 > "$OUT/diag.json" 2>&1
  echo "diag ok"
fi
timeout -k 10 180 python -u tools/betti_rc10.py 16 2 > "$OUT/rc10.log" 2>&1
cat "$OUT/rc10.log"
