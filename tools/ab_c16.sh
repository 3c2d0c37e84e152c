#!/bin/bash
# A/B: wide kernel on u16 rank codes (default) vs f32 distances (DGN_WIDE_C16=0) at 10 A
set -eo pipefail
mkdir -p gpurun_out/c16
timeout -k 10 300 python -u -m pytest tests/test_gpu_betti_wide.py tests/test_gpu_betti_envelope.py -x -q --timeout 200 --timeout-method thread > gpurun_out/c16/pytest.log 2>&1
tail -2 gpurun_out/c16/pytest.log
for v in 1 0 1 0; do
  echo "== C16=$v"
  DGN_WIDE_C16=$v timeout -k 10 100 python -u tools/betti_rc10.py 32 3 2>&1 | grep "rep [12]"
done
