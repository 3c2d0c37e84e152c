#!/bin/bash
# round-3 call: bench multi-rank test, wide natural-retry probe, then the hang-repro variants
# (last: a hang ends the script)
set -eo pipefail
OUT=gpurun_out/r03_call3
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_dist.py -x -v --timeout 280 --timeout-method thread > "$OUT/dist.log" 2>&1
tail -3 "$OUT/dist.log"
bash tools/ab_betti.sh r03_ab_pv defect-gnn-cpp_amd/lib/libdgn_base.so defect-gnn-cpp_amd/lib/libdgn.so
timeout -k 10 200 python -u tools/retry_probe.py wide > "$OUT/probe_wide.log" 2>&1
cat "$OUT/probe_wide.log"
bash tools/hang_repro.sh gpurun_out/hang repro_uni repro
