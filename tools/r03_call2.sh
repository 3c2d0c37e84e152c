#!/bin/bash
# round-3 call: natural-retry probe, bench multi-rank test, then the hang-repro variants (last:
# a hang ends the script)
set -eo pipefail
OUT=gpurun_out/r03_call2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/retry_probe.py > "$OUT/probe.log" 2>&1
cat "$OUT/probe.log"
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_dist.py -x -v --timeout 280 --timeout-method thread > "$OUT/dist.log" 2>&1
tail -3 "$OUT/dist.log"
bash tools/hang_repro.sh gpurun_out/hang repro_uni repro
