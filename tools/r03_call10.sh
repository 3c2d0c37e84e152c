#!/bin/bash
# round-3 call: kernel trace of the tiered narrow dispatch (NP 44 main + NP 48 mid)
set -eo pipefail
OUT=gpurun_out/r03_call10
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-side --no-alt-rbf > "$OUT/bench.json" 2> "$OUT/err.log"
find "$OUT/tr" -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-8 | head -20
