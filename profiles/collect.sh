#!/bin/bash
# Collect the per-round rocprofv3 evidence on the GPU box (run from the repo root):
#   bash profiles/collect.sh r01
# 1. kernel trace + stats of the default bench (N=1, 8192 FCC-256 structures, graph + Betti)
# 2. two separate PMC passes (FETCH_SIZE, WRITE_SIZE; they do not fit one TCC pass on gfx950) on
#    the graph-only bench (the headline's f64 RBF, no other-dtype side run): HBM bytes of prep,
#    graph_count, block_scan and graph_emit, summed into the bytes per neighbour-path launch set the
#    roofline quotes
# 3. parse_profiles.py folds them into profiles/<round>_*.{csv,json} and profiles/traffic_latest.json
set -eo pipefail
R=${1:-r01}
OUT=gpurun_out/prof_$R
mkdir -p "$OUT"
cd "$(dirname "$0")/.." 
export TMPDIR=/tmp
BENCH="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 $BENCH > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 $BENCH --no-betti --no-alt-rbf > "$OUT/fetch_bench.json" 2> "$OUT/fetch_bench.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 $BENCH --no-betti --no-alt-rbf > "$OUT/write_bench.json" 2> "$OUT/write_bench.err"
[ "${NO_PARSE:-0}" = 1 ] || python3 profiles/parse_profiles.py --round "$R" --dir "$OUT"
