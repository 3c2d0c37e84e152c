#!/bin/bash
# Round-6 rocprofv3 evidence (run from the repo root on the GPU box):
#   bash profiles/collect_r06.sh <outdir>
# 1. kernel trace + stats of the default bench step (N=1, 8,192 FCC-256, graph + Betti)
# 2. FETCH_SIZE / WRITE_SIZE passes (separate; gfx950 TCC limits) of the graph-only bench
# 3. the 10 A path (tools/betti_rc10.py 32 1: 8,192 complexes, one slice): kernel trace, and for the
#    walk pass (betti_walk_kernel) and the reduction kernel (betti_wide_kernel_c16<6, true>) SQ
#    issue / wait / instruction mix and FETCH / WRITE
# 4. kernel trace of the small-batch graph side lines (BASELINE configs 2 and 5, tools/side_graph.py)
set -eo pipefail
OUT=${1:-gpurun_out/prof_r06}
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 $BENCH > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err"; echo "1 trace ok"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 $BENCH --no-betti --no-alt-rbf > "$OUT/fetch_bench.json" 2> "$OUT/fetch_bench.err"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 $BENCH --no-betti --no-alt-rbf > "$OUT/write_bench.json" 2> "$OUT/write_bench.err"; echo "2 traffic ok"
W="tools/betti_rc10.py 32 1"
K="betti_walk|betti_wide_kernel_c16"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/rc10_trace" -o run -- python3 $W > "$OUT/rc10_trace.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$K" --output-format csv -d "$OUT/rc10_fetch" -o run -- python3 $W > "$OUT/rc10_fetch.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$K" --output-format csv -d "$OUT/rc10_write" -o run -- python3 $W > "$OUT/rc10_write.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
    --kernel-include-regex "$K" --output-format csv -d "$OUT/rc10_sq1" -o run -- python3 $W > "$OUT/rc10_sq1.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM \
    --kernel-include-regex "$K" --output-format csv -d "$OUT/rc10_sq2" -o run -- python3 $W > "$OUT/rc10_sq2.log" 2>&1; echo "3 rc10 ok"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/side" -o run -- python3 tools/side_graph.py 20 > "$OUT/side.log" 2>&1; echo "4 side ok"
