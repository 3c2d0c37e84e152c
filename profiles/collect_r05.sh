#!/bin/bash
# Round-5 rocprofv3 evidence (run from the repo root on the GPU box):
#   bash profiles/collect_r05.sh <outdir>
# 1. kernel trace + stats of the default bench step (N=1, 8,192 FCC-256, graph + Betti)
# 2. FETCH_SIZE / WRITE_SIZE passes (separate; gfx950 TCC limits) of the graph-only bench
# 3. SQ counters of the distance kernel (betti_dist_search_kernel: f64 VALU pairs) inside the bench step
# 4. narrow Betti kernel SQ instruction mix / waits / LDS bank conflicts and TCP/TCC requests
#    (tools/betti_run.py: 2,048 FCC-256 structures at 5 A)
# 5. the 10 A wide kernel: FETCH/WRITE and SQ issue/wait (tools/betti_rc10.py, 16 FCC-256)
# 6. kernel trace of the small-batch graph side lines (BASELINE configs 2 and 5, tools/side_graph.py)
set -eo pipefail
OUT=${1:-gpurun_out/prof_r05}
mkdir -p "$OUT"
export TMPDIR=/tmp
BENCH="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 $BENCH > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err"; echo "1 trace ok"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- \
    python3 $BENCH --no-betti --no-alt-rbf > "$OUT/fetch_bench.json" 2> "$OUT/fetch_bench.err"
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- \
    python3 $BENCH --no-betti --no-alt-rbf > "$OUT/write_bench.json" 2> "$OUT/write_bench.err"; echo "2 traffic ok"
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS \
    --kernel-include-regex betti_dist --output-format csv -d "$OUT/dist" -o run -- \
    python3 $BENCH > "$OUT/dist_bench.json" 2> "$OUT/dist_bench.err"; echo "3 dist ok"
RUN="tools/betti_run.py fcc 4 2048 5.0 1"
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
    --kernel-include-regex betti_kernel --output-format csv -d "$OUT/narrow_sq1" -o run -- python3 $RUN > "$OUT/narrow_sq1.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS \
    --kernel-include-regex betti_kernel --output-format csv -d "$OUT/narrow_sq2" -o run -- python3 $RUN > "$OUT/narrow_sq2.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc TCP_TCC_WRITE_REQ_sum TCP_TCC_READ_REQ_sum TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_sum \
    --kernel-include-regex betti_kernel --output-format csv -d "$OUT/narrow_mem" -o run -- python3 $RUN > "$OUT/narrow_mem.log" 2>&1; echo "4 narrow ok"
W="tools/betti_rc10.py 16 1"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/wide_trace" -o run -- python3 $W > "$OUT/wide_trace.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex betti_wide --output-format csv -d "$OUT/wide_fetch" -o run -- python3 $W > "$OUT/wide_fetch.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex betti_wide --output-format csv -d "$OUT/wide_write" -o run -- python3 $W > "$OUT/wide_write.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
    --kernel-include-regex betti_wide --output-format csv -d "$OUT/wide_sq1" -o run -- python3 $W > "$OUT/wide_sq1.log" 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH \
    --kernel-include-regex betti_wide --output-format csv -d "$OUT/wide_sq2" -o run -- python3 $W > "$OUT/wide_sq2.log" 2>&1; echo "5 wide ok"
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/side" -o run -- python3 tools/side_graph.py 20 > "$OUT/side.log" 2>&1; echo "6 side ok"
