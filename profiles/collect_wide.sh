#!/bin/bash
# rocprofv3 evidence for the wide Betti kernel at the reference's default 10 A cutoff
# (32 FCC-256 structures = 8,192 complexes of ~340 points):
#   bash profiles/collect_wide.sh r02
# 1. kernel trace + stats; 2. FETCH_SIZE and WRITE_SIZE passes (separate, gfx950 TCC limits);
# 3. two SQ passes (instruction mix, wave cycles, waits)
set -eo pipefail
R=${1:-r02}
OUT=gpurun_out/wide_$R
mkdir -p "$OUT"
export TMPDIR=/tmp
RUN="tools/betti_rc10.py 32 1"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $RUN > "$OUT/trace.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $RUN > "$OUT/fetch.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 $RUN > "$OUT/write.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d "$OUT/sq1" -o run -- python3 $RUN > "$OUT/sq1.log" 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH --output-format csv -d "$OUT/sq2" -o run -- python3 $RUN > "$OUT/sq2.log" 2>&1
echo done
