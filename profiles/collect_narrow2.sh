#!/bin/bash
# Narrow Betti kernel counters, round 3 after the NP = 44 tier: SQ issue/wait split, LDS, the
# instruction cache (SQC) -- one rocprofv3 --pmc pass per group over tools/betti_run.py (2,048
# FCC-256 structures at 5 A, one rep).
#   gpurun --timeout 600 -- bash profiles/collect_narrow2.sh <outdir>
set -eo pipefail
OUT=${1:-gpurun_out/r03_narrow2}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="fcc 4 2048 5.0 1"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_INSTS_VMEM" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH" \
           "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 tools/betti_run.py $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; }
  echo "pass $i done"
done
python3 tools/pmc_summary.py "$OUT" betti_kernel > "$OUT/summary.txt"
cat "$OUT/summary.txt"
