#!/bin/bash
# Narrow Betti kernel memory-hierarchy counters (L2 hit/miss, HBM requests, L1 accesses) over
# tools/betti_run.py (2,048 FCC-256 structures at 5 A): one rocprofv3 --pmc pass per group.
#   gpurun --timeout 600 -- bash profiles/collect_narrow_mem.sh <outdir>
set -eo pipefail
OUT=${1:-gpurun_out/r03_narrow_mem}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="fcc 4 2048 5.0 1"
i=0
for grp in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 tools/betti_run.py $ARGS > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; }
  echo "pass $i done"
done
python3 tools/pmc_summary.py "$OUT" betti_kernel > "$OUT/summary.txt"
cat "$OUT/summary.txt"
