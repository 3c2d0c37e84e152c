#!/bin/bash
# WG kernel v3 (LDS-only barriers in the pivot search, edge units from the LDS adjacency)
set -eo pipefail
OUT=gpurun_out/r03_wg4
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_gpu_betti_wide.py -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest_wide.log" 2>&1 || { tail -40 "$OUT/pytest_wide.log"; exit 1; }
tail -3 "$OUT/pytest_wide.log"
DGN_WIDE_WG=1 timeout -k 10 240 python -u tools/betti_rc10.py 32 2 > "$OUT/rc10_wg.log" 2>&1
cat "$OUT/rc10_wg.log"
DGN_WIDE_WG=1 timeout -k 10 180 python -u tools/diag_wide.py 16 > "$OUT/diag_wg.json" 2>&1
cat "$OUT/diag_wg.json"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_INSTS_VMEM"; do
  i=$((i+1))
  DGN_WIDE_WG=1 timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 tools/betti_rc10.py 8 1 > "$OUT/p$i.log" 2>&1 || { echo "pass $i failed"; tail -5 "$OUT/p$i.log"; }
done
python3 tools/pmc_summary.py "$OUT" betti_wg > "$OUT/pmc_summary.txt"
cat "$OUT/pmc_summary.txt"
