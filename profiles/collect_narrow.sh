#!/bin/bash
# Narrow Betti kernel SQ counters (3 rocprofv3 --pmc passes over tools/betti_run.py: 2,048 FCC-256
# structures at 5 A) + the diagnostics build's phase split (tools/diag_phases.py).
#   gpurun --timeout 600 -- bash profiles/collect_narrow.sh <outdir>
set -eo pipefail
OUT=${1:-gpurun_out/r03_base}
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="fcc 4 2048 5.0 1"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM" \
           "SQ_LDS_IDX_ACTIVE SQ_INST_CYCLES_VMEM SQ_INSTS_VALU_CVT SQ_WAIT_INST_ANY SQ_INSTS_VALU_TRANS_F32"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 tools/betti_run.py $ARGS > "$OUT/p$i.log" 2>&1
  echo "pass $i ok"
done
python3 tools/pmc_summary.py "$OUT" betti_kernel > "$OUT/summary.txt"
cat "$OUT/summary.txt"
DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_diag.so timeout -k 10 120 python -u tools/diag_phases.py fcc 4 1024 5.0 > "$OUT/diag.json" 2>&1
cat "$OUT/diag.json"
