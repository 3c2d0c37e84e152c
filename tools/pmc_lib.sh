#!/bin/bash
# Two SQ counter passes over the graph-only bench with a given libdgn build:
#   bash tools/pmc_lib.sh <outdir> <lib.so>
set -eo pipefail
OUT=$1; LIB=$2
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM" \
           "SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_INSTS_VALU_CVT"; do
  i=$((i+1))
  DGN_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-side --no-betti --no-alt-rbf > "$OUT/p$i.log" 2>&1
done
python3 tools/pmc_summary.py "$OUT" count emit > "$OUT/summary.txt"
