#!/bin/bash
# PMC passes over the Betti kernel alone (tools/betti_run.py), one rocprofv3 run per counter group.
#   bash tools/pmc_betti.sh <outdir> [kind m B rc]
set -eo pipefail
OUT=${1:-gpurun_out/pmc_betti}; shift || true
ARGS=${@:-fcc 4 1024 5.0 1}
mkdir -p "$OUT"
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
           "SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d "$OUT/p$i" -o run -- python3 tools/betti_run.py $ARGS > "$OUT/p$i.log" 2>&1
done
