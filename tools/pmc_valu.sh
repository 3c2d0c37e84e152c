#!/bin/bash
# One SQ instruction-count pass (graph-only bench) per libdgn build:
#   bash tools/pmc_valu.sh <outdir> lib1.so lib2.so ...
set -eo pipefail
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for LIB in "$@"; do
  n=$(basename "$LIB" .so)
  DGN_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES --output-format csv -d "$OUT/$n" -o run -- \
      python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-betti --no-alt-rbf > "$OUT/$n.log" 2>&1
  echo "== $n" >> "$OUT/summary.txt"
  python3 tools/pmc_summary.py "$OUT/$n" count emit >> "$OUT/summary.txt"
done
