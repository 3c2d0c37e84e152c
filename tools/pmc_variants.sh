#!/bin/bash
# One SQ counter pass over the Betti workload (tools/betti_run.py) per libdgn variant:
#   bash tools/pmc_variants.sh <outdir> "<betti_run args>" <tag>...   (tag "base" = libdgn.so, else libdgn_<tag>.so)
set -eo pipefail
OUT=$1; ARGS=$2; shift 2
mkdir -p "$OUT"
export TMPDIR=/tmp
CTRS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
for tag in "$@"; do
  lib=defect-gnn-cpp_amd/lib/libdgn.so; [ "$tag" != base ] && lib=defect-gnn-cpp_amd/lib/libdgn_$tag.so
  DGN_LIB=$lib timeout -s KILL 100 rocprofv3 --pmc $CTRS --kernel-trace --stats --output-format csv -d "$OUT/$tag" -o run -- \
      python3 tools/betti_run.py $ARGS > "$OUT/$tag.log" 2>&1
  echo "== $tag"; python3 tools/pmc_summary.py "$OUT/$tag" betti_kernel | tee "$OUT/$tag.txt"
  grep -h "betti_kernel" $(find "$OUT/$tag" -name '*kernel_stats.csv') | cut -d, -f1-4 || true
done
