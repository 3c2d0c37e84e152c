#!/bin/bash
# A/B of wide-kernel variants at the default 10 A cutoff (FCC-256, 32 structures, 2 reps each):
#   bash tools/ab_wide.sh tag1 tag2 ...   (tag "base" = libdgn.so, else lib/libdgn_<tag>.so)
set -eo pipefail
for t in "$@"; do
  if [ "$t" = base ]; then L=defect-gnn-cpp_amd/lib/libdgn.so; else L=defect-gnn-cpp_amd/lib/libdgn_$t.so; fi
  echo "== $t"
  DGN_LIB=$L timeout -k 10 100 python -u tools/betti_rc10.py 32 3 2>&1 | grep rep
done
