#!/bin/bash
# round-3 call: narrow-kernel occupancy sensitivity (16 -> 11 waves per CU via LDS padding)
set -eo pipefail
bash tools/ab_betti.sh r03_ab_occ defect-gnn-cpp_amd/lib/libdgn.so defect-gnn-cpp_amd/lib/libdgn_occ3.so
