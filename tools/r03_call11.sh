#!/bin/bash
# round-3 call: issue-port probe -- 16 extra SALU vs 16 extra VALU instructions per pivot-search step
set -eo pipefail
export TMPDIR=/tmp
bash tools/ab_betti.sh r03_probe_salu defect-gnn-cpp_amd/lib/libdgn.so defect-gnn-cpp_amd/lib/libdgn_psalu.so
bash tools/ab_betti.sh r03_probe_valu defect-gnn-cpp_amd/lib/libdgn.so defect-gnn-cpp_amd/lib/libdgn_pvalu.so
