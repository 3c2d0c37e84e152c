#!/bin/bash
# Build a variant of libdgn.so with extra compile flags (A/B experiments; never used by tests):
#   bash tools/build_variant.sh <tag> "-DFOO=1 ..." [sources...]  -> defect-gnn-cpp_amd/lib/libdgn_<tag>.so
# Only the listed sources (default: all) are rebuilt with the flags; the rest are the main build's objects.
set -eo pipefail
TAG=$1; FLAGS=${2:-}; shift 2 || true
SRCS=${@:-graph_kernels betti_kernels betti_wide betti_rank betti_split node_kernels dgn_api}
cd "$(dirname "$0")/.."
make -s defect-gnn-cpp_amd/lib/libdgn.so
B=defect-gnn-cpp_amd/build_var_$TAG
mkdir -p "$B"
cp defect-gnn-cpp_amd/build/*.o "$B/"
HF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Idefect-gnn-cpp_amd/csrc -Iinclude -mllvm -amdgpu-atomic-optimizer-strategy=DPP $FLAGS"
for f in $SRCS; do
  if [ "$f" = dgn_api ]; then
    /opt/rocm/bin/hipcc $HF -x hip -c defect-gnn-cpp_amd/csrc/dgn_api.cpp -o $B/dgn_api.o &
  else
    PF=""; [ "$f" = betti_kernels ] && [[ "$FLAGS" != *sched-strategy* ]] && PF="-mllvm -amdgpu-sched-strategy=iterative-minreg"  # Makefile per-source flag
    /opt/rocm/bin/hipcc $HF $PF -c defect-gnn-cpp_amd/csrc/$f.hip -o $B/$f.o &
  fi
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o defect-gnn-cpp_amd/lib/libdgn_$TAG.so $B/*.o
