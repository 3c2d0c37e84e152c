#!/bin/bash
# Build an experimental libdgn_<tag>.so from a patched COPY of csrc/ (A/B experiments; never used by
# tests; the product sources stay untouched):
#   bash tools/build_patched.sh <tag> <edit.py> ["-DFOO=1 ..."]
# <edit.py> runs with the copy's directory as argv[1] and edits the sources there (str.replace).
set -eo pipefail
TAG=$1; EDIT=$2; FLAGS=${3:-}
cd "$(dirname "$0")/.."
make -s defect-gnn-cpp_amd/lib/libdgn.so
R=$(mktemp -d /tmp/dgn_patch_XXXX)
T=$R/pkg/csrc  # dgn_api.cpp includes ../../include/dgn.h
mkdir -p "$T" && ln -s "$PWD/include" "$R/include"
cp defect-gnn-cpp_amd/csrc/* "$T/"
python3 "$EDIT" "$T"
B=defect-gnn-cpp_amd/build_var_$TAG
mkdir -p "$B"
HF="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -I$T -Iinclude -mllvm -amdgpu-atomic-optimizer-strategy=DPP $FLAGS"
rm -f "$B"/*.o
pids=()
for f in graph_kernels betti_kernels betti_wide betti_rank betti_split node_kernels; do
  PF=""; [ "$f" = betti_kernels ] && PF="-mllvm -amdgpu-sched-strategy=iterative-minreg"  # Makefile per-source flag
  /opt/rocm/bin/hipcc $HF $PF -c "$T/$f.hip" -o "$B/$f.o" & pids+=($!)
done
/opt/rocm/bin/hipcc $HF -x hip -c "$T/dgn_api.cpp" -o "$B/dgn_api.o" & pids+=($!)
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o defect-gnn-cpp_amd/lib/libdgn_$TAG.so "$B"/*.o
rm -rf "$R"
