#!/bin/bash
# graph path after the tile-size change: GPU graph tests, then per-launch emit durations (fused /
# split rows+RBF / rows only) for f64 and f32 RBF, and the side-line kernels
set -eo pipefail
OUT=gpurun_out/r03_graph2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_fused.py tests/test_gpu_edges.py tests/test_gpu_node.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest_graph.log" 2>&1 || { tail -30 "$OUT/pytest_graph.log"; exit 1; }
tail -2 "$OUT/pytest_graph.log"
EXP_TAG=r03_graph2 VARIANTS="libdgn libdgn_split libdgn_norbf" bash tools/r03_graph_exp.sh
