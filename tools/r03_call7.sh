#!/bin/bash
# round-3 call: full GPU suite + smoke + the driver's bench command on the async-step build
set -eo pipefail
OUT=gpurun_out/r03_call7
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
bash tools/ab_rc10.sh r03_ab_rc10 defect-gnn-cpp_amd/lib/libdgn_base.so defect-gnn-cpp_amd/lib/libdgn.so defect-gnn-cpp_amd/lib/libdgn_pv32.so
DTYPES=f64 EXP_TAG=r03_buf VARIANTS="libdgn libdgn_buf8k libdgn_buf2k" bash tools/r03_graph_exp.sh
