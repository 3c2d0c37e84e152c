#!/bin/bash
# graph emit past 1,024 candidates (2,048-candidate streamed instantiation): graph tests
set -eo pipefail
OUT=gpurun_out/r03_env
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_fused.py -m gpu -x -v --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
grep -E "17A|12A" "$OUT/pytest.log"
tail -2 "$OUT/pytest.log"
