#!/bin/bash
# round-3 evidence on one fresh MI355X: every GPU test + smoke, the default bench (side lines and
# CPU baseline included), then the rocprofv3 kernel trace/stats and the FETCH/WRITE PMC passes
# (profiles/collect.sh; parsed locally after the merge back)
set -eo pipefail
OUT=gpurun_out/r03_final
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
tail -1 "$OUT/smoke.log"
timeout -k 10 400 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
cat "$OUT/bench.json"
NO_PARSE=1 bash profiles/collect.sh r03
echo collect ok
