#!/bin/bash
# word-major hit masks: graph / fused / Betti parity, then the count pass's WRITE_SIZE and the path times
set -eo pipefail
OUT=gpurun_out/r03_mask
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_fused.py tests/test_gpu_betti.py tests/test_gpu_edges.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-side > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 -c "import json; r=json.load(open('$OUT/bench.json')); print(r['value'], r['kernel_ms_per_step'], r['roofline']['frac'], r['roofline']['rbf_f32']['frac'])"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-side --no-betti --no-alt-rbf > "$OUT/w.log" 2>&1
python3 tools/pmc_summary.py "$OUT/write" graph_count graph_emit
