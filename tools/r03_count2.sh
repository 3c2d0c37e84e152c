#!/bin/bash
# round 3: one-image count kernel split from the general one (graph_count_one_kernel + deferred
# list): neighbour / fused / Betti parity tests, then the default bench and a kernel trace
set -eo pipefail
OUT=gpurun_out/r03_count2
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_fused.py tests/test_gpu_betti.py tests/test_gpu_edges.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/bench.json" 2> "$OUT/bench.err"
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['kernel_ms_per_step'], d['roofline']['frac'], d['roofline']['emit_only'], d['side']['config2'], d['side']['config5'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side --no-betti > "$OUT/trace.json" 2> "$OUT/trace.err"
grep -i "count\|scan\|prep" "$OUT/trace/run_kernel_stats.csv" | cut -c1-200
