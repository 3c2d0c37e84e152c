#!/bin/bash
# f32-prefiltered general search (config 2's SC-64 cells): graph / fused / Betti parity, config-2/5
# kernel times and the config-4 bench, each vs the build without it (nogen)
set -eo pipefail
OUT=gpurun_out/r03_gen
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_fused.py tests/test_gpu_betti.py tests/test_gpu_edges.py tests/test_facade.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for v in libdgn libdgn_nogen libdgn libdgn_nogen; do
  DGN_LIB=defect-gnn-cpp_amd/lib/$v.so timeout -k 10 120 python -u tools/side_graph.py 20 > "$OUT/side_$v.log" 2>&1
  echo "$v $(head -2 $OUT/side_$v.log | tail -2 | tr '\n' ' ')"
  DGN_LIB=defect-gnn-cpp_amd/lib/$v.so timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-side > "$OUT/b_$v.json" 2>> "$OUT/err.log"
  python3 -c "import json; r=json.load(open('$OUT/b_$v.json')); k=r['kernel_ms_per_step']; print('$v', r['value'], k['graph_count'], k['graph_emit'], r['roofline']['frac'])"
done
