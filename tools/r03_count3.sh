#!/bin/bash
# round 3: count split with per-tile defer flags: neighbour / fused / Betti parity tests, then an
# A/B of the one-image count kernel's waves per SIMD (8 = default, 6, 5) on the graph path
set -eo pipefail
OUT=gpurun_out/r03_count3
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_fused.py tests/test_gpu_betti.py tests/test_gpu_edges.py tests/test_gpu_multiproc.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for r in 1 2; do
  for lib in defect-gnn-cpp_amd/lib/libdgn.so defect-gnn-cpp_amd/lib/libdgn_c6.so defect-gnn-cpp_amd/lib/libdgn_c5.so; do
    name=$(basename "$lib" .so)
    DGN_LIB=$lib timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/${name}_$r.json" 2>> "$OUT/err.log"
    python3 -c "import json;d=json.load(open('$OUT/${name}_$r.json'));k=d['kernel_ms_per_step'];print('$name', d['value'], k['graph_count'], k['graph_emit'], d['roofline']['frac'], d['side']['config2']['path_ms'], d['side']['config5']['graph_path_kernels_ms'])"
  done
done
