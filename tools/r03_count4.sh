#!/bin/bash
# round 3: count split (one-image count kernel + per-tile defer flags, query position read only in
# the borderline test): every GPU test, then the default bench twice
set -eo pipefail
OUT=gpurun_out/r03_count4
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline > "$OUT/bench_$r.json" 2>> "$OUT/err.log"
  python3 -c "import json;d=json.load(open('$OUT/bench_$r.json'));k=d['kernel_ms_per_step'];print(d['value'], k['graph_count'], k['graph_emit'], k['betti_vr'], d['roofline']['frac'], d['side']['config2']['path_ms'], d['side']['config5']['graph_path_kernels_ms'])"
done
