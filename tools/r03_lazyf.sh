#!/bin/bash
# round 3 A/B: (1) the one-image count kernel at 8 / 7 / 6 waves per SIMD (count pass alone);
# (2) the narrow Betti kernel's per-column fence only once the spilled pivot table is in use
# (-DDGN_COL_FENCE_LAZY): Betti parity tests on that build, then the bench against the default
set -eo pipefail
OUT=gpurun_out/r03_lazyf
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2; do
  for lib in libdgn libdgn_c7 libdgn_c6; do
    DGN_LIB=defect-gnn-cpp_amd/lib/$lib.so timeout -k 10 120 python -u tools/count_probe.py 30 >> "$OUT/probe.txt" 2>> "$OUT/err.log"
  done
done
cat "$OUT/probe.txt"
DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_lazyf.so timeout -k 10 400 python -u -m pytest tests/test_gpu_betti.py tests/test_gpu_betti_envelope.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
for r in 1 2; do
  for lib in libdgn libdgn_lazyf; do
    DGN_LIB=defect-gnn-cpp_amd/lib/$lib.so timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-side > "$OUT/${lib}_$r.json" 2>> "$OUT/err.log"
    python3 -c "import json;d=json.load(open('$OUT/${lib}_$r.json'));k=d['kernel_ms_per_step'];print('$lib', d['value'], k['betti_vr'])"
  done
done
