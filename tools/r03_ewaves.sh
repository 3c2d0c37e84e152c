#!/bin/bash
# round 3 A/B: waves-per-SIMD target of the fused emit (default = none: 88 VGPRs, 5 waves; 6; 7), via a
# temporary amdgpu_waves_per_eu(DGN_EMIT_WAVES) hook on graph_emit_kernel (not kept: no gain),
# libdgn_e6/e7 built with tools/build_variant.sh; graph-only bench (f64 RBF headline configuration)
set -eo pipefail
OUT=gpurun_out/r03_ewaves
mkdir -p "$OUT"
export TMPDIR=/tmp
for r in 1 2 3; do
  for lib in libdgn libdgn_e6 libdgn_e7; do
    DGN_LIB=defect-gnn-cpp_amd/lib/$lib.so timeout -k 10 200 python -u bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-side --no-betti > "$OUT/${lib}_$r.json" 2>> "$OUT/err.log"
    python3 -c "import json;d=json.load(open('$OUT/${lib}_$r.json'));k=d['kernel_ms_per_step'];print('$lib', k['graph_emit'], k['graph_count'], d['roofline']['frac'])"
  done
done
