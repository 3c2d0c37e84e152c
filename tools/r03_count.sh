#!/bin/bash
# count-pass A/B: 5 waves per SIMD (12 VGPRs spilled, scratch writes) vs 4 (no spills)
set -eo pipefail
OUT=gpurun_out/r03_count
mkdir -p "$OUT"
export TMPDIR=/tmp
for v in libdgn libdgn_count4 libdgn libdgn_count4; do
  DGN_LIB=defect-gnn-cpp_amd/lib/$v.so timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-side > "$OUT/b_$v.json" 2>> "$OUT/err.log"
  python3 -c "import json; r=json.load(open('$OUT/b_$v.json')); k=r['kernel_ms_per_step']; print('$v', r['value'], k['graph_count'], k['graph_emit'], r['roofline']['frac'], r['roofline']['rbf_f32']['frac'])"
done
DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_count4.so timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write4" -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-side --no-betti --no-alt-rbf > "$OUT/w4.log" 2>&1
python3 tools/pmc_summary.py "$OUT/write4" graph_count
