#!/bin/bash
# A/B of the Betti distance kernel (betti_dist ms) between libdgn.so and lib/libdgn_d4.so
set -eo pipefail
mkdir -p gpurun_out/abd
for arm in base d4 base d4; do  # d4: a variant lib (tools/build_variant.sh d4 "...")
  L=defect-gnn-cpp_amd/lib/libdgn.so; [ $arm = d4 ] && L=defect-gnn-cpp_amd/lib/libdgn_d4.so
  DGN_LIB=$L timeout -k 10 180 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side --no-alt-rbf > gpurun_out/abd/$arm.json 2>/dev/null
  python -c "import json; r=json.load(open('gpurun_out/abd/$arm.json')); k=r['kernel_ms_per_step']; print('$arm', r['value'], k['betti_dist'], k['betti_vr'])"
done
