#!/bin/bash
# round 3: Betti dim-2 triangle enumeration reading the edge list through a register window (A/B
# against the previous build, libdgn_base.so): Betti parity tests, diag phase split, bench x2
set -eo pipefail
OUT=gpurun_out/r03_ewin
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_betti.py tests/test_gpu_betti_envelope.py tests/test_gpu_fused.py -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -30 "$OUT/pytest.log"; exit 1; }
tail -2 "$OUT/pytest.log"
timeout -k 10 200 python -u tools/diag_phases.py fcc 4 512 5.0 > "$OUT/phases.json" 2> "$OUT/phases.err"
python3 -c "import json;d=json.load(open('$OUT/phases.json'));print('enum', d['dim2_enumerate_cycles_per_complex'], 'dim2app', d['phase_cycles_per_complex']['dim2 apparent'], 'tot', d['cycles_per_complex'])"
for r in 1 2; do
  for lib in defect-gnn-cpp_amd/lib/libdgn_base.so defect-gnn-cpp_amd/lib/libdgn.so; do
    name=$(basename "$lib" .so)
    DGN_LIB=$lib timeout -k 10 200 python -u bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-side > "$OUT/${name}_$r.json" 2>> "$OUT/err.log"
    python3 -c "import json;d=json.load(open('$OUT/${name}_$r.json'));k=d['kernel_ms_per_step'];print('$name', d['value'], k['betti_vr'])"
  done
done
