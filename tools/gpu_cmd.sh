# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/ab_c1f
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_graph.py tests/test_gpu_betti.py tests/test_gpu_fused.py > gpurun_out/ab_c1f/t.log 2>&1 || { tail -30 gpurun_out/ab_c1f/t.log; exit 1; }
tail -1 gpurun_out/ab_c1f/t.log
for r in 1 2; do
  for t in base old; do
    lib=defect-gnn-cpp_amd/lib/libdgn.so; [ $t != base ] && lib=defect-gnn-cpp_amd/lib/libdgn_$t.so
    DGN_LIB=$lib timeout -k 10 120 python -u bench.py --steps 5 --warmup 1 --no-betti --no-cpu-baseline --no-side --no-alt-rbf > gpurun_out/ab_c1f/${t}_$r.json 2>gpurun_out/ab_c1f/err.log || exit 1
    python3 -c "import json; r=json.load(open('gpurun_out/ab_c1f/${t}_$r.json')); k=r['kernel_ms_per_step']; print('$t', r['roofline']['frac'], k)"
    DGN_LIB=$lib timeout -k 10 120 python -u tools/side_graph.py 20 2>/dev/null | grep '^config2 ' 
  done
done
