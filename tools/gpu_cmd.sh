# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/ab_par
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_betti_wide.py tests/test_gpu_betti_envelope.py tests/test_gpu_betti.py > gpurun_out/ab_par/t.log 2>&1 || { tail -30 gpurun_out/ab_par/t.log; exit 1; }
tail -1 gpurun_out/ab_par/t.log
for r in 1 2; do
  for t in base old; do
    lib=defect-gnn-cpp_amd/lib/libdgn.so; [ $t != base ] && lib=defect-gnn-cpp_amd/lib/libdgn_$t.so
    DGN_LIB=$lib timeout -k 10 150 python -u tools/betti_rc10.py 128 2 > gpurun_out/ab_par/${t}_$r.log 2>&1 || exit 1
    echo "$t $(grep -o '= [0-9.]* structures/s' gpurun_out/ab_par/${t}_$r.log | tail -1)"
  done
done
