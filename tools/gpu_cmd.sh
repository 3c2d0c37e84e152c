# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_betti_wide.py tests/test_gpu_betti_envelope.py -k "not 16A" > gpurun_out/t_wide.log 2>&1; rc=$?; tail -3 gpurun_out/t_wide.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 env DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_r4b.so python -u tools/betti_rc10.py 32 2 > gpurun_out/ab_b$r.log 2>&1 || exit 1
  grep "rep 1" gpurun_out/ab_b$r.log | sed 's/^/r4b /'
  timeout -k 10 200 python -u tools/betti_rc10.py 32 2 > gpurun_out/ab_n$r.log 2>&1 || exit 1
  grep "rep 1" gpurun_out/ab_n$r.log | sed 's/^/new /'
done
timeout -k 10 200 python -u tools/diag_wide.py 4 > gpurun_out/diag3.log 2>&1; head -14 gpurun_out/diag3.log
