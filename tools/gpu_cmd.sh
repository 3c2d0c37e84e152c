# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_betti.py tests/test_gpu_betti_wide.py tests/test_gpu_graph.py tests/test_gpu_fused.py > gpurun_out/t_core.log 2>&1; rc=$?; tail -3 gpurun_out/t_core.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab.sh gpurun_out/ab_lane 2 r4b base || exit 1
for r in 1 2; do
  timeout -k 10 200 env DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_r4b.so python -u tools/betti_rc10.py 32 2 2>&1 | grep "rep 1" | sed 's/^/r4b /' || exit 1
  timeout -k 10 200 python -u tools/betti_rc10.py 32 2 2>&1 | grep "rep 1" | sed 's/^/new /' || exit 1
done
