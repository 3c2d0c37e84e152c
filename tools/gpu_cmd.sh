# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_betti_wide.py tests/test_gpu_fused.py tests/test_gpu_graph.py > gpurun_out/t_last.log 2>&1 || { tail -30 gpurun_out/t_last.log; exit 1; }
tail -1 gpurun_out/t_last.log
