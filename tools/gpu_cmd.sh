# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_graph.py -k "few or epsilon" > gpurun_out/t_few2.log 2>&1 || { tail -30 gpurun_out/t_few2.log; exit 1; }
tail -3 gpurun_out/t_few2.log
