# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g44
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_graph.py -k "large_rows" > gpurun_out/g44/t.log 2>&1 || { tail -30 gpurun_out/g44/t.log; exit 1; }
tail -1 gpurun_out/g44/t.log
