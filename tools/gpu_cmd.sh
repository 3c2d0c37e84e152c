# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g36
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_betti.py tests/test_gpu_betti_envelope.py tests/test_gpu_betti_cellist.py > gpurun_out/g36/t.log 2>&1 || { tail -30 gpurun_out/g36/t.log; exit 1; }
tail -1 gpurun_out/g36/t.log
timeout -k 10 600 bash tools/ab.sh gpurun_out/g36/ab 2 pre base
