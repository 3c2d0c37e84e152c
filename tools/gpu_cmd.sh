# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
O=gpurun_out/r6p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -k "single_component or fails_loudly" tests/test_gpu_betti_envelope.py -m gpu > $O/t1.txt 2>&1 || { tail -30 $O/t1.txt; exit 1; }
tail -3 $O/t1.txt
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_betti_envelope.py tests/test_gpu_betti_wide.py tests/test_gpu_betti.py tests/test_gpu_betti_cellist.py -m gpu > $O/t2.txt 2>&1 || { tail -30 $O/t2.txt; exit 1; }
tail -2 $O/t2.txt
