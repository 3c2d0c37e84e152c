# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
O=gpurun_out/salu2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_betti.py tests/test_gpu_betti_cellist.py tests/test_gpu_fused.py -x -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -3 $O/tests.txt
