# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_betti.py tests/test_gpu_betti_cellist.py tests/test_gpu_fused.py tests/test_gpu_betti_envelope.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3
