set -eo pipefail
mkdir -p gpurun_out/w1
timeout -k 10 300 python -u -m pytest tests/test_gpu_betti_wide.py tests/test_gpu_betti_envelope.py tests/test_gpu_betti.py -x -q --timeout 200 --timeout-method thread > gpurun_out/w1/pytest.log 2>&1
tail -2 gpurun_out/w1/pytest.log
timeout -k 10 120 python -u tools/diag_wide.py 4 > gpurun_out/w1/diag.json 2>&1
cat gpurun_out/w1/diag.json
timeout -k 10 150 python -u tools/betti_rc10.py 32 2 2>&1 | grep rep
