# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g51
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_betti.py tests/test_gpu_fused.py tests/test_gpu_betti_envelope.py -m gpu > gpurun_out/g51/tests.txt 2>&1 || { tail -30 gpurun_out/g51/tests.txt; exit 1; }
tail -3 gpurun_out/g51/tests.txt
bash tools/ab.sh gpurun_out/g51/ab 3 base r0
