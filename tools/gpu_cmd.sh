# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
bash tools/ab.sh gpurun_out/fork1 3 base nofork && \
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_graph.py tests/test_gpu_bench_dist.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3
