set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_graph.py -k "large_rows or 17A" > gpurun_out/t_graph.log 2>&1 && \
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_betti_envelope.py -k "grow_levels or above_1024 or above_2048 or above_512" > gpurun_out/t_env.log 2>&1
echo "rc=$?"
tail -5 gpurun_out/t_graph.log; tail -15 gpurun_out/t_env.log
