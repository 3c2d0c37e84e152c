# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
O=gpurun_out/r6q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench_dist.py -m gpu > $O/t1.txt 2>&1 || { tail -40 $O/t1.txt; exit 1; }
tail -4 $O/t1.txt
