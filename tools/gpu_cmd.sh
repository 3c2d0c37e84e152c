# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
O=gpurun_out/r6r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_betti_wide.py tests/test_gpu_betti_envelope.py -m gpu > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u tools/betti_rc10.py 32 1 > $O/rc10_32.txt 2>&1 || { tail -20 $O/rc10_32.txt; exit 1; }
timeout -k 10 200 python3 -u tools/betti_rc10.py 128 2 > $O/rc10_128.txt 2>&1 || { tail -20 $O/rc10_128.txt; exit 1; }
grep "rep" $O/rc10_128.txt
