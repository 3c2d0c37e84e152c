# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
O=gpurun_out/r6h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_betti_wide.py -m gpu > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u tools/betti_rc10.py 128 1 > $O/rc10.txt 2>&1 || { tail -20 $O/rc10.txt; exit 1; }
grep "rep 0" $O/rc10.txt
timeout -k 10 200 python3 -u tools/betti_rc10.py 128 3 > $O/rc10_128.txt 2>&1 || { tail -20 $O/rc10_128.txt; exit 1; }
grep "rep" $O/rc10_128.txt
