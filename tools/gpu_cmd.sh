# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
O=gpurun_out/r6l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_betti_wide.py tests/test_gpu_betti_envelope.py tests/test_gpu_betti_cellist.py -m gpu > $O/tests.txt 2>&1 || { tail -30 $O/tests.txt; exit 1; }
tail -2 $O/tests.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 -u tools/betti_rc10.py 32 1 > $O/rc10_32.txt 2>&1 || { tail -20 $O/rc10_32.txt; exit 1; }
timeout -k 10 200 python3 -u tools/betti_rc10.py 128 2 > $O/rc10_128.txt 2>&1 || { tail -20 $O/rc10_128.txt; exit 1; }
grep "rep" $O/rc10_128.txt
DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_chk.so timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -k "triangles or betti_dist or fcc256_batch or test_kat or random_clouds or persistence_from or wide_random" tests/test_gpu_betti.py tests/test_gpu_betti_cellist.py tests/test_gpu_betti_envelope.py tests/test_gpu_betti_wide.py -m gpu > $O/chk_tests.txt 2>&1 || { tail -30 $O/chk_tests.txt; exit 1; }
tail -3 $O/chk_tests.txt
