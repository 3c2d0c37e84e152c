# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g56
export TMPDIR=/tmp
DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_st5.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_betti.py tests/test_gpu_betti_cellist.py -m gpu > gpurun_out/g56/tests.txt 2>&1 || { tail -30 gpurun_out/g56/tests.txt; exit 1; }
tail -2 gpurun_out/g56/tests.txt
bash tools/ab.sh gpurun_out/g56/ab 3 base st4 st5
