# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
export TMPDIR=/tmp
rm -rf gpurun_out/prof_r05c
mkdir -p gpurun_out/g39
DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_chk.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_betti.py tests/test_gpu_betti_wide.py tests/test_gpu_betti_cellist.py tests/test_gpu_fused.py > gpurun_out/g39/chk.log 2>&1 || { tail -30 gpurun_out/g39/chk.log; exit 1; }
tail -1 gpurun_out/g39/chk.log
timeout -k 10 1000 bash profiles/collect_r05.sh gpurun_out/prof_r05c
