# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g24
export TMPDIR=/tmp
DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_dbg.so timeout -k 10 300 python -u tools/betti_rc10.py 1 1 > gpurun_out/g24/dbg.log 2>&1 || { tail -20 gpurun_out/g24/dbg.log; exit 1; }
grep DBG gpurun_out/g24/dbg.log | head -20
