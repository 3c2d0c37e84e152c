# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g29
export TMPDIR=/tmp
DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_ndbg.so timeout -k 10 300 python -u tools/betti_run.py fcc 4 1 5.0 1 > gpurun_out/g29/dbg.log 2>&1 || { tail -20 gpurun_out/g29/dbg.log; exit 1; }
grep DBG gpurun_out/g29/dbg.log | head -40
