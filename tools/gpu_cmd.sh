# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log; return $rc; }
run t_wide 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_betti_wide.py && \
run t_env 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_betti_envelope.py -k "grow_levels or above_1024 or above_512 or wide_in_kernel or clique_200" && \
run ab_base 300 env DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_r4a.so python -u tools/betti_rc10.py 32 2 && \
run ab_new 300 python -u tools/betti_rc10.py 32 2 && \
run ab_base2 300 env DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_r4a.so python -u tools/betti_rc10.py 32 2 && \
run ab_new2 300 python -u tools/betti_rc10.py 32 2 && \
run diag 300 python -u tools/diag_wide.py 4
