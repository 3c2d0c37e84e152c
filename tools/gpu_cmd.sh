# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -4 gpurun_out/$name.log; return $rc; }
run t_graph 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_graph.py -k "large_rows or 17A" && \
run t_env 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_betti_envelope.py -k "grow_levels or above_1024 or above_2048 or above_512" && \
run t_wide 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_betti_wide.py && \
run ab_base 300 env DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_r4a.so python -u tools/betti_rc10.py 16 2 && \
run ab_new 300 python -u tools/betti_rc10.py 16 2 && \
run ab_base2 300 env DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_r4a.so python -u tools/betti_rc10.py 16 2 && \
run ab_new2 300 python -u tools/betti_rc10.py 16 2
