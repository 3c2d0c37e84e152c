# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g35
export TMPDIR=/tmp
for v in al1 al2; do
DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_$v.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_betti.py > gpurun_out/g35/t_$v.log 2>&1 || { tail -30 gpurun_out/g35/t_$v.log; exit 1; }
tail -1 gpurun_out/g35/t_$v.log
done
timeout -k 10 600 bash tools/ab.sh gpurun_out/g35/ab 2 pre al1 al2
