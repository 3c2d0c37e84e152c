# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g50
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_betti_wide.py -m gpu > gpurun_out/g50/tests.txt 2>&1 || { tail -30 gpurun_out/g50/tests.txt; exit 1; }
tail -3 gpurun_out/g50/tests.txt
for tag in base r0 base r0; do
  lib=defect-gnn-cpp_amd/lib/libdgn.so; [ "$tag" != base ] && lib=defect-gnn-cpp_amd/lib/libdgn_$tag.so
  echo "== $tag"
  DGN_LIB=$lib timeout -k 10 300 python -u tools/betti_rc10.py 64 2 2>&1 | grep "rep 1" || exit 1
done
