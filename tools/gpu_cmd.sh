# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g37
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_betti_wide.py tests/test_gpu_betti_envelope.py > gpurun_out/g37/t.log 2>&1 || { tail -30 gpurun_out/g37/t.log; exit 1; }
tail -1 gpurun_out/g37/t.log
for tag in pre base pre base; do
  lib=defect-gnn-cpp_amd/lib/libdgn.so; [ "$tag" != base ] && lib=defect-gnn-cpp_amd/lib/libdgn_$tag.so
  echo "== $tag"
  DGN_LIB=$lib timeout -k 10 300 python -u tools/betti_rc10.py 64 2 2>&1 | grep "rep 1" || exit 1
done
