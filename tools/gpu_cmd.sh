# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g55
export TMPDIR=/tmp
bash tools/ab.sh gpurun_out/g55/ab 2 base gkilp gkmc
for tag in base bwmc bwilp base bwmc bwilp; do
  lib=defect-gnn-cpp_amd/lib/libdgn.so; [ "$tag" != base ] && lib=defect-gnn-cpp_amd/lib/libdgn_$tag.so
  echo "== $tag"
  DGN_LIB=$lib timeout -k 10 300 python -u tools/betti_rc10.py 64 2 2>&1 | grep "rep 1" || exit 1
done
