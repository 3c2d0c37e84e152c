# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
O=gpurun_out/r6s
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
for v in base pw7 pw8; do
  lib=defect-gnn-cpp_amd/lib/libdgn.so; [ $v != base ] && lib=defect-gnn-cpp_amd/lib/libdgn_$v.so
  DGN_LIB=$lib timeout -k 10 200 python3 -u tools/betti_rc10.py 128 2 > $O/rc10_${v}_$r.txt 2>&1 || { tail -20 $O/rc10_${v}_$r.txt; exit 1; }
  echo $v $(grep "rep 1" $O/rc10_${v}_$r.txt | cut -c1-90)
done
done
