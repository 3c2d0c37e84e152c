# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
O=gpurun_out/r6t
mkdir -p $O
export TMPDIR=/tmp
for v in base ws3 ws6 ws8; do
  lib=defect-gnn-cpp_amd/lib/libdgn.so; [ $v != base ] && lib=defect-gnn-cpp_amd/lib/libdgn_$v.so
  DGN_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run -- python3 -u tools/betti_rc10.py 32 1 > $O/rc10_${v}.txt 2>&1 || { tail -20 $O/rc10_${v}.txt; exit 1; }
  echo $v done
done
