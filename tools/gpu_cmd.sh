# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g47
export TMPDIR=/tmp
for B in 2 4 8 16 32 64; do
  echo "== B=$B"
  timeout -k 10 300 python -u tools/betti_rc10.py $B 2 2>&1 | grep "rep 1" || exit 1
done
for wv in 1024 2048 3072; do
  echo "== waves=$wv B=64"
  DGN_WIDE_WAVES=$wv timeout -k 10 300 python -u tools/betti_rc10.py 64 2 2>&1 | grep "rep 1" || exit 1
done
