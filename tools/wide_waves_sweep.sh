set -eo pipefail
mkdir -p gpurun_out/wv
for w in 2048 1024 512 256; do
  echo "waves $w"
  DGN_WIDE_WAVES=$w timeout -k 10 150 python -u tools/betti_rc10.py 32 2 2>&1 | grep rep
done
