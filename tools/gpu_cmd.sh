# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g43
export TMPDIR=/tmp
timeout -k 10 600 bash tools/ab.sh gpurun_out/g43/ab 2 base pv2 pv8 as2
