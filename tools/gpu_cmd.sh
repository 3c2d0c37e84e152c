# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g42
export TMPDIR=/tmp
timeout -k 10 600 bash tools/ab.sh gpurun_out/g42/ab 2 base ch2 ch4
