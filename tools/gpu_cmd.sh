# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
bash tools/ab.sh gpurun_out/t64 3 base t64
