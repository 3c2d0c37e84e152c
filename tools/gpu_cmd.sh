# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g54
export TMPDIR=/tmp
bash tools/ab.sh gpurun_out/g54/ab 2 base ilp mrnc mro2 mrnurp
