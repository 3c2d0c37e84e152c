# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
bash tools/ab.sh gpurun_out/salu1 2 base s12 s123 s124 s1234
