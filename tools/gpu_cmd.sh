# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
export TMPDIR=/tmp
rm -rf gpurun_out/prof_r05c
timeout -k 10 1000 bash profiles/collect_r05.sh gpurun_out/prof_r05c
