# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g34
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/g34/bench.json 2> gpurun_out/g34/bench.err || { tail -20 gpurun_out/g34/bench.err; exit 1; }
tail -c 400 gpurun_out/g34/bench.json
timeout -k 10 900 bash profiles/collect_r05.sh gpurun_out/prof_r05b
