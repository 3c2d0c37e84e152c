# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g10
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py > gpurun_out/g10/bench.json 2> gpurun_out/g10/bench.err || { tail -20 gpurun_out/g10/bench.err; exit 1; }
tail -c 3000 gpurun_out/g10/bench.json
timeout -k 10 1200 bash profiles/collect_r05.sh gpurun_out/prof_r05a
