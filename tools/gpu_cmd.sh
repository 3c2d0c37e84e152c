# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/prof_r04
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04/side -o run -- python3 tools/side_graph.py 20 > gpurun_out/prof_r04/side_graph.log 2>&1 || { tail -20 gpurun_out/prof_r04/side_graph.log; exit 1; }
tail -4 gpurun_out/prof_r04/side_graph.log
