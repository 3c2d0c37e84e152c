# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/prof_r04
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/t_all.log 2>&1 || { tail -30 gpurun_out/t_all.log; exit 1; }
tail -1 gpurun_out/t_all.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench_final.log 2>&1 || { tail -30 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r04/side -o run -- python3 tools/side_graph.py 20 > gpurun_out/prof_r04/side_graph.log 2>&1 || { tail -20 gpurun_out/prof_r04/side_graph.log; exit 1; }
grep -E "^config" gpurun_out/prof_r04/side_graph.log
NO_PARSE=1 timeout -k 10 1000 bash profiles/collect.sh r04 > gpurun_out/collect.log 2>&1 || { tail -20 gpurun_out/collect.log; exit 1; }
echo collected
