# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/final5
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final5/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/final5/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/final5/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final5/smoke.txt 2>&1 || { tail -20 gpurun_out/final5/smoke.txt; exit 1; }
tail -1 gpurun_out/final5/smoke.txt
timeout -k 10 400 python -u bench.py > gpurun_out/final5/bench.json 2> gpurun_out/final5/bench.err || { tail -20 gpurun_out/final5/bench.err; exit 1; }
python3 -c "import json; r=json.loads(open('gpurun_out/final5/bench.json').read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'], r['roofline']['frac'], r['cpu_baseline']['value'])"
