# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/final5b
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/final5b/gpu_tests.txt 2>&1 || { tail -30 gpurun_out/final5b/gpu_tests.txt; exit 1; }
tail -2 gpurun_out/final5b/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final5b/smoke.txt 2>&1 || { tail -20 gpurun_out/final5b/smoke.txt; exit 1; }
tail -1 gpurun_out/final5b/smoke.txt
timeout -k 10 400 python -u bench.py > gpurun_out/final5b/bench.json 2> gpurun_out/final5b/bench.err || { tail -20 gpurun_out/final5b/bench.err; exit 1; }
python3 -c "import json; r=json.loads(open('gpurun_out/final5b/bench.json').read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'], r['kernel_ms_per_step']['betti_vr'], r['roofline']['frac'])"
bash profiles/collect_r05.sh gpurun_out/prof_r05i
