# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/r04_full
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_betti_wide.py > gpurun_out/t_wide.log 2>&1; rc=$?; tail -1 gpurun_out/t_wide.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r04_full/bench2.json 2> gpurun_out/r04_full/bench2.err; rc=$?; python3 -c "
import json; r=json.load(open('gpurun_out/r04_full/bench2.json')); print(r['value'], r['side']['betti_rc10'], r['side']['config2'])"; exit $rc
