# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u bench.py > gpurun_out/bench_final.log 2>&1 || { tail -30 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], json.dumps(d['side']['config2']), json.dumps(d['side']['betti_rc10']), json.dumps(d['side']['betti_rc10_b128']))"
