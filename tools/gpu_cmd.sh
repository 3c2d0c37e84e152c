# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
O=gpurun_out/r6g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.txt 2>&1 || { tail -30 $O/gpu_tests.txt; exit 1; }
tail -1 $O/gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo bench ok
bash profiles/collect_r06.sh $O/prof
bash tools/pmc_variants.sh $O/pmc "fcc 4 1024 5.0 1" base > $O/pmc.log 2>&1; echo pmc ok
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum --output-format csv -d $O/narrow_mem -o run -- python3 tools/betti_run.py fcc 4 1024 5.0 1 > $O/narrow_mem.log 2>&1
python3 tools/pmc_summary.py $O/narrow_mem betti_kernel > $O/narrow_mem.txt; echo done
