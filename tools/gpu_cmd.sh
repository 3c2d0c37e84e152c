# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
mkdir -p gpurun_out/g8
export TMPDIR=/tmp
bash tools/pmc_betti.sh gpurun_out/g8/pmc fcc 4 1024 5.0 1 || exit 1
python3 tools/pmc_summary.py gpurun_out/g8/pmc betti > gpurun_out/g8/pmc.txt
bash profiles/collect_wide.sh r05base || exit 1
timeout -k 10 120 python -u tools/side_graph.py 20 > gpurun_out/g8/side_graph.json 2>&1 || exit 1
echo done
