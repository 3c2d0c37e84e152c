# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_facade.py -m gpu -x -v --timeout 300 --timeout-method thread 2>&1 | tail -12
