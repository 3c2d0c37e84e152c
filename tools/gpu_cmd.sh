# scratch driver for one gpurun call (edited per call; not used by tests or the bench)
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
