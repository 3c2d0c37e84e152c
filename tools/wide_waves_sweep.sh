#!/bin/bash
# Wide-kernel resident-wave sweep at 10 A (DGN_WIDE_WAVES caps the launch; A/B only)
set -eo pipefail
for w in ${@:-2048 1536 1024 768}; do
  echo "waves $w"
  DGN_WIDE_WAVES=$w timeout -k 10 100 python -u tools/betti_rc10.py 32 2 2>&1 | grep "rep 1"
done
