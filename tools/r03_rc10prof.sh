#!/bin/bash
# kernel trace of the 10 A Betti path (rank pass, wide launches), for the phase budget
set -eo pipefail
OUT=gpurun_out/r03_rc10prof
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/tr" -o run -- python3 tools/betti_rc10.py 32 1 > "$OUT/rc10.log" 2>&1
cat "$OUT/rc10.log" | tail -2
python3 - "$OUT/tr" <<'PY'
import csv, glob, sys
f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True))[-1]
for r in list(csv.DictReader(open(f)))[:14]:
    print(r["Name"][:70], r["Calls"], round(float(r["TotalDurationNs"]) / 1e6, 2), "ms")
PY
