#!/bin/bash
# Kernel trace of the graph-only bench with a given libdgn: per-launch emit durations.
#   bash tools/emit_trace.sh <outdir> <lib.so>
set -eo pipefail
OUT=$1; LIB=$2
mkdir -p "$OUT"
export TMPDIR=/tmp
DGN_LIB=$LIB timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr" -o run -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-betti --no-alt-rbf > "$OUT/b.log" 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = sorted(glob.glob(sys.argv[1] + "/tr/**/*kernel_trace.csv", recursive=True))[-1]
rows = [r for r in csv.DictReader(open(f)) if "graph_emit" in r["Kernel_Name"] or "graph_count" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
for r in rows[-40:]:
    print(r["Kernel_Name"][:40], r["Grid_Size_X"] if "Grid_Size_X" in r else r.get("Grid_Size", ""),
          (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0, "us")
PY
