#!/bin/bash
# round-3 graph-path experiment: per-launch emit durations (rocprofv3 kernel trace) of the fused
# emit, the split emit (rows launch, then RBF launch) and rows only, for f64 and f32 RBF
set -eo pipefail
OUT=gpurun_out/${EXP_TAG:-r03_graph_exp}
mkdir -p "$OUT"
export TMPDIR=/tmp
for dt in ${DTYPES:-f64 f32}; do
  for v in ${VARIANTS:-libdgn libdgn_split libdgn_norbf}; do
    DGN_LIB=defect-gnn-cpp_amd/lib/$v.so timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr_${v}_$dt" -o run -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-side --no-betti --no-alt-rbf --rbf-dtype $dt > "$OUT/b_${v}_$dt.log" 2>&1
    python3 - "$OUT/tr_${v}_$dt" "$v $dt" <<'PY'
import csv, glob, sys, collections
f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True))[-1]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "")
    acc[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
print(sys.argv[2], {k[-26:]: [round(x, 3) for x in v[-6:]] for k, v in acc.items() if "graph_emit" in k or "graph_count" in k})
PY
  done
done
