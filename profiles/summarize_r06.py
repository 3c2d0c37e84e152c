"""Round-6 evidence beside parse_profiles.py (bench trace + path PMC): folds profiles/collect_r06.sh's
10 A and side-line output into committed summaries.
    python profiles/summarize_r06.py [gpurun_out/r6o/prof]
Writes (profiles/):
  r06_rc10.json        the 10 A path (tools/betti_rc10.py 32 1: 8,192 complexes of ~340 points, one
                       slice): per-kernel times from the trace; per complex, the walk pass
                       (betti_walk_kernel, one workgroup per complex, code triangle in LDS) and the
                       reduction kernel (betti_wide_kernel_c16<6, true>): HBM bytes and the SQ mix
  r06_side_graph.json  per-kernel medians of BASELINE configs 2 and 5 (f32 / f64 RBF)
SQ cycle counters are in quad-cycles (MI355X_MICROARCH.md); instruction counters per wave instruction.
"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
D = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(HERE), "gpurun_out", "r6o", "prof")
NC = 8192  # complexes of tools/betti_rc10.py 32 1


def counters(sub):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in sorted(glob.glob(os.path.join(D, sub, "**", "*counter_collection.csv"), recursive=True)):
        with open(p) as f:
            for r in csv.DictReader(f):
                k = "walk" if "betti_walk" in r["Kernel_Name"] else ("reduce" if "c16" in r["Kernel_Name"] else None)
                if k:
                    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    return acc


def trace(sub):
    out = collections.defaultdict(list)
    for p in glob.glob(os.path.join(D, sub, "**", "*kernel_trace.csv"), recursive=True):
        with open(p) as f:
            for r in csv.DictReader(f):
                n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
                n = n[:n.find("(")] if "(" in n else n
                out[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    return out


def main():
    tr = trace("rc10_trace")
    c = collections.defaultdict(dict)
    for sub in ("rc10_fetch", "rc10_write", "rc10_sq1", "rc10_sq2"):
        for k, cs in counters(sub).items():
            c[k].update(cs)
    per = {}
    for k, cs in c.items():
        d = {n: round(v / NC, 1) for n, v in sorted(cs.items())}
        if "FETCH_SIZE" in cs:
            d["fetch_mb_x1"] = round(cs["FETCH_SIZE"] * 1024 / NC / 1e6, 3)
        if "WRITE_SIZE" in cs:
            d["write_mb"] = round(cs["WRITE_SIZE"] * 1024 / NC / 1e6, 3)
        if cs.get("SQ_WAVE_CYCLES"):
            d["issue_frac"] = round(cs["SQ_ACTIVE_INST_ANY"] / cs["SQ_WAVE_CYCLES"], 3)
            d["wait_frac"] = round(cs["SQ_WAIT_ANY"] / cs["SQ_WAVE_CYCLES"], 3)
        per[k] = d
    rc = {"workload": "tools/betti_rc10.py 32 1: 32 FCC-256 structures at rc 10 (8,192 complexes of ~340 points, one slice)",
          "kernel_ms": {k: [round(x, 3) for x in v] for k, v in tr.items() if max(v) > 1.0},
          "per_complex": per,
          "note": ("walk = betti_walk_kernel (one 1,024-thread workgroup per complex: the u16 code triangle and the "
                   "adjacency bitsets in LDS; forest, dim-1 pass, dim-2 apparent walk); reduce = "
                   "betti_wide_kernel_c16<6, true> (no LDS, 8 waves per SIMD: the reductions, statistics, outputs). "
                   "FETCH_SIZE / WRITE_SIZE in KB (x1: the x2 gfx950 read correction is calibrated for streaming "
                   "reads); round 5's per-wave kernel: FETCH 83.2 MB x1 and WRITE 25.5 MB per complex, "
                   "profiles/r05_rc10_wide.json")}
    json.dump(rc, open(os.path.join(HERE, "r06_rc10.json"), "w"), indent=1)
    side = {"hip_events_us_per_batch": {}}
    for line in open(os.path.join(D, "side.log")):
        if line.startswith("config"):
            name, js = line.split(" ", 1)
            side["hip_events_us_per_batch"][name] = json.loads(js)
    st = trace("side")
    side["trace_median_ms"] = {k: round(statistics.median(v), 4) for k, v in st.items()}
    side["note"] = ("tools/side_graph.py 20 under rocprofv3: config 2 = 1,024 x SC-64 graph only, config 5 = one "
                    "4,096-atom SC supercell graph only; f32 and f64 RBF runs in one trace (medians over both)")
    json.dump(side, open(os.path.join(HERE, "r06_side_graph.json"), "w"), indent=1)
    print(json.dumps(rc, indent=1)[:3000])


if __name__ == "__main__":
    main()
