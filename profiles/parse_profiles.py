"""Fold one round's rocprofv3 output (profiles/collect.sh) into committed summaries:
  profiles/<round>_kernel_stats.csv   rocprofv3 --stats table of the default bench
  profiles/<round>_summary.json       per-kernel avg duration + PMC HBM bytes per launch of every
                                      neighbour-path kernel (prep, count, scan, emit) and their sum
  profiles/traffic_latest.json        what bench.py reads for roofline.traffic
HBM bytes per launch = 2 x FETCH_SIZE (gfx950 tallies 128-B read requests at 64 B,
MI355X_MICROARCH.md "HBM") + WRITE_SIZE (exact for wide streaming stores); FETCH/WRITE_SIZE are in KB.
"""
import argparse
import csv
import glob
import json
import os
import shutil

HERE = os.path.dirname(os.path.abspath(__file__))
# the neighbour + RBF path (bench.py roofline): prep_structures = prep_meta + prep_atoms
# (round 3: the count pass is graph_count_one_kernel + graph_count_kernel over the flagged tiles)
PATH_KERNELS = ("prep_meta_kernel", "prep_atoms_kernel", "graph_count_one_kernel", "graph_count_kernel", "block_scan_kernel",
                "graph_emit_kernel")


def find(d, pattern):
    hits = sorted(glob.glob(os.path.join(d, "**", pattern), recursive=True))
    return hits[-1] if hits else None


def pmc_per_launch(path, kernel_substr, counter):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel_substr in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--round", required=True)
    ap.add_argument("--dir", required=True)
    a = ap.parse_args()
    summary = {"round": a.round}
    stats = find(os.path.join(a.dir, "trace"), "*kernel_stats.csv")
    if stats:
        shutil.copy(stats, os.path.join(HERE, f"{a.round}_kernel_stats.csv"))
        with open(stats) as f:
            summary["kernel_stats"] = {r["Name"]: {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                                                   "total_ns": float(r["TotalDurationNs"]),
                                                   "percent": float(r["Percentage"])} for r in csv.DictReader(f)}
    # per-launch durations of the path kernels and the Betti kernels in dispatch order (the stats'
    # averages mix the timed full-shard launches with the bench's warm-up, parity and f32 side
    # launches; the bench's HIP-event averages cover the timed launches only)
    trace = find(os.path.join(a.dir, "trace"), "*kernel_trace.csv")
    if trace:
        launches = {}
        with open(trace) as f:
            for r in csv.DictReader(f):
                name = r["Kernel_Name"]
                for k in PATH_KERNELS + ("betti_dist_search_kernel", "betti_kernel<44>", "betti_kernel<48>", "betti_kernel<64>"):
                    if k in name:
                        ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
                        launches.setdefault(k, []).append(round(ms, 4))
        summary["trace_launch_ms"] = launches
    for name in ("trace_bench", "fetch_bench", "write_bench"):
        p = os.path.join(a.dir, f"{name}.json")
        if os.path.exists(p):
            lines = [l for l in open(p) if l.startswith("{")]
            if lines:
                summary[name] = json.loads(lines[-1])
    fetch = find(os.path.join(a.dir, "fetch"), "*counter_collection.csv")
    write = find(os.path.join(a.dir, "write"), "*counter_collection.csv")
    if fetch and write:
        per_kernel = {}
        for k in PATH_KERNELS:
            fv = pmc_per_launch(fetch, k, "FETCH_SIZE")
            wv = pmc_per_launch(write, k, "WRITE_SIZE")
            if fv and wv:
                f_kb = sum(fv) / len(fv)
                w_kb = sum(wv) / len(wv)
                per_kernel[k] = {"launches": len(fv), "fetch_kb": f_kb, "write_kb": w_kb,
                                 "hbm_bytes_per_launch": 2 * f_kb * 1024 + w_kb * 1024}
        if "graph_emit_kernel" in per_kernel:
            gb = summary.get("fetch_bench", {})
            cfg = gb.get("config", {})
            roof = summary.get("trace_bench", {}).get("roofline") or {}
            # must match bench.py's workload_key for the default run
            rbf = "f32" if "RBF 50xf32" in cfg.get("workload", "") else "f64"
            key = "fcc4x%d_rc5.0_k20_nb50_%s" % (cfg.get("structures_per_gpu", 0), rbf) if cfg else None
            path = sum(v["hbm_bytes_per_launch"] for v in per_kernel.values())
            summary["graph_path_pmc"] = {"per_kernel": per_kernel, "hbm_bytes_per_path": path,
                                         "algorithmic_bytes_per_path": roof.get("algorithmic_bytes_per_launch"),
                                         "workload_key": key}
            with open(os.path.join(HERE, "traffic_latest.json"), "w") as f:
                json.dump({"round": a.round, "workload_key": key, "hbm_bytes_per_path": path,
                           "hbm_bytes_per_emit": per_kernel["graph_emit_kernel"]["hbm_bytes_per_launch"],
                           "per_kernel": per_kernel, "source": f"profiles/{a.round}_summary.json"}, f, indent=1)
    with open(os.path.join(HERE, f"{a.round}_summary.json"), "w") as f:
        json.dump(summary, f, indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != "kernel_stats"}, indent=1)[:4000])


if __name__ == "__main__":
    main()
