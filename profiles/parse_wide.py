"""Fold profiles/collect_wide.sh output into profiles/<round>_wide_rc10.json: the wide Betti
kernel's duration (kernel trace), HBM bytes (FETCH_SIZE / WRITE_SIZE passes; the gfx950 FETCH
correction of MI355X_MICROARCH.md: x2) and SQ instruction mix, per complex.
    python3 profiles/parse_wide.py --round r02 --dir gpurun_out/wide_r02 [--complexes 8192]"""
import argparse
import csv
import json
import os

ap = argparse.ArgumentParser()
ap.add_argument("--round", default="r02")
ap.add_argument("--dir", required=True)
ap.add_argument("--complexes", type=int, default=8192)
a = ap.parse_args()
KEY = "betti_wide_kernel"


def counters(sub):
    out = {}
    path = os.path.join(a.dir, sub, "run_counter_collection.csv")
    for r in csv.DictReader(open(path)):
        if KEY in r["Kernel_Name"]:
            out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            out["_vgpr"] = int(r["VGPR_Count"])
            out["_lds"] = int(r["LDS_Block_Size"])
    return out


stats = {}
for r in csv.DictReader(open(os.path.join(a.dir, "trace", "run_kernel_stats.csv"))):
    stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "percent": float(r["Percentage"])}
wide = {k: v for k, v in stats.items() if KEY in k}
dur_ns = sum(v["avg_ns"] * v["calls"] for v in wide.values())
f, w = counters("fetch"), counters("write")
s1, s2 = counters("sq1"), counters("sq2")
C = a.complexes
fetch_b = 2 * f.get("FETCH_SIZE", 0.0) * 1024  # KB, doubled (gfx950 correction)
write_b = w.get("WRITE_SIZE", 0.0) * 1024
res = {
    "round": a.round, "workload": f"{C} FCC-256 local complexes at rc 10 (~340 points), one wide launch",
    "kernel": list(wide), "duration_ms": dur_ns / 1e6, "complexes_per_s": C / (dur_ns * 1e-9),
    "vgpr": s1.get("_vgpr"), "lds_bytes_per_wave": s1.get("_lds"),
    "hbm_bytes_per_complex": (fetch_b + write_b) / C, "hbm_gbs": (fetch_b + write_b) / (dur_ns * 1e-9) / 1e9,
    "per_complex": {k: v / C for k, v in {**s1, **s2}.items() if not k.startswith("_")},
    "issue_fraction": s1.get("SQ_ACTIVE_INST_ANY", 0) / max(s1.get("SQ_WAVE_CYCLES", 1), 1),
    "wait_fraction": s1.get("SQ_WAIT_ANY", 0) / max(s1.get("SQ_WAVE_CYCLES", 1), 1),
    "kernel_stats": stats,
}
json.dump(res, open(os.path.join(os.path.dirname(os.path.abspath(__file__)), f"{a.round}_wide_rc10.json"), "w"), indent=1)
print(json.dumps({k: v for k, v in res.items() if k != "kernel_stats"}, indent=1))
