"""Round-5 evidence beside parse_profiles.py (bench trace + path PMC): folds profiles/collect_r05.sh's
output (and the round's narrow-kernel A/B counter runs) into committed summaries.
    python profiles/summarize_r05.py [gpurun_out/prof_r05a]
Writes (profiles/):
  r05_narrow_sq.txt / r05_narrow_mem.txt   per-kernel PMC of the narrow Betti kernels (2,048 FCC-256 at 5 A)
  r05_narrow_before_after.json             narrow kernels per complex: round 4 (f32 LDS matrix, NP 44 + 48 tiers)
                                           -> u16 rank codes at 6 and 8 waves per SIMD (1,024 FCC-256 at 5 A,
                                           tools/pmc_betti.sh; gpurun_out/g4, g8)
  r05_dist.json                            distance kernel SQ counters (f64 VALU pairs) + derived rates
  r05_rc10_wide.json                       the 10 A wide kernel: time, HBM bytes and SQ mix per complex
  r05_side_graph.json                      per-kernel medians of BASELINE configs 2 and 5 (f32 / f64 RBF)
SQ cycle counters are in quad-cycles (MI355X_MICROARCH.md); instruction counters per wave instruction.
"""
import collections
import csv
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
D = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(HERE), "gpurun_out", "prof_r05a")
CLOCK_GHZ = 2.4
SIMDS = 1024


def rows(sub):
    out = []
    for p in sorted(glob.glob(os.path.join(D, sub, "**", "*counter_collection.csv"), recursive=True)):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def per_kernel(sub, want=None):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in rows(sub):
        name = r["Kernel_Name"]
        name = name[:name.rfind("(")] if name.endswith(")") else name
        if want and want not in name:
            continue
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def pmc_text(sub, path):
    with open(path, "w") as f:
        for k, cs in sorted(per_kernel(sub).items()):
            if "betti_kernel" not in k:
                continue
            f.write(f"{k}\n")
            for c, v in sorted(cs.items()):
                f.write(f"    {c:32s} {v:18.1f}\n")


def parse_txt(path):
    out, cur = {}, None
    for line in open(path):
        if not line.startswith(" "):
            cur = line.strip()
            out[cur] = {}
        elif cur:
            p = line.split()
            out[cur][p[0]] = float(p[1])
    return out




def narrow_before_after():
    global D
    g = os.path.join(os.path.dirname(D))
    runs = {"r04_f32_np44_np48": os.path.join(g, "g4", "pmc_r04"), "r05_codes_6waves": os.path.join(g, "g4", "pmc_new"),
            "r05_codes_8waves": os.path.join(g, "g8", "pmc")}
    nc = 1024 * 256
    out = {"workload": "tools/betti_run.py fcc 4 1024 5.0 1 (1,024 FCC-256 structures at 5 A: 262,144 complexes); "
                       "counters summed over the narrow launches (r04: betti_kernel<44> + <48>; r05: betti_kernel<48>, "
                       "and the empty dense launch betti_kernel<64>), per complex", "per_complex": {}}
    keep = D
    for tag, d in runs.items():
        if not os.path.isdir(d):
            continue
        D = os.path.dirname(d)
        sub = os.path.basename(d)
        tot = collections.defaultdict(float)
        for k, cs in per_kernel(sub).items():
            if "betti_kernel<" in k:
                for c, v in cs.items():
                    tot[c] += v
        out["per_complex"][tag] = {c: round(v / nc, 1) for c, v in sorted(tot.items())}
    D = keep
    json.dump(out, open(os.path.join(HERE, "r05_narrow_before_after.json"), "w"), indent=1)


def main():
    pmc_text("narrow_sq1", os.path.join(HERE, "r05_narrow_sq.txt"))
    with open(os.path.join(HERE, "r05_narrow_sq.txt"), "a") as f:
        for k, cs in sorted(per_kernel("narrow_sq2").items()):
            if "betti_kernel" in k:
                f.write(f"{k} (pass 2)\n")
                for c, v in sorted(cs.items()):
                    f.write(f"    {c:32s} {v:18.1f}\n")
    pmc_text("narrow_mem", os.path.join(HERE, "r05_narrow_mem.txt"))
    narrow_before_after()
    # SQ counters of the distance kernel (betti_dist_search_kernel<64>), durations from the bench trace
    m = per_kernel("dist").get("void dgn::betti_dist_search_kernel<64>", {})
    summ = json.load(open(os.path.join(HERE, "r05_summary.json")))
    dur = summ["trace_launch_ms"]["betti_dist_search_kernel"]
    ms = sum(dur) / len(dur)
    nc = 8192 * 256
    mf = {"kernel": "betti_dist_search_kernel<64> (config-4 shard: 2,097,152 local complexes of <= 64 points)",
          "counters_per_launch": m, "avg_launch_ms": round(ms, 4),
          "per_complex": {c: round(v / nc, 1) for c, v in m.items()},
          "issue_frac": round(m["SQ_ACTIVE_INST_ANY"] / m["SQ_WAVE_CYCLES"], 3) if m.get("SQ_WAVE_CYCLES") else None,
          "useful": summ["trace_bench"].get("roofline_dist"),
          "note": "one packed pair per lane on the f64 VALU (Gram arithmetic in the reference's order, lean f64 "
                  "square root); SQ cycle counters in quad-cycles"}
    json.dump(mf, open(os.path.join(HERE, "r05_dist.json"), "w"), indent=1)

    # the 10 A wide kernel (tools/betti_rc10.py 16 1: 4,096 complexes)
    nc = 4096
    wide = {}
    for sub in ("wide_fetch", "wide_write", "wide_sq1", "wide_sq2"):
        for r in rows(sub):
            # the u16-code wide launch (the device-driven retry launch beside it is empty here)
            if "betti_wide_kernel_c16" in r["Kernel_Name"]:
                wide[r["Counter_Name"]] = wide.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    st = {}
    p = glob.glob(os.path.join(D, "wide_trace", "**", "*kernel_stats.csv"), recursive=True)
    if p:
        with open(p[0]) as f:
            st = {r["Name"][:90]: round(float(r["AverageNs"]) / 1e6, 3) for r in csv.DictReader(f)}
    rc = {"workload": "tools/betti_rc10.py 16 1: 16 FCC-256 structures at rc 10 (4,096 complexes of ~340 points)",
          "kernel_ms": st,
          "per_complex": {k: round(v / nc, 1) for k, v in wide.items()},
          "hbm_mb_per_complex": {"fetch_x1": round(wide.get("FETCH_SIZE", 0) * 1024 / nc / 1e6, 1),
                                 "fetch_x2": round(2 * wide.get("FETCH_SIZE", 0) * 1024 / nc / 1e6, 1),
                                 "write": round(wide.get("WRITE_SIZE", 0) * 1024 / nc / 1e6, 1)},
          "note": "FETCH_SIZE / WRITE_SIZE in KB; the x2 gfx950 correction is calibrated for 16-B-per-lane streaming "
                  "reads, these are 2-byte scattered reads (uncalibrated: both readings given)"}
    if wide.get("SQ_WAVE_CYCLES"):
        rc["issue_frac"] = round(wide["SQ_ACTIVE_INST_ANY"] / wide["SQ_WAVE_CYCLES"], 3)
        rc["wait_frac"] = round(wide["SQ_WAIT_ANY"] / wide["SQ_WAVE_CYCLES"], 3)
    json.dump(rc, open(os.path.join(HERE, "r05_rc10_wide.json"), "w"), indent=1)

    # BASELINE configs 2 and 5 (tools/side_graph.py 20 runs config2, config5 with the f32 RBF, then
    # both with f64, one after the other): dispatches in time order, a new phase whenever the
    # one-image count kernel's grid changes (config 2: 2,048 blocks, config 5: 1,024)
    tr = glob.glob(os.path.join(D, "side", "**", "*kernel_trace.csv"), recursive=True)
    if tr:
        rs = sorted(csv.DictReader(open(tr[0])), key=lambda r: int(r["Start_Timestamp"]))
        phases, cur, grid = [], None, None
        for r in rs:
            if "dgn::" not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("dgn::", "")
            if name == "graph_count_one_kernel" and r["Grid_Size_X"] != grid:
                grid = r["Grid_Size_X"]
                cur = collections.defaultdict(list)
                phases.append(cur)
            if cur is not None:
                cur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        out = {"config2": {}, "config5": {}}
        for (cfg, dt), ph in zip((("config2", "f32"), ("config5", "f32"), ("config2", "f64"), ("config5", "f64")), phases):
            med = {k: round(sorted(v)[len(v) // 2], 2) for k, v in ph.items()}
            med["path_us"] = round(sum(med.values()), 1)
            out[cfg][dt] = med
        out["note"] = ("median kernel durations (us) per dispatch, rocprofv3 --kernel-trace of tools/side_graph.py 20; "
                       "config 2 = 1,024 SC-64 cells (grid 2,048 blocks; cells narrower than 2 rc: the few-image search), "
                       "config 5 = one 4,096-atom SC supercell (1,024 blocks of 4 atoms; cell list); graph rc 5, K 20, 50-bin RBF")
        json.dump(out, open(os.path.join(HERE, "r05_side_graph.json"), "w"), indent=1)




if __name__ == "__main__":
    main()
