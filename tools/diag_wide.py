"""Diagnostics: phase breakdown of the wide Betti kernel (libdgn_diag.so) at the default 10 A cutoff.
Usage: python tools/diag_wide.py [B]"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("DGN_LIB", os.path.join(ROOT, "defect-gnn-cpp_amd", "lib", "libdgn_diag.so"))
sys.path[:0] = [os.path.join(ROOT, "defect-gnn-cpp_amd", "python")]
import dgn  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 2
ctx = dgn.Context(0)
batch = dgn.synth_batch("fcc", 4, B)
A = batch["positions"].shape[0]
t0 = time.perf_counter()
f, c = ctx.host_betti(batch, 10.0)
dt = time.perf_counter() - t0
ph = (C.c_ulonglong * 32)()
dgn.lib().dgn_diag_phase_cycles(ctx.h, ph)
ph = list(ph)
names = ["load", "prim+edges", "dim1 apparent", "dim1 reduce", "dim2 apparent", "dim2 reduce", "stats"]
tot = sum(ph[:7])
print(json.dumps({"complexes": A, "s": round(dt, 3), "cycles_per_complex": round(tot / A),
                  "phase_share": {n: round(ph[i] / tot, 4) for i, n in enumerate(names)},
                  "edges": ph[10] / A, "na1": ph[8] / A, "na2": ph[9] / A,
                  "reduce_sub_cycles_per_complex": {n: round(ph[16 + i] / A) for i, n in enumerate(
                      ["sort", "hfind", "apparent_owner", "toggles", "pivot_of_V", "finalize"])},
                  "adds_per_complex": ph[24] / A, "reduced_columns_per_complex": ph[22] / A,
                  "dim2_walk": {"columns_walked": ph[28] / A, "mean_steps": ph[26] / max(ph[28], 1),
                                "wave_iterations_per_complex": ph[27] / A,
                                "lane_efficiency": ph[26] / max(64 * ph[27], 1)}, "mean_V_per_pivot_search": ph[25] / max(ph[24], 1),
                  "pivot_searches_per_complex": ph[29] / A, "floor_rounds_per_search": ph[30] / max(ph[29], 1)}, indent=1))
