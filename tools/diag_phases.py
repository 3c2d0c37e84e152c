"""Diagnostics: per-phase cycle breakdown of the Betti kernel (libdgn_diag.so, s_memtime stamps).
Usage: DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_diag.so python tools/diag_phases.py [kind] [m] [B] [rc]"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("DGN_LIB", os.path.join(ROOT, "defect-gnn-cpp_amd", "lib", "libdgn_diag.so"))
sys.path[:0] = [os.path.join(ROOT, "defect-gnn-cpp_amd", "python")]
import numpy as np  # noqa: E402

import dgn  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "fcc"
m = int(sys.argv[2]) if len(sys.argv) > 2 else 4
B = int(sys.argv[3]) if len(sys.argv) > 3 else 512
rc = float(sys.argv[4]) if len(sys.argv) > 4 else 5.0
ctx = dgn.Context(0)
batch = dgn.synth_batch(kind, m, B)
A = batch["positions"].shape[0]
ctx.host_betti(batch, rc)  # warm-up
ctx.reset_timing()
ctx.enable_timing(True)
t0 = time.perf_counter()
f, c = ctx.host_betti(batch, rc)
dt = time.perf_counter() - t0
kt = ctx.kernel_times()
ctx.enable_timing(False)
ph = (C.c_ulonglong * 32)()
dgn.lib().dgn_diag_phase_cycles(ctx.h, ph)
ph = list(ph)
names = ["load+gram", "adj+prim+edges", "dim1 apparent", "dim1 serial", "dim2 apparent", "dim2 serial",
         "stats+write", "dequeue/gap"]
sub = ["serial:sort", "serial:col-start", "serial:find_pivot", "serial:apparent_owner", "serial:toggles", "serial:pivot_of_V", "serial:finalize"]
tot = sum(ph[:8]) + sum(ph[16:23]) + ph[26]
out = {"kind": kind, "m": m, "B": B, "rc": rc, "atoms": A, "host_betti_s": round(dt, 4),
       "betti_vr_ms": round(kt.get("betti_vr", {}).get("total_ms", 0.0), 3),
       "cycles_per_complex": round(tot / A), "phase_cycles_per_complex": {n: round(ph[i] / A) for i, n in enumerate(names)},
       "phase_share": {n: round(ph[i] / tot, 4) for i, n in enumerate(names)},
       "na1_per_complex": ph[8] / A, "na2_per_complex": ph[9] / A, "adds1": ph[10] / A, "adds2": ph[11] / A,
       "spills_per_complex": ph[12] / A, "dim2_complexes": ph[13],
       "pivot_V_entries_per_complex": ph[14] / A, "pivot_V_sq_per_complex": ph[15] / A,
       "max_V": ph[23], "pivot_iters_per_complex": ph[24] / A, "pivot_iter_entries_per_complex": ph[25] / A,
       "trivial_columns_per_complex": ph[27] / A, "zero_columns_per_complex": ph[28] / A,
       "dim2_enumerate_cycles_per_complex": round(ph[26] / A),
       "dim2_walk_steps_per_complex": ph[29] / A, "dim2_rounds_per_complex": ph[31] / A,
       "dim2_walk_lane_efficiency": ph[29] / max(1, 64 * ph[30]), "serial_sub_cycles_per_complex": {n: round(ph[16 + i] / A) for i, n in enumerate(sub)}}
print(json.dumps(out, indent=1))
