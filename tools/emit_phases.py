"""Diagnostics: per-phase s_memtime cycles of the graph emit (libdgn built with -DDGN_EMIT_PHASES).
    DGN_LIB=defect-gnn-cpp_amd/lib/libdgn_diag_ph.so python tools/emit_phases.py [reps] [kind m B]
    (default fcc 4 8192 = config 4; sc 4 1024 = config 2)"""
import ctypes as C
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "defect-gnn-cpp_amd", "python")]
import torch  # noqa: E402
import dgn  # noqa: E402
from dgn import abi  # noqa: E402

NAMES = ["setup", "stage+loop", "hits+exact", "rank+put", "rbf", "-", "-", "-"]
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
ctx = dgn.Context(0)
kind = sys.argv[2] if len(sys.argv) > 2 else "fcc"
m_, B_ = (int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (4, 8192)
host = dgn.synth_batch(kind, m_, B_)
batch = {k: torch.from_numpy(v).cuda() for k, v in host.items()}
gp = abi.graph_params(r_cutoff=5.0, max_neighbors=20, rbf_cutoff=5.0, rbf_dr=0.1, rbf_dtype=dgn.DGN_F32)
E = ctx.dev_graph_count(batch, gp)
A = host["positions"].shape[0]
rp = torch.empty(A + 1, dtype=torch.int64, device="cuda")
col = torch.empty(E, dtype=torch.int32, device="cuda")
dist = torch.empty(E, dtype=torch.float64, device="cuda")
rbf = torch.empty((E, 50), dtype=torch.float32, device="cuda")
fn = abi.lib().dgn_diag_emit_phases
fn.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
out = (C.c_ulonglong * 8)()
ctx.dev_graph_emit(batch, gp, rp, col, dist, None, rbf)
ctx.synchronize()
fn(out, 1)
ctx.enable_timing(True)
for _ in range(reps):
    ctx.dev_graph_count(batch, gp)
    ctx.dev_graph_emit(batch, gp, rp, col, dist, None, rbf)
ctx.synchronize()
fn(out, 0)
kt = ctx.kernel_times()
tot = sum(out)
print({k: round(v["total_ms"] / reps, 4) for k, v in kt.items()})
for i, n in enumerate(NAMES):
    if out[i]:
        print(f"{n:12s} {out[i] * 64 / reps / (A / 16):10.1f} cycles per wave per query (sampled 1/64 blocks)  {100 * out[i] / tot:5.1f}%")
