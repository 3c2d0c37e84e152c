"""Debug: run count + emit on growing FCC batches and report the deferred emit flag."""
import sys, os
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "defect-gnn-cpp_amd", "python")]
import numpy as np, torch
import dgn
from dgn import abi
ctx = dgn.Context(0)
for B in [int(x) for x in sys.argv[1:]]:
    host = dgn.synth_batch("fcc", 4, B)
    batch = {k: torch.from_numpy(v).cuda() for k, v in host.items()}
    if os.environ.get("DBG_SYNC"):
        torch.cuda.synchronize()
    gp = abi.graph_params(r_cutoff=5.0, max_neighbors=20, rbf_cutoff=5.0, rbf_dr=0.1, rbf_dtype=dgn.DGN_F32)
    E = ctx.dev_graph_count(batch, gp)
    A = host["positions"].shape[0]
    rp = torch.empty(A + 1, dtype=torch.int64, device="cuda"); col = torch.empty(E, dtype=torch.int32, device="cuda")
    dist = torch.empty(E, dtype=torch.float64, device="cuda"); rbf = torch.empty((E, 50), dtype=torch.float32, device="cuda")
    ctx.dev_graph_emit(batch, gp, rp, col, dist, None, rbf)
    try:
        ctx.synchronize(); print(B, "ok", E, flush=True)
    except Exception as e:
        print(B, "FAIL", e, flush=True)
