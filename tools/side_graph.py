"""Per-kernel times of the small-batch graph side lines (BASELINE configs 2 and 5):
python tools/side_graph.py [reps]  -- prints kernel_times() per config (HIP events on the launch
stream); run under rocprofv3 --kernel-trace --stats for the trace."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "defect-gnn-cpp_amd", "python")]
import torch  # noqa: E402
import dgn  # noqa: E402
from dgn import abi  # noqa: E402
from dgn.shard import Shard  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
ctx = dgn.Context(0)
ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
nb = abi.lib().dgn_rbf_bins(5.0, 0.1)
out = {}
for name, kind, m, B, dt in (("config2", "sc", 4, 1024, "f32"), ("config5", "sc", 16, 1, "f32"),
                             ("config2_f64", "sc", 4, 1024, "f64"), ("config5_f64", "sc", 16, 1, "f64")):
    gp = abi.graph_params(r_cutoff=5.0, max_neighbors=20, rbf_cutoff=5.0, rbf_dr=0.1,
                          rbf_dtype=dgn.DGN_F64 if dt == "f64" else dgn.DGN_F32)
    sh = Shard(dgn, abi, kind, m, B, 0, dev)
    sh.alloc_graph(ctx, gp, nb, torch.float64 if dt == "f64" else torch.float32)
    sh.step(ctx, gp, 5.0, betti=False)
    torch.cuda.synchronize(dev)
    ctx.reset_timing()
    ctx.enable_timing(True)
    for _ in range(reps):
        sh.step(ctx, gp, 5.0, betti=False)
    torch.cuda.synchronize(dev)
    kt = ctx.kernel_times()
    ctx.enable_timing(False)
    out[name] = {"atoms": sh.A, "edges": sh.E, **{k: round(v["total_ms"] / reps * 1e3, 2) for k, v in kt.items()}}
    print(name, json.dumps(out[name]), flush=True)
    del sh
