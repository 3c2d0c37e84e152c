"""Diagnostics: time the neighbour count pass alone on the config-4 shard (8,192 x FCC-256, rc 5),
for A/B builds of the count kernels (DGN_LIB=...; -DDGN_COUNT1_PROBE builds give wrong counts and
are never used by tests or the bench). python tools/count_probe.py [reps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "defect-gnn-cpp_amd", "python")]
import torch  # noqa: E402
import dgn  # noqa: E402
from dgn import abi  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
ctx = dgn.Context(0)
ctx.set_stream(torch.cuda.current_stream(dev).cuda_stream)
host = dgn.synth_batch("fcc", 4, 8192)
batch = {k: torch.from_numpy(v).to(dev) for k, v in host.items()}
gp = abi.graph_params(r_cutoff=5.0, max_neighbors=20, rbf_cutoff=5.0, rbf_dr=0.1, rbf_dtype=dgn.DGN_F64)
ctx.dev_graph_count(batch, gp)
torch.cuda.synchronize(dev)
ctx.reset_timing()
ctx.enable_timing(True)
for _ in range(reps):
    ctx.dev_graph_count(batch, gp)
torch.cuda.synchronize(dev)
kt = ctx.kernel_times()
print(json.dumps({"lib": os.path.basename(os.environ.get("DGN_LIB", "libdgn.so")),
                  **{k: round(v["total_ms"] / reps, 4) for k, v in kt.items()}}), flush=True)
