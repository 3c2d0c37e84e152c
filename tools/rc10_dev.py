"""10 A Betti through the device entry (dgn_dev_betti, as bench.py's side line) and the host entry
(dgn_host_betti, as tools/betti_rc10.py) in one fresh process: python tools/rc10_dev.py [B] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "defect-gnn-cpp_amd", "python")]
import torch  # noqa: E402
import dgn  # noqa: E402
from dgn import abi  # noqa: E402
from dgn.shard import Shard  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 128
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
dev = torch.device("cuda:0")
ctx = dgn.Context(0)
if os.environ.get("DGN_WIDE_CAP"):  # A/B knob for this tool only
    ctx.set_debug(abi.DEBUG_WIDE_CAP, int(os.environ["DGN_WIDE_CAP"]))
if os.environ.get("PRE_HEADLINE"):  # the bench's config-4 shard (graph + Betti at rc 5) first, kept alive
    head = Shard(dgn, abi, "fcc", 4, 8192, 0, dev)
    gp = abi.graph_params(r_cutoff=5.0, max_neighbors=20, rbf_cutoff=5.0, rbf_dr=0.1, rbf_dtype=dgn.DGN_F64)
    head.alloc_graph(ctx, gp, abi.lib().dgn_rbf_bins(5.0, 0.1), torch.float64)
    head.alloc_betti()
    for _ in range(3):
        head.step(ctx, gp, 5.0)
    torch.cuda.synchronize(dev)
    f, t = torch.cuda.mem_get_info(dev)
    print(f"headline shard done; free {f / 2**30:.1f} of {t / 2**30:.1f} GiB", flush=True)
if os.environ.get("PRE_B"):  # a smaller batch through the same context first (bench.py's side-line order)
    pre = Shard(dgn, abi, "fcc", 4, int(os.environ["PRE_B"]), 0, dev)
    pre.alloc_betti()
    for _ in range(2):
        ctx.dev_betti(pre.batch, 10.0, pre.out["feat"], pre.out["counts"])
    torch.cuda.synchronize(dev)
    del pre
sh = Shard(dgn, abi, "fcc", 4, B, 0, dev)
sh.alloc_betti()
for r in range(reps + 1):
    torch.cuda.synchronize(dev)
    ctx.reset_timing()
    ctx.enable_timing(True)
    t0 = time.perf_counter()
    ctx.dev_betti(sh.batch, 10.0, sh.out["feat"], sh.out["counts"])
    torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    kt = ctx.kernel_times()
    ctx.enable_timing(False)
    print(f"dev rep {r}: {B / dt:.2f} structures/s; " + ", ".join(f"{k} {v['total_ms']:.1f}" for k, v in kt.items()), flush=True)
for r in range(reps):
    t0 = time.perf_counter()
    ctx.host_betti(sh.host, 10.0)
    dt = time.perf_counter() - t0
    print(f"host rep {r}: {B / dt:.2f} structures/s", flush=True)
