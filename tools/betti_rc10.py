"""Time the Betti path at the reference default 10 A cutoff (wide kernel) on FCC-256 structures:
python tools/betti_rc10.py [B] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "defect-gnn-cpp_amd", "python")]
import dgn  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ctx = dgn.Context(0)
# A/B knobs for this tool only (the library never reads the environment)
if os.environ.get("DGN_WIDE_WAVES"):
    ctx.set_debug(dgn.abi.DEBUG_WIDE_WAVES, int(os.environ["DGN_WIDE_WAVES"]))
if os.environ.get("DGN_WIDE_C16"):
    ctx.set_debug(dgn.abi.DEBUG_WIDE_C16, int(os.environ["DGN_WIDE_C16"]))
if os.environ.get("DGN_WIDE_WALK"):
    ctx.set_debug(dgn.abi.DEBUG_WIDE_WALK, int(os.environ["DGN_WIDE_WALK"]))
batch = dgn.synth_batch("fcc", 4, B)
for r in range(reps):
    ctx.reset_timing()
    ctx.enable_timing(True)
    t0 = time.perf_counter()
    f, c = ctx.host_betti(batch, 10.0)
    dt = time.perf_counter() - t0
    kt = ctx.kernel_times()
    ctx.enable_timing(False)
    print(f"rep {r}: {B} structures ({B * 256} complexes, max n {int(c.sum(1).max())}) {dt:.3f} s "
          f"= {B / dt:.1f} structures/s; " + ", ".join(f"{k} {v['total_ms']:.1f} ms" for k, v in kt.items()), flush=True)
