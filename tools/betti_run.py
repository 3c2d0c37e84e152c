"""Minimal Betti workload for profiling: python tools/betti_run.py [kind] [m] [B] [rc] [reps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "defect-gnn-cpp_amd", "python")]
import dgn  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "fcc"
m = int(sys.argv[2]) if len(sys.argv) > 2 else 4
B = int(sys.argv[3]) if len(sys.argv) > 3 else 2048
rc = float(sys.argv[4]) if len(sys.argv) > 4 else 5.0
reps = int(sys.argv[5]) if len(sys.argv) > 5 else 2
ctx = dgn.Context(0)
batch = dgn.synth_batch(kind, m, B)
for r in range(reps):
    t0 = time.perf_counter()
    ctx.host_betti(batch, rc)
    print(f"rep {r}: {time.perf_counter() - t0:.4f} s", flush=True)
