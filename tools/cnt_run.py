"""Per-complex reduction counters of an instrumented narrow-kernel build (tools only)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "defect-gnn-cpp_amd", "python")]
import numpy as np  # noqa: E402
import dgn  # noqa: E402
ctx = dgn.Context(0)
b = dgn.synth_batch("fcc", 4, 64)
f, c = ctx.host_betti(b, 5.0)
c = np.asarray(c, dtype=np.int64)
print("complexes", len(c), "per complex: stored-list toggles %.1f, lazy/apparent toggles %.1f, pivot searches %.1f, V entries scanned %.1f" % tuple(c.mean(0)))
