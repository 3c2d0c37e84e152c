"""Per-dispatch kernel durations from a rocprofv3 rocpd database (default output format):
python tools/rpd_kernels.py <results.db> [min_ms]"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
mn = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
for name, dur, gx, wx, lds in db.execute("select name, duration, grid_x, workgroup_x, lds_size from kernels order by start"):
    if dur / 1e6 >= mn:
        print(f"{dur / 1e6:10.3f} ms  grid {gx:>9} wg {wx:>5} lds {lds:>7}  {name[:90]}")
