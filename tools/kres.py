"""Per-kernel register / LDS / occupancy summary of one HIP source (hipcc -Rpass-analysis).
    python tools/kres.py defect-gnn-cpp_amd/csrc/graph_kernels.hip [extra hipcc flags]"""
import re
import subprocess
import sys

src = sys.argv[1]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Wall",
       "-Idefect-gnn-cpp_amd/csrc", "-Iinclude", "-Rpass-analysis=kernel-resource-usage", "-c", src, "-o", "/tmp/kres.o"]
cmd += sys.argv[2:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    if "error" in line or ("warning" in line and "remark" not in line):
        print(line)
    m = re.search(r"remark:\s*(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k.split()[0]] = v
for r in rows:
    n = r["name"]
    n = re.sub(r"^_ZN3dgn\d+", "", n)[:60]
    print(f"{n:62s} vgpr={r.get('VGPRs')} agpr={r.get('AGPRs')} scratch={r.get('ScratchSize')} occ={r.get('Occupancy')} lds={r.get('LDS')}")
