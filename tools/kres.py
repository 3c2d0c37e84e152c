"""Per-kernel register / spill / LDS / occupancy summary of HIP sources (hipcc -Rpass-analysis),
compiled with the product flags (Makefile HIPFLAGS).
    python tools/kres.py defect-gnn-cpp_amd/csrc/*.hip [-- extra hipcc flags]"""
import re
import subprocess
import sys

args = sys.argv[1:]
extra = []
if "--" in args:
    i = args.index("--")
    args, extra = args[:i], args[i + 1:]
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-Idefect-gnn-cpp_amd/csrc",
         "-Iinclude", "-mllvm", "-amdgpu-atomic-optimizer-strategy=DPP", "-Rpass-analysis=kernel-resource-usage"]
KEYS = {"TotalSGPRs": "sgpr", "VGPRs": "vgpr", "AGPRs": "agpr", "ScratchSize [bytes/lane]": "scratch",
        "Occupancy [waves/SIMD]": "occ", "SGPRs Spill": "sgpr_spill", "VGPRs Spill": "vgpr_spill",
        "LDS Size [bytes/block]": "lds"}
print(f"{'kernel':70s} {'vgpr':>5s} {'sgpr':>5s} {'vspill':>6s} {'sspill':>6s} {'scratch':>7s} {'lds':>7s} {'occ':>4s}")
# per-source flags of the Makefile
PER_SRC = {"betti_kernels.hip": ["-mllvm", "-amdgpu-sched-strategy=iterative-minreg"]}
for src in args:
    cmd = ["/opt/rocm/bin/hipcc"] + FLAGS + PER_SRC.get(src.split("/")[-1], []) + extra + ["-c", src, "-o", "/tmp/kres.o"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        if " error:" in line:
            print(line)
        m = re.search(r"remark:\s*(Function Name|" + "|".join(re.escape(k) for k in KEYS) + r"): (\S+)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[KEYS[k]] = v
    print(f"# {src}")
    for r in rows:
        if "rocprim" in r["name"]:
            continue  # the library's sort kernels (betti_rank.hip instantiates them)
        n = re.sub(r"^_ZN3dgn(12_GLOBAL__N_1)?\d+", "", r["name"])[:70]
        print(f"{n:70s} {r.get('vgpr', ''):>5s} {r.get('sgpr', ''):>5s} {r.get('vgpr_spill', '0'):>6s} "
              f"{r.get('sgpr_spill', '0'):>6s} {r.get('scratch', ''):>7s} {r.get('lds', ''):>7s} {r.get('occ', ''):>4s}")
