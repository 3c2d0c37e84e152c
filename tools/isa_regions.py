"""ISA instruction mix per code region of the narrow Betti kernel (CPU only, no GPU):
inserts `; MARK_*` asm comments at fixed anchors into a copy of the sources, compiles with
--save-temps and counts instructions between consecutive markers of betti_kernel<NP>.
    ISA_NP=44 python tools/isa_regions.py [outdir]"""
import collections
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.environ.get("ISA_CSRC") or os.path.join(ROOT, "defect-gnn-cpp_amd", "csrc")
MARKS = [
    ("        for (int ci = 0; ci < nna; ++ci) {\n", "COL_TOP", True),
    ("            int owner = (int)uni((uint32_t)find_pivot(npiv, tau));\n", "AFTER_FIND", True),
    ("            int v = 0;  // 0 = lazy: V == {this column}\n", "AFTER_APP", True),
    ("                    tau = uni64(v > 0 ? pivot_of_V(dim, v, tau) : kInf);\n", "PIV", False),
    ("                    tau = uni64(v > 0 ? pivot_of_V(dim, v, tau) : kInf);\n", "AFTER_PIV", True),
    ("            // ---- tau is the pivot of this column ----\n", "FINAL", True),
    ("            npiv = (int)uni((uint32_t)(npiv + 1));\n            lds_sync();\n", "FINAL_END", True),
]


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "/tmp/isa_regions"
    shutil.rmtree(out, ignore_errors=True)
    os.makedirs(out)
    for f in os.listdir(CSRC):
        shutil.copy(os.path.join(CSRC, f), out)
    p = os.path.join(out, "betti_kernels.hip")
    s = open(p).read()
    for anchor, name, after in MARKS:
        assert anchor in s, name
        m = f'asm volatile("; MARK_{name}");\n'
        s = s.replace(anchor, anchor + m if after else m + anchor, 1)
    open(p, "w").write(s)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                    "-I" + out, "-I" + os.path.join(ROOT, "include"), "-mllvm", "-amdgpu-sched-strategy=iterative-minreg", "--save-temps", "-c", p, "-o",
                    os.path.join(out, "bk.o")], cwd=out, check=True, capture_output=True)
    asm = open(os.path.join(out, "betti_kernels-hip-amdgcn-amd-amdhsa-gfx950.s")).read().split("\n")
    np_ = os.environ.get("ISA_NP", "48")  # instantiation: 32, 44, 48 or 64
    start = next(i for i, l in enumerate(asm) if l.startswith(f"_ZN3dgn12betti_kernelILi{np_}EEEvNS_11BettiLaunchE:"))
    end = next(i for i in range(start, len(asm)) if asm[i].startswith(".Lfunc_end") )
    region, counts = "ENTRY", collections.defaultdict(collections.Counter)
    for l in asm[start:end]:
        m = re.search(r"MARK_(\w+)", l)
        if m:
            region = m.group(1) + ("#2" if (m.group(1) + "#1") in counts else "#1")
            continue
        t = l.strip().split()
        if not t or t[0].startswith((";", ".")) or t[0].endswith(":"):
            continue
        op = t[0]
        cls = ("branch" if op.startswith("s_cbranch") or op == "s_branch" else "waitcnt" if op == "s_waitcnt" else
               "salu" if op.startswith("s_") else "lds" if op.startswith("ds_") else
               "scratch" if op.startswith("scratch_") else
               "vmem" if op.startswith(("global_", "buffer_", "flat_")) else "valu" if op.startswith("v_") else "other")
        counts[region][cls] += 1
    for r, c in counts.items():
        print(f"{r:14s} " + " ".join(f"{k}={c[k]}" for k in ("valu", "salu", "branch", "lds", "vmem", "scratch", "waitcnt")))
    for l in asm:
        if "NumVgprs:" in l or "ScratchSize:" in l:
            pass
    vg = [l for l in asm[end:end + 40] if "NumVgprs" in l or "ScratchSize" in l or "Occupancy" in l]
    print("\n".join(vg))


if __name__ == "__main__":
    main()
