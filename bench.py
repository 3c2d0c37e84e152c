#!/usr/bin/env python3
"""Bench: structures/sec (graph + Betti) on synthetic crystal batches, 1..8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--structures B] [...]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[3], one shard per GPU, weak scaling): every rank owns B = 8,192
jittered 256-atom FCC structures (structure ids [rank*B, (rank+1)*B)), inputs resident in HBM.
One step = the whole hot path over the shard through the C ABI (libdgn.so):
  graph : NeighborList(rc=5, K=20) + CrystalGraph edge RBF (rc=5, dr=0.1 -> 50 bins, f32)
  Betti : compute_structure_betti_features(rc=5): NeighborList(rc, inf) + per-atom local VR
          (Gram distances on MFMA, dim 0/1/2, Z/2) + 35 statistics (f64)
Shards are independent (no collective on the data path); the only collectives are the barrier
and the max-over-ranks of the timed region.
Rank 0 prints ONE JSON line (metric/unit from BASELINE.json) with a `roofline` object for the
neighbour+RBF emit kernel (HBM-bound; HIP events on the launch stream) and a `cpu_baseline`
timed on this host with the reference's verbatim vendored Ripser (oracle/_ref) on a bounded
sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "defect-gnn-cpp_amd", "python"), os.path.join(ROOT, "oracle")]

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_MFMA_PEAK_TFS = 78.6  # MI355X dense FP64 matrix (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--structures", type=int, default=8192, help="structures per GPU (weak scaling)")
    ap.add_argument("--kind", default="fcc", choices=["fcc", "sc"])
    ap.add_argument("--m", type=int, default=4)
    ap.add_argument("--rc", type=float, default=5.0)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--rbf-rc", type=float, default=5.0)
    ap.add_argument("--dr", type=float, default=0.1)
    ap.add_argument("--betti-rc", type=float, default=5.0)
    ap.add_argument("--no-betti", action="store_true", help="graph only (config 2 style)")
    ap.add_argument("--cpu-sample", type=int, default=128, help="structures in the CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="PMC-derived HBM bytes per emit launch (written by profiles/collect.sh)")
    return ap.parse_args()


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    import dgn
    from dgn import abi

    # ---- synthetic shard, resident in HBM ----
    B = args.structures
    host = dgn.synth_batch(args.kind, args.m, B, first_id=rank * B)
    batch = {k: torch.from_numpy(v).to(dev) for k, v in host.items()}
    A = int(host["positions"].shape[0])
    n_atoms = A // B

    ctx = dgn.Context(local)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    gp = abi.graph_params(r_cutoff=args.rc, max_neighbors=args.k, rbf_cutoff=args.rbf_rc, rbf_dr=args.dr,
                          rbf_dtype=dgn.DGN_F32)
    nbins = abi.lib().dgn_rbf_bins(args.rbf_rc, args.dr)
    E = ctx.dev_graph_count(batch, gp)
    out = {"row_ptr": torch.empty(A + 1, dtype=torch.int64, device=dev),
           "col": torch.empty(max(E, 1), dtype=torch.int32, device=dev),
           "dist": torch.empty(max(E, 1), dtype=torch.float64, device=dev),
           "rbf": torch.empty((max(E, 1), nbins), dtype=torch.float32, device=dev),
           "feat": torch.empty((A, 35), dtype=torch.float64, device=dev),
           "counts": torch.empty((A, 4), dtype=torch.int32, device=dev)}

    def step():
        e = ctx.dev_graph_count(batch, gp)
        assert e == E
        ctx.dev_graph_emit(batch, gp, out["row_ptr"], out["col"], out["dist"], None, out["rbf"])
        if not args.no_betti:
            ctx.dev_betti(batch, args.betti_rc, out["feat"], out["counts"])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ctx.reset_timing()
    ctx.enable_timing(True)

    # ---- timed region: barrier + sync on both sides, max over ranks ----
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ktimes = ctx.kernel_times()
    ctx.enable_timing(False)

    # sanity: no NaN features (NaN marks a complex outside the kernel envelope)
    if not args.no_betti:
        bad = int(torch.isnan(out["feat"]).any(dim=1).sum().item())
        if bad:
            raise SystemExit(f"rank {rank}: {bad} atoms with NaN features")

    total_structures = B * world * args.steps
    value = total_structures / elapsed

    emit = ktimes.get("graph_emit", {})
    roof = None
    if emit.get("launches"):
        avg_s = emit["total_ms"] / emit["launches"] / 1e3
        bytes_per_launch = emit["bytes"] / emit["launches"]
        achieved = bytes_per_launch / avg_s / 1e9
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                tj = json.load(open(args.traffic_json))
                if tj.get("workload_key") == f"{args.kind}{args.m}x{B}_rc{args.rc}_k{args.k}_nb{nbins}":
                    traffic = tj.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        roof = {"bound": "hbm", "kernel": "graph_emit", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "algorithmic_bytes_per_launch": int(bytes_per_launch), "avg_launch_ms": round(avg_s * 1e3, 4)}
    dk = ktimes.get("betti_dist", {})
    mfma = None
    if dk.get("launches") and dk["total_ms"] > 0:
        dk_s = dk["total_ms"] / dk["launches"] / 1e3
        tfs = dk["flops"] / dk["launches"] / dk_s / 1e12
        gbs = dk["bytes"] / dk["launches"] / dk_s / 1e9
        mfma = {"bound": "mfma", "kernel": "betti_dist (f64 MFMA Gram product -> f32 triangles)", "achieved": round(tfs, 6),
                "peak": FP64_MFMA_PEAK_TFS, "unit": "TFLOP/s", "frac": tfs / FP64_MFMA_PEAK_TFS,
                "hbm_achieved_gbs": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
                "note": "useful 6n^2 flops per local complex (K=3 Gram); the kernel is bound by its triangle writes"}
    step_ms = elapsed / args.steps * 1e3
    kernel_ms = {k: round(v["total_ms"] / args.steps, 3) for k, v in ktimes.items()}

    result = {
        "metric": "structures/sec (graph+Betti) at 1/2/4/8 MI355X; HBM GB/s vs peak",
        "value": round(value, 2), "unit": "structures/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_ms, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": (f"config4 shard: {B} x {n_atoms}-atom jittered {args.kind.upper()} per GPU; "
                                f"graph rc={args.rc} K={args.k} RBF {nbins}xf32"
                                + ("" if args.no_betti else f" + Betti-0/1/2 rc={args.betti_rc}")),
                   "structures_per_gpu": B, "atoms_per_structure": n_atoms, "edges_per_gpu": E,
                   "parallelism": f"shard{world}"},
        "roofline": roof,
        "roofline_mfma": mfma,
        "kernel_ms_per_step": kernel_ms,
    }

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args, host, n_atoms)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline(args, host, n_atoms):
    """Reference CPU path on this host: restated neighbour list + RBF (nanoflann/Eigen absent
    offline) and the reference's VERBATIM vendored Ripser for the topology (oracle/_ref),
    OpenMP over atoms x 1 Ripser thread, on the first `cpu_sample` structures of the shard."""
    import numpy as np
    import oracle_py as O
    if not O.ref_available():
        return {"value": None, "unit": "structures/s", "cores": 0, "kind": "reference",
                "sample": "oracle/_ref/libdgn_ref.so not built"}
    S = args.cpu_sample
    t0 = time.perf_counter()
    for s in range(S):
        sl = slice(s * n_atoms, (s + 1) * n_atoms)
        lat, pos, sp = host["lattice"][s], host["positions"][sl], host["species"][sl]
        O.structure_graph(lat, pos, args.rc, args.k, args.rbf_rc, args.dr)
        if not args.no_betti:
            O.ref_structure_betti(lat, pos, sp, args.betti_rc, omp_threads=args.cpu_threads, ripser_threads=1)
    dt = time.perf_counter() - t0
    return {"value": round(S / dt, 4), "unit": "structures/s", "cores": args.cpu_threads, "kind": "reference",
            "sample": (f"{S} of the shard's {n_atoms}-atom structures, graph (restated NeighborList+RBF, 1 thread) + "
                       f"Betti (verbatim vendored Ripser, OpenMP {args.cpu_threads} x Ripser 1 thread), "
                       f"{dt:.1f} s on {os.cpu_count()} visible CPUs")}


if __name__ == "__main__":
    main()
