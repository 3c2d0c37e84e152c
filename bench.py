#!/usr/bin/env python3
"""Bench: structures/sec (graph + Betti) on synthetic crystal batches, 1..8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--structures B] [...]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[3], one shard per GPU, weak scaling): every rank owns B = 8,192
jittered 256-atom FCC structures (structure ids [rank*B, (rank+1)*B)), inputs resident in HBM.
One step = the whole hot path over the shard through the C ABI (libdgn.so):
  graph : NeighborList(rc=5, K=20) + CrystalGraph edge RBF (rc=5, dr=0.1 -> 50 bins, f64 as the
          reference's edge_attr, crystal_graph.cpp:30,37; --rbf-dtype f32 for the narrower variant)
  Betti : compute_structure_betti_features(rc=5): NeighborList(rc, inf) + per-atom local VR
          (Gram distances, dim 0/1/2, Z/2) + 35 statistics (f64)
Shards are independent (no collective on the data path); the only collectives are the barrier
and the max-over-ranks of the timed region.
Rank 0 prints ONE JSON line (metric/unit from BASELINE.json) with
  roofline      the neighbour + RBF path (prep + count + scan + emit, HBM-bound) at SURVEY 8(d)'s
                algorithmic bytes over its HIP-event time on the launch stream; the emit launch
                alone and the f32-RBF variant (measured after the timed loop) beside it
  side          beside the headline, never part of `value`: BASELINE configs 1, 2, 3 and 5 (the
                741.vasp POSCAR through the reference CPU path and the GPU path; 1,024 x SC-64 graph
                / graph + Betti; one 4,096-atom supercell) and the Betti pass at the reference's
                default 10 A cutoff (32 FCC-256 structures, wide kernel)
  cpu_baseline  the reference CPU path on this host on a bounded sample of the same shard
                (restated neighbour list + the reference's verbatim vendored Ripser), at the
                reference's default nesting and at OMP x 1 Ripser thread; its outputs double as the
                parity check of the GPU results for the same structures (`parity`)
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
FP64_PEAK_TFS = 78.6  # MI355X FP64 vector (and dense matrix) peak (spec)
GRAPH_KERNELS = ("prep_structures", "graph_count", "block_scan", "graph_emit")


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
    ap.add_argument("--rbf-dtype", default="f64", choices=["f64", "f32"],
                    help="edge_attr dtype of the timed step (the reference's is f64)")
    ap.add_argument("--no-alt-rbf", action="store_true", help="skip the other-RBF-dtype side measurement")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for the timing barrier / max (nccl = RCCL)")
    ap.add_argument("--dump-shards", default=None,
                    help="directory: each rank writes its shard's Betti counts/features and CSR (tests)")
    ap.add_argument("--no-side", action="store_true",
                    help="skip the side lines (BASELINE configs 2/3/5 and the 10 A Betti line)")
    ap.add_argument("--side-reps", type=int, default=3)
    ap.add_argument("--cpu-sample", type=int, default=64, help="structures in each CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=8)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--config", default=None, help="label of the BASELINE config this run measures")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "traffic_latest.json"),
                    help="PMC-derived HBM bytes per neighbour-path launch set (profiles/collect.sh)")
    return ap.parse_args()


def graph_bytes_8d(n_atoms, n_struct, edges, nbins, rbf_bytes):
    """SURVEY 8(d) algorithmic bytes of the neighbour + RBF path: positions 24N + lattice 72 +
    species 4N + row_ptr 8(N+1) + col 4E + dist 4E (+4E: the distance is written as f64) + RBF
    rbf_bytes * E * n_rbf, summed over the shard."""
    return (24 * n_atoms + 72 * n_struct + 4 * n_atoms + 8 * (n_atoms + n_struct) + 4 * edges + 8 * edges
            + rbf_bytes * edges * nbins)


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # one process per GPU; ranks beyond the visible devices share them (gloo tests on one GPU)
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    # under torch.distributed.run (WORLD_SIZE set, the driver's N > 1 launches) the timing barrier and
    # the max-over-ranks reduction go through the process group, even for one rank
    distributed = "WORLD_SIZE" in os.environ
    if distributed:
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    # the collective's tensors live where the backend expects them
    cdev = dev if args.dist_backend == "nccl" else torch.device("cpu")

    import dgn
    from dgn import abi
    from dgn.shard import Shard

    # ---- synthetic shard, resident in HBM ----
    sh = Shard(dgn, abi, args.kind, args.m, args.structures, rank, dev)
    B, A, n_atoms = sh.B, sh.A, sh.n_atoms
    ctx = dgn.Context(local)
    stream = torch.cuda.current_stream(dev)
    ctx.set_stream(stream.cuda_stream)
    f64 = args.rbf_dtype == "f64"
    gp = abi.graph_params(r_cutoff=args.rc, max_neighbors=args.k, rbf_cutoff=args.rbf_rc, rbf_dr=args.dr,
                          rbf_dtype=dgn.DGN_F64 if f64 else dgn.DGN_F32)
    nbins = abi.lib().dgn_rbf_bins(args.rbf_rc, args.dr)
    E = sh.alloc_graph(ctx, gp, nbins, torch.float64 if f64 else torch.float32)
    if not args.no_betti:
        sh.alloc_betti()

    def step():
        sh.step(ctx, gp, args.betti_rc, betti=not args.no_betti)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ctx.reset_timing()
    ctx.enable_timing(True)

    # ---- timed region: barrier + sync on both sides, max over ranks ----
    if distributed:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if distributed:
        t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ctx.synchronize()  # raises if an emit reported a count/emit disagreement
    ktimes = ctx.kernel_times()
    ctx.enable_timing(False)

    # sanity: no NaN features (NaN marks a complex outside the kernel envelope)
    if not args.no_betti:
        bad = int(torch.isnan(sh.out["feat"]).any(dim=1).sum().item())
        if bad:
            raise SystemExit(f"rank {rank}: {bad} atoms with NaN features")

    total_structures = B * world * args.steps
    value = total_structures / elapsed
    step_ms = elapsed / args.steps * 1e3
    kernel_ms = {k: round(v["total_ms"] / args.steps, 4) for k, v in ktimes.items()}

    # ---- neighbour + RBF path roofline (HIP events on the launch stream) ----
    roof = None
    if all(ktimes.get(k, {}).get("launches") for k in GRAPH_KERNELS):
        path_ms = sum(ktimes[k]["total_ms"] for k in GRAPH_KERNELS) / args.steps
        emit_ms = ktimes["graph_emit"]["total_ms"] / ktimes["graph_emit"]["launches"]
        algo = graph_bytes_8d(A, B, E, nbins, 8 if f64 else 4)
        achieved = algo / (path_ms * 1e-3) / 1e9
        traffic = None
        if os.path.exists(args.traffic_json):
            try:
                tj = json.load(open(args.traffic_json))
                if tj.get("workload_key") == f"{args.kind}{args.m}x{B}_rc{args.rc}_k{args.k}_nb{nbins}_{args.rbf_dtype}":
                    traffic = tj.get("hbm_bytes_per_path")
            except Exception:
                traffic = None
        roof = {"bound": "hbm", "kernel": "neighbour+RBF path: prep_structures + graph_count + block_scan + graph_emit",
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "algorithmic_bytes_per_launch": int(algo), "avg_launch_ms": round(path_ms, 4),
                "bytes_formula": ("SURVEY 8(d): 24N+72+4N+8(N+1)+4E+4E(+4E f64 dist)+%d*E*n_rbf per structure (%s RBF)"
                                  % (8 if f64 else 4, args.rbf_dtype)),
                "emit_only": {"avg_launch_ms": round(emit_ms, 4),
                              "achieved": round(algo / (emit_ms * 1e-3) / 1e9, 1),
                              "frac": round(algo / (emit_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}}
        if not args.no_alt_rbf:
            alt = "f32" if f64 else "f64"
            roof["rbf_" + alt] = alt_rbf_measurement(ctx, sh, args, nbins, abi, dgn, torch, alt)
    dk = ktimes.get("betti_dist", {})
    dist_roof = None
    if dk.get("launches") and dk["total_ms"] > 0:
        dk_s = dk["total_ms"] / dk["launches"] / 1e3
        tfs = dk["flops"] / dk["launches"] / dk_s / 1e12
        gbs = dk["bytes"] / dk["launches"] / dk_s / 1e9
        dist_roof = {"bound": "valu", "kernel": "betti_dist (neighbour search + f64 Gram distances -> f32 triangles)",
                "achieved": round(tfs, 6), "peak": FP64_PEAK_TFS, "unit": "TFLOP/s",
                "frac": tfs / FP64_PEAK_TFS, "hbm_achieved_gbs": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
                "note": ("useful 6n^2 flops per local complex (K=3 Gram); one packed pair per lane on the f64 VALU "
                         "(the square root's Newton steps and the pair index are not counted; SQ counters in "
                         "profiles/r05_dist.json)")}

    label = args.config or ("config4" if (args.kind, args.m) == ("fcc", 4) else f"{args.kind}{args.m}")
    result = {
        "metric": "structures/sec (graph+Betti) at 1/2/4/8 MI355X; HBM GB/s vs peak",
        "value": round(value, 2), "unit": "structures/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(step_ms, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f64" if f64 else "f64 (RBF f32)", "data": "synthetic",
        "config": {"workload": (f"{label} shard: {B} x {n_atoms}-atom jittered {args.kind.upper()} per GPU; "
                                f"graph rc={args.rc} K={args.k} RBF {nbins}x{args.rbf_dtype}"
                                + ("" if args.no_betti else f" + Betti-0/1/2 rc={args.betti_rc}")),
                   "structures_per_gpu": B, "atoms_per_structure": n_atoms, "edges_per_gpu": E,
                   "parallelism": f"shard{world}"},
        "roofline": roof,
        "roofline_dist": dist_roof,
        "kernel_ms_per_step": kernel_ms,
    }
    if args.dump_shards:
        dump_shard(args.dump_shards, rank, sh, args)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"], result["parity"] = cpu_baseline(args, sh, n_atoms, torch)
    if not args.no_side and world == 1:
        result["side"] = side_lines(dgn, abi, ctx, dev, args, torch)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if distributed:
        dist.barrier()
        dist.destroy_process_group()


def dump_shard(d, rank, sh, args):
    """Tests: this rank's shard outputs (structure ids [rank*B, (rank+1)*B)) as .npy files."""
    import numpy as np
    os.makedirs(d, exist_ok=True)
    for k in ("row_ptr", "col", "dist", "feat", "counts"):
        if k in sh.out:
            np.save(os.path.join(d, f"rank{rank}_{k}.npy"), sh.out[k].cpu().numpy())


def alt_rbf_measurement(ctx, sh, args, nbins, abi, dgn, torch, alt):
    """The same neighbour path with the other edge_attr dtype (the reference's is f64,
    crystal_graph.cpp:30,37), measured after the timed loop (HIP events), 3 repetitions."""
    f64 = alt == "f64"
    gpa = abi.graph_params(r_cutoff=args.rc, max_neighbors=args.k, rbf_cutoff=args.rbf_rc, rbf_dr=args.dr,
                           rbf_dtype=dgn.DGN_F64 if f64 else dgn.DGN_F32)
    rbfa = torch.empty((max(sh.E, 1), nbins), dtype=torch.float64 if f64 else torch.float32, device=sh.dev)
    reps = 3
    ctx.reset_timing()
    ctx.enable_timing(True)
    for _ in range(reps):
        ctx.dev_graph_count(sh.batch, gpa)
        ctx.dev_graph_emit(sh.batch, gpa, sh.out["row_ptr"], sh.out["col"], sh.out["dist"], None, rbfa)
    ctx.synchronize()
    kt = ctx.kernel_times()
    ctx.enable_timing(False)
    del rbfa
    path_ms = sum(kt[k]["total_ms"] for k in GRAPH_KERNELS) / reps
    emit_ms = kt["graph_emit"]["total_ms"] / reps
    algo = graph_bytes_8d(sh.A, sh.B, sh.E, nbins, 8 if f64 else 4)
    return {"algorithmic_bytes_per_launch": int(algo), "avg_launch_ms": round(path_ms, 4),
            "achieved": round(algo / (path_ms * 1e-3) / 1e9, 1),
            "frac": round(algo / (path_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "emit_ms": round(emit_ms, 4)}


def side_lines(dgn, abi, ctx, dev, args, torch):
    """Beside the headline (never part of `value`): the other BASELINE configs on one GPU and the
    Betti pass at the reference's default 10 A cutoff (preprocess_betti.cpp:117). Each: the
    whole path through the C ABI, inputs resident, `reps` timed repetitions after one warm-up."""
    from dgn.shard import Shard
    out = {}

    def timed(sh, gp, betti_rc, betti, graph=True):
        sh.step(ctx, gp, betti_rc, betti=betti, graph=graph)
        torch.cuda.synchronize(dev)
        ctx.reset_timing()
        ctx.enable_timing(True)
        t0 = time.perf_counter()
        for _ in range(args.side_reps):
            sh.step(ctx, gp, betti_rc, betti=betti, graph=graph)
        torch.cuda.synchronize(dev)
        dt = (time.perf_counter() - t0) / args.side_reps
        kt = ctx.kernel_times()
        ctx.enable_timing(False)
        return dt, {k: round(v["total_ms"] / args.side_reps, 4) for k, v in kt.items()}

    out["config1"] = config1_line(dgn, abi, ctx, dev, args, torch)
    gp = abi.graph_params(r_cutoff=5.0, max_neighbors=20, rbf_cutoff=5.0, rbf_dr=0.1, rbf_dtype=dgn.DGN_F32)
    nb = abi.lib().dgn_rbf_bins(5.0, 0.1)
    # configs 2 and 3: 1,024 jittered SC-64 cells, graph only / graph + Betti (rc 5)
    sh = Shard(dgn, abi, "sc", 4, 1024, 0, dev)
    sh.alloc_graph(ctx, gp, nb, torch.float32)
    sh.alloc_betti()
    dt, kt = timed(sh, gp, 5.0, False)
    gk = sum(kt.get(k, 0.0) for k in GRAPH_KERNELS)
    algo = graph_bytes_8d(sh.A, sh.B, sh.E, nb, 4)
    out["config2"] = {"workload": "1024 x SC-64, NeighborList(5, 20) + 50-bin f32 RBF", "structures_per_s": round(sh.B / dt, 1),
                      "ms": round(dt * 1e3, 4), "path_ms": round(gk, 4),
                      "path_hbm_frac": round(algo / (gk * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if gk else None}
    dt, kt = timed(sh, gp, 5.0, True)
    out["config3"] = {"workload": "1024 x SC-64, graph + Betti-0/1/2 (rc 5)", "structures_per_s": round(sh.B / dt, 1),
                      "ms": round(dt * 1e3, 4), "betti_vr_ms": kt.get("betti_vr")}
    del sh
    # config 5: one 4,096-atom SC supercell (27 images), graph + Betti
    sh = Shard(dgn, abi, "sc", 16, 1, 0, dev)
    sh.alloc_graph(ctx, gp, nb, torch.float32)
    sh.alloc_betti()
    dt, kt = timed(sh, gp, 5.0, False)
    gk = sum(kt.get(k, 0.0) for k in GRAPH_KERNELS)
    dt2, kt2 = timed(sh, gp, 5.0, True, graph=False)
    out["config5"] = {"workload": "1 x SC-4096 supercell (L = 37.1 A), graph rc 5 K 20 + Betti rc 5",
                      "graph_ms": round(dt * 1e3, 4), "graph_path_kernels_ms": round(gk, 4),
                      "graph_path_hbm_frac": round(graph_bytes_8d(sh.A, 1, sh.E, nb, 4) / (gk * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                      if gk else None, "betti_ms": round(dt2 * 1e3, 4)}
    # the cell-list Betti search (> 512 atoms): every atom of the timed supercell vs the oracle
    import numpy as np
    import oracle_py as O
    fo, co = O.structure_betti(sh.host["lattice"][0], sh.host["positions"], sh.host["species"], 5.0)
    gf, gc = sh.out["feat"].cpu().numpy(), sh.out["counts"].cpu().numpy()
    rel = np.abs(gf - fo) / np.maximum(np.abs(fo), 1e-12)
    out["config5"]["betti_parity"] = {"atoms_checked": int(sh.A), "counts_exact": bool(np.array_equal(gc, co)),
                                      "feat_within_1e-6": bool(np.all((rel <= 1e-6) | (np.abs(gf - fo) <= 1e-12))),
                                      "checker": "oracle structure_betti (pinned to verbatim Ripser, cellist.npz)"}
    del sh
    # the reference's default Betti cutoff, 10 A (~340-point complexes, wide kernel)
    sh = Shard(dgn, abi, "fcc", 4, 32, 0, dev)
    sh.alloc_betti()
    dt, kt = timed(sh, gp, 10.0, True, graph=False)
    out["betti_rc10"] = {"workload": "32 x FCC-256 (8,192 complexes of ~340 points), Betti-0/1/2 at rc 10",
                         "structures_per_s": round(sh.B / dt, 2), "complexes_per_s": round(sh.A / dt, 1),
                         "ms": round(dt * 1e3, 2), "betti_vr_ms": kt.get("betti_vr")}
    del sh
    # the same at a 128-structure batch (32,768 complexes, ~7 per resident wave): the steady-state
    # rate; at 32 structures each resident wave reduces one or two complexes and the last ones idle
    sh = Shard(dgn, abi, "fcc", 4, 128, 0, dev)
    sh.alloc_betti()
    dt, kt = timed(sh, gp, 10.0, True, graph=False)
    out["betti_rc10_b128"] = {"workload": "128 x FCC-256 (32,768 complexes of ~340 points), Betti-0/1/2 at rc 10",
                              "structures_per_s": round(sh.B / dt, 2), "complexes_per_s": round(sh.A / dt, 1),
                              "ms": round(dt * 1e3, 2), "betti_vr_ms": kt.get("betti_vr")}
    return out


def config1_line(dgn, abi, ctx, dev, args, torch):
    """BASELINE config 1: one POSCAR at 5 A (preprocess_betti.cpp:30-107 on the reference's
    web/public/data/structures/741.vasp, N = 120, kept as input data in tests/golden/poscar_rc5.npz):
    NeighborList(5, K = 20) + f64 RBF + compute_structure_betti_features(rc = 5). The GPU path
    (inputs resident, one dgn_dev_graph_count + dgn_dev_graph_betti per repetition) beside the
    reference CPU path on this host (restated neighbour list + RBF, verbatim vendored Ripser with
    OpenMP 8 x 1 Ripser thread), and the GPU outputs checked against the CPU ones."""
    import numpy as np
    import oracle_py as O
    fx = np.load(os.path.join(ROOT, "tests", "golden", "poscar_rc5.npz"))
    host = {"lattice": fx["741/lattice"][None].copy(), "positions": fx["741/positions"].copy(),
            "species": fx["741/species"].astype(np.int32),
            "atom_offset": np.array([0, len(fx["741/positions"])], np.int64)}
    N = len(host["positions"])
    batch = {k: torch.from_numpy(v).to(dev) for k, v in host.items()}
    gp = abi.graph_params(r_cutoff=5.0, max_neighbors=20, rbf_cutoff=5.0, rbf_dr=0.1, rbf_dtype=dgn.DGN_F64)
    nb = abi.lib().dgn_rbf_bins(5.0, 0.1)
    E = ctx.dev_graph_count(batch, gp)
    o = {"row_ptr": torch.empty(N + 1, dtype=torch.int64, device=dev), "col": torch.empty(E, dtype=torch.int32, device=dev),
         "dist": torch.empty(E, dtype=torch.float64, device=dev), "rbf": torch.empty((E, nb), dtype=torch.float64, device=dev),
         "feat": torch.empty((N, 35), dtype=torch.float64, device=dev), "counts": torch.empty((N, 4), dtype=torch.int32, device=dev)}

    def gpu_step():
        ctx.dev_graph_count(batch, gp)
        ctx.dev_graph_betti(batch, gp, o["row_ptr"], o["col"], o["dist"], None, o["rbf"], 5.0, o["feat"], o["counts"])

    gpu_step()
    torch.cuda.synchronize(dev)
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        gpu_step()
    torch.cuda.synchronize(dev)
    gpu_s = (time.perf_counter() - t0) / reps
    line = {"workload": "741.vasp (N = 120): NeighborList(5, 20) + 50-bin f64 RBF + Betti-0/1/2 rc 5",
            "gpu_ms": round(gpu_s * 1e3, 4), "gpu_structures_per_s": round(1 / gpu_s, 1)}
    if O.ref_available():
        t0 = time.perf_counter()
        O.structure_graph(host["lattice"][0], host["positions"], 5.0, 20, 5.0, 0.1, want_rbf=True)
        f, c = O.ref_structure_betti(host["lattice"][0], host["positions"], host["species"], 5.0, omp_threads=8,
                                     ripser_threads=1)
        cpu_s = time.perf_counter() - t0
        gf, gc = o["feat"].cpu().numpy(), o["counts"].cpu().numpy()
        rel = np.abs(gf - f) / np.maximum(np.abs(f), 1e-12)
        line.update(cpu_ms=round(cpu_s * 1e3, 2), cpu_kind="reference (restated NeighborList + RBF, verbatim Ripser)",
                    cpu_threads="OpenMP 8 x Ripser 1", cpu_model=cpu_model(), nproc=os.cpu_count(),
                    counts_exact=bool(np.array_equal(gc, c)))
        line["feat_within_1e-6"] = bool(np.all((rel <= 1e-6) | (np.abs(gf - f) <= 1e-12)))
    return line


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(args, sh, n_atoms, torch):
    """Reference CPU path on this host: restated neighbour list + RBF (nanoflann/Eigen absent
    offline) and the reference's VERBATIM vendored Ripser for the topology (oracle/_ref), on the
    shard's first structures, at the reference's default nesting (OpenMP 8 over atoms x Ripser 8
    threads, preprocess_betti.cpp:119) and at OpenMP 8 x Ripser 1 thread. The GPU outputs for the
    same structures are compared with these reference outputs (the `parity` field)."""
    import numpy as np
    import oracle_py as O
    host = sh.host
    cores = args.cpu_threads
    info = {"cpu_model": cpu_model(), "nproc": os.cpu_count()}
    if not O.ref_available():
        return ({"value": None, "unit": "structures/s", "cores": 0, "kind": "reference",
                 "sample": "oracle/_ref/libdgn_ref.so not built", **info}, None)
    S = min(args.cpu_sample, sh.B)
    variants = {}
    feats = {}
    # the whole host the process may run on (OpenMP over every visible core x Ripser 1), on a sample
    # scaled with the thread count so the leg still takes about as long as the 8-thread ones
    # (the cgroup's CPU quota caps it: the GPU box shows 256 CPUs but grants a job 16 of them, and 256
    # threads time-sliced over 16 CPUs measured slower than 8)
    host_threads = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 8)
    try:
        info["cgroup_cpu_max"] = open("/sys/fs/cgroup/cpu.max").read().strip()
        quota, period = info["cgroup_cpu_max"].split()[:2]
        if quota != "max":
            host_threads = max(1, min(host_threads, -(-int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    info["host_threads"] = host_threads
    runs = [("omp8_x_ripser8_reference_default", cores, 8, S), ("omp8_x_ripser1", cores, 1, S)]
    if host_threads > cores:
        runs.append((f"omp{host_threads}_x_ripser1_full_host", host_threads, 1,
                     min(sh.B, max(S, S * min(host_threads // cores, 8)))))
    for name, omp, rt, n_s in runs:
        t0 = time.perf_counter()
        for s in range(n_s):
            sl = slice(s * n_atoms, (s + 1) * n_atoms)
            lat, pos, sp = host["lattice"][s], host["positions"][sl], host["species"][sl]
            O.structure_graph(lat, pos, args.rc, args.k, args.rbf_rc, args.dr)
            if not args.no_betti:
                f, c = O.ref_structure_betti(lat, pos, sp, args.betti_rc, omp_threads=omp, ripser_threads=rt)
                if s < S:
                    feats[s] = (f, c)
        dt = time.perf_counter() - t0
        variants[name] = {"value": round(n_s / dt, 4), "seconds": round(dt, 2), "threads": omp * rt,
                          "structures": n_s}
    best = max(variants.values(), key=lambda v: v["value"])
    if host_threads > cores and os.cpu_count() and os.cpu_count() > host_threads:
        full = variants[f"omp{host_threads}_x_ripser1_full_host"]
        # the whole machine, were the job granted it: the full-host rate scaled linearly (an upper bound)
        info["projected_all_cpus"] = {"value": round(full["value"] * os.cpu_count() / host_threads, 2),
                                      "threads": os.cpu_count(), "kind": "linear projection, not measured"}
    base = {"value": best["value"], "unit": "structures/s", "cores": best["threads"], "kind": "reference",
            "sample": (f"first {S} of the shard's {n_atoms}-atom structures per 8-thread variant (the full-host "
                       f"variant: its `structures`): graph = restated NeighborList + RBF (1 thread; nanoflann/Eigen "
                       f"absent offline), Betti = verbatim vendored Ripser; value = the fastest variant"),
            "variants": variants, **info}
    parity = None
    if not args.no_betti:
        feat = sh.out["feat"][:S * n_atoms].cpu().numpy()
        cnt = sh.out["counts"][:S * n_atoms].cpu().numpy()
        ref_f = np.concatenate([feats[s][0] for s in range(S)])
        ref_c = np.concatenate([feats[s][1] for s in range(S)])
        rel = np.abs(feat - ref_f) / np.maximum(np.abs(ref_f), 1e-12)
        # graph rows of the first and last sampled structure vs the oracle (bit-exact CSR)
        rp = sh.out["row_ptr"].cpu().numpy()
        col = sh.out["col"].cpu().numpy()
        dist = sh.out["dist"].cpu().numpy()
        g_ok = True
        rbf_rel = 0.0
        rbf_gpu = sh.out["rbf"]
        for s in (0, S - 1):
            lat_s, pos_s = host["lattice"][s], host["positions"][s * n_atoms:(s + 1) * n_atoms]
            nl = O.neighbor_list(lat_s, pos_s, args.rc, args.k)
            a, b = rp[s * n_atoms], rp[(s + 1) * n_atoms]
            g_ok = g_ok and np.array_equal(rp[s * n_atoms:(s + 1) * n_atoms + 1] - a, nl["row_ptr"]) and \
                np.array_equal(col[a:b], nl["col"]) and np.array_equal(dist[a:b], nl["dist"])
            # the timed shard's RBF rows of the same structures vs the oracle (gaussian_rbf,
            # edge_features.cpp:7-24, one row per edge in CSR order)
            ref = O.structure_graph(lat_s, pos_s, args.rc, args.k, args.rbf_rc, args.dr, want_rbf=True)
            got = rbf_gpu[a:b].double().cpu().numpy()
            if got.shape != ref.shape:
                rbf_rel = float("inf")
            else:
                rbf_rel = max(rbf_rel, float(np.max(np.abs(got - ref) / np.maximum(np.abs(ref), 1e-300))))
        parity = {"betti_atoms_checked": int(S * n_atoms), "betti_counts_exact": bool(np.array_equal(cnt, ref_c)),
                  "betti_feat_max_rel": float(np.max(np.where(np.abs(ref_f) > 1e-12, rel, 0.0))),
                  "betti_feat_within_1e-6": bool(np.all((rel <= 1e-6) | (np.abs(feat - ref_f) <= 1e-12))),
                  "graph_structures_checked": 2, "graph_csr_bit_exact": bool(g_ok),
                  "rbf_structures_checked": 2, "rbf_max_rel": rbf_rel,
                  "rbf_within_tol": bool(rbf_rel <= (1e-12 if args.rbf_dtype == "f64" else 1e-6)),
                  "reference": "verbatim vendored Ripser (oracle/_ref) + restated neighbour list"}
    return base, parity


if __name__ == "__main__":
    main()
