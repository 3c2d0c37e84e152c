"""Per-structure sharding across GPUs: one process per GPU, each owns a
contiguous block of structures; no collective on the data path. The only exchange is the
optional final gather of results to one rank, done here with per-shard sizes first so CSR
row pointers can be rebased (host-side exclusive scan of shard edge counts)."""
from __future__ import annotations

import numpy as np


def shard_bounds(num_structures: int, world: int, rank: int) -> tuple[int, int]:
    """Contiguous block [lo, hi) of structure ids for `rank` (remainder spread over low ranks)."""
    base, rem = divmod(num_structures, world)
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def merge_csr(shards: list[dict]) -> dict:
    """Concatenate per-shard CSR results (row_ptr local to each shard) into one batch-level CSR.
    Keys: row_ptr [A_s + 1] int64, and any per-edge arrays (col, dist, disp, rbf) and per-atom
    arrays (features, counts) which are simply concatenated."""
    out = {}
    offs = np.cumsum([0] + [int(s["row_ptr"][-1]) for s in shards])
    out["row_ptr"] = np.concatenate([shards[0]["row_ptr"][:1] * 0] +
                                    [np.asarray(s["row_ptr"][1:], np.int64) + offs[i] for i, s in enumerate(shards)])
    for k in shards[0]:
        if k != "row_ptr":
            out[k] = np.concatenate([np.asarray(s[k]) for s in shards])
    return out


class Shard:
    """One rank's share of a synthetic bench workload (bench.py and the multi-process tests):
    structures [rank*B, (rank+1)*B) of `synth_batch(kind, m)`, inputs resident on `dev`, output
    buffers allocated once; `step` runs the whole hot path over the shard through the C ABI."""

    def __init__(self, dgn, abi, kind: str, m: int, structures: int, rank: int, dev):
        import torch
        self.dgn, self.abi, self.dev = dgn, abi, dev
        self.B = int(structures)
        self.host = dgn.synth_batch(kind, m, self.B, first_id=rank * self.B)
        self.batch = {k: torch.from_numpy(v).to(dev) for k, v in self.host.items()}
        self.A = int(self.host["positions"].shape[0])
        self.n_atoms = self.A // self.B
        self.E = 0
        self.out = {}

    def alloc_graph(self, ctx, gp, nbins: int, rbf_dtype) -> int:
        import torch
        self.E = ctx.dev_graph_count(self.batch, gp)
        e = max(self.E, 1)
        self.out.update(row_ptr=torch.empty(self.A + 1, dtype=torch.int64, device=self.dev),
                        col=torch.empty(e, dtype=torch.int32, device=self.dev),
                        dist=torch.empty(e, dtype=torch.float64, device=self.dev),
                        rbf=torch.empty((e, nbins), dtype=rbf_dtype, device=self.dev))
        return self.E

    def alloc_betti(self):
        import torch
        self.out.update(feat=torch.empty((self.A, 35), dtype=torch.float64, device=self.dev),
                        counts=torch.empty((self.A, 4), dtype=torch.int32, device=self.dev))

    def step(self, ctx, gp, betti_rc: float, betti: bool = True, graph: bool = True, fused: bool = True):
        """graph: NeighborList count + emit (CSR + RBF); betti: the Betti pass. Both with fused:
        dgn_dev_graph_betti, which shares the neighbour count when the cutoffs agree."""
        o = self.out
        if graph:
            e = ctx.dev_graph_count(self.batch, gp)
            if e != self.E:
                raise RuntimeError(f"edge count changed between steps: {e} != {self.E}")
            if betti and fused:
                ctx.dev_graph_betti(self.batch, gp, o["row_ptr"], o["col"], o["dist"], None, o["rbf"], betti_rc,
                                    o["feat"], o["counts"])
                return
            ctx.dev_graph_emit(self.batch, gp, o["row_ptr"], o["col"], o["dist"], None, o["rbf"])
        if betti:
            ctx.dev_betti(self.batch, betti_rc, o["feat"], o["counts"])

    def results(self) -> dict:
        """Host copies of every output buffer (row_ptr local to the shard)."""
        return {k: v.cpu().numpy() for k, v in self.out.items()}


def gather_csr(local: dict, dst: int = 0, group=None):
    """Gather every rank's CSR dict to rank `dst` (torch.distributed, any backend; objects are
    sent as numpy arrays). Returns the merged CSR on dst, None elsewhere."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    objs = [None] * world if dist.get_rank(group) == dst else None
    dist.gather_object({k: np.asarray(v) for k, v in local.items()}, objs, dst=dst, group=group)
    return merge_csr(objs) if objs is not None else None
