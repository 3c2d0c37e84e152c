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


def gather_csr(local: dict, dst: int = 0, group=None):
    """Gather every rank's CSR dict to rank `dst` (torch.distributed, any backend; objects are
    sent as numpy arrays). Returns the merged CSR on dst, None elsewhere."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    objs = [None] * world if dist.get_rank(group) == dst else None
    dist.gather_object({k: np.asarray(v) for k, v in local.items()}, objs, dst=dst, group=group)
    return merge_csr(objs) if objs is not None else None
