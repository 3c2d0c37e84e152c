"""Multi-process path on CPU (gloo, world size 2): per-structure shards computed independently
and gathered with rebased row pointers equal the single-process result; the bench's
max-over-ranks timing reduction. Compute here uses the CPU oracle (test infrastructure); the
GPU ranks run the same host logic around libdgn."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT  # noqa: F401  (sys.path setup)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _graph_shard(lo, hi):
    import oracle_py as O
    from dgn import synth
    b = synth.make_batch("sc", 4, hi - lo, first_id=lo)
    n = 64
    parts = []
    for s in range(hi - lo):
        nl = O.neighbor_list(b["lattice"][s], b["positions"][s * n:(s + 1) * n], 5.0, 20)
        parts.append({"row_ptr": nl["row_ptr"], "col": nl["col"], "dist": nl["dist"]})
    from dgn.shard import merge_csr
    return merge_csr(parts)


def _worker(rank, world, port, total, out_path):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dgn.shard import gather_csr, shard_bounds
    lo, hi = shard_bounds(total, world, rank)
    merged = gather_csr(_graph_shard(lo, hi))
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # bench.py: max over ranks of the timed region
    if rank == 0:
        np.savez(out_path, **merged, tmax=t.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_shard_bounds_cover():
    from dgn.shard import shard_bounds
    for total in (0, 1, 7, 8, 65536):
        for world in (1, 2, 3, 8):
            spans = [shard_bounds(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))


def test_gloo_world2_gather_matches_single(tmp_path):
    total, world = 5, 2
    out = str(tmp_path / "g.npz")
    mp.start_processes(_worker, args=(world, _free_port(), total, out), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    ref = _graph_shard(0, total)
    for k in ("row_ptr", "col", "dist"):
        assert np.array_equal(got[k], ref[k]), k
    assert float(got["tmax"][0]) == 2.0
