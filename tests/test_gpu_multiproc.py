"""Multi-process GPU path: two ranks, each running libdgn in its own process on
device 0 over its own shard with the bench's rank logic (dgn.shard.Shard, the helper bench.py
uses), results gathered over gloo with rebased row pointers, must be byte-identical to one
process computing the whole batch. The max-over-ranks reduction of the timed region rides along."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT  # noqa: F401  (sys.path setup)

pytestmark = pytest.mark.gpu

KIND, M, PER_RANK, RC, K, BETTI_RC = "sc", 4, 6, 5.0, 20, 5.0


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run_shard(structures, rank):
    import torch
    import dgn
    from dgn import abi
    from dgn.shard import Shard
    dev = torch.device("cuda", 0)
    sh = Shard(dgn, abi, KIND, M, structures, rank, dev)
    ctx = dgn.Context(0)
    gp = abi.graph_params(r_cutoff=RC, max_neighbors=K, rbf_cutoff=RC, rbf_dr=0.1, rbf_dtype=dgn.DGN_F32)
    nbins = abi.lib().dgn_rbf_bins(RC, 0.1)
    sh.alloc_graph(ctx, gp, nbins, torch.float32)
    sh.alloc_betti()
    sh.step(ctx, gp, BETTI_RC)
    ctx.synchronize()
    res = sh.results()
    res["row_ptr"] = res["row_ptr"] - res["row_ptr"][0]
    ctx.close()
    return res


def _worker(rank, world, port, out_path):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dgn.shard import gather_csr
    merged = gather_csr(_run_shard(PER_RANK, rank))
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        np.savez(out_path, **merged, tmax=t.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_world2_shards_on_device0_match_single_process(tmp_path):
    world = 2
    out = str(tmp_path / "g.npz")
    env_keep = os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = env_keep or "0"
    mp.start_processes(_worker, args=(world, _free_port(), out), nprocs=world, join=True, start_method="spawn")
    got = np.load(out)
    ref = _run_shard(PER_RANK * world, 0)
    assert set(ref) <= set(got.files)
    for k, v in ref.items():
        assert got[k].dtype == v.dtype and got[k].shape == v.shape, k
        assert got[k].tobytes() == v.tobytes(), k
    assert float(got["tmax"][0]) == 2.0
    assert not np.isnan(ref["feat"]).any()
