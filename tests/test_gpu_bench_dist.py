"""bench.py's multi-rank path (one process per GPU) on one MI355X: two
ranks launched by torch.distributed.run with the gloo backend for the timing collectives (the
8-GPU driver run uses nccl = RCCL; the data path has no collective either way). Checks the JSON
line's n_gpus / value / ms_per_step and that every rank's shard outputs equal the library's on the
same structure ids computed in this process (reference parallel axis: the per-structure loop of
preprocess_betti.cpp:61-85 / the OpenMP loop of betti_features.cpp:111)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import dgn
from dgn import abi

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
B = 64


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_gloo(tmp_path, ctx):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--structures", str(B), "--steps", "2", "--warmup", "1", "--no-side", "--no-cpu-baseline",
           "--no-alt-rbf", "--dist-backend", "gloo", "--dump-shards", str(tmp_path)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints one JSON line
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["steps"] == 2 and j["warmup"] == 1 and j["scaling"] == "weak"
    assert j["config"]["structures_per_gpu"] == B and j["dtype"] == "f64"
    # value = structures of all ranks over the max-over-ranks timed region
    assert j["value"] > 0 and abs(j["value"] - B * 2 / (j["ms_per_step"] * 1e-3)) / j["value"] < 0.01
    gp = abi.graph_params(r_cutoff=5.0, max_neighbors=20, rbf_cutoff=5.0, rbf_dr=0.1, rbf_dtype=dgn.DGN_F64)
    for rank in range(2):
        batch = dgn.synth_batch("fcc", 4, B, first_id=rank * B)
        f, c = ctx.host_betti(batch, 5.0)
        assert np.array_equal(np.load(tmp_path / f"rank{rank}_counts.npy"), c), rank
        assert np.array_equal(np.load(tmp_path / f"rank{rank}_feat.npy"), f), rank
        g = ctx.host_graph(batch, gp)
        assert np.array_equal(np.load(tmp_path / f"rank{rank}_row_ptr.npy"), g["row_ptr"]), rank
        assert np.array_equal(np.load(tmp_path / f"rank{rank}_col.npy"), g["col"]), rank
        assert np.array_equal(np.load(tmp_path / f"rank{rank}_dist.npy"), g["dist"]), rank


def test_bench_one_rank_nccl(tmp_path):
    """The launcher path the 8-GPU driver run takes -- torch.distributed.run with the default nccl
    (RCCL) backend for the timing barrier and the max-over-ranks reduction -- on the one GPU this box
    has (one rank: RCCL needs a device per rank). The line reports n_gpus 1 and the rank's value."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "1", "--structures", str(B), "--steps", "2", "--warmup", "1", "--no-side", "--no-cpu-baseline",
           "--no-alt-rbf", "--dump-shards", str(tmp_path)]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    j = json.loads(lines[0])
    assert j["n_gpus"] == 1 and j["value"] > 0 and j["config"]["structures_per_gpu"] == B
    assert (tmp_path / "rank0_counts.npy").exists()
