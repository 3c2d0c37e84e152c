"""Flat float32 edge arrays (the WasmAPI graph accessors, reference
src/viz/wasm_bindings.cpp:206-294) through the C ABI and the C++ facade's viz::WasmAPI, vs the
oracle neighbour list: sources = the row atom's index within its structure, targets = Neighbor::idx,
distances / displacements = static_cast<float> of the f64 values — bit-exact."""
import os
import subprocess

import numpy as np
import pytest
import torch
from conftest import GOLDEN, ROOT

import dgn
import oracle_py as O
from dgn import abi

pytestmark = pytest.mark.gpu


def _oracle_edges(batch, rc, k):
    src, tgt, dist, disp = [], [], [], []
    off = batch["atom_offset"]
    for s in range(len(off) - 1):
        a, b = off[s], off[s + 1]
        nl = O.neighbor_list(batch["lattice"][s], batch["positions"][a:b], rc, k)
        rp = nl["row_ptr"]
        src.append(np.repeat(np.arange(b - a, dtype=np.int32), np.diff(rp)))
        tgt.append(nl["col"].astype(np.int32))
        dist.append(nl["dist"].astype(np.float32))
        disp.append(nl["disp"].astype(np.float32))
    return np.concatenate(src), np.concatenate(tgt), np.concatenate(dist), np.concatenate(disp)


@pytest.mark.parametrize("k", [20, None])
def test_host_edge_arrays_ragged_batch(ctx, k):
    sc = dgn.synth_batch("sc", 4, 3)
    fcc = dgn.synth_batch("fcc", 2, 2, first_id=7)
    batch = {"lattice": np.concatenate([sc["lattice"], fcc["lattice"]]),
             "positions": np.concatenate([sc["positions"], fcc["positions"]]),
             "species": np.concatenate([sc["species"], fcc["species"]]),
             "atom_offset": np.concatenate([sc["atom_offset"], sc["atom_offset"][-1] + fcc["atom_offset"][1:]])}
    got = ctx.host_edge_arrays(batch, 5.0, abi.UINT64_MAX if k is None else k)
    ref = _oracle_edges(batch, 5.0, k)
    for g, r in zip(got, ref):
        assert g.dtype == r.dtype and np.array_equal(g, r)


def test_dev_edge_arrays_partial_outputs(ctx):
    batch = dgn.synth_batch("fcc", 4, 2)
    dev = torch.device("cuda", 0)
    db = {k: torch.from_numpy(v).to(dev) for k, v in batch.items()}
    p = abi.graph_params(r_cutoff=5.0, max_neighbors=20, rbf_dtype=dgn.DGN_NONE, write_displacement=True)
    E = ctx.dev_graph_count(db, p)
    A = batch["positions"].shape[0]
    rp = torch.empty(A + 1, dtype=torch.int64, device=dev)
    col = torch.empty(E, dtype=torch.int32, device=dev)
    dist = torch.empty(E, dtype=torch.float64, device=dev)
    disp = torch.empty((E, 3), dtype=torch.float64, device=dev)
    ctx.dev_graph_emit(db, p, rp, col, dist, disp)
    src = torch.full((E,), -7, dtype=torch.int32, device=dev)
    d32 = torch.empty(E, dtype=torch.float32, device=dev)
    ctx.dev_edge_arrays(db, rp, None, dist, None, src, None, d32, None)
    torch.cuda.synchronize()
    ref = _oracle_edges(batch, 5.0, 20)
    assert np.array_equal(src.cpu().numpy(), ref[0])
    assert np.array_equal(d32.cpu().numpy(), ref[2])
    assert np.array_equal(d32.cpu().numpy(), dist.cpu().numpy().astype(np.float32))


@pytest.mark.parametrize("name", ["1", "741"])
def test_facade_wasm_api(tmp_path, name):
    """viz::WasmAPI: load_structure(POSCAR text) + build_graph(rc, K) + every accessor."""
    golden = np.load(os.path.join(GOLDEN, "poscar_rc5.npz"))
    out = tmp_path / "w.txt"
    r = subprocess.run([os.path.join(ROOT, "defect-gnn-cpp_amd", "bin", "facade_check"), "wasm",
                        os.path.join(GOLDEN, "poscar", f"{name}.vasp"), "5.0", "12", str(out)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    d = {}
    for line in open(out):
        parts = line.split()
        d[parts[0]] = np.array([float(x) for x in parts[2:2 + int(parts[1])]])
    lat, pos = golden[f"{name}/lattice"], golden[f"{name}/positions"]
    n = pos.shape[0]
    assert int(d["num_atoms"][0]) == n
    assert np.array_equal(d["positions"].astype(np.float32), pos.astype(np.float32).ravel())
    assert np.array_equal(d["lattice"].astype(np.float32), lat.astype(np.float32).ravel())
    assert np.array_equal(d["atom_types"], golden[f"{name}/species"])
    assert d["element_counts"].sum() == n
    batch = {"lattice": lat[None], "positions": pos, "species": golden[f"{name}/species"],
             "atom_offset": np.array([0, n], np.int64)}
    src, tgt, dist, disp = _oracle_edges(batch, 5.0, 12)
    assert int(d["num_edges"][0]) == len(src)
    assert np.array_equal(d["sources"], src) and np.array_equal(d["targets"], tgt)
    assert np.array_equal(d["distances"].astype(np.float32), dist)
    assert np.array_equal(d["displacements"].astype(np.float32), disp.ravel())
