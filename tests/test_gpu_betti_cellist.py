"""The Betti pass on structures above 512 atoms, where its neighbour search enumerates a cell list
instead of staging the structure in LDS (betti_dist_search_kernel, cell-list branch; reference
src/topology/betti_features.cpp:103-119 over src/graph/neighbor_list.cpp:27-66 with K = inf).

  * config 5's SC-4096 supercell (BASELINE.json configs[4]) at rc 5: every atom's counts bit-exact
    and features within 1e-6 of the oracle, every 8th atom against verbatim Ripser (cellist.npz);
    through the host entry point, the device entry point and the fused graph + Betti step;
  * a 688-atom triclinic cell (sheared, atoms outside the cell, a dense pocket: complexes of 34..88
    points, so the main, mid, overflow and wide tiers all run on cell-list clouds): every atom
    against verbatim Ripser;
  * the search's clouds themselves: the f32 triangles of selected SC-4096 atoms bit-identical to
    the reference arithmetic over NeighborList(rc, inf) (the displacement rows of the cell-list
    enumeration)."""
import os

import numpy as np
import pytest
import torch
from conftest import GOLDEN
from test_gpu_betti import _kernel_vs_reference_triangles

import dgn
import oracle_py as O
from dgn import abi

pytestmark = pytest.mark.gpu
FEAT_RTOL, FEAT_ATOL = 1e-6, 1e-12


def _fx():
    return np.load(os.path.join(GOLDEN, "cellist.npz"))


def _check(f, c, fo, co, what):
    bad = np.argwhere(np.any(c != co, axis=1)).ravel()
    assert bad.size == 0, (what, bad[:10], c[bad[:3]], co[bad[:3]])
    np.testing.assert_allclose(f, fo, rtol=FEAT_RTOL, atol=FEAT_ATOL, err_msg=what)


def test_sc4096_every_atom_host(ctx):
    fx = _fx()
    batch = dgn.synth_batch("sc", 16, 1)
    assert batch["positions"].shape[0] == 4096
    f, c = ctx.host_betti(batch, 5.0)
    fo, co = O.structure_betti(batch["lattice"][0], batch["positions"], batch["species"], 5.0)
    _check(f, c, fo, co, "sc4096 vs oracle")
    a = fx["sc4096/atoms"]
    _check(f[a], c[a], fx["sc4096/features"], fx["sc4096/counts"], "sc4096 vs verbatim Ripser")


def test_sc4096_device_and_fused(ctx):
    """dgn_dev_betti and dgn_dev_graph_betti (the bench's config-5 step) on the resident supercell."""
    fx = _fx()
    host = dgn.synth_batch("sc", 16, 1)
    dev = torch.device("cuda", 0)
    batch = {k: torch.from_numpy(v).to(dev) for k, v in host.items()}
    A = 4096
    feat = torch.empty((A, 35), dtype=torch.float64, device=dev)
    cnt = torch.empty((A, 4), dtype=torch.int32, device=dev)
    ctx.dev_betti(batch, 5.0, feat, cnt)
    ctx.synchronize()
    fo, co = O.structure_betti(host["lattice"][0], host["positions"], host["species"], 5.0)
    _check(feat.cpu().numpy(), cnt.cpu().numpy(), fo, co, "dev_betti")
    gp = abi.graph_params(r_cutoff=5.0, max_neighbors=20, rbf_cutoff=5.0, rbf_dr=0.1, rbf_dtype=dgn.DGN_F32)
    nb = abi.lib().dgn_rbf_bins(5.0, 0.1)
    E = ctx.dev_graph_count(batch, gp)
    rp = torch.empty(A + 1, dtype=torch.int64, device=dev)
    col = torch.empty(E, dtype=torch.int32, device=dev)
    dist = torch.empty(E, dtype=torch.float64, device=dev)
    rbf = torch.empty((E, nb), dtype=torch.float32, device=dev)
    feat.fill_(0.0)
    cnt.fill_(0)
    ctx.dev_graph_betti(batch, gp, rp, col, dist, None, rbf, 5.0, feat, cnt)
    ctx.synchronize()
    _check(feat.cpu().numpy(), cnt.cpu().numpy(), fo, co, "dev_graph_betti")
    a = fx["sc4096/atoms"]
    _check(feat.cpu().numpy()[a], cnt.cpu().numpy()[a], fx["sc4096/features"], fx["sc4096/counts"], "fused vs Ripser")


def test_triclinic_688_every_atom(ctx):
    fx = _fx()
    pos = fx["tri688/positions"]
    one = {"lattice": fx["tri688/lattice"][None].copy(), "positions": pos.copy(),
           "species": fx["tri688/species"].astype(np.int32), "atom_offset": np.array([0, len(pos)], np.int64)}
    nl = O.neighbor_list(one["lattice"][0], pos, 5.0, None)
    sizes = np.diff(nl["row_ptr"]) + 1
    # every Betti tier runs on cell-list clouds here
    assert sizes.min() <= 44 and np.any((sizes > 44) & (sizes <= 48)) and np.any((sizes > 48) & (sizes <= 64)) \
        and sizes.max() > 64, (sizes.min(), sizes.max())
    f, c = ctx.host_betti(one, 5.0)
    _check(f, c, fx["tri688/features"], fx["tri688/counts"], "tri688 vs verbatim Ripser")


def test_sc4096_search_triangles(ctx):
    """The cell-list search + Gram triangles (f64 VALU pairs) of SC-4096 atoms (corners, faces, interior)
    bit-identical to the reference arithmetic over the oracle's NeighborList(5, inf)."""
    batch = dgn.synth_batch("sc", 16, 1)
    lat, pos = batch["lattice"][0], batch["positions"]
    for a in (0, 15, 255, 2047, 2730, 4095):
        lower, npts, keys = ctx.debug_betti_clouds(batch, 5.0, a, 1, 64)
        got, mapped, _, _ = _kernel_vs_reference_triangles(lower[0], npts[0], keys[0], lat, pos, a, 5.0)
        assert np.array_equal(got.view(np.uint32), mapped.view(np.uint32)), a
