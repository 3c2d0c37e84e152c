"""HIP neighbour search + CSR + RBF through the C ABI vs the CPU oracle (bit-exact CSR and
distances; RBF within 1e-6 relative as north_star states)."""
import os

import numpy as np
import pytest
from conftest import GOLDEN, mixed_batch

import dgn
import oracle_py as O
from dgn import abi

pytestmark = pytest.mark.gpu

RBF_RTOL = 1e-6  # north_star: RBF/distance floats within 1e-6 relative


def oracle_batch_csr(batch, rc, k, epsilon=1e-10):
    rp_all, col_all, dist_all, disp_all = [np.zeros(1, np.int64)], [], [], []
    off = batch["atom_offset"]
    base = 0
    for s in range(len(off) - 1):
        a, b = off[s], off[s + 1]
        nl = O.neighbor_list(batch["lattice"][s], batch["positions"][a:b], rc, k, epsilon=epsilon)
        rp_all.append(nl["row_ptr"][1:] + base)
        base += nl["row_ptr"][-1]
        col_all.append(nl["col"])
        dist_all.append(nl["dist"])
        disp_all.append(nl["disp"])
    return (np.concatenate(rp_all), np.concatenate(col_all), np.concatenate(dist_all), np.concatenate(disp_all))


def check_rbf(rbf, dist, rc, dr):
    ref = np.stack([O.gaussian_rbf(d, rc, dr) for d in dist])
    rel = np.abs(rbf.astype(np.float64) - ref) / np.abs(ref)
    assert rel.max() < RBF_RTOL, rel.max()


@pytest.mark.parametrize("k", [20, 12, None])
def test_sc64_batch(ctx, k):
    batch = dgn.synth_batch("sc", 4, 16)
    p = abi.graph_params(r_cutoff=5.0, max_neighbors=k, rbf_cutoff=5.0, rbf_dr=0.1, write_displacement=True)
    g = ctx.host_graph(batch, p)
    rp, col, dist, disp = oracle_batch_csr(batch, 5.0, k)
    assert np.array_equal(g["row_ptr"], rp)
    assert np.array_equal(g["col"], col)
    assert np.array_equal(g["dist"], dist)  # bit-exact: same op order, correctly rounded sqrt
    assert np.array_equal(g["disp"], disp)
    check_rbf(g["rbf"], dist, 5.0, 0.1)


def test_fcc256_rbf_f64_default_cutoff(ctx):
    batch = dgn.synth_batch("fcc", 4, 4)
    p = abi.graph_params(r_cutoff=5.0, max_neighbors=20, rbf_cutoff=10.0, rbf_dr=0.1, rbf_dtype=dgn.DGN_F64)
    g = ctx.host_graph(batch, p)
    rp, col, dist, _ = oracle_batch_csr(batch, 5.0, 20)
    assert np.array_equal(g["row_ptr"], rp) and np.array_equal(g["col"], col) and np.array_equal(g["dist"], dist)
    assert g["rbf"].shape == (len(dist), 100)
    ref = np.stack([O.gaussian_rbf(d, 10.0, 0.1) for d in dist])
    np.testing.assert_allclose(g["rbf"], ref, rtol=1e-13, atol=0)


@pytest.mark.parametrize("name", ["1", "1_1", "1_2", "741", "741_1", "741_2", "1046", "1046_1", "1046_2"])
@pytest.mark.parametrize("k", [12, 20])
def test_poscar_fixtures(ctx, name, k):
    fx = np.load(os.path.join(GOLDEN, "poscar_rc5.npz"))
    batch = {"lattice": fx[f"{name}/lattice"][None].copy(), "positions": fx[f"{name}/positions"].copy(),
             "species": fx[f"{name}/species"].astype(np.int32), "atom_offset": np.array([0, len(fx[f"{name}/positions"])], np.int64)}
    p = abi.graph_params(r_cutoff=5.0, max_neighbors=k, rbf_cutoff=5.0, rbf_dr=0.1)
    g = ctx.host_graph(batch, p)
    rp = fx[f"{name}/k{k}/row_ptr"]
    assert np.array_equal(g["row_ptr"], rp)
    assert np.array_equal(g["dist"], fx[f"{name}/k{k}/dist"])
    # CSR indices bit-exact; rows with exact distance ties compare as multisets (tie order is
    # implementation-defined in the reference)
    col, ref_col, d = g["col"], fx[f"{name}/k{k}/col"], fx[f"{name}/k{k}/dist"]
    for i in range(len(rp) - 1):
        a, b = rp[i], rp[i + 1]
        if np.array_equal(col[a:b], ref_col[a:b]):
            continue
        assert sorted(zip(d[a:b], col[a:b])) == sorted(zip(d[a:b], ref_col[a:b])), (name, i)
    if name in ("1", "741"):
        np.testing.assert_allclose(g["rbf"], fx[f"{name}/k{k}/rbf"], rtol=RBF_RTOL, atol=0)


def test_supercell_4096(ctx):
    batch = dgn.synth_batch("sc", 16, 1)
    p = abi.graph_params(r_cutoff=5.0, max_neighbors=20, rbf_cutoff=5.0, rbf_dr=0.1)
    g = ctx.host_graph(batch, p)
    rp, col, dist, _ = oracle_batch_csr(batch, 5.0, 20)
    assert np.array_equal(g["row_ptr"], rp) and np.array_equal(g["col"], col) and np.array_equal(g["dist"], dist)


@pytest.mark.parametrize("k,rbf_rc,dtype", [(None, 5.0, dgn.DGN_F32), (7, 4.95, dgn.DGN_F64), (20, 4.95, dgn.DGN_F32)])
def test_empty_and_ragged(ctx, k, rbf_rc, dtype):
    # structures of different sizes in one batch, including a 1-atom cell with no neighbours and
    # an empty structure; odd RBF bin counts exercise the unaligned head/tail of the RBF stream
    a = dgn.synth_batch("sc", 2, 1)
    b = dgn.synth_batch("fcc", 2, 1)
    c = dgn.synth_batch("sc", 3, 2)
    lone = {"lattice": np.eye(3)[None] * 20.0, "positions": np.array([[1.0, 2.0, 3.0]]),
            "species": np.zeros(1, np.int32)}
    empty = {"lattice": np.eye(3)[None] * 10.0, "positions": np.zeros((0, 3)), "species": np.zeros(0, np.int32)}
    parts = [a, lone, empty, b, c]
    batch = {"lattice": np.concatenate([x["lattice"] for x in parts]),
             "positions": np.concatenate([x["positions"] for x in parts]),
             "species": np.concatenate([x["species"] for x in parts]).astype(np.int32)}
    sizes = [len(x["positions"]) for x in parts]
    batch["atom_offset"] = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    p = abi.graph_params(r_cutoff=5.0, max_neighbors=k, rbf_cutoff=rbf_rc, rbf_dr=0.1, rbf_dtype=dtype,
                         write_displacement=True)
    g = ctx.host_graph(batch, p)
    rp, col, dist, disp = oracle_batch_csr(batch, 5.0, k)
    assert np.array_equal(g["row_ptr"], rp) and np.array_equal(g["col"], col) and np.array_equal(g["dist"], dist)
    assert np.array_equal(g["disp"], disp)
    lone_row = sizes[0]
    assert rp[lone_row + 1] - rp[lone_row] == 0
    ref = np.stack([O.gaussian_rbf(d, rbf_rc, 0.1) for d in dist])
    assert g["rbf"].shape == ref.shape
    np.testing.assert_allclose(g["rbf"], ref, rtol=1e-13 if dtype == dgn.DGN_F64 else RBF_RTOL, atol=0)


@pytest.mark.parametrize("npairs", [8, 520])
def test_mixed_one_image_and_general_tiles(ctx, npairs):
    # 8 pairs: 2,560 atoms, 4-atom count tiles; 520 pairs: 166,400 atoms, 64-atom tiles (some
    # straddle an FCC and an SC cell)
    batch = mixed_batch(npairs)
    p = abi.graph_params(r_cutoff=5.0, max_neighbors=20, rbf_cutoff=5.0, rbf_dr=0.1, rbf_dtype=dgn.DGN_F64,
                         write_displacement=True)
    g = ctx.host_graph(batch, p)
    rp, col, dist, disp = oracle_batch_csr(batch, 5.0, 20)
    assert np.array_equal(g["row_ptr"], rp) and np.array_equal(g["col"], col) and np.array_equal(g["dist"], dist)
    assert np.array_equal(g["disp"], disp)


def few_image_batch(seed, B=24, rc=5.0, nmax=90, hlo=0.5, hhi=0.98):
    """Cells whose perpendicular widths lie between rc and 2 rc (max H_k in (0.5, 1): at most two
    images per axis reach rc, the `few` staged search), triclinic and axis-aligned, 5..nmax atoms
    with fractional coordinates in [-0.2, 1.2) (atoms outside the cell: images n = +-2)."""
    rng = np.random.default_rng(seed)
    lat, pos, sizes = [], [], []
    while len(lat) < B:
        lo = 1.0 / hhi if hhi > 0.98 else 1.05  # cells just wider than rc when hhi is near 1
        L = np.diag(rng.uniform(lo, 1.9, 3) * rc) + np.triu(rng.uniform(-0.35, 0.35, (3, 3)) * rc, 1)
        if len(lat) % 3 == 0:
            L = np.diag(np.diag(L))
        H = rc * np.linalg.norm(np.linalg.inv(L), axis=0)
        if not (hlo < H.max() < hhi) or np.linalg.norm(L, axis=1).min() < rc:
            continue
        n = int(rng.integers(5, nmax))
        lat.append(L)
        pos.append(rng.uniform(-0.2, 1.2, (n, 3)) @ L)
        sizes.append(n)
    return {"lattice": np.stack(lat), "positions": np.concatenate(pos),
            "species": (np.arange(sum(sizes)) % 3).astype(np.int32),
            "atom_offset": np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)}


@pytest.mark.parametrize("seed,k,hlo,hhi", [(1, 20, 0.5, 0.98), (2, None, 0.5, 0.98), (3, 7, 0.5, 0.98),
                                             (4, None, 0.95, 0.9995)])
def test_few_image_cells(ctx, seed, k, hlo, hhi):
    """Cells narrower than 2 rc but wider than rc (search_staged_few / count_few: up to 2^3 images
    of an atom decided in f32, borderline ones exactly): CSR, distances and displacements bit-exact
    vs the oracle's (2 nref + 1)^3 image scan; the last case has a width within 0.05 % of rc on some
    axis (two images per axis for nearly every pair)."""
    batch = few_image_batch(seed, hlo=hlo, hhi=hhi)
    p = abi.graph_params(r_cutoff=5.0, max_neighbors=k, rbf_cutoff=5.0, rbf_dr=0.1, write_displacement=True)
    g = ctx.host_graph(batch, p)
    rp, col, dist, disp = oracle_batch_csr(batch, 5.0, k)
    assert np.array_equal(g["row_ptr"], rp)
    assert np.array_equal(g["col"], col)
    assert np.array_equal(g["dist"], dist)
    assert np.array_equal(g["disp"], disp)


@pytest.mark.parametrize("eps", [0.0, 1e-10, 5.0])
def test_self_image_epsilon(ctx, eps):
    """NeighborList's epsilon skips only images of the query atom closer than eps
    (neighbor_list.cpp:47): eps = 0 keeps the atom itself at distance 0, eps = 5 also drops its
    periodic images inside a 4.64 A cell. One-image (FCC-256), few-image (SC-64) and general
    (SC-8, L < rc) structures in one batch, CSR bit-exact vs the oracle at the same epsilon."""
    parts = [dgn.synth_batch("fcc", 4, 1), dgn.synth_batch("sc", 4, 2), dgn.synth_batch("sc", 2, 2)]
    batch = {k: np.concatenate([x[k] for x in parts]) for k in ("lattice", "positions", "species")}
    sizes = np.concatenate([np.diff(x["atom_offset"]) for x in parts])
    batch["atom_offset"] = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    p = abi.graph_params(r_cutoff=5.0, max_neighbors=None, epsilon=eps, rbf_cutoff=5.0, rbf_dr=0.1,
                         write_displacement=True)
    g = ctx.host_graph(batch, p)
    rp, col, dist, disp = oracle_batch_csr(batch, 5.0, None, epsilon=eps)
    assert np.array_equal(g["row_ptr"], rp)
    assert np.array_equal(g["col"], col)
    assert np.array_equal(g["dist"], dist)
    assert np.array_equal(g["disp"], disp)
    if eps == 0.0:
        assert (g["dist"] == 0.0).sum() == len(batch["positions"])  # every atom lists itself once


@pytest.mark.parametrize("layout", [0, 1])
def test_rbf_of_given_distances(ctx, layout):
    d = np.linspace(0.0, 9.99, 777)
    for dt, tol in ((dgn.DGN_F64, 1e-13), (dgn.DGN_F32, RBF_RTOL)):
        out = ctx.host_rbf(d, 10.0, 0.1, dt, layout)
        ref = np.stack([O.gaussian_rbf(x, 10.0, 0.1) for x in d])
        assert out.shape == ref.shape
        assert np.max(np.abs(out - ref) / ref) < tol


def test_device_count_emit_full_shard(ctx):
    """The bench's device-level path (dgn_dev_graph_count -> dgn_dev_graph_emit on torch tensors)
    at the full config-4 shard size, twice: the emit's deferred consistency flag must stay clear
    and sampled structures must match the oracle bit for bit."""
    import torch
    B = 8192
    host = dgn.synth_batch("fcc", 4, B)
    batch = {k: torch.from_numpy(v).cuda() for k, v in host.items()}
    gp = abi.graph_params(r_cutoff=5.0, max_neighbors=20, rbf_cutoff=5.0, rbf_dr=0.1, rbf_dtype=dgn.DGN_F32)
    A = host["positions"].shape[0]
    for _ in range(2):
        E = ctx.dev_graph_count(batch, gp)
        rp = torch.empty(A + 1, dtype=torch.int64, device="cuda")
        col = torch.empty(E, dtype=torch.int32, device="cuda")
        dist = torch.empty(E, dtype=torch.float64, device="cuda")
        rbf = torch.empty((E, 50), dtype=torch.float32, device="cuda")
        ctx.dev_graph_emit(batch, gp, rp, col, dist, None, rbf)
        ctx.synchronize()  # raises on a count/emit disagreement
    rp, col, dist, rbf = rp.cpu().numpy(), col.cpu().numpy(), dist.cpu().numpy(), rbf.cpu().numpy()
    n = 256
    for s in (0, 1, 4095, B - 1):
        nl = O.neighbor_list(host["lattice"][s], host["positions"][s * n:(s + 1) * n], 5.0, 20)
        a, b = rp[s * n], rp[(s + 1) * n]
        assert np.array_equal(rp[s * n:(s + 1) * n + 1] - a, nl["row_ptr"])
        assert np.array_equal(col[a:b], nl["col"]) and np.array_equal(dist[a:b], nl["dist"])
        check_rbf(rbf[a:b], nl["dist"], 5.0, 0.1)


def test_fcc256_cutoff_17A_above_1024_candidates(ctx):
    """NeighborList(rc = 17, K = 20): ~1,650 candidates per atom (the 2,048-candidate streamed
    emit), CSR bit-exact."""
    batch = dgn.synth_batch("fcc", 4, 1)
    p = abi.graph_params(r_cutoff=17.0, max_neighbors=20, rbf_cutoff=17.0, rbf_dr=0.1, write_displacement=True)
    g = ctx.host_graph(batch, p)
    rp, col, dist, disp = oracle_batch_csr(batch, 17.0, 20)
    assert np.array_equal(g["row_ptr"], rp)
    assert np.array_equal(g["col"], col)
    assert np.array_equal(g["dist"], dist)
    assert np.array_equal(g["disp"], disp)
    check_rbf(g["rbf"], dist, 17.0, 0.1)


@pytest.mark.parametrize("rc,k", [(17.0, None), (20.0, 20), (20.0, None)])
def test_fcc256_large_rows_global_keys(ctx, rc, k):
    """Rows past the LDS hit lists (more than 2,048 candidates, or more than 1,024 without a
    neighbour cap; neighbor_list.cpp:27-66 has no cap): the emit keeps each wave's hit list, keys
    and sorted distances in HBM (kEmitGlobalKeys). FCC-256 at 17 A (~1,650 candidates, K = inf)
    and 20 A (~2,700), CSR, distances and displacements bit-exact vs the oracle, f32 RBF (0.5 A
    bins to the cutoff) within 1e-6."""
    batch = dgn.synth_batch("fcc", 4, 1)
    p = abi.graph_params(r_cutoff=rc, max_neighbors=k, rbf_cutoff=rc, rbf_dr=0.5, write_displacement=True)
    g = ctx.host_graph(batch, p)
    rp, col, dist, disp = oracle_batch_csr(batch, rc, k)
    if k is None:
        assert np.diff(rp).max() > (2048 if rc == 20.0 else 1024)
    assert np.array_equal(g["row_ptr"], rp)
    assert np.array_equal(g["col"], col)
    assert np.array_equal(g["dist"], dist)
    assert np.array_equal(g["disp"], disp)
    check_rbf(g["rbf"], dist, rc, 0.5)


def test_large_rows_chunked_launches(ctx):
    """The global-key emit's chunk loop: key rows are reused launch after launch, a few tiles at a
    time (DGN_DEBUG_EMIT_CHUNK = 3 instead of the 256 MB budget's count, which covers a single
    structure in one launch). FCC-256 at 17 A, K = inf: CSR, distances and displacements bit-exact
    vs the oracle."""
    batch = dgn.synth_batch("fcc", 4, 1)
    p = abi.graph_params(r_cutoff=17.0, max_neighbors=None, rbf_cutoff=17.0, rbf_dr=0.5, write_displacement=True)
    ctx.set_debug(abi.DEBUG_EMIT_CHUNK, 3)
    try:
        g = ctx.host_graph(batch, p)
    finally:
        ctx.set_debug(abi.DEBUG_EMIT_CHUNK, 0)
    rp, col, dist, disp = oracle_batch_csr(batch, 17.0, None)
    assert np.array_equal(g["row_ptr"], rp)
    assert np.array_equal(g["col"], col)
    assert np.array_equal(g["dist"], dist)
    assert np.array_equal(g["disp"], disp)
    check_rbf(g["rbf"], dist, 17.0, 0.5)


@pytest.mark.parametrize("k", [20, None])
def test_fcc256_cutoff_12A_above_512_candidates(ctx, k):
    """NeighborList(rc = 12): ~580 candidates per atom (the 1,024-candidate emit), CSR bit-exact."""
    batch = dgn.synth_batch("fcc", 4, 1)
    p = abi.graph_params(r_cutoff=12.0, max_neighbors=k, rbf_cutoff=12.0, rbf_dr=0.1, write_displacement=True)
    g = ctx.host_graph(batch, p)
    rp, col, dist, disp = oracle_batch_csr(batch, 12.0, k)
    if k is None:
        assert np.diff(rp).max() > 512
    assert np.array_equal(g["row_ptr"], rp)
    assert np.array_equal(g["col"], col)
    assert np.array_equal(g["dist"], dist)
    assert np.array_equal(g["disp"], disp)
    check_rbf(g["rbf"], dist, 12.0, 0.1)
