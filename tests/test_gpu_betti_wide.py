"""Wide local complexes (65..512 points: the reference's default 10 A cutoff) through the C ABI
vs the reference's verbatim vendored Ripser (oracle/_ref) — counts and pairs bit-exact, the 35
statistics within 1e-6 relative. Every atom of 741.vasp and of one FCC-256 structure at 10 A is
checked against committed verbatim-Ripser fixtures (tests/golden/rc10.npz, made by
tests/golden/make_golden.py rc10); other 10 A checks spot-check atoms live (~1 s per complex)."""
import os

import numpy as np
import pytest
from conftest import GOLDEN

import dgn
import oracle_py as O

pytestmark = pytest.mark.gpu
FEAT_RTOL, FEAT_ATOL = 1e-6, 1e-12


def _ref(low, n, thr):
    return O.ref_persistence(low, n, thr) if O.ref_available() else O.persistence(low, n, thr)


def _check_clouds(ctx, clouds, npts, thr, cap):
    pairs, counts = ctx.host_persistence(clouds, npts, thr, cap=cap)
    bad = []
    for c in range(len(npts)):
        n = int(npts[c])
        r = _ref(O.local_distances(clouds[c, :n]), n, np.float32(thr))
        got = {"dim0": pairs[c, 0, :counts[c, 0]], "dim1": pairs[c, 1, :counts[c, 2]], "dim2": pairs[c, 2, :counts[c, 3]]}
        ok = all(np.array_equal(np.array(sorted(map(tuple, got[d]))).reshape(-1, 2), r[d].reshape(-1, 2))
                 for d in got) and counts[c, 1] == r["n_inf0"]
        if not ok:
            bad.append((c, n, counts[c].tolist(), [len(r[d]) for d in ("dim0", "dim1", "dim2")], r["n_inf0"]))
    assert not bad, bad[:8]


def test_wide_random_clouds(ctx):
    rng = np.random.default_rng(21)
    C, maxp = 24, 200
    npts = rng.integers(65, maxp + 1, size=C).astype(np.int32)
    clouds = np.zeros((C, maxp, 3))
    for c in range(C):
        if c % 4 == 0:
            clouds[c, :npts[c]] = rng.integers(0, 6, size=(npts[c], 3))  # exact ties
        else:
            clouds[c, :npts[c]] = rng.uniform(0, 6, size=(npts[c], 3))
    _check_clouds(ctx, clouds, npts, 2.0, 4096)


def test_all_three_tiers_in_one_batch(ctx):
    """2..150 points: <= 48 main launch, 49..64 overflow launch, 65.. wide kernel."""
    rng = np.random.default_rng(23)
    C, maxp = 60, 150
    npts = rng.integers(2, maxp + 1, size=C).astype(np.int32)
    npts[:4] = [40, 60, 100, 150]
    clouds = np.zeros((C, maxp, 3))
    for c in range(C):
        clouds[c, :npts[c]] = rng.uniform(0, 5.5, size=(npts[c], 3))
    _check_clouds(ctx, clouds, npts, 1.8, 4096)


def _rc10_inputs(name):
    if name == "741":
        fx = np.load(os.path.join(GOLDEN, "poscar_rc5.npz"))
        pos = fx["741/positions"]
        return {"lattice": fx["741/lattice"][None].copy(), "positions": pos.copy(),
                "species": fx["741/species"].astype(np.int32), "atom_offset": np.array([0, len(pos)], np.int64)}
    return dgn.synth_batch("fcc", 4, 1)


@pytest.mark.parametrize("name", ["741", "fcc256_0"])
def test_default_cutoff_10A_every_atom(ctx, name):
    """compute_structure_betti_features at the reference's default r_cutoff = 10
    (preprocess_betti.cpp:117; betti_features.cpp:103-119) for EVERY atom of 741.vasp (120 atoms,
    ~300-point complexes) and of FCC-256 structure 0 (256 atoms, ~340 points) against the
    verbatim-Ripser fixtures: counts bit-exact, statistics within 1e-6."""
    fx = np.load(os.path.join(GOLDEN, "rc10.npz"))
    batch = _rc10_inputs(name)
    if name == "fcc256_0":
        assert np.array_equal(batch["positions"], fx["fcc256_0/positions"])  # generator bit-identity
    f, c = ctx.host_betti(batch, 10.0)
    fo, co = fx[f"{name}/features"], fx[f"{name}/counts"]
    assert f.shape == fo.shape and not np.isnan(f).any()
    bad = np.nonzero((c != co).any(axis=1))[0]
    assert bad.size == 0, (bad[:8], c[bad[:4]], co[bad[:4]])
    np.testing.assert_allclose(f, fo, rtol=FEAT_RTOL, atol=FEAT_ATOL)


def test_f32_instantiations_363_to_512_points(ctx):
    """Complexes of 363..512 points keep f32 distances (u16 rank codes need C(n, 2) < 2^16): the
    6- and 8-word instantiations, against verbatim Ripser."""
    rng = np.random.default_rng(29)
    sizes = [450, 380]
    clouds = np.zeros((len(sizes), max(sizes), 3))
    for c, n in enumerate(sizes):
        clouds[c, :n] = rng.uniform(0, 8.0, size=(n, 3))
    _check_clouds(ctx, clouds, np.array(sizes, dtype=np.int32), 1.7, 8192)


def test_f32_fallback_matches_rank_codes(ctx):
    """DGN_DEBUG_WIDE_C16 = 0 (f32 distances for every wide complex) gives the same pairs as the
    default u16 rank codes; both against verbatim Ripser."""
    rng = np.random.default_rng(31)
    sizes = [300, 150, 70]
    clouds = np.zeros((len(sizes), max(sizes), 3))
    for c, n in enumerate(sizes):
        clouds[c, :n] = rng.uniform(0, 6.0, size=(n, 3))
    npts = np.array(sizes, dtype=np.int32)
    _check_clouds(ctx, clouds, npts, 1.9, 8192)
    p16, k16 = ctx.host_persistence(clouds, npts, 1.9, cap=8192)
    ctx.set_debug(dgn.abi.DEBUG_WIDE_C16, 0)
    try:
        p32, k32 = ctx.host_persistence(clouds, npts, 1.9, cap=8192)
    finally:
        ctx.set_debug(dgn.abi.DEBUG_WIDE_C16, 1)
    assert np.array_equal(k32, k16)
    for c in range(len(sizes)):  # the emitted pairs (entries past each count are not written)
        for d, col in ((0, 0), (1, 2), (2, 3)):
            n = k16[c, col]
            assert np.array_equal(p32[c, d, :n], p16[c, d, :n]), (c, d)


def test_10A_fused_step_never_waits_for_the_host(ctx):
    """dgn_dev_graph_betti at the reference's default 10 A cutoff (every complex ~340 points: the
    wide tier on u16 rank codes) returns without waiting for the stream: the rank-code slices are
    sized from the count pass's census of wide complexes and take their lengths on the device, and
    the capacity retry is device-driven. Its outputs equal the verbatim-Ripser fixtures of FCC-256
    structure 0 (counts exact, statistics within 1e-6)."""
    import torch
    from dgn import abi
    fx = np.load(os.path.join(GOLDEN, "rc10.npz"))
    host = dgn.synth_batch("fcc", 4, 1)
    dev = torch.device("cuda", 0)
    batch = {k: torch.from_numpy(v).to(dev) for k, v in host.items()}
    A = host["positions"].shape[0]
    gp = abi.graph_params(r_cutoff=10.0, max_neighbors=20, rbf_cutoff=10.0, rbf_dr=0.1, rbf_dtype=dgn.DGN_F32)
    nb = abi.lib().dgn_rbf_bins(10.0, 0.1)
    feat = torch.empty((A, 35), dtype=torch.float64, device=dev)
    cnt = torch.empty((A, 4), dtype=torch.int32, device=dev)
    for rep in range(2):  # the first call allocates and initialises the workspaces
        E = ctx.dev_graph_count(batch, gp)
        rp = torch.empty(A + 1, dtype=torch.int64, device=dev)
        col = torch.empty(E, dtype=torch.int32, device=dev)
        dist = torch.empty(E, dtype=torch.float64, device=dev)
        rbf = torch.empty((E, nb), dtype=torch.float32, device=dev)
        ctx.host_syncs()
        ctx.dev_graph_betti(batch, gp, rp, col, dist, None, rbf, 10.0, feat, cnt)
        assert ctx.host_syncs() == 0, rep
        ctx.synchronize()
    bad = np.nonzero((cnt.cpu().numpy() != fx["fcc256_0/counts"]).any(axis=1))[0]
    assert bad.size == 0, bad[:8]
    np.testing.assert_allclose(feat.cpu().numpy(), fx["fcc256_0/features"], rtol=FEAT_RTOL, atol=FEAT_ATOL)


def test_walk_pass_matches_per_wave_walk(ctx):
    """The u16-coded wide complexes' dim-2 apparent walk as a workgroup-per-complex pass with the
    code triangle in LDS (default) against the per-wave kernel's own walk (DGN_DEBUG_WIDE_WALK = 0):
    identical counts, pairs and statistics; random clouds (with exact ties) of 65..362 points, both
    against verbatim Ripser, and every atom of FCC-256 structure 0 at 10 A byte for byte."""
    rng = np.random.default_rng(37)
    sizes = [362, 65, 129, 200, 257, 330]
    clouds = np.zeros((len(sizes), max(sizes), 3))
    for c, n in enumerate(sizes):
        clouds[c, :n] = rng.integers(0, 7, size=(n, 3)) if c % 2 else rng.uniform(0, 6.5, size=(n, 3))
    npts = np.array(sizes, dtype=np.int32)
    _check_clouds(ctx, clouds, npts, 1.9, 8192)
    p1, k1 = ctx.host_persistence(clouds, npts, 1.9, cap=8192)
    batch = dgn.synth_batch("fcc", 4, 1)
    f1, c1 = ctx.host_betti(batch, 10.0)
    ctx.set_debug(dgn.abi.DEBUG_WIDE_WALK, 0)
    try:
        p0, k0 = ctx.host_persistence(clouds, npts, 1.9, cap=8192)
        f0, c0 = ctx.host_betti(batch, 10.0)
    finally:
        ctx.set_debug(dgn.abi.DEBUG_WIDE_WALK, 1)
    assert np.array_equal(k0, k1)
    for c in range(len(sizes)):
        for d, col in ((0, 0), (1, 2), (2, 3)):
            n = k1[c, col]
            a0 = np.array(sorted(map(tuple, p0[c, d, :n])))
            a1 = np.array(sorted(map(tuple, p1[c, d, :n])))
            assert np.array_equal(a0, a1), (c, d)
    assert np.array_equal(c0, c1) and np.array_equal(f0.view(np.uint64), f1.view(np.uint64))
