"""HIP Betti path (Gram distances + wave-parallel VR reduction + statistics) through the C ABI
vs the oracle and the verbatim-Ripser golden fixtures. Counts and pairs bit-exact; the 35
statistics within 1e-6 relative (absolute floor 1e-12: std of near-constant sets)."""
import os

import numpy as np
import pytest
from conftest import GOLDEN, mixed_batch

import dgn
import oracle_py as O

pytestmark = pytest.mark.gpu
FEAT_RTOL, FEAT_ATOL = 1e-6, 1e-12


def test_kat_pairs(ctx):
    kat = np.load(os.path.join(GOLDEN, "kat.npz"))
    names = sorted({k.split("/")[0] for k in kat.files})
    for name in names:
        pts = kat[f"{name}/cloud"]
        thr = float(kat[f"{name}/threshold"])
        pairs, counts = ctx.host_persistence(pts[None], [pts.shape[0]], thr, cap=64)
        for di, d in enumerate(("dim0", "dim1", "dim2")):
            n = counts[0, [0, 2, 3][di]]
            assert np.array_equal(pairs[0, di, :n], kat[f"{name}/{d}"]), (name, d, pairs[0, di, :n])
        assert counts[0, 1] == int(kat[f"{name}/n_inf0"]), name


def test_random_clouds_pairs_exact(ctx):
    rng = np.random.default_rng(5)
    C, maxp = 300, 48
    clouds = np.zeros((C, maxp, 3))
    npts = rng.integers(2, maxp + 1, size=C).astype(np.int32)
    thr = 2.5
    for c in range(C):
        if c % 4 == 0:
            clouds[c, :npts[c]] = rng.integers(0, 3, size=(npts[c], 3))  # exact ties
        else:
            clouds[c, :npts[c]] = rng.uniform(0, 4, size=(npts[c], 3))
    pairs, counts = ctx.host_persistence(clouds, npts, thr, cap=512)
    bad = []
    for c in range(C):
        n = npts[c]
        low = O.local_distances(clouds[c, :n])
        r = O.persistence(low, n, np.float32(thr))
        got = {"dim0": pairs[c, 0, :counts[c, 0]], "dim1": pairs[c, 1, :counts[c, 2]], "dim2": pairs[c, 2, :counts[c, 3]]}
        ok = all(np.array_equal(got[d], r[d]) for d in got) and counts[c, 1] == r["n_inf0"]
        if not ok:
            bad.append((c, n, counts[c].tolist(), [len(r[d]) for d in ("dim0", "dim1", "dim2")], r["n_inf0"]))
    assert not bad, bad[:10]


@pytest.mark.parametrize("s", range(8))
def test_sc64_fixture(ctx, s):
    fx = np.load(os.path.join(GOLDEN, "sc64_rc5.npz"))
    batch = dgn.synth_batch("sc", 4, 8)
    n = 64
    one = {"lattice": batch["lattice"][s:s + 1].copy(), "positions": batch["positions"][s * n:(s + 1) * n].copy(),
           "species": batch["species"][s * n:(s + 1) * n].copy(), "atom_offset": np.array([0, n], np.int64)}
    f, c = ctx.host_betti(one, 5.0)
    assert np.array_equal(c, fx[f"{s}/counts"]), np.argwhere(c != fx[f"{s}/counts"])[:5]
    np.testing.assert_allclose(f, fx[f"{s}/features"], rtol=FEAT_RTOL, atol=FEAT_ATOL)


@pytest.mark.parametrize("name", ["1", "1046", "1046_1", "1046_2", "1_1", "1_2", "741", "741_1", "741_2"])
def test_poscar_fixture(ctx, name):
    fx = np.load(os.path.join(GOLDEN, "poscar_rc5.npz"))
    pos = fx[f"{name}/positions"]
    one = {"lattice": fx[f"{name}/lattice"][None].copy(), "positions": pos.copy(),
           "species": fx[f"{name}/species"].astype(np.int32), "atom_offset": np.array([0, len(pos)], np.int64)}
    f, c = ctx.host_betti(one, 5.0)
    assert np.array_equal(c, fx[f"{name}/betti5/counts"])
    np.testing.assert_allclose(f, fx[f"{name}/betti5/features"], rtol=FEAT_RTOL, atol=FEAT_ATOL)


def test_fcc256_batch_vs_oracle(ctx):
    batch = dgn.synth_batch("fcc", 4, 3)
    f, c = ctx.host_betti(batch, 5.0)
    n = 256
    for s in range(3):
        sl = slice(s * n, (s + 1) * n)
        fo, co = O.structure_betti(batch["lattice"][s], batch["positions"][sl], batch["species"][sl], 5.0)
        assert np.array_equal(c[sl], co)
        np.testing.assert_allclose(f[sl], fo, rtol=FEAT_RTOL, atol=FEAT_ATOL)


def test_mixed_one_image_and_general_tiles(ctx):
    # FCC-256 (one-image count kernel + its hit masks) alternating with SC-64 (general search):
    # the Betti search reads the masks of the one-image tiles only
    batch = mixed_batch(2)
    f, c = ctx.host_betti(batch, 5.0)
    off = batch["atom_offset"]
    for s in range(len(off) - 1):
        sl = slice(off[s], off[s + 1])
        fo, co = O.structure_betti(batch["lattice"][s], batch["positions"][sl], batch["species"][sl], 5.0)
        assert np.array_equal(c[sl], co)
        np.testing.assert_allclose(f[sl], fo, rtol=FEAT_RTOL, atol=FEAT_ATOL)


def test_few_image_cells(ctx):
    # cells between rc and 2 rc wide (the `few` staged search builds the local clouds): triclinic
    # and axis-aligned, atoms partly outside the cell
    from test_gpu_graph import few_image_batch
    batch = few_image_batch(5, B=8, nmax=36)
    f, c = ctx.host_betti(batch, 5.0)
    off = batch["atom_offset"]
    for s in range(len(off) - 1):
        sl = slice(off[s], off[s + 1])
        fo, co = O.structure_betti(batch["lattice"][s], batch["positions"][sl], batch["species"][sl], 5.0)
        assert np.array_equal(c[sl], co)
        np.testing.assert_allclose(f[sl], fo, rtol=FEAT_RTOL, atol=FEAT_ATOL)


def test_isolated_atom(ctx):
    one = {"lattice": np.eye(3)[None] * 30.0, "positions": np.array([[1.0, 1.0, 1.0], [15.0, 15.0, 15.0]]),
           "species": np.array([0, 1], np.int32), "atom_offset": np.array([0, 2], np.int64)}
    f, c = ctx.host_betti(one, 5.0)
    assert np.all(f == 0.0)
    assert c.tolist() == [[0, 1, 0, 0], [0, 1, 0, 0]]


def test_persistence_from_distance_matrix(ctx):
    # compute_persistence_from_distances input mode: the packed f32 lower triangle
    rng = np.random.default_rng(9)
    maxp, C = 40, 50
    npts = rng.integers(2, maxp + 1, size=C).astype(np.int32)
    lows = np.zeros((C, maxp * (maxp - 1) // 2), np.float32)
    refs = []
    for c in range(C):
        pts = rng.uniform(0, 4, size=(npts[c], 3))
        low = O.local_distances(pts)
        lows[c, :low.shape[0]] = low
        refs.append(O.persistence(low, npts[c], np.float32(2.5)))
    # the kernel reads row i at offset i*(i-1)/2 of a max_points-sized triangle: same packing
    pairs, counts = ctx.host_persistence_lower(lows, npts, maxp, 2.5, cap=256)
    for c in range(C):
        r = refs[c]
        assert np.array_equal(pairs[c, 1, :counts[c, 2]], r["dim1"]) and np.array_equal(pairs[c, 2, :counts[c, 3]], r["dim2"])
        assert np.array_equal(pairs[c, 0, :counts[c, 0]], r["dim0"])


def test_mixed_sizes_two_level_dispatch(ctx):
    """Complexes of 2..64 points in one batch: <= 48 go to the main launch, the rest through
    the bucket pass to the NP = 64 overflow launch; every complex must match the oracle."""
    rng = np.random.default_rng(11)
    C, maxp = 160, 64
    clouds = np.zeros((C, maxp, 3))
    npts = rng.integers(2, maxp + 1, size=C).astype(np.int32)
    npts[:8] = maxp  # guarantee overflow members
    for c in range(C):
        clouds[c, :npts[c]] = rng.uniform(0, 4.5, size=(npts[c], 3))
    pairs, counts = ctx.host_persistence(clouds, npts, 2.5, cap=1024)
    for c in range(C):
        n = npts[c]
        r = O.persistence(O.local_distances(clouds[c, :n]), n, np.float32(2.5))
        assert counts[c, 1] == r["n_inf0"], c
        for di, d in enumerate(("dim0", "dim1", "dim2")):
            assert np.array_equal(pairs[c, di, :counts[c, [0, 2, 3][di]]], r[d]), (c, n, d)


def test_betti_batch_with_dense_outlier(ctx):
    """A compressed FCC cell (about 50 neighbours within rc) inside a batch of ordinary ones:
    its atoms take the overflow launch, the others the main launch."""
    batch = dgn.synth_batch("fcc", 4, 3)
    n = 256
    batch["lattice"][1] *= 0.95
    batch["positions"][n:2 * n] *= 0.95
    f, c = ctx.host_betti(batch, 5.0)
    sizes = []
    for s in range(3):
        sl = slice(s * n, (s + 1) * n)
        nl = O.neighbor_list(batch["lattice"][s], batch["positions"][sl], 5.0, None)
        sizes.append(int(np.diff(nl["row_ptr"]).max()) + 1)
        fo, co = O.structure_betti(batch["lattice"][s], batch["positions"][sl], batch["species"][sl], 5.0)
        assert np.array_equal(c[sl], co), s
        np.testing.assert_allclose(f[sl], fo, rtol=FEAT_RTOL, atol=FEAT_ATOL)
    assert sizes[1] > 48 and max(sizes[0], sizes[2]) <= 48, sizes


def _kernel_vs_reference_triangles(lower, npts, keys, lat, pos, a, rc):
    """Map the Betti distance kernel's cloud rows to the reference's (centre, then the
    NeighborList(rc, inf) rows in canonical order, betti_features.cpp:67-73) through the (j, image)
    keys, and return (kernel triangle, reference triangle re-indexed into the kernel's order)."""
    nl = O.neighbor_list(lat, pos, rc, None)
    r0, r1 = nl["row_ptr"][a], nl["row_ptr"][a + 1]
    n = int(npts)
    assert n == r1 - r0 + 1
    cloud = np.vstack([pos[a], pos[a] + nl["disp"][r0:r1]])
    ref_low = O.local_distances(cloud)
    row_of = {(int(nl["col"][e]), *map(int, nl["image"][e])): e - r0 + 1 for e in range(r0, r1)}
    perm = [0]
    for p in range(n - 1):
        k = int(keys[p])
        j, na, nb, nc = k >> 24, ((k >> 16) & 255) - 128, ((k >> 8) & 255) - 128, (k & 255) - 128
        perm.append(row_of[(j, na, nb, nc)])
    assert sorted(perm) == list(range(n))
    tri = lambda i, j: i * (i - 1) // 2 + j  # noqa: E731  (i > j)
    mapped = np.empty(n * (n - 1) // 2, np.float32)
    for i in range(1, n):
        for j in range(i):
            pi, pj = perm[i], perm[j]
            mapped[tri(i, j)] = ref_low[tri(max(pi, pj), min(pi, pj))]
    return lower[:n * (n - 1) // 2], mapped, cloud, ref_low


@pytest.mark.parametrize("s", [0, 3, 7])
def test_betti_dist_triangles_sc64_fixture(ctx, s):
    """The Betti pass's own neighbour search + Gram distances (f64 VALU pairs): every entry of the f32 lower
    triangle bit-identical to the reference arithmetic (sc64_rc5.npz lower0 / lower37, i.e.
    ripser_wrapper.cpp:20-24 over betti_features.cpp:67-73's cloud)."""
    fx = np.load(os.path.join(GOLDEN, "sc64_rc5.npz"))
    batch = dgn.synth_batch("sc", 4, 8)
    n = 64
    one = {"lattice": batch["lattice"][s:s + 1].copy(), "positions": batch["positions"][s * n:(s + 1) * n].copy(),
           "species": batch["species"][s * n:(s + 1) * n].copy(), "atom_offset": np.array([0, n], np.int64)}
    for a in (0, 37):
        lower, npts, keys = ctx.debug_betti_clouds(one, 5.0, a, 1, 64)
        got, mapped, cloud, ref_low = _kernel_vs_reference_triangles(lower[0], npts[0], keys[0], one["lattice"][0],
                                                                     one["positions"], a, 5.0)
        assert np.array_equal(cloud, fx[f"{s}/cloud{a}"])
        assert np.array_equal(ref_low, fx[f"{s}/lower{a}"])
        assert np.array_equal(got.view(np.uint32), mapped.view(np.uint32)), (s, a)


def test_betti_dist_triangles_fcc256(ctx):
    """Same on FCC-256 complexes (43 points) against oracle_local_distances."""
    batch = dgn.synth_batch("fcc", 4, 2)
    n = 256
    atoms = [0, 1, 100, 255, 256, 300, 511]
    lower, npts, keys = ctx.debug_betti_clouds(batch, 5.0, 0, 2 * n, 64)
    for gi in atoms:
        s, a = divmod(gi, n)
        got, mapped, _, _ = _kernel_vs_reference_triangles(lower[gi], npts[gi], keys[gi], batch["lattice"][s],
                                                           batch["positions"][s * n:(s + 1) * n], a, 5.0)
        assert np.array_equal(got.view(np.uint32), mapped.view(np.uint32)), gi


def test_rank_code_tiers_dense_complexes(ctx):
    """The narrow kernels rank the distances <= thr of a complex in registers (512 keys in the
    32/48-point tiers, 1,024 in the 64-point tier): denser complexes take the dense launch (NP = 64
    after the main one) or the capacity retry (wide kernel). Clouds in a ball of radius thr/2 (every
    pair within thr), some with exact ties, across every route; pairs bit-exact vs the oracle."""
    rng = np.random.default_rng(21)
    thr = 2.0
    sizes = [12, 31, 33, 40, 46, 48, 52, 60, 64]
    maxp = max(sizes)
    clouds = np.zeros((2 * len(sizes), maxp, 3))
    npts = np.array(sizes * 2, np.int32)
    for c, n in enumerate(npts):
        d = rng.normal(size=(n, 3))
        d *= (rng.uniform(0, 1, (n, 1)) ** (1 / 3)) / np.linalg.norm(d, axis=1, keepdims=True)
        pts = d * (thr / 2 * 0.999)
        if c >= len(sizes):  # exact ties: a coarse grid inside the same ball
            pts = np.round(pts * 2) / 2
        clouds[c, :n] = pts
    pairs, counts = ctx.host_persistence(clouds, npts, thr, cap=4096)
    for c, n in enumerate(npts):
        r = O.persistence(O.local_distances(clouds[c, :n]), n, np.float32(thr))
        assert counts[c, 1] == r["n_inf0"], c
        for di, d in enumerate(("dim0", "dim1", "dim2")):
            assert np.array_equal(pairs[c, di, :counts[c, [0, 2, 3][di]]], r[d]), (c, n, d)


@pytest.mark.parametrize("thr", [np.inf, 1e39])
def test_unbounded_threshold(ctx, thr):
    """threshold = +inf (or a double above FLT_MAX, +inf after ripser_wrapper.cpp:28's cast):
    every pair is an edge. The narrow rank codes must not take the lanes past the packed
    triangle as edges (their mirrored stores would overwrite real codes). Clouds of
    fewer points than their tier, through the main, dense and retry routes, vs the oracle."""
    rng = np.random.default_rng(23)
    sizes = [3, 17, 30, 31, 40, 44, 47, 60]
    maxp = max(sizes)
    clouds = np.zeros((len(sizes), maxp, 3))
    npts = np.array(sizes, np.int32)
    for c, n in enumerate(npts):
        clouds[c, :n] = rng.uniform(0, 4, size=(n, 3))
    pairs, counts = ctx.host_persistence(clouds, npts, thr, cap=4096)
    for c, n in enumerate(npts):
        r = O.persistence(O.local_distances(clouds[c, :n]), n, np.float32(np.inf))
        assert counts[c, 1] == r["n_inf0"] == 1, c
        for di, d in enumerate(("dim0", "dim1", "dim2")):
            assert np.array_equal(pairs[c, di, :counts[c, [0, 2, 3][di]]], r[d]), (c, n, d)
    lows = np.zeros((len(sizes), maxp * (maxp - 1) // 2), np.float32)
    for c, n in enumerate(npts):
        low = O.local_distances(clouds[c, :n])
        lows[c, :low.shape[0]] = low
    pairs2, counts2 = ctx.host_persistence_lower(lows, npts, maxp, thr, cap=4096)
    assert np.array_equal(counts2, counts)
    for c in range(len(sizes)):  # the emitted pairs (entries past each count are not written)
        for di, col in ((0, 0), (1, 2), (2, 3)):
            assert np.array_equal(pairs2[c, di, :counts[c, col]], pairs[c, di, :counts[c, col]]), (c, di)
