"""Envelope of the Betti reduction vs the reference's verbatim vendored Ripser (oracle/_ref), which
has no workspace caps (third_party/ripser/ripser.cpp:514-1269): complexes whose reduction outgrows
a kernel's per-wave workspace (cliques: every pairwise distance <= threshold) must be reduced again
by the capacity-retry launch (betti_wide_kernel, big layout) instead of failing; a complex that
outgrows the big layout's tables is listed again and reduced with 4x the tables, up to 2^30
entries (betti_wide_layout grow levels). Complexes of up to 2,048 points (the HUGE instantiation);
larger clouds given to dgn_host_persistence are reduced per connected component of their threshold
graph (each component of up to 2,048 points).
Counts and (birth, death) pairs bit-exact, compared as sorted multisets."""
import os

import numpy as np
import pytest
from conftest import GOLDEN

import dgn
import oracle_py as O

pytestmark = pytest.mark.gpu


def _ref(low, n, thr):
    return O.ref_persistence(low, n, thr) if O.ref_available() else O.persistence(low, n, thr)


def _check(ctx, clouds, npts, thr, cap):
    """Pairs and counts vs verbatim Ripser; returns the number of complexes the capacity-retry launch
    reduced (dgn_debug_retry_count: the retry launch itself runs on every pass, device-driven)."""
    ctx.retry_count()
    pairs, counts = ctx.host_persistence(clouds, npts, thr, cap=cap)
    kt = ctx.retry_count()
    bad = []
    for c in range(len(npts)):
        n = int(npts[c])
        r = _ref(O.local_distances(clouds[c, :n]), n, np.float32(thr))
        assert max(len(r[d]) for d in ("dim0", "dim1", "dim2")) <= cap, "raise the pair cap of this test"
        got = {"dim0": pairs[c, 0, :counts[c, 0]], "dim1": pairs[c, 1, :counts[c, 2]], "dim2": pairs[c, 2, :counts[c, 3]]}
        ok = all(np.array_equal(np.array(sorted(map(tuple, got[d]))).reshape(-1, 2), r[d].reshape(-1, 2))
                 for d in got) and counts[c, 1] == r["n_inf0"]
        if not ok:
            bad.append((c, n, counts[c].tolist(), [len(r[d]) for d in ("dim0", "dim1", "dim2")], r["n_inf0"]))
    assert not bad, bad[:8]
    return kt


def _check_lower(ctx, lowers, npts, thr, cap):
    """host_persistence_lower (compute_persistence_from_distances) on caller-given f32 triangles."""
    ctx.retry_count()
    maxp = int(max(npts))
    pairs, counts = ctx.host_persistence_lower(lowers, npts, maxp, thr, cap=cap)
    kt = ctx.retry_count()
    bad = []
    for c in range(len(npts)):
        n = int(npts[c])
        r = _ref(lowers[c, :n * (n - 1) // 2], n, np.float32(thr))
        got = {"dim0": pairs[c, 0, :counts[c, 0]], "dim1": pairs[c, 1, :counts[c, 2]], "dim2": pairs[c, 2, :counts[c, 3]]}
        ok = all(np.array_equal(np.array(sorted(map(tuple, got[d]))).reshape(-1, 2), r[d].reshape(-1, 2))
                 for d in got) and counts[c, 1] == r["n_inf0"]
        if not ok:
            bad.append((c, n, counts[c].tolist(), [len(r[d]) for d in ("dim0", "dim1", "dim2")], r["n_inf0"]))
    assert not bad, bad[:8]
    return kt


def _sphere(rng, n):
    x = rng.standard_normal((n, 3))
    return x / np.linalg.norm(x, axis=1, keepdims=True)


def _cliques(rng, sizes, side=1.0):
    maxp = max(sizes)
    clouds = np.zeros((len(sizes), maxp, 3))
    for c, n in enumerate(sizes):
        clouds[c, :n] = rng.uniform(0, side, size=(n, 3))
    return clouds, np.array(sizes, dtype=np.int32)


def test_clique_64_points(ctx):
    """64 points, all pairwise distances <= threshold (the narrow kernel's largest tier)."""
    rng = np.random.default_rng(31)
    clouds, npts = _cliques(rng, [64, 64, 60, 48])
    _check(ctx, clouds, npts, 2.0, 1 << 15)


def test_clique_200_points(ctx):
    """A 200-point clique of a random cube cloud: 1.3 M triangle columns in the wide kernel's
    regular layout (it fits the natural caps: no retry; the retry paths are exercised by the
    natural-overflow tests below)."""
    rng = np.random.default_rng(37)
    clouds, npts = _cliques(rng, [200])
    kt = _check(ctx, clouds, npts, 2.0, 1 << 17)
    assert kt == 0, kt


def test_forced_capacity_retry_all_tiers(ctx):
    """Every complex of a batch spanning the three tiers (<= 48, 49..64, 65..) is routed through
    the capacity-retry launch (DGN_DEBUG_FORCE_RETRY, a test knob) and still matches Ripser."""
    rng = np.random.default_rng(41)
    sizes = [5, 30, 48, 55, 64, 90, 130]
    clouds = np.zeros((len(sizes), max(sizes), 3))
    for c, n in enumerate(sizes):
        clouds[c, :n] = rng.uniform(0, 5.0, size=(n, 3))
    ctx.set_debug(dgn.abi.DEBUG_FORCE_RETRY, 1)
    try:
        kt = _check(ctx, clouds, np.array(sizes, dtype=np.int32), 1.9, 4096)
    finally:
        ctx.set_debug(dgn.abi.DEBUG_FORCE_RETRY, 0)
    assert kt >= 1, kt
    kt = _check(ctx, clouds, np.array(sizes, dtype=np.int32), 1.9, 4096)
    assert kt == 0, kt


@pytest.mark.skipif(not O.ref_available(), reason="verbatim Ripser (oracle/_ref) not built")
def test_cloud_above_512_points(ctx):
    """Complexes of 513..1024 points: the bucket pass lists them for the retry launch, which runs
    the rank-coded (BIG) instantiation (126 KB of adjacency LDS at 1,000 points); 1,000-, 700- and
    520-point clouds plus a small one in the same batch, against verbatim Ripser."""
    rng = np.random.default_rng(43)
    sizes = [1000, 700, 520, 90]
    clouds = np.zeros((len(sizes), max(sizes), 3))
    for c, n in enumerate(sizes):
        clouds[c, :n] = rng.uniform(0, 9.0 * (n / 700) ** (1 / 3), size=(n, 3))
    clouds[2, 10] = clouds[2, 3]  # a duplicate point: zero distance, dim-0 pair not emitted
    kt = _check(ctx, clouds, np.array(sizes, dtype=np.int32), 1.6, 1 << 14)
    assert kt >= 1, kt


@pytest.mark.skipif(not O.ref_available(), reason="verbatim Ripser (oracle/_ref) not built")
def test_fcc256_cutoff_12A_above_512_points(ctx):
    """compute_structure_betti_features at r_cutoff = 12: FCC-256 local complexes of ~580 points
    (neighbour search at K = inf with up to 1,024 candidates, the rank-coded retry launch); one
    atom spot-checked against the verbatim Ripser."""
    batch = dgn.synth_batch("fcc", 4, 1)
    f, c = ctx.host_betti(batch, 12.0)
    assert not np.isnan(f).any()
    assert c[:, 0].max() + 1 > 512  # complexes above the regular wide envelope
    atoms = [5]
    fo, co = O.ref_atom_betti(batch["lattice"][0], batch["positions"], batch["species"], 12.0, atoms)
    assert np.array_equal(c[atoms], co), (c[atoms], co)
    np.testing.assert_allclose(f[atoms], fo, rtol=1e-6, atol=1e-12)


def test_natural_retry_narrow_clouds(ctx):
    """Clouds whose reduction outgrows the narrow kernel's caps on its own (no forced retry): points
    on a unit sphere and on a circle, every pair within the threshold. Their dim-2 (sphere) and
    dim-1 (circle) columns need long V lists / many non-apparent columns, so the narrow launch
    appends them to the retry list in the kernel and the big-layout wide launch reduces them;
    against verbatim Ripser."""
    rng = np.random.default_rng(53)
    sizes = [48, 64, 48, 30]
    clouds = np.zeros((len(sizes), max(sizes), 3))
    clouds[0, :48] = _sphere(rng, 48)
    clouds[1, :64] = _sphere(rng, 64)
    t = rng.uniform(0, 2 * np.pi, 48)
    clouds[2, :48] = np.stack([np.cos(t), np.sin(t), 0.01 * rng.standard_normal(48)], 1)
    clouds[3, :30] = rng.uniform(0, 1.0, size=(30, 3))  # an ordinary complex in the same batch
    kt = _check(ctx, clouds, np.array(sizes, dtype=np.int32), 3.0, 1 << 12)
    assert kt >= 1, kt


def test_natural_retry_narrow_matrices(ctx):
    """compute_persistence_from_distances on non-Euclidean symmetric matrices (uniform random
    lengths; lengths from {1, 2, 3, 4}: massive exact ties) of 48 and 64 points: the narrow kernel
    overflows on its own and the retry launch reduces them; against verbatim Ripser."""
    rng = np.random.default_rng(59)
    sizes = [48, 48, 64]
    maxp = max(sizes)
    lowers = np.zeros((len(sizes), maxp * (maxp - 1) // 2), np.float32)
    for c, (n, kind) in enumerate(zip(sizes, ("uniform", "ties4", "uniform"))):
        M = rng.uniform(0.0, 1.0, (n, n)) if kind == "uniform" else rng.integers(1, 5, (n, n)).astype(np.float64)
        lowers[c, :n * (n - 1) // 2] = np.array([M[i, j] for i in range(1, n) for j in range(i)], np.float32)
    kt = _check_lower(ctx, lowers, np.array(sizes, dtype=np.int32), 5.0, 1 << 12)
    assert kt >= 1, kt


def test_wide_in_kernel_overflow_retry(ctx):
    """The wide kernel's own overflow detection and retry append (betti_wide.hip finish(): restore
    the scratch invariants, list the complex, leave its outputs to the retry launch): with the
    regular layout's column / pivot / pair tables shrunk to 256 entries (DGN_DEBUG_WIDE_CAP, a test
    knob; the overflow is detected in the kernel, not listed by the host), ordinary 65..200-point
    complexes overflow and are reduced again by the big-layout launch; against verbatim Ripser.
    (Inputs that overflow the natural 2^17-entry caps, e.g. dense cliques of a few hundred points,
    take minutes in Ripser too.)"""
    rng = np.random.default_rng(61)
    sizes = [150, 90, 200, 70]
    clouds = np.zeros((len(sizes), max(sizes), 3))
    for c, n in enumerate(sizes):
        clouds[c, :n] = rng.uniform(0, 6.0, size=(n, 3))
    npts = np.array(sizes, dtype=np.int32)
    ctx.set_debug(dgn.abi.DEBUG_WIDE_CAP, 256)
    try:
        kt = _check(ctx, clouds, npts, 2.0, 4096)
    finally:
        ctx.set_debug(dgn.abi.DEBUG_WIDE_CAP, 0)
    assert kt >= 1, kt
    kt = _check(ctx, clouds, npts, 2.0, 4096)  # natural caps again: no retry
    assert kt == 0, kt


def test_capacity_retry_grow_levels(ctx):
    """A complex that outgrows the capacity-retry layout is listed again and reduced with 4x the
    tables (betti_wide_layout grow levels; the reference's Ripser has no caps). With the first
    level shrunk to 256-entry tables (DGN_DEBUG_BIG_LOG2 = 8, a test knob) and every complex
    routed to the retry launch (DGN_DEBUG_FORCE_RETRY), 65..200-point complexes need the later
    levels (more than one retry launch); against verbatim Ripser."""
    rng = np.random.default_rng(67)
    sizes = [200, 150, 90, 30]
    clouds = np.zeros((len(sizes), max(sizes), 3))
    for c, n in enumerate(sizes):
        clouds[c, :n] = rng.uniform(0, 6.0, size=(n, 3))
    npts = np.array(sizes, dtype=np.int32)
    ctx.set_debug(dgn.abi.DEBUG_BIG_LOG2, 8)
    ctx.set_debug(dgn.abi.DEBUG_FORCE_RETRY, 1)
    ctx.enable_timing(True)
    ctx.reset_timing()
    try:
        kt = _check(ctx, clouds, npts, 2.0, 4096)
        launches = ctx.kernel_times().get("betti_retry", {}).get("launches", 0)
    finally:
        ctx.set_debug(dgn.abi.DEBUG_FORCE_RETRY, 0)
        ctx.set_debug(dgn.abi.DEBUG_BIG_LOG2, 0)
        ctx.enable_timing(False)
    assert kt == len(sizes), kt  # each complex reduced once, at the level it fits
    assert launches >= 2, launches


@pytest.mark.skipif(not O.ref_available(), reason="verbatim Ripser (oracle/_ref) not built")
def test_cloud_above_1024_points(ctx):
    """Complexes of 1,025..2,048 points: the HUGE instantiation (11-bit vertices, 64-bit packed
    triangles, the adjacency bitsets in the wave's scratch); 1,900-, 1,300- and 1,030-point clouds
    plus a small one in the same batch, against verbatim Ripser."""
    rng = np.random.default_rng(45)
    sizes = [1900, 1300, 1030, 80]
    clouds = np.zeros((len(sizes), max(sizes), 3))
    for c, n in enumerate(sizes):
        clouds[c, :n] = rng.uniform(0, 9.0 * (n / 700) ** (1 / 3), size=(n, 3))
    clouds[1, 40] = clouds[1, 7]  # a duplicate point
    kt = _check(ctx, clouds, np.array(sizes, dtype=np.int32), 1.6, 1 << 14)
    assert kt >= 1, kt


def test_fcc256_cutoff_16A_every_dim(ctx):
    """The reference's Betti path at r_cutoff = 16 (betti_features.cpp:67-73, 103-119): FCC-256
    local complexes of ~1,370 points. Three atoms' clouds (the oracle's NeighborList(16, inf)) and
    their verbatim-Ripser pairs are committed fixtures (tests/golden/rc16.npz, make_golden.py rc16;
    ~15 min of Ripser per atom); pairs and counts bit-exact."""
    fx = np.load(os.path.join(GOLDEN, "rc16.npz"))
    atoms = sorted({int(k.split("/")[0]) for k in fx.files})
    clouds_l = [fx[f"{a}/cloud"] for a in atoms]
    npts = np.array([c.shape[0] for c in clouds_l], np.int32)
    assert npts.min() > 1024
    clouds = np.zeros((len(atoms), npts.max(), 3))
    for c, cl in enumerate(clouds_l):
        clouds[c, :cl.shape[0]] = cl
    pairs, counts = ctx.host_persistence(clouds, npts, 16.0, cap=1 << 12)
    for c, a in enumerate(atoms):
        got = {"dim0": pairs[c, 0, :counts[c, 0]], "dim1": pairs[c, 1, :counts[c, 2]], "dim2": pairs[c, 2, :counts[c, 3]]}
        for d in got:
            assert np.array_equal(np.array(sorted(map(tuple, got[d]))).reshape(-1, 2), fx[f"{a}/{d}"].reshape(-1, 2)), (a, d)
        assert counts[c, 1] == fx[f"{a}/n_inf0"]


def test_fcc256_cutoff_16A_search_triangles(ctx):
    """The device half of compute_structure_betti_features at r_cutoff = 16 (betti_features.cpp:
    67-73, 107; ripser_wrapper.cpp:60-70): the Betti neighbour search at K = inf (up to 2,048
    candidates, betti_dist_search_kernel<2048>) and the MFMA distance triangles of two ~1,400-point
    complexes, bit-exact against the oracle's NeighborList(16, inf) clouds (the reduction of the
    same clouds is checked against the verbatim-Ripser fixtures above; the whole structure, 256 such
    complexes, takes minutes)."""
    from test_gpu_betti import _kernel_vs_reference_triangles
    batch = dgn.synth_batch("fcc", 4, 1)
    for a in (0, 97):
        lower, npts, keys = ctx.debug_betti_clouds(batch, 16.0, a, 1, 2048)
        assert npts[0] > 1024
        got, mapped, _, _ = _kernel_vs_reference_triangles(lower[0], npts[0], keys[0], batch["lattice"][0],
                                                           batch["positions"], a, 16.0)
        assert np.array_equal(got.view(np.uint32), mapped.view(np.uint32)), a


def _clustered(rng, n, k, spread, big=0):
    """n points in k Gaussian clusters (plus, if big > 0, one cluster of `big` points) in a 60 A box."""
    centers = rng.uniform(0, 60, (k, 3))
    lab = rng.integers(0, k, n - big)
    pts = centers[lab] + rng.normal(0, spread, (n - big, 3))
    if big:
        pts = np.vstack([pts, rng.uniform(0, 60, 3) + rng.normal(0, 2.2, (big, 3))])
    return pts


def test_above_2048_points_split_into_components(ctx):
    """Clouds of 2,100..3,000 points (dgn_host_persistence / _lower: compute_persistence and
    compute_persistence_from_distances, ripser_wrapper.cpp:11-70), reduced per connected component of
    the threshold graph (betti_split.hip; the pairs of a disjoint union are the union of the pairs):
    clusters of ~20..200 points and isolated points, one 600-point cluster (the rank-coded BIG tier),
    against verbatim Ripser on the whole cloud."""
    rng = np.random.default_rng(7)
    specs = [(2100, 30, 0), (2600, 20, 600), (3000, 60, 0)]
    npts = np.array([n for n, _, _ in specs], np.int32)
    clouds = np.zeros((len(specs), npts.max(), 3))
    for c, (n, k, big) in enumerate(specs):
        clouds[c, :n] = _clustered(rng, n, k, 1.2, big)
    thr = 1.6
    pairs, counts = ctx.host_persistence(clouds, npts, thr, cap=4096)
    lows = []
    for c, n in enumerate(npts):
        low = O.local_distances(clouds[c, :n])
        lows.append(low)
        r = O.ref_persistence(low, int(n), np.float32(thr))
        assert counts[c, 1] == r["n_inf0"], c
        for di, d in enumerate(("dim0", "dim1", "dim2")):
            assert np.array_equal(pairs[c, di, :counts[c, [0, 2, 3][di]]], r[d]), (c, n, d)
    # the caller-given distance matrices (the same packed triangles)
    m = int(npts.max())
    L = np.zeros((len(specs), m * (m - 1) // 2), np.float32)
    for c, low in enumerate(lows):
        L[c, :low.shape[0]] = low
    pl, cl = ctx.host_persistence_lower(L, npts, m, thr, cap=4096)
    assert np.array_equal(cl, counts)
    for c in range(len(specs)):
        for di, col in enumerate((0, 2, 3)):
            assert np.array_equal(pl[c, di, :cl[c, col]], pairs[c, di, :counts[c, col]])


def _many_small(rng, big, npair, nsingle, spread):
    """One Gaussian cluster of `big` points, `npair` 2-point components and `nsingle` isolated points
    on a 4 A grid beside it."""
    clus = rng.uniform(0, 10, 3) + rng.normal(0, spread, (big, 3))
    g = np.stack(np.meshgrid(np.arange(20), np.arange(20), np.arange(20)), -1).reshape(-1, 3) * 4.0 + np.array([40.0, 0, 0])
    sel = rng.permutation(len(g))[:npair + nsingle]
    a = g[sel[:npair]] + rng.normal(0, 0.05, (npair, 3))
    b = a + rng.normal(0, 0.3, (npair, 3))
    return np.vstack([clus, a, b, g[sel[npair:]]])


def test_split_many_small_components_beside_a_large_one(ctx):
    """The component split groups components by size (each group's triangle stride and pair block
    are its largest member's, within a byte budget): clouds of ~5,000 points with one
    ~1,100-point cluster, 1,500 two-point components and 1,000 isolated points, taken one cloud per
    chunk (DGN_DEBUG_SPLIT_CHUNK = 1: the chunk loop), both input modes, against verbatim Ripser."""
    rng = np.random.default_rng(41)
    clouds = [_many_small(rng, 1100, 1500, 1000, 1.3), _many_small(rng, 900, 1600, 700, 1.6)]
    npts = np.array([len(x) for x in clouds], np.int32)
    m = int(npts.max())
    C = np.zeros((len(clouds), m, 3))
    for c, x in enumerate(clouds):
        C[c, :len(x)] = x
    thr = 1.0
    ctx.set_debug(dgn.abi.DEBUG_SPLIT_CHUNK, 1)
    try:
        pairs, counts = ctx.host_persistence(C, npts, thr, cap=8192)
        lows = [O.local_distances(x) for x in clouds]
        L = np.zeros((len(clouds), m * (m - 1) // 2), np.float32)
        for c, low in enumerate(lows):
            L[c, :low.shape[0]] = low
        pl, cl = ctx.host_persistence_lower(L, npts, m, thr, cap=8192)
    finally:
        ctx.set_debug(dgn.abi.DEBUG_SPLIT_CHUNK, 0)
    for c, n in enumerate(npts):
        r = O.ref_persistence(lows[c], int(n), np.float32(thr))
        assert counts[c, 1] == r["n_inf0"], c
        for di, d in enumerate(("dim0", "dim1", "dim2")):
            assert np.array_equal(pairs[c, di, :counts[c, [0, 2, 3][di]]], r[d]), (c, n, d)
    assert np.array_equal(cl, counts)
    for c in range(len(clouds)):  # the emitted pairs (entries past each count are not written)
        for di, col in ((0, 0), (1, 2), (2, 3)):
            assert np.array_equal(pl[c, di, :counts[c, col]], pairs[c, di, :counts[c, col]]), (c, di)


def _tube(rng, n, ds, radius):
    """n points in a tube of the given radius around a slowly turning random walk of step ds: one
    connected component at threshold 1 with a few thousand 1- and 2-cycles."""
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    for i in range(1, n):
        d[i] = 0.97 * d[i - 1] + 0.03 * d[i]
        d[i] /= np.linalg.norm(d[i])
    c = np.cumsum(d * ds, axis=0)
    off = rng.normal(size=(n, 3))
    off -= (off * d).sum(1, keepdims=True) * d
    off /= np.linalg.norm(off, axis=1, keepdims=True)
    return c + off * radius * np.sqrt(rng.uniform(0, 1, (n, 1)))


@pytest.mark.skipif(not O.ref_available(), reason="verbatim Ripser (oracle/_ref) not built")
def test_single_component_above_2048_points(ctx):
    """One connected component of 2,100..3,000 points (dgn_host_persistence / _lower): the GIANT
    instantiation (12-bit vertices, keys (code << 44) | ~index, no min-cofacet table), against
    verbatim Ripser on the whole cloud (ripser.cpp:154, 514-1269 have no point cap)."""
    rng = np.random.default_rng(61)
    specs = [(2100, 0.12, 0.6), (2600, 0.1, 0.7), (3000, 0.15, 0.6)]
    npts = np.array([n for n, _, _ in specs], np.int32)
    clouds = np.zeros((len(specs), npts.max(), 3))
    for c, (n, ds, rad) in enumerate(specs):
        clouds[c, :n] = _tube(rng, n, ds, rad)
    thr = 1.0
    pairs, counts = ctx.host_persistence(clouds, npts, thr, cap=4096)
    lows = []
    for c, n in enumerate(npts):
        low = O.local_distances(clouds[c, :n])
        lows.append(low)
        r = O.ref_persistence(low, int(n), np.float32(thr))
        assert r["n_inf0"] == 1 and counts[c, 1] == 1, c  # a single component
        for di, d in enumerate(("dim0", "dim1", "dim2")):
            assert np.array_equal(pairs[c, di, :counts[c, [0, 2, 3][di]]], r[d]), (c, n, d)
    m = int(npts.max())
    L = np.zeros((len(specs), m * (m - 1) // 2), np.float32)
    for c, low in enumerate(lows):
        L[c, :low.shape[0]] = low
    pl, cl = ctx.host_persistence_lower(L, npts, m, thr, cap=4096)
    assert np.array_equal(cl, counts)
    for c in range(len(specs)):
        for di, col in enumerate((0, 2, 3)):
            assert np.array_equal(pl[c, di, :cl[c, col]], pairs[c, di, :counts[c, col]])


def test_above_2048_points_fails_loudly(ctx):
    # outside the envelope: an explicit DGN_ERR_UNSUPPORTED, never a silent or
    # truncated result -- one connected component above 4,096 points; a 2,100-point component whose
    # distances within the threshold number 2^20 or more (every pair: the GIANT keys hold codes below
    # 2^20); and FCC-256 at 21 A (~3,100-point atom-centred complexes, above the distance search's
    # 2,048 candidates: the count pass finds them before any Betti launch)
    rng = np.random.default_rng(5)
    cloud = _tube(rng, 4200, 0.12, 0.6)[None]
    with pytest.raises(dgn.DgnError) as e:
        ctx.host_persistence(cloud, np.array([4200], np.int32), 1.0)
    assert e.value.status == 5
    dense = rng.uniform(0.0, 1.0, size=(1, 2100, 3))
    with pytest.raises(dgn.DgnError) as e:
        ctx.host_persistence(dense, np.array([2100], np.int32), 3.0)
    assert e.value.status == 5
    with pytest.raises(dgn.DgnError) as e:
        ctx.host_betti(dgn.synth_batch("fcc", 4, 1), 21.0)
    assert e.value.status == 5
    # the context stays usable
    f, c = ctx.host_betti(dgn.synth_batch("fcc", 4, 1), 5.0)
    assert (c >= 0).all()
