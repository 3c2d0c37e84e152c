"""The CPU oracle, pinned against the golden fixtures (verbatim Ripser + restated front end)
and against independent numpy restatements. CPU only."""
import os

import numpy as np
import pytest
from conftest import GOLDEN

import oracle_py as O
from dgn import synth


@pytest.fixture(scope="module")
def kat():
    return np.load(os.path.join(GOLDEN, "kat.npz"))


@pytest.fixture(scope="module")
def sc64():
    return np.load(os.path.join(GOLDEN, "sc64_rc5.npz"))


@pytest.fixture(scope="module")
def poscar():
    return np.load(os.path.join(GOLDEN, "poscar_rc5.npz"))


KATS = ["square", "octahedron", "cube", "tetrahedron", "hexagon", "two_points", "duplicate", "octahedron_t15"]


@pytest.mark.parametrize("name", KATS)
def test_kat_against_verbatim_ripser_fixture(kat, name):
    pts = kat[f"{name}/cloud"]
    thr = float(kat[f"{name}/threshold"])
    low = O.local_distances(pts)
    r = O.persistence(low, pts.shape[0], np.float32(thr))
    for d in ("dim0", "dim1", "dim2"):
        assert np.array_equal(r[d], kat[f"{name}/{d}"]), (name, d)
    assert r["n_inf0"] == int(kat[f"{name}/n_inf0"])


def test_kat_values_match_survey_table(kat):
    # SURVEY.md section 4 table
    s2 = np.float32(np.sqrt(2.0))
    assert kat["square/dim1"].tolist() == [[1.0, s2]]
    assert kat["octahedron/dim2"].tolist() == [[s2, 2.0]] and len(kat["octahedron/dim1"]) == 0
    assert len(kat["octahedron_t15/dim2"]) == 0  # essential class not emitted
    assert len(kat["cube/dim1"]) == 5 and len(kat["cube/dim0"]) == 7
    assert len(kat["tetrahedron/dim1"]) == 0 and len(kat["tetrahedron/dim2"]) == 0
    assert kat["hexagon/dim1"].shape == (1, 2) and kat["hexagon/dim2"].shape == (1, 2)
    assert kat["two_points/dim0"].tolist() == [[0.0, 3.0]]
    assert kat["duplicate/dim0"].tolist() == [[0.0, 1.0]]  # zero-length pair dropped


def test_isolated_point_defined():
    r = O.persistence(np.zeros(0, np.float32), 1, np.float32(5.0))
    assert r["n_inf0"] == 1 and len(r["dim0"]) == 0


@pytest.mark.parametrize("s", range(8))
def test_sc64_betti_against_fixture(sc64, s):
    bt = synth.make_batch("sc", 4, 8)
    n = 64
    lat, pos, sp = bt["lattice"][s], bt["positions"][s * n:(s + 1) * n], bt["species"][s * n:(s + 1) * n]
    f, c = O.structure_betti(lat, pos, sp, 5.0)
    assert np.array_equal(c, sc64[f"{s}/counts"])
    np.testing.assert_allclose(f, sc64[f"{s}/features"], rtol=1e-12, atol=1e-12)
    nl = O.neighbor_list(lat, pos, 5.0, 20)
    assert np.array_equal(nl["row_ptr"], sc64[f"{s}/row_ptr"])
    assert np.array_equal(nl["col"], sc64[f"{s}/col"])
    assert np.array_equal(nl["dist"], sc64[f"{s}/dist"])
    for a in (0, 37):
        low = O.local_distances(sc64[f"{s}/cloud{a}"])
        assert np.array_equal(low, sc64[f"{s}/lower{a}"])
        r = O.persistence(low, sc64[f"{s}/cloud{a}"].shape[0], np.float32(5.0))
        for d in ("dim0", "dim1", "dim2"):
            assert np.array_equal(r[d], sc64[f"{s}/pairs{a}/{d}"])


@pytest.mark.parametrize("name", ["1", "1046", "1046_1", "1046_2", "1_1", "1_2", "741", "741_1", "741_2"])
def test_poscar_betti_against_fixture(poscar, name):
    f, c = O.structure_betti(poscar[f"{name}/lattice"], poscar[f"{name}/positions"], poscar[f"{name}/species"], 5.0)
    assert np.array_equal(c, poscar[f"{name}/betti5/counts"])
    np.testing.assert_allclose(f, poscar[f"{name}/betti5/features"], rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("name", ["1", "1046", "1046_1", "1046_2", "1_1", "1_2", "741", "741_1", "741_2"])
@pytest.mark.parametrize("k", [12, 20])
def test_poscar_neighbors_against_fixture(poscar, name, k):
    nl = O.neighbor_list(poscar[f"{name}/lattice"], poscar[f"{name}/positions"], 5.0, k)
    assert np.array_equal(nl["row_ptr"], poscar[f"{name}/k{k}/row_ptr"])
    assert np.array_equal(nl["col"], poscar[f"{name}/k{k}/col"])
    assert np.array_equal(nl["dist"], poscar[f"{name}/k{k}/dist"])


def test_perfect_sc_shells():
    # perfect SC, a = 2.32, rc = 5 -> 6 + 12 + 8 + 6 = 32 neighbours
    a = 2.32
    idx = np.stack(np.meshgrid(np.arange(4), np.arange(4), np.arange(4), indexing="ij"), -1).reshape(-1, 3)
    pos = (idx + 0.5) * a
    lat = np.eye(3) * 4 * a
    nl = O.neighbor_list(lat, pos, 5.0, None)
    assert np.all(np.diff(nl["row_ptr"]) == 32)
    assert O.num_images(lat, 5.0) == 2  # ceil(5 / 9.28) + 1


def test_rbf_matches_numpy_restatement():
    # edge_features.cpp:7-24 restated independently in numpy
    for d in (0.0, 1.234, 4.999, 7.5):
        rc, dr = 5.0, 0.1
        n = int(np.floor(rc / dr))
        sigma = rc / 3
        g = (1 / (sigma * np.sqrt(2 * np.pi))) * np.exp(-0.5 * (np.arange(n) * dr - d) ** 2 * (1 / sigma ** 2))
        np.testing.assert_allclose(O.gaussian_rbf(d, rc, dr), g, rtol=1e-14)
    assert len(O.gaussian_rbf(1.0)) == 100  # defaults rc=10, dr=0.1 -> 100 bins


def test_local_distances_gram_order():
    rng = np.random.default_rng(3)
    X = rng.uniform(-20, 20, size=(40, 3))
    low = O.local_distances(X)
    sq = (X[:, 0] * X[:, 0] + X[:, 1] * X[:, 1]) + X[:, 2] * X[:, 2]
    i, j = np.tril_indices(40, -1)
    order = np.lexsort((j, i))
    i, j = i[order], j[order]
    dot = (X[i, 0] * X[j, 0] + X[i, 1] * X[j, 1]) + X[i, 2] * X[j, 2]
    d = np.sqrt(np.maximum((sq[i] + sq[j]) - 2.0 * dot, 0.0)).astype(np.float32)
    assert np.array_equal(low, d)


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built")
def test_restated_reduction_vs_verbatim_ripser_random():
    rng = np.random.default_rng(11)
    for t in range(150):
        n = int(rng.integers(2, 40))
        if t % 3 == 0:
            pts = rng.integers(0, 3, size=(n, 3)).astype(float)  # many exact ties
        else:
            pts = rng.uniform(0, 4, size=(n, 3))
        thr = np.float32(rng.uniform(1.0, 5.0))
        low = O.local_distances(pts)
        a, b = O.persistence(low, n, thr), O.ref_persistence(low, n, thr)
        for d in ("dim0", "dim1", "dim2"):
            assert np.array_equal(a[d], b[d]), (t, d)
        assert a["n_inf0"] == b["n_inf0"]


def test_cellist_fixture_sc4096():
    """The oracle over config 5's SC-4096 supercell vs verbatim Ripser (every 8th atom of
    cellist.npz): pins the checker the > 512-atom GPU tests compare against."""
    fx = np.load(os.path.join(GOLDEN, "cellist.npz"))
    bt = synth.make_batch("sc", 16, 1)
    f, c = O.structure_betti(bt["lattice"][0], bt["positions"], bt["species"], 5.0)
    a = fx["sc4096/atoms"]
    assert np.array_equal(c[a], fx["sc4096/counts"])
    np.testing.assert_allclose(f[a], fx["sc4096/features"], rtol=1e-12, atol=1e-12)
