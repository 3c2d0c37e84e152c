"""The library's synthetic generator (C++) equals the numpy restatement bit for bit. CPU only."""
import numpy as np
import pytest

import dgn
from dgn import synth


@pytest.mark.parametrize("kind,m,B,first", [("sc", 4, 5, 0), ("fcc", 4, 3, 7), ("sc", 16, 1, 0), ("fcc", 2, 4, 100)])
def test_generator_bit_identical(kind, m, B, first):
    a = dgn.synth_batch(kind, m, B, first)
    b = synth.make_batch(kind, m, B, first)
    for k in ("lattice", "positions", "species", "atom_offset"):
        assert np.array_equal(a[k], b[k]), k


def test_generator_shapes_and_density():
    b = synth.make_batch("fcc", 4, 2)
    assert b["positions"].shape == (512, 3)
    L = b["lattice"][0, 0, 0]
    assert abs(256 / L ** 3 - 0.08) < 1e-9
    assert np.all(b["positions"][:256] > 0) and np.all(b["positions"][:256] < L)
    s = synth.make_batch("sc", 4, 1)
    assert abs(64 / s["lattice"][0, 0, 0] ** 3 - 0.0801) < 1e-3


def test_rc10_fixture_inputs_match_generator():
    """tests/golden/rc10.npz holds verbatim-Ripser outputs at 10 A for FCC-256 structure 0: its
    stored positions are the generator's (so the GPU test feeds the same input), and its counts
    are plausible (one essential dim-0 class per atom: every 10 A complex is connected)."""
    import os
    fx = np.load(os.path.join(os.path.dirname(__file__), "golden", "rc10.npz"))
    b = synth.make_batch("fcc", 4, 1)
    assert np.array_equal(fx["fcc256_0/positions"], b["positions"])
    for name, n in (("fcc256_0", 256), ("741", 120)):
        c = fx[f"{name}/counts"]
        assert c.shape == (n, 4) and fx[f"{name}/features"].shape == (n, 35)
        assert np.all(c[:, 1] == 1) and np.all(c[:, 2] > 0)


def test_rc16_fixture_clouds_match_oracle_neighbour_list():
    """tests/golden/rc16.npz holds three FCC-256 atoms' local clouds at r_cutoff = 16 (centre +
    NeighborList(16, inf) displacements, betti_features.cpp:67-73) with their verbatim-Ripser pairs:
    the clouds are the oracle's for the generator's structure 0, so the GPU test feeds the same
    complexes; each is past the 1,024-point envelope of round 3."""
    import os
    import oracle_py as O
    fx = np.load(os.path.join(os.path.dirname(__file__), "golden", "rc16.npz"))
    b = synth.make_batch("fcc", 4, 1)
    nl = O.neighbor_list(b["lattice"][0], b["positions"], 16.0, None)
    rp = nl["row_ptr"]
    for a in (0, 97, 203):
        cloud = np.vstack([b["positions"][a], b["positions"][a] + nl["disp"][rp[a]:rp[a + 1]]])
        assert np.array_equal(fx[f"{a}/cloud"], cloud)
        assert cloud.shape[0] > 1024
        assert len(fx[f"{a}/dim0"]) + int(fx[f"{a}/n_inf0"]) == cloud.shape[0]
