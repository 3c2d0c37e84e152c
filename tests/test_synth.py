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
