"""Shared test setup: paths, the `gpu` marker, and helpers.

`-m "not gpu"` runs here (no GPU): oracle vs golden vectors / verbatim Ripser, host logic,
ABI exports. `-m gpu` runs on an MI355X: the HIP path through the C ABI vs the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "defect-gnn-cpp_amd", "python")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through libdgn.so)")
    config.addinivalue_line("markers", "slow: longer CPU test")


@pytest.fixture(scope="session")
def ctx():
    """One libdgn context for the whole GPU session (tests run in one process)."""
    import dgn
    c = dgn.Context(0)
    yield c
    c.close()


def mixed_batch(npairs):
    """FCC-256 cells (one image per axis at rc 5: the one-image count kernel) alternating with
    SC-64 cells (L = 9.28 A < 2 rc: the general search), so count tiles are one-image, general or
    straddle both (flagged for the general count kernel)."""
    import numpy as np
    import dgn

    f, s = dgn.synth_batch("fcc", 4, npairs), dgn.synth_batch("sc", 4, npairs)
    fo, so = f["atom_offset"], s["atom_offset"]
    lat, pos, spc, sizes = [], [], [], []
    for i in range(npairs):
        lat += [f["lattice"][i], s["lattice"][i]]
        pos += [f["positions"][fo[i]:fo[i + 1]], s["positions"][so[i]:so[i + 1]]]
        spc += [f["species"][fo[i]:fo[i + 1]], s["species"][so[i]:so[i + 1]]]
        sizes += [fo[i + 1] - fo[i], so[i + 1] - so[i]]
    return {"lattice": np.stack(lat), "positions": np.concatenate(pos), "species": np.concatenate(spc).astype(np.int32),
            "atom_offset": np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)}
