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
