"""The C-ABI library loads and exports every symbol include/dgn.h declares. CPU only (no compute)."""
import os
import re
import subprocess

import pytest
from conftest import ROOT

import dgn
from dgn import abi as L


def declared_functions():
    src = open(os.path.join(ROOT, "include", "dgn.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(dgn_[a-z0-9_]+)\s*\(", src))
    return sorted(names)


def test_header_declarations_match_binding_list():
    assert declared_functions() == sorted(L.EXPORTS)


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", L.lib_path], capture_output=True, text=True, check=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, missing
    lib = dgn.lib()
    for n in declared_functions():
        assert hasattr(lib, n)


def test_status_strings():
    lib = dgn.lib()
    assert lib.dgn_status_string(0) == b"ok"
    assert b"no GPU" in lib.dgn_status_string(4)


def test_no_oracle_in_product_library():
    # the product library must not link or reference the CPU oracle
    out = subprocess.run(["nm", "-D", L.lib_path], capture_output=True, text=True, check=True).stdout
    assert "oracle_" not in out and "ref_ripser" not in out
    ldd = subprocess.run(["ldd", L.lib_path], capture_output=True, text=True).stdout
    assert "oracle" not in ldd


def test_context_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(dgn.DgnError) as e:
        dgn.Context(0)
    assert e.value.status in (4, 2)


def test_rbf_bins_and_defaults():
    lib = dgn.lib()
    assert lib.dgn_rbf_bins(10.0, 0.1) == 100 and lib.dgn_rbf_bins(5.0, 0.1) == 50
    p = L.GraphParams()
    lib.dgn_graph_params_default(p)
    assert (p.r_cutoff, p.max_neighbors, p.epsilon, p.rbf_cutoff, p.rbf_dr) == (10.0, 20, 1e-10, 10.0, 0.1)


def test_wide_layouts_keep_power_of_two_caps():
    """Every wide / capacity-retry scratch layout (65..2,048 points, every growth level) keeps its
    int32 table capacities positive powers of two (the pivot hash of the last
    growth level overflowed int32). Host arithmetic only: runs without a GPU."""
    import ctypes
    bad = ctypes.c_int64(0)
    st = dgn.lib().dgn_debug_check_wide_layouts(ctypes.byref(bad))
    assert st == 0, f"layout nmax={bad.value // 64} big={(bad.value // 16) & 1} grow={bad.value % 16}"
