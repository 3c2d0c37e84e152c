"""ctypes bindings for the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
liboracle.so is the restatement (oracle.cpp); _ref/libdgn_ref.so wraps the reference's own
vendored Ripser (ref_ripser_shim.cpp) when it has been built in the survey container.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_lib = None
_ref = None


class Counts(C.Structure):
    _fields_ = [("n_dim0_finite", C.c_int32), ("n_dim0_inf", C.c_int32),
                ("n_dim1", C.c_int32), ("n_dim2", C.c_int32)]


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t)) if a is not None else None


def lib():
    global _lib
    if _lib is None:
        _lib = C.CDLL(os.path.join(HERE, "liboracle.so"))
        _lib.oracle_neighbor_list.restype = C.c_int64
        _lib.oracle_neighbor_list.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int64,
                                              C.c_double, C.c_uint64, C.c_double, C.POINTER(C.c_int64),
                                              C.POINTER(C.c_int32), C.POINTER(C.c_double),
                                              C.POINTER(C.c_double), C.POINTER(C.c_int32)]
        _lib.oracle_num_images.restype = C.c_int
        _lib.oracle_num_images.argtypes = [C.POINTER(C.c_double), C.c_double]
        _lib.oracle_rbf_bins.restype = C.c_int
        _lib.oracle_rbf_bins.argtypes = [C.c_double, C.c_double]
        _lib.oracle_structure_graph.restype = C.c_int64
        _lib.oracle_structure_graph.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double), C.c_int64, C.c_double,
                                                C.c_uint64, C.c_double, C.c_double, C.c_double,
                                                C.POINTER(C.c_double)]
        _lib.oracle_gaussian_rbf.argtypes = [C.c_double, C.c_double, C.c_double, C.POINTER(C.c_double)]
        _lib.oracle_local_distances.argtypes = [C.POINTER(C.c_double), C.c_int, C.POINTER(C.c_float)]
        _lib.oracle_persistence.restype = C.c_int
        _lib.oracle_persistence.argtypes = [C.POINTER(C.c_float), C.c_int, C.c_float, C.POINTER(C.c_float),
                                            C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int,
                                            C.POINTER(Counts), C.POINTER(C.c_int64)]
        _lib.oracle_statistics.argtypes = [C.POINTER(C.c_float), C.c_int, C.c_int, C.c_double,
                                           C.POINTER(C.c_double)]
        _lib.oracle_structure_betti.restype = C.c_int
        _lib.oracle_structure_betti.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double),
                                                C.POINTER(C.c_int32), C.c_int64, C.c_double,
                                                C.POINTER(C.c_double), C.POINTER(C.c_int32)]
    return _lib


def ref_available() -> bool:
    return os.path.exists(os.path.join(HERE, "_ref", "libdgn_ref.so"))


def ref():
    global _ref
    if _ref is None:
        _ref = C.CDLL(os.path.join(HERE, "_ref", "libdgn_ref.so"))
        _ref.ref_ripser_persistence.restype = C.c_int
        _ref.ref_ripser_persistence.argtypes = [C.POINTER(C.c_float), C.c_int, C.c_float, C.c_uint,
                                                C.POINTER(C.c_float), C.POINTER(C.c_float),
                                                C.POINTER(C.c_float), C.c_int, C.POINTER(Counts)]
        _ref.ref_structure_betti.restype = C.c_int
        _ref.ref_structure_betti.argtypes = [C.POINTER(C.c_double), C.POINTER(C.c_double),
                                             C.POINTER(C.c_int32), C.c_int64, C.c_double, C.c_int,
                                             C.c_uint, C.POINTER(C.c_double), C.POINTER(C.c_int32)]
    return _ref


def neighbor_list(lattice, pos, r_cutoff, max_neighbors=None, epsilon=1e-10):
    """Returns dict(row_ptr, col, dist, disp, image) for one structure."""
    L = np.ascontiguousarray(lattice, dtype=np.float64)
    P = np.ascontiguousarray(pos, dtype=np.float64)
    n = P.shape[0]
    k = (1 << 64) - 1 if max_neighbors is None else int(max_neighbors)
    rp = np.zeros(n + 1, dtype=np.int64)
    e = lib().oracle_neighbor_list(_p(L, C.c_double), _p(P, C.c_double), n, r_cutoff, k, epsilon,
                                   _p(rp, C.c_int64), None, None, None, None)
    col = np.zeros(e, dtype=np.int32)
    dist = np.zeros(e)
    disp = np.zeros((e, 3))
    img = np.zeros((e, 3), dtype=np.int32)
    lib().oracle_neighbor_list(_p(L, C.c_double), _p(P, C.c_double), n, r_cutoff, k, epsilon,
                               _p(rp, C.c_int64), _p(col, C.c_int32), _p(dist, C.c_double),
                               _p(disp, C.c_double), _p(img, C.c_int32))
    return {"row_ptr": rp, "col": col, "dist": dist, "disp": disp, "image": img}


def num_images(lattice, r_cutoff):
    L = np.ascontiguousarray(lattice, dtype=np.float64)
    return lib().oracle_num_images(_p(L, C.c_double), r_cutoff)


def gaussian_rbf(distance, r_cutoff=10.0, dr=0.1):
    n = lib().oracle_rbf_bins(r_cutoff, dr)
    out = np.zeros(n)
    lib().oracle_gaussian_rbf(distance, r_cutoff, dr, _p(out, C.c_double))
    return out


def local_distances(cloud):
    X = np.ascontiguousarray(cloud, dtype=np.float64)
    n = X.shape[0]
    out = np.zeros(n * (n - 1) // 2, dtype=np.float32)
    lib().oracle_local_distances(_p(X, C.c_double), n, _p(out, C.c_float))
    return out


def _pairs_call(fn, lower, n, thr, extra=(), cap=None, stats=False):
    lower = np.ascontiguousarray(lower, dtype=np.float32)
    cap = cap or max(16, n * n * 4)
    d0 = np.zeros((cap, 2), np.float32)
    d1 = np.zeros((cap, 2), np.float32)
    d2 = np.zeros((cap, 2), np.float32)
    cnt = Counts()
    st = np.zeros(8, np.int64)
    args = [_p(lower, C.c_float), n, thr, *extra, _p(d0, C.c_float), _p(d1, C.c_float),
            _p(d2, C.c_float), cap, C.byref(cnt)]
    if stats:
        args.append(_p(st, C.c_int64))
    rc = fn(*args)
    if rc != 0:
        raise RuntimeError(f"persistence call failed rc={rc}")
    out = {"dim0": d0[:cnt.n_dim0_finite].copy(), "n_inf0": cnt.n_dim0_inf,
           "dim1": d1[:cnt.n_dim1].copy(), "dim2": d2[:cnt.n_dim2].copy()}
    if stats:
        out["stats"] = st
    return out


def persistence(lower, n, thr, stats=False):
    return _pairs_call(lib().oracle_persistence, lower, n, thr, stats=True) if stats else \
        _pairs_call(lambda *a: lib().oracle_persistence(*a, None), lower, n, thr)


def ref_persistence(lower, n, thr, threads=1):
    return _pairs_call(ref().ref_ripser_persistence, lower, n, thr, extra=(threads,))


def structure_betti(lattice, pos, species, r_cutoff):
    L = np.ascontiguousarray(lattice, dtype=np.float64)
    P = np.ascontiguousarray(pos, dtype=np.float64)
    S = np.ascontiguousarray(species, dtype=np.int32)
    n = P.shape[0]
    f = np.zeros((n, 35))
    c = np.zeros((n, 4), np.int32)
    lib().oracle_structure_betti(_p(L, C.c_double), _p(P, C.c_double), _p(S, C.c_int32), n, r_cutoff,
                                 _p(f, C.c_double), _p(c, C.c_int32))
    return f, c


def ref_structure_betti(lattice, pos, species, r_cutoff, omp_threads=8, ripser_threads=1):
    L = np.ascontiguousarray(lattice, dtype=np.float64)
    P = np.ascontiguousarray(pos, dtype=np.float64)
    S = np.ascontiguousarray(species, dtype=np.int32)
    n = P.shape[0]
    f = np.zeros((n, 35))
    c = np.zeros((n, 4), np.int32)
    ref().ref_structure_betti(_p(L, C.c_double), _p(P, C.c_double), _p(S, C.c_int32), n, r_cutoff,
                              omp_threads, ripser_threads, _p(f, C.c_double), _p(c, C.c_int32))
    return f, c


def structure_graph(lattice, pos, r_cutoff, max_neighbors, rbf_cutoff, dr, want_rbf=False):
    L = np.ascontiguousarray(lattice, dtype=np.float64)
    P = np.ascontiguousarray(pos, dtype=np.float64)
    k = (1 << 64) - 1 if max_neighbors is None else int(max_neighbors)
    if not want_rbf:
        return lib().oracle_structure_graph(_p(L, C.c_double), _p(P, C.c_double), P.shape[0], r_cutoff, k, 1e-10,
                                            rbf_cutoff, dr, None)
    e = lib().oracle_structure_graph(_p(L, C.c_double), _p(P, C.c_double), P.shape[0], r_cutoff, k, 1e-10,
                                     rbf_cutoff, dr, None)
    out = np.zeros((e, lib().oracle_rbf_bins(rbf_cutoff, dr)))
    lib().oracle_structure_graph(_p(L, C.c_double), _p(P, C.c_double), P.shape[0], r_cutoff, k, 1e-10, rbf_cutoff,
                                 dr, _p(out, C.c_double))
    return out


def statistics(pairs, which, weight):
    """compute_statistics over one diagram (betti_features.cpp:24-55): which 0 birth, 1 death,
    2 persistence; pairs [m][2] f32 sorted."""
    P = np.ascontiguousarray(pairs, dtype=np.float32).reshape(-1, 2)
    out = np.zeros(5)
    lib().oracle_statistics(_p(P, C.c_float), P.shape[0], which, weight, _p(out, C.c_double))
    return out


def atom_betti_from_pairs(r, weight):
    """The 35 features of one atom from its persistence dict (betti_features.cpp:87-98)."""
    f = [statistics(r["dim0"], 1, weight)]
    for d in ("dim1", "dim2"):
        f += [statistics(r[d], 2, weight), statistics(r[d], 0, weight), statistics(r[d], 1, weight)]
    return np.concatenate(f)


def ref_atom_betti(lattice, pos, species, r_cutoff, atoms, ripser=True):
    """Features + counts of selected atoms (compute_atom_betti_features, betti_features.cpp:57-101)
    with the verbatim vendored Ripser (or the restatement): for spot checks at large cutoffs."""
    nl = neighbor_list(lattice, pos, r_cutoff, None)
    rp = nl["row_ptr"]
    feats, counts = [], []
    for i in atoms:
        cloud = np.vstack([pos[i], pos[i] + nl["disp"][rp[i]:rp[i + 1]]])
        n = cloud.shape[0]
        low = local_distances(cloud)
        thr = np.float32(r_cutoff)
        r = ref_persistence(low, n, thr) if ripser else persistence(low, n, thr)
        w = 1.0 / float(np.sum(np.asarray(species) == species[i]))
        feats.append(atom_betti_from_pairs(r, w))
        counts.append([len(r["dim0"]), r["n_inf0"], len(r["dim1"]), len(r["dim2"])])
    return np.array(feats), np.array(counts, np.int32)
