"""ctypes view of include/dgn.h. Loads the in-tree libdgn.so (built by `make` / build())."""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(os.path.dirname(HERE))  # defect-gnn-cpp_amd/
lib_path = os.environ.get("DGN_LIB") or os.path.join(PKG, "lib", "libdgn.so")

DGN_NONE, DGN_F32, DGN_F64 = 0, 1, 2
STATUS = {0: "DGN_OK", 1: "DGN_ERR_ARG", 2: "DGN_ERR_HIP", 3: "DGN_ERR_CAPACITY", 4: "DGN_ERR_NODEVICE",
          5: "DGN_ERR_UNSUPPORTED", 6: "DGN_ERR_INTERNAL"}
UINT64_MAX = (1 << 64) - 1

# exported symbols of include/dgn.h (checked by tests/test_abi.py)
EXPORTS = [
    "dgn_status_string", "dgn_ctx_create", "dgn_ctx_destroy", "dgn_ctx_set_stream", "dgn_ctx_synchronize",
    "dgn_ctx_last_error", "dgn_ctx_enable_timing", "dgn_ctx_kernel_times", "dgn_ctx_reset_timing",
    "dgn_graph_params_default", "dgn_rbf_bins", "dgn_dev_graph_count", "dgn_dev_graph_emit", "dgn_host_graph",
    "dgn_graph_result_free", "dgn_dev_betti", "dgn_host_betti", "dgn_host_persistence",
    "dgn_host_persistence_lower", "dgn_host_rbf", "dgn_debug_betti_clouds", "dgn_dev_node_features",
    "dgn_dev_edge_arrays", "dgn_host_edge_arrays", "dgn_edge_arrays_free", "dgn_dev_graph_betti",
    "dgn_synth_atoms_per_structure", "dgn_synth_batch", "dgn_ctx_set_debug", "dgn_debug_retry_count",
    "dgn_debug_host_syncs", "dgn_debug_check_wide_layouts",
]
DEBUG_FORCE_RETRY, DEBUG_WIDE_WAVES, DEBUG_WIDE_C16, DEBUG_WIDE_CAP, DEBUG_BIG_LOG2, DEBUG_EMIT_CHUNK = 1, 2, 3, 4, 6, 7
DEBUG_WIDE_WALK, DEBUG_SPLIT_CHUNK = 8, 9


class DgnError(RuntimeError):
    def __init__(self, status, msg=""):
        self.status = status
        super().__init__(f"{STATUS.get(status, status)}: {msg}")


class Batch(C.Structure):
    _fields_ = [("num_structures", C.c_int64), ("num_atoms", C.c_int64), ("lattice", C.c_void_p),
                ("positions", C.c_void_p), ("species", C.c_void_p), ("atom_offset", C.c_void_p)]


class GraphParams(C.Structure):
    _fields_ = [("r_cutoff", C.c_double), ("max_neighbors", C.c_uint64), ("epsilon", C.c_double),
                ("rbf_cutoff", C.c_double), ("rbf_dr", C.c_double), ("rbf_dtype", C.c_int32),
                ("write_displacement", C.c_int32)]


class GraphOut(C.Structure):
    _fields_ = [("col_idx", C.c_void_p), ("distance", C.c_void_p), ("displacement", C.c_void_p),
                ("rbf", C.c_void_p)]


class GraphResult(C.Structure):
    _fields_ = [("num_atoms", C.c_int64), ("num_edges", C.c_int64), ("n_rbf", C.c_int32),
                ("rbf_dtype", C.c_int32), ("row_ptr", C.POINTER(C.c_int64)), ("col_idx", C.POINTER(C.c_int32)),
                ("distance", C.POINTER(C.c_double)), ("displacement", C.POINTER(C.c_double)),
                ("rbf", C.c_void_p)]


class BettiParams(C.Structure):
    _fields_ = [("r_cutoff", C.c_double)]


class EdgeArrays(C.Structure):
    _fields_ = [("num_edges", C.c_int64), ("sources", C.POINTER(C.c_int32)), ("targets", C.POINTER(C.c_int32)),
                ("distances", C.POINTER(C.c_float)), ("displacements", C.POINTER(C.c_float))]


class KernelTime(C.Structure):
    _fields_ = [("name", C.c_char * 48), ("launches", C.c_int64), ("total_ms", C.c_double),
                ("bytes", C.c_double), ("flops", C.c_double)]


_lib = None


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(lib_path):
        raise FileNotFoundError(f"{lib_path} missing: run `make` (or __graft_entry__.build()) first")
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64 / libhsa-runtime64 (SONAMEs
    # libamdhip64.so.7 / libhsa-runtime64.so.1), which libdgn's DT_NEEDED entries bind to when torch is
    # loaded first; loaded the other way round the process would hold two runtimes and torch would
    # find no device. So torch, when installed, is imported before libdgn.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(lib_path)
    vp, i32, i64, dbl = C.c_void_p, C.c_int32, C.c_int64, C.c_double
    L.dgn_status_string.restype = C.c_char_p
    L.dgn_status_string.argtypes = [C.c_int]
    L.dgn_ctx_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.dgn_ctx_destroy.argtypes = [vp]
    L.dgn_ctx_destroy.restype = None
    L.dgn_ctx_set_stream.argtypes = [vp, vp]
    L.dgn_ctx_synchronize.argtypes = [vp]
    if hasattr(L, "dgn_ctx_set_debug"):  # absent from older A/B builds
        L.dgn_ctx_set_debug.argtypes = [vp, C.c_int, C.c_int]
    if hasattr(L, "dgn_debug_retry_count"):
        L.dgn_debug_retry_count.argtypes = [vp, C.POINTER(i64)]
    if hasattr(L, "dgn_debug_host_syncs"):
        L.dgn_debug_host_syncs.argtypes = [vp, C.POINTER(i64)]
    if hasattr(L, "dgn_debug_check_wide_layouts"):
        L.dgn_debug_check_wide_layouts.argtypes = [C.POINTER(i64)]
    L.dgn_ctx_last_error.restype = C.c_char_p
    L.dgn_ctx_last_error.argtypes = [vp]
    L.dgn_ctx_enable_timing.argtypes = [vp, C.c_int]
    L.dgn_ctx_kernel_times.argtypes = [vp, C.POINTER(KernelTime), C.c_int]
    L.dgn_ctx_reset_timing.argtypes = [vp]
    L.dgn_graph_params_default.argtypes = [C.POINTER(GraphParams)]
    L.dgn_graph_params_default.restype = None
    L.dgn_rbf_bins.argtypes = [dbl, dbl]
    L.dgn_dev_graph_count.argtypes = [vp, C.POINTER(Batch), C.POINTER(GraphParams), C.POINTER(i64)]
    L.dgn_dev_graph_emit.argtypes = [vp, C.POINTER(Batch), C.POINTER(GraphParams), vp, C.POINTER(GraphOut)]
    L.dgn_host_graph.argtypes = [vp, C.POINTER(Batch), C.POINTER(GraphParams), C.POINTER(C.POINTER(GraphResult))]
    L.dgn_graph_result_free.argtypes = [C.POINTER(GraphResult)]
    L.dgn_graph_result_free.restype = None
    L.dgn_dev_betti.argtypes = [vp, C.POINTER(Batch), C.POINTER(BettiParams), vp, vp]
    L.dgn_host_betti.argtypes = [vp, C.POINTER(Batch), C.POINTER(BettiParams), vp, vp]
    L.dgn_host_persistence.argtypes = [vp, vp, vp, i64, i32, dbl, vp, i32, vp]
    L.dgn_host_persistence_lower.argtypes = [vp, vp, vp, i64, i32, dbl, vp, i32, vp]
    L.dgn_host_rbf.argtypes = [vp, vp, i64, dbl, dbl, i32, i32, vp]
    if hasattr(L, "dgn_dev_node_features"):  # absent from older A/B builds
        L.dgn_dev_node_features.argtypes = [vp, C.POINTER(Batch), vp, i32, i32, vp, vp, vp, i32, vp]
    if hasattr(L, "dgn_dev_graph_betti"):  # absent from older A/B builds
        L.dgn_dev_graph_betti.argtypes = [vp, C.POINTER(Batch), C.POINTER(GraphParams), vp, C.POINTER(GraphOut),
                                          C.POINTER(BettiParams), vp, vp]
    if hasattr(L, "dgn_dev_edge_arrays"):  # absent from older A/B builds
        L.dgn_dev_edge_arrays.argtypes = [vp, C.POINTER(Batch), vp, vp, vp, vp, vp, vp, vp, vp]
        L.dgn_host_edge_arrays.argtypes = [vp, C.POINTER(Batch), dbl, C.c_uint64, dbl, C.POINTER(C.POINTER(EdgeArrays))]
        L.dgn_edge_arrays_free.argtypes = [C.POINTER(EdgeArrays)]
        L.dgn_edge_arrays_free.restype = None
    if hasattr(L, "dgn_debug_betti_clouds"):  # absent from older A/B builds
        L.dgn_debug_betti_clouds.argtypes = [vp, vp, dbl, i64, i64, i32, vp, vp, vp]
    L.dgn_synth_atoms_per_structure.restype = i64
    L.dgn_synth_atoms_per_structure.argtypes = [C.c_int, C.c_int]
    L.dgn_synth_batch.argtypes = [C.c_int, C.c_int, i64, i64, vp, vp, vp, vp]
    _lib = L
    return L


def _ptr(a):
    if a is None:
        return None
    if hasattr(a, "data_ptr"):  # torch tensor (device pointer)
        return a.data_ptr()
    return a.ctypes.data


def synth_batch(kind: str, m: int, num_structures: int, first_id: int = 0):
    """Synthetic batch from the library's own generator (host numpy arrays)."""
    k = {"sc": 0, "fcc": 1}[kind]
    n = lib().dgn_synth_atoms_per_structure(k, m)
    A = n * num_structures
    out = {"lattice": np.zeros((num_structures, 3, 3)), "positions": np.zeros((A, 3)),
           "species": np.zeros(A, np.int32), "atom_offset": np.zeros(num_structures + 1, np.int64)}
    st = lib().dgn_synth_batch(k, m, num_structures, first_id, _ptr(out["lattice"]), _ptr(out["positions"]),
                               _ptr(out["species"]), _ptr(out["atom_offset"]))
    if st:
        raise DgnError(st, "dgn_synth_batch")
    return out


def make_batch(d) -> Batch:
    """dgn_batch over a dict of numpy arrays (host) or torch tensors (device)."""
    b = Batch()
    b.num_structures = int(d["atom_offset"].shape[0] - 1)
    b.num_atoms = int(d["positions"].shape[0])
    b.lattice = _ptr(d["lattice"])
    b.positions = _ptr(d["positions"])
    b.species = _ptr(d.get("species"))
    b.atom_offset = _ptr(d["atom_offset"])
    return b


def graph_params(r_cutoff=10.0, max_neighbors=20, epsilon=1e-10, rbf_cutoff=10.0, rbf_dr=0.1, rbf_dtype=DGN_F32,
                 write_displacement=False) -> GraphParams:
    p = GraphParams()
    p.r_cutoff = r_cutoff
    p.max_neighbors = UINT64_MAX if max_neighbors is None else int(max_neighbors)
    p.epsilon = epsilon
    p.rbf_cutoff = rbf_cutoff
    p.rbf_dr = rbf_dr
    p.rbf_dtype = rbf_dtype
    p.write_displacement = 1 if write_displacement else 0
    return p


class Context:
    def __init__(self, device: int = 0):
        self.h = C.c_void_p()
        st = lib().dgn_ctx_create(device, C.byref(self.h))
        if st:
            raise DgnError(st, "dgn_ctx_create")

    def close(self):
        if self.h:
            lib().dgn_ctx_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, st, what):
        if st:
            msg = lib().dgn_ctx_last_error(self.h)
            raise DgnError(st, f"{what}: {msg.decode() if msg else ''}")

    def set_stream(self, stream_handle: int | None):
        self._check(lib().dgn_ctx_set_stream(self.h, stream_handle), "set_stream")

    def set_debug(self, knob: int, value: int):
        """Debug / A-B knob (DEBUG_FORCE_RETRY, DEBUG_WIDE_WAVES, DEBUG_WIDE_C16, DEBUG_WIDE_CAP,
        DEBUG_BIG_LOG2, DEBUG_EMIT_CHUNK, DEBUG_WIDE_WALK, DEBUG_SPLIT_CHUNK); tests and tools only."""
        self._check(lib().dgn_ctx_set_debug(self.h, knob, value), "set_debug")

    def retry_count(self) -> int:
        """Complexes the capacity-retry launches reduced since the last call (synchronizes)."""
        n = C.c_int64()
        self._check(lib().dgn_debug_retry_count(self.h, C.byref(n)), "retry_count")
        return n.value

    def host_syncs(self) -> int:
        """Host waits on the context's stream since the last call (no synchronization itself)."""
        n = C.c_int64()
        self._check(lib().dgn_debug_host_syncs(self.h, C.byref(n)), "host_syncs")
        return n.value

    def synchronize(self):
        self._check(lib().dgn_ctx_synchronize(self.h), "synchronize")

    def enable_timing(self, on=True):
        self._check(lib().dgn_ctx_enable_timing(self.h, 1 if on else 0), "enable_timing")

    def reset_timing(self):
        self._check(lib().dgn_ctx_reset_timing(self.h), "reset_timing")

    def kernel_times(self):
        n = lib().dgn_ctx_kernel_times(self.h, None, 0)
        arr = (KernelTime * max(n, 1))()
        n = lib().dgn_ctx_kernel_times(self.h, arr, n)
        return {arr[i].name.decode(): {"launches": arr[i].launches, "total_ms": arr[i].total_ms,
                                       "bytes": arr[i].bytes, "flops": arr[i].flops} for i in range(n)}

    # ---- host-level API ----
    def host_graph(self, batch: dict, params: GraphParams):
        b = make_batch(batch)
        res = C.POINTER(GraphResult)()
        self._check(lib().dgn_host_graph(self.h, C.byref(b), C.byref(params), C.byref(res)), "dgn_host_graph")
        r = res.contents
        A, E = r.num_atoms, r.num_edges
        out = {"row_ptr": np.ctypeslib.as_array(r.row_ptr, (A + 1,)).copy(),
               "col": np.ctypeslib.as_array(r.col_idx, (max(E, 1),))[:E].copy(),
               "dist": np.ctypeslib.as_array(r.distance, (max(E, 1),))[:E].copy()}
        if r.displacement:
            out["disp"] = np.ctypeslib.as_array(r.displacement, (max(E, 1) * 3,))[:3 * E].reshape(E, 3).copy()
        if r.rbf:
            dt = np.float32 if r.rbf_dtype == DGN_F32 else np.float64
            ct = C.c_float if r.rbf_dtype == DGN_F32 else C.c_double
            arr = np.ctypeslib.as_array(C.cast(r.rbf, C.POINTER(ct)), (max(E, 1) * r.n_rbf,))
            out["rbf"] = arr[:E * r.n_rbf].reshape(E, r.n_rbf).astype(dt, copy=True)
        lib().dgn_graph_result_free(res)
        return out

    def host_betti(self, batch: dict, r_cutoff: float):
        b = make_batch(batch)
        p = BettiParams()
        p.r_cutoff = r_cutoff
        A = b.num_atoms
        f = np.zeros((A, 35))
        c = np.zeros((A, 4), np.int32)
        self._check(lib().dgn_host_betti(self.h, C.byref(b), C.byref(p), _ptr(f), _ptr(c)), "dgn_host_betti")
        return f, c

    def host_persistence(self, clouds, npoints, threshold: float, cap: int = 512):
        clouds = np.ascontiguousarray(clouds, dtype=np.float64)
        npoints = np.ascontiguousarray(npoints, dtype=np.int32)
        Cn, maxp = clouds.shape[0], clouds.shape[1]
        pairs = np.zeros((Cn, 3, cap, 2), np.float32)
        counts = np.zeros((Cn, 4), np.int32)
        self._check(lib().dgn_host_persistence(self.h, _ptr(clouds), _ptr(npoints), Cn, maxp, threshold,
                                               _ptr(pairs), cap, _ptr(counts)), "dgn_host_persistence")
        return pairs, counts

    def host_persistence_lower(self, lower, npoints, max_points: int, threshold: float, cap: int = 512):
        lower = np.ascontiguousarray(lower, dtype=np.float32)
        npoints = np.ascontiguousarray(npoints, dtype=np.int32)
        Cn = npoints.shape[0]
        assert lower.shape == (Cn, max_points * (max_points - 1) // 2)
        pairs = np.zeros((Cn, 3, cap, 2), np.float32)
        counts = np.zeros((Cn, 4), np.int32)
        self._check(lib().dgn_host_persistence_lower(self.h, _ptr(lower), _ptr(npoints), Cn, max_points, threshold,
                                                     _ptr(pairs), cap, _ptr(counts)), "dgn_host_persistence_lower")
        return pairs, counts

    def dev_node_features(self, batch: dict, embed, betti, pca_mean, pca_components, out):
        """Device tensors: embed [S][D], betti [A][35] (or None), pca_mean [35], pca_components
        [35][k] (row-major), out [A][D + k] f64."""
        b = make_batch(batch)
        S, D = int(embed.shape[0]), int(embed.shape[1])
        k = 0 if betti is None else int(pca_components.shape[1])
        self._check(lib().dgn_dev_node_features(self.h, C.byref(b), _ptr(embed), S, D, _ptr(betti), _ptr(pca_mean),
                                                _ptr(pca_components), k, _ptr(out)), "dgn_dev_node_features")

    def debug_betti_clouds(self, batch: dict, r_cutoff: float, atom_first: int, count: int, max_points: int):
        """Diagnostics: the Betti pass's local complexes of atoms [atom_first, atom_first + count):
        (lower [count][C(max_points, 2)] f32 in the kernel's row order, npoints [count],
        keys [count][max_points] int64 packed (j, image) of cloud rows 1..npoints-1)."""
        b = make_batch(batch)
        lower = np.zeros((count, max_points * (max_points - 1) // 2), np.float32)
        npoints = np.zeros(count, np.int32)
        keys = np.zeros((count, max_points), np.int64)
        self._check(lib().dgn_debug_betti_clouds(self.h, C.byref(b), r_cutoff, atom_first, count, max_points,
                                                 _ptr(lower), _ptr(npoints), _ptr(keys)), "dgn_debug_betti_clouds")
        return lower, npoints, keys

    def host_edge_arrays(self, batch: dict, r_cutoff=10.0, max_neighbors=20, epsilon=1e-10):
        """WasmAPI::build_graph + graph accessors: (sources, targets, distances f32, displacements f32 [E][3])."""
        b = make_batch(batch)
        res = C.POINTER(EdgeArrays)()
        self._check(lib().dgn_host_edge_arrays(self.h, C.byref(b), r_cutoff, max_neighbors, epsilon, C.byref(res)),
                    "dgn_host_edge_arrays")
        r = res.contents
        E, m = r.num_edges, max(r.num_edges, 1)
        out = (np.ctypeslib.as_array(r.sources, (m,))[:E].copy(), np.ctypeslib.as_array(r.targets, (m,))[:E].copy(),
               np.ctypeslib.as_array(r.distances, (m,))[:E].copy(),
               np.ctypeslib.as_array(r.displacements, (3 * m,))[:3 * E].reshape(E, 3).copy())
        lib().dgn_edge_arrays_free(res)
        return out

    def dev_edge_arrays(self, batch: dict, row_ptr, col, dist, disp, sources, targets, dist32, disp32):
        b = make_batch(batch)
        self._check(lib().dgn_dev_edge_arrays(self.h, C.byref(b), _ptr(row_ptr), _ptr(col), _ptr(dist), _ptr(disp),
                                              _ptr(sources), _ptr(targets), _ptr(dist32), _ptr(disp32)),
                    "dgn_dev_edge_arrays")

    def host_rbf(self, distances, rbf_cutoff=10.0, rbf_dr=0.1, dtype=DGN_F64, layout=0):
        d = np.ascontiguousarray(distances, dtype=np.float64)
        nb = lib().dgn_rbf_bins(rbf_cutoff, rbf_dr)
        out = np.zeros(d.shape[0] * nb, np.float32 if dtype == DGN_F32 else np.float64)
        self._check(lib().dgn_host_rbf(self.h, _ptr(d), d.shape[0], rbf_cutoff, rbf_dr, dtype, layout, _ptr(out)),
                    "dgn_host_rbf")
        return out.reshape(d.shape[0], nb) if layout == 0 else out.reshape(nb, d.shape[0]).T

    # ---- device-level API (torch tensors on cuda) ----
    def dev_graph_count(self, batch: dict, params: GraphParams) -> int:
        b = make_batch(batch)
        E = C.c_int64()
        self._check(lib().dgn_dev_graph_count(self.h, C.byref(b), C.byref(params), C.byref(E)), "dgn_dev_graph_count")
        return E.value

    def dev_graph_emit(self, batch: dict, params: GraphParams, row_ptr, col, dist, disp=None, rbf=None):
        b = make_batch(batch)
        o = GraphOut()
        o.col_idx = _ptr(col)
        o.distance = _ptr(dist)
        o.displacement = _ptr(disp)
        o.rbf = _ptr(rbf)
        self._check(lib().dgn_dev_graph_emit(self.h, C.byref(b), C.byref(params), _ptr(row_ptr), C.byref(o)),
                    "dgn_dev_graph_emit")

    def dev_graph_betti(self, batch: dict, params: GraphParams, row_ptr, col, dist, disp, rbf, r_cutoff: float,
                        features, counts=None):
        """dgn_dev_graph_emit + dgn_dev_betti after a dgn_dev_graph_count, sharing the count when the
        cutoffs agree."""
        b = make_batch(batch)
        o = GraphOut()
        o.col_idx = _ptr(col)
        o.distance = _ptr(dist)
        o.displacement = _ptr(disp)
        o.rbf = _ptr(rbf)
        p = BettiParams()
        p.r_cutoff = r_cutoff
        self._check(lib().dgn_dev_graph_betti(self.h, C.byref(b), C.byref(params), _ptr(row_ptr), C.byref(o),
                                              C.byref(p), _ptr(features), _ptr(counts)), "dgn_dev_graph_betti")

    def dev_betti(self, batch: dict, r_cutoff: float, features, counts=None):
        b = make_batch(batch)
        p = BettiParams()
        p.r_cutoff = r_cutoff
        self._check(lib().dgn_dev_betti(self.h, C.byref(b), C.byref(p), _ptr(features), _ptr(counts)), "dgn_dev_betti")
