"""Python bindings over libdgn.so (the C ABI in include/dgn.h), used by tests/ and bench.py.

The product is the C ABI + HIP kernels; this module is plumbing (ctypes). It never falls back
to a CPU implementation: without a GPU, every compute call raises DgnError(DGN_ERR_NODEVICE).
"""
from .abi import (DGN_F32, DGN_F64, DGN_NONE, Batch, Context, DgnError, GraphParams, lib, lib_path,
                  synth_batch)

__all__ = ["DGN_F32", "DGN_F64", "DGN_NONE", "Batch", "Context", "DgnError", "GraphParams", "lib",
           "lib_path", "synth_batch"]
