"""Synthetic crystal batches, bit-reproducible across C++ and numpy.

RNG: splitmix64 seeded with 0x5EED0000 + structure_id; draw k of a structure is
mix(seed + (k + 1) * GAMMA); uniform u = (z >> 11) * 2**-53. Coordinates are drawn in site order
x, y, z. Jitter = (0.1 * u - 0.05) * spacing (uniform in [-0.05, 0.05) spacings).

  * "sc"  : simple cubic m x m x m sites, spacing s (default 2.32 A, rho ~ 0.080 A^-3);
            site (ix, iy, iz) -> i = (ix*m + iy)*m + iz; pos = (idx + 0.5)*s + jitter;
            species = (ix + iy + iz) % 2.                    configs 2, 3 (m=4) and 5 (m=16)
  * "fcc" : m^3 conventional cells, a = (4/0.08)^(1/3) = 3.684 A, 4-atom basis
            {000, hh0, h0h, 0hh}; cell-major, basis-minor; pos = (c + basis + 0.25)*a + jitter;
            species = basis % 2.                              config 4 (m=4, 256 atoms)

The product library exports the same generator (dgn_synth_batch in include/dgn.h); tests check
the two agree bit for bit.
"""
from __future__ import annotations

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
SEED_BASE = 0x5EED0000
SC_SPACING = 2.32
FCC_A = (4.0 / 0.08) ** (1.0 / 3.0)


def _mix(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def uniforms(struct_ids: np.ndarray, ndraw: int) -> np.ndarray:
    """[B, ndraw] uniforms in [0, 1)."""
    with np.errstate(over="ignore"):
        seeds = (np.uint64(SEED_BASE) + struct_ids.astype(np.uint64))[:, None]
        k = np.arange(1, ndraw + 1, dtype=np.uint64)[None, :]
        z = _mix(seeds + k * GAMMA)
    return (z >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def structure_sites(kind: str, m: int):
    """Return (site_frac_in_spacing_units [N,3], species [N], spacing, box_length)."""
    if kind == "sc":
        ix, iy, iz = np.meshgrid(np.arange(m), np.arange(m), np.arange(m), indexing="ij")
        idx = np.stack([ix.ravel(), iy.ravel(), iz.ravel()], axis=1).astype(np.float64)
        base = idx + 0.5
        species = ((ix + iy + iz) % 2).ravel().astype(np.int32)
        s = SC_SPACING
    elif kind == "fcc":
        basis = np.array([[0, 0, 0], [0.5, 0.5, 0], [0.5, 0, 0.5], [0, 0.5, 0.5]], dtype=np.float64)
        cx, cy, cz = np.meshgrid(np.arange(m), np.arange(m), np.arange(m), indexing="ij")
        cells = np.stack([cx.ravel(), cy.ravel(), cz.ravel()], axis=1).astype(np.float64)
        base = ((cells[:, None, :] + basis[None, :, :]) + 0.25).reshape(-1, 3)
        species = np.tile(np.arange(4) % 2, cells.shape[0]).astype(np.int32)
        s = FCC_A
    else:
        raise ValueError(f"unknown lattice kind {kind!r}")
    return base, species, s, m * s


def make_batch(kind: str, m: int, num_structures: int, first_id: int = 0):
    """Synthetic batch in the dgn_batch layout (host numpy arrays).

    Returns dict(lattice [B,3,3] rows a,b,c; positions [A,3] Cartesian; species [A] int32;
    atom_offset [B+1] int64).
    """
    base, species, s, L = structure_sites(kind, m)
    n = base.shape[0]
    ids = np.arange(first_id, first_id + num_structures, dtype=np.int64)
    u = uniforms(ids, 3 * n).reshape(num_structures, n, 3)
    jitter = (0.1 * u - 0.05) * s
    pos = base[None, :, :] * s + jitter
    lattice = np.zeros((num_structures, 3, 3))
    lattice[:, 0, 0] = L
    lattice[:, 1, 1] = L
    lattice[:, 2, 2] = L
    return {
        "lattice": np.ascontiguousarray(lattice),
        "positions": np.ascontiguousarray(pos.reshape(-1, 3)),
        "species": np.ascontiguousarray(np.tile(species, num_structures)),
        "atom_offset": np.arange(num_structures + 1, dtype=np.int64) * n,
    }
