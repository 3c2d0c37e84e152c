"""Generate the committed golden fixtures (run ONLY in the survey/build container).

    python tests/golden/make_golden.py          # everything
    python tests/golden/make_golden.py rc10     # only the 10 A fixtures (rc10.npz)
    python tests/golden/make_golden.py rc16     # only the 16 A fixtures (rc16.npz; ~45 min, ~34 GB)
    python tests/golden/make_golden.py cellist  # only the > 512-atom fixtures (cellist.npz)

Inputs: the reference's own POSCAR files (/root/reference/web/public/data/structures/*.vasp,
parsed here as data) and synthetic SC cells from the bit-reproducible generator.
Expected outputs: the CPU restatement (oracle/liboracle.so) for the neighbour list, RBF and Gram
distances, and the reference's VERBATIM vendored Ripser (oracle/_ref/libdgn_ref.so, compiled from
/root/reference/third_party/ripser) for persistence pairs, counts and the 35 statistics. The script
asserts that the restated reduction agrees with verbatim Ripser on every complex it writes.

Outputs (tests/golden/*.npz, small): no reference source text is stored, only arrays.
"""
from __future__ import annotations

import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "defect-gnn-cpp_amd", "python")]
import oracle_py as O  # noqa: E402
from dgn import synth  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
REF_POSCARS = "/root/reference/web/public/data/structures"


def parse_poscar(path):
    """vasp_parser.cpp:13-78 + Structure ctor (structure.cpp:7-20), as data extraction."""
    lines = open(path).read().splitlines()
    scale = float(lines[1].split()[0])
    lat = np.array([[float(x) for x in lines[2 + i].split()[:3]] for i in range(3)]) * scale
    counts = [int(x) for x in lines[6].split()]
    direct = lines[7].strip()[:1] in ("d", "D")
    n = sum(counts)
    coords = np.array([[float(x) for x in lines[8 + i].split()[:3]] for i in range(n)])
    species = np.concatenate([np.full(c, k, np.int32) for k, c in enumerate(counts)])
    frac = coords if direct else coords @ np.linalg.inv(lat)
    # pos = L^T * frac; Eigen fixed-size redux order x0 + (x1 + x2) (unpinned)
    pos = np.empty((n, 3))
    for k in range(3):
        pos[:, k] = lat[0, k] * frac[:, 0] + (lat[1, k] * frac[:, 1] + lat[2, k] * frac[:, 2])
    return lat, pos, species


def betti_ref(lat, pos, species, rc):
    f, c = O.ref_structure_betti(lat, pos, species, rc, omp_threads=8, ripser_threads=1)
    f2, c2 = O.structure_betti(lat, pos, species, rc)
    assert np.array_equal(c, c2), "restated reduction disagrees with verbatim Ripser"
    assert np.allclose(f, f2, rtol=1e-12, atol=1e-12)
    return f, c


def rc10_fixtures():
    """(iv) The reference's default Betti cutoff, r_cutoff = 10 (preprocess_betti.cpp:117): verbatim
    Ripser counts and 35 statistics for EVERY atom of 741.vasp (N = 120) and of FCC-256 structure 0
    of the synthetic generator (the bench workload; ~340-point complexes). The restated reduction
    is not re-run here (minutes per structure single-threaded); the GPU tests compare against these
    arrays directly. Written to rc10.npz."""
    out = {}
    lat, pos, sp = parse_poscar(os.path.join(REF_POSCARS, "741.vasp"))
    f, c = O.ref_structure_betti(lat, pos, sp, 10.0, omp_threads=8, ripser_threads=1)
    out["741/features"], out["741/counts"] = f, c
    print("rc10 741", pos.shape[0], "atoms")
    bt = synth.make_batch("fcc", 4, 1)
    f, c = O.ref_structure_betti(bt["lattice"][0], bt["positions"], bt["species"], 10.0, omp_threads=8,
                                 ripser_threads=1)
    out["fcc256_0/features"], out["fcc256_0/counts"] = f, c
    out["fcc256_0/positions"] = bt["positions"]  # the generator's output, for a bit-identity check
    print("rc10 fcc256", bt["positions"].shape[0], "atoms")
    np.savez_compressed(os.path.join(OUT, "rc10.npz"), **out)


RC16_ATOMS = (0, 97, 203)


def _rc16_one(a):
    bt = synth.make_batch("fcc", 4, 1)
    pos, lat = bt["positions"], bt["lattice"][0]
    nl = O.neighbor_list(lat, pos, 16.0, None)
    rp = nl["row_ptr"]
    cloud = np.vstack([pos[a], pos[a] + nl["disp"][rp[a]:rp[a + 1]]])
    r = O.ref_persistence(O.local_distances(cloud), cloud.shape[0], np.float32(16.0))
    return a, cloud, r


def rc16_fixtures():
    """(v) Past the 1,024-point envelope of round 3: FCC-256 structure 0 at r_cutoff = 16
    (~1,400-point complexes, the HUGE wide instantiation), three atoms' clouds (the oracle's
    NeighborList(16, inf), betti_features.cpp:67-73) and their verbatim-Ripser pairs. Ripser needs
    ~15 min and ~34 GB per atom here: one atom at a time, rc16.npz rewritten after each."""
    out = {}
    for a in RC16_ATOMS:
        a, cloud, r = _rc16_one(a)
        out[f"{a}/cloud"] = cloud
        for d in ("dim0", "dim1", "dim2"):
            out[f"{a}/{d}"] = r[d]
        out[f"{a}/n_inf0"] = np.int32(r["n_inf0"])
        print("rc16 atom", a, cloud.shape[0], "points", [len(r[d]) for d in ("dim0", "dim1", "dim2")], flush=True)
        np.savez_compressed(os.path.join(OUT, "rc16.npz"), **out)


def triclinic_cell_688():
    """A 688-atom triclinic cell (above the 512-atom cell-list threshold of the Betti search): a
    jittered 8 x 9 x 9 grid in fractional coordinates of a sheared cell at 0.08 atoms/A^3, every
    37th atom moved one cell out (images n = +-1 in the reference's scan), and a 40-atom pocket
    around site 100 so that the local complexes span every tier (34..88 points at rc 5)."""
    rng = np.random.default_rng(2025)
    g = (8, 9, 9)
    n0 = int(np.prod(g))
    lat = np.array([[20.0, 0, 0], [3.5, 19.0, 0], [-2.5, 4.0, 21.0]]) * ((n0 / 0.08) / (20 * 19 * 21)) ** (1 / 3)
    idx = np.stack(np.meshgrid(*[np.arange(k) for k in g], indexing="ij"), -1).reshape(-1, 3)
    frac = (idx + 0.5 + rng.uniform(-0.3, 0.3, (n0, 3))) / np.array(g)
    frac[::37] += rng.choice([-1, 1], (len(frac[::37]), 3))
    pocket = frac[100] @ lat + rng.normal(0, 1.2, (40, 3))
    pos = np.vstack([frac @ lat, pocket])
    return lat, pos, (np.arange(pos.shape[0]) % 3).astype(np.int32)


CELLIST_SC_STRIDE = 8


def cellist_fixtures():
    """(vi) Structures above 512 atoms, where the Betti pass's neighbour search uses the cell list
    (betti_features.cpp:103-119 over neighbor_list.cpp:27-66): verbatim-Ripser counts + 35
    statistics of
      * config 5's SC-4096 supercell (synthetic generator, sc m = 16) at rc 5, every 8th atom;
      * the 688-atom triclinic cell above (positions stored) at rc 5, every atom.
    Written to cellist.npz."""
    out = {}
    bt = synth.make_batch("sc", 16, 1)
    f, c = O.ref_structure_betti(bt["lattice"][0], bt["positions"], bt["species"], 5.0, omp_threads=8,
                                 ripser_threads=1)
    out["sc4096/atoms"] = np.arange(0, bt["positions"].shape[0], CELLIST_SC_STRIDE, dtype=np.int32)
    out["sc4096/features"] = f[::CELLIST_SC_STRIDE]
    out["sc4096/counts"] = c[::CELLIST_SC_STRIDE]
    lat, pos, sp = triclinic_cell_688()
    f, c = betti_ref(lat, pos, sp, 5.0)
    out["tri688/lattice"], out["tri688/positions"], out["tri688/species"] = lat, pos, sp
    out["tri688/features"], out["tri688/counts"] = f, c
    np.savez_compressed(os.path.join(OUT, "cellist.npz"), **out)
    print("cellist: sc4096", bt["positions"].shape[0], "atoms; tri688", pos.shape[0], "atoms")


def main():
    assert O.ref_available(), "build oracle/_ref first (make -C oracle)"
    if sys.argv[1:] == ["rc10"]:
        rc10_fixtures()
        return
    if sys.argv[1:] == ["cellist"]:
        cellist_fixtures()
        return
    if sys.argv[1:] == ["rc16"]:
        rc16_fixtures()
        return
    # (i) POSCARs: inputs + CSR at rc=5, K=12/20, RBF (rc=5, dr=0.1) of 1 / 741, Betti at rc=5 of all
    poscar = {}
    for path in sorted(glob.glob(os.path.join(REF_POSCARS, "*.vasp"))):
        name = os.path.basename(path)[:-5]
        lat, pos, sp = parse_poscar(path)
        poscar[f"{name}/lattice"] = lat
        poscar[f"{name}/positions"] = pos
        poscar[f"{name}/species"] = sp
        for k in (12, 20):
            nl = O.neighbor_list(lat, pos, 5.0, k)
            poscar[f"{name}/k{k}/row_ptr"] = nl["row_ptr"]
            poscar[f"{name}/k{k}/col"] = nl["col"]
            poscar[f"{name}/k{k}/dist"] = nl["dist"]
            if name in ("1", "741"):
                poscar[f"{name}/k{k}/rbf"] = np.stack([O.gaussian_rbf(d, 5.0, 0.1) for d in nl["dist"]]).astype(
                    np.float64)
        # Betti at 5 A for all nine files: the (birth, death) multisets (hence the features) do not
        # depend on how distance ties are ordered, so the tied 1046* / *_1 / *_2 files pin too
        if True:
            f, c = betti_ref(lat, pos, sp, 5.0)
            poscar[f"{name}/betti5/features"] = f
            poscar[f"{name}/betti5/counts"] = c
        print("poscar", name, pos.shape[0], "atoms")
    np.savez_compressed(os.path.join(OUT, "poscar_rc5.npz"), **poscar)

    # (ii) 8 jittered SC-64 cells: CSR K=20 + all-atom Betti (verbatim Ripser), local distances of 2 atoms
    sc = {}
    bt = synth.make_batch("sc", 4, 8)
    n = 64
    for s in range(8):
        lat = bt["lattice"][s]
        pos = bt["positions"][s * n:(s + 1) * n]
        sp = bt["species"][s * n:(s + 1) * n]
        nl = O.neighbor_list(lat, pos, 5.0, 20)
        sc[f"{s}/row_ptr"] = nl["row_ptr"]
        sc[f"{s}/col"] = nl["col"]
        sc[f"{s}/dist"] = nl["dist"]
        f, c = betti_ref(lat, pos, sp, 5.0)
        sc[f"{s}/features"] = f
        sc[f"{s}/counts"] = c
        full = O.neighbor_list(lat, pos, 5.0, None)
        for a in (0, 37):
            r0, r1 = full["row_ptr"][a], full["row_ptr"][a + 1]
            cloud = np.vstack([pos[a], pos[a] + full["disp"][r0:r1]])
            sc[f"{s}/cloud{a}"] = cloud
            sc[f"{s}/lower{a}"] = O.local_distances(cloud)
            pr = O.ref_persistence(sc[f"{s}/lower{a}"], cloud.shape[0], np.float32(5.0))
            for d in ("dim0", "dim1", "dim2"):
                sc[f"{s}/pairs{a}/{d}"] = pr[d]
        print("sc64", s)
    np.savez_compressed(os.path.join(OUT, "sc64_rc5.npz"), **sc)

    # (iii) known-answer tests, expected pairs from verbatim Ripser
    kat = {}
    clouds = {
        "square": [[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0]],
        "octahedron": [[1, 0, 0], [-1, 0, 0], [0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1]],
        "cube": [[x, y, z] for x in (0, 1) for y in (0, 1) for z in (0, 1)],
        "tetrahedron": [[1, 1, 1], [1, -1, -1], [-1, 1, -1], [-1, -1, 1]],
        "hexagon": [[np.cos(k * np.pi / 3), np.sin(k * np.pi / 3), 0] for k in range(6)],
        "two_points": [[0, 0, 0], [3, 0, 0]],
        "duplicate": [[0, 0, 0], [0, 0, 0], [1, 0, 0]],
    }
    thresholds = {"octahedron_t15": 1.5}
    for name, pts in list(clouds.items()) + [("octahedron_t15", clouds["octahedron"])]:
        pts = np.asarray(pts, float)
        if name == "tetrahedron":
            pts = pts / np.sqrt(8.0)  # unit edge length
        thr = np.float32(thresholds.get(name, 10.0))
        low = O.local_distances(pts)
        pr = O.ref_persistence(low, pts.shape[0], thr)
        mine = O.persistence(low, pts.shape[0], thr)
        for d in ("dim0", "dim1", "dim2"):
            assert np.array_equal(pr[d], mine[d]), (name, d)
        kat[f"{name}/cloud"] = pts
        kat[f"{name}/threshold"] = np.float32(thr)
        for d in ("dim0", "dim1", "dim2"):
            kat[f"{name}/{d}"] = pr[d]
        kat[f"{name}/n_inf0"] = np.int32(pr["n_inf0"])
    np.savez_compressed(os.path.join(OUT, "kat.npz"), **kat)
    rc10_fixtures()
    cellist_fixtures()
    for f in sorted(glob.glob(os.path.join(OUT, "*.npz"))):
        print(f, os.path.getsize(f), "bytes")


if __name__ == "__main__":
    main()
