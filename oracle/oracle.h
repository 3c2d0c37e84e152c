/*
 * oracle.h — CPU restatement of the reference hot path (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the checker for the MI355X product path. Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it. The product
 * library (libdgn.so) never links, loads or calls it, and has no CPU fallback.
 *
 * Every function restates the behaviour of bamarler/Defect-GNN-cpp
 * (reference mounted read-only at /root/reference) and cites file:line:
 *   neighbour search   src/graph/neighbor_list.cpp:27-94   (nanoflann v1.5.5 -> exhaustive scan)
 *   Gaussian RBF       src/graph/edge_features.cpp:7-24
 *   Gram distances     src/topology/ripser_wrapper.cpp:11-33,60-70
 *   VR persistence     third_party/ripser/ripser.cpp:514-1269 (semantics; own reduction code)
 *   35 statistics      src/topology/betti_features.cpp:24-119, include/utils/math.hpp:9-28
 *
 * Parity pinning: the VR restatement is pinned against the verbatim vendored Ripser built
 * from /root/reference by oracle/Makefile (oracle/_ref/libdgn_ref.so) and against the SURVEY
 * section 4 known-answer tests (tests/golden/). The Eigen / nanoflann arithmetic orders are
 * restated from their upstream sources (Eigen 3.4.0, nanoflann 1.5.5 — both absent offline):
 * parity on those two boundaries is UNPINNED ("Oracle").
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- neighbour list (CSR) ------------------------------------------------------------ */
/* One structure: lattice rows a,b,c (row-major 3x3), Cartesian positions [n][3].
 * Emits the reference NeighborList rows (neighbor_list.cpp:35-65) in canonical order
 * (distance, j, n_a, n_b, n_c). row_ptr[n+1] must be provided; when col==NULL only counts
 * are produced. Returns total edges. max_neighbors == UINT64_MAX means unlimited. */
int64_t oracle_neighbor_list(const double* lattice, const double* pos, int64_t n, double r_cutoff,
                             uint64_t max_neighbors, double epsilon, int64_t* row_ptr,
                             int32_t* col, double* dist, double* disp /* [E][3] or NULL */,
                             int32_t* image /* [E][3] or NULL */);

/* Reference image count: ceil(rc / min row norm) + 1 (neighbor_list.cpp:68-72). */
int oracle_num_images(const double* lattice, double r_cutoff);

/* ---- Gaussian RBF (edge_features.cpp:7-24) -------------------------------------------- */
int oracle_rbf_bins(double r_cutoff, double dr);
void oracle_gaussian_rbf(double distance, double r_cutoff, double dr, double* out);

/* CrystalGraph edge part for one structure (neighbour rows + one RBF per edge); rbf_out may be
 * NULL (timing only). Returns E. */
int64_t oracle_structure_graph(const double* lattice, const double* pos, int64_t n, double r_cutoff,
                               uint64_t max_neighbors, double epsilon, double rbf_cutoff, double dr,
                               double* rbf_out);

/* ---- local distance matrix (ripser_wrapper.cpp:60-70 then :17-24) --------------------- */
/* cloud [n][3] f64 -> strict lower triangle, row i=1..n-1, j<i, as float32. */
void oracle_local_distances(const double* cloud, int n, float* lower);

/* ---- VR persistence (Ripser semantics, own reduction) ----------------------------------- */
typedef struct {
    int32_t n_dim0_finite, n_dim0_inf, n_dim1, n_dim2;
} oracle_counts;

/* Pairs are written as (birth, death) float pairs into caller buffers of capacity cap each
 * (dim0 finite pairs only; infinite dim0 pairs are counted). Output pairs are sorted
 * ascending by (birth, death). Returns 0, or -1 if a buffer was too small.
 * stats (optional, 8 int64): columns d1, apparent d1, additions d1, columns d2, apparent d2,
 * additions d2, triangles, tetrahedra-visited. */
int oracle_persistence(const float* lower, int n, float threshold, float* dim0, float* dim1,
                       float* dim2, int cap, oracle_counts* counts, int64_t* stats);

/* ---- 35 statistics (betti_features.cpp:24-55 + math.hpp:9-28) -------------------------- */
/* pairs: (birth,death) float pairs. which: 0 birth, 1 death, 2 persistence. out[5]. */
void oracle_statistics(const float* pairs, int m, int which, double weight, double* out);

/* ---- whole structure Betti features (betti_features.cpp:57-119) -------------------------- */
/* species[n] are used for the 1/count weight (betti_features.cpp:62-63,77). features is
 * row-major [n][35]; counts [n][4]. Isolated atom (reference UB) -> 35 zeros + (0,1,0,0). */
int oracle_structure_betti(const double* lattice, const double* pos, const int32_t* species,
                           int64_t n, double r_cutoff, double* features, int32_t* counts);

#ifdef __cplusplus
}
#endif
