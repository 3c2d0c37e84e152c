/*
 * dgn.h — C ABI of the MI355X-native crystal-graph + Betti feature path (libdgn.so).
 *
 * Drop-in boundary for the reference's include/graph and include/topology hot path
 * (bamarler/Defect-GNN-cpp). Plain pointers and sizes only; no exceptions cross this
 * boundary; every entry point returns a dgn_status. Each function names the reference
 * interface it replaces (file:line in the reference tree).
 *
 * Two levels:
 *   dgn_dev_*  : device pointers (HBM-resident inputs/outputs), asynchronous on the context's
 *                stream except where noted. This is what the bench times.
 *   dgn_host_* : host pointers; the library stages through its own device buffers. This is
 *                what the C++ facade (defect-gnn-cpp_amd/cpp) and FFI callers use.
 *
 * Threading: one context per device/stream; calls on different contexts are thread-safe;
 * a context must not be used from two threads at once (reference: NeighborList is immutable
 * after construction, include/graph/neighbor_list.hpp:19-24; Ripser spawns its own threads —
 * num_threads is accepted and ignored on this path).
 */
#ifndef DGN_H
#define DGN_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status ------------------------------------------------------------------------- */
typedef enum {
    DGN_OK = 0,
    DGN_ERR_ARG = 1,         /* bad argument (reference: std::out_of_range / UB)            */
    DGN_ERR_HIP = 2,         /* HIP runtime error                                         */
    DGN_ERR_CAPACITY = 3,    /* caller buffer too small / per-complex workspace overflow  */
    DGN_ERR_NODEVICE = 4,    /* no GPU visible — there is NO CPU fallback                  */
    DGN_ERR_UNSUPPORTED = 5, /* outside the implemented envelope           */
    DGN_ERR_INTERNAL = 6     /* a device-side consistency check failed                    */
} dgn_status;

const char* dgn_status_string(int status);

/* ---- context -------------------------------------------------------------------------- */
typedef struct dgn_ctx dgn_ctx;

/* A context owns its device workspaces, grown on demand and kept until dgn_ctx_destroy. The first
 * Betti pass with complexes of at most kWideRegular (512) points also allocates the device-driven
 * capacity-retry workspace once: 8..32 first-level big-layout waves within an eighth of the free HBM
 * and at most 32 GB (about 0.3 GB at 64 points, about 13 GB at the 10 A cutoff's ~340 points),
 * whether or not any complex overflows, so that later passes never wait for the host; several
 * contexts on one GPU each hold their own. Per-wave Betti scratch (narrow kernel ~1 MB per resident
 * wave, wide kernel 15-60 MB per wave, at most half of the free HBM) is held the same way. */
int dgn_ctx_create(int device, dgn_ctx** out);
void dgn_ctx_destroy(dgn_ctx* ctx);
/* Use an external hipStream_t (e.g. torch's current stream); NULL = the context's own. */
int dgn_ctx_set_stream(dgn_ctx* ctx, void* hip_stream);
int dgn_ctx_synchronize(dgn_ctx* ctx);
/* Debug / A-B knobs (tests and experiments only; the library never reads the environment):
 * DGN_DEBUG_FORCE_RETRY  1 = every complex of a Betti pass is reduced again by the capacity-retry
 *                        launch (the path is then checked on every tier);
 * DGN_DEBUG_WIDE_WAVES   cap on the wide Betti launch's resident waves (0 = none);
 * DGN_DEBUG_WIDE_C16     0 = f32 distances for every wide complex (default 1: u16 rank codes);
 * DGN_DEBUG_WIDE_CAP     > 0: the wide launch's column / pivot / pair tables hold at most this many
 *                        entries (rounded up to a power of two), so ordinary complexes overflow in the
 *                        kernel and take the in-kernel capacity-retry path; 0 = the natural caps;
 * DGN_DEBUG_BIG_LOG2     > 0: the capacity-retry layout's first level holds 2^value-entry column /
 *                        pivot / pair tables and V store (default 2^24), so ordinary complexes outgrow it
 *                        and are reduced again at the next levels (4x the tables each); 0 = natural;
 * DGN_DEBUG_EMIT_CHUNK   > 0: the large-row graph emit (per-wave key rows in HBM) launches this many
 *                        tiles at a time instead of its byte budget's count (its chunk loop on small
 *                        inputs); 0 = natural;
 * DGN_DEBUG_WIDE_WALK    0 = the u16-coded wide complexes' whole apparent phase inside the per-wave
 *                        wide kernel (default 1: the workgroup-per-complex walk pass before it);
 * DGN_DEBUG_SPLIT_CHUNK  > 0: the component split of dgn_host_persistence[_lower] above 2,048 points
 *                        takes at most this many clouds per chunk (its chunk loop on small inputs). */
enum {
    DGN_DEBUG_FORCE_RETRY = 1,
    DGN_DEBUG_WIDE_WAVES = 2,
    DGN_DEBUG_WIDE_C16 = 3,
    DGN_DEBUG_WIDE_CAP = 4,
    /* 5: removed (the round-3 workgroup-per-complex kernel) */
    DGN_DEBUG_BIG_LOG2 = 6,
    DGN_DEBUG_EMIT_CHUNK = 7,
    DGN_DEBUG_WIDE_WALK = 8,
    DGN_DEBUG_SPLIT_CHUNK = 9
};
int dgn_ctx_set_debug(dgn_ctx* ctx, int knob, int value);
/* Diagnostics: complexes the capacity-retry launches reduced since the last call (synchronizes). */
int dgn_debug_retry_count(dgn_ctx* ctx, int64_t* count);
/* Diagnostics: how many times the context's calls waited for its stream since the last call
 * (no synchronization itself; tests of the asynchronous device entry points). */
int dgn_debug_host_syncs(dgn_ctx* ctx, int64_t* count);
/* Diagnostics (host arithmetic only, no device, no context): every wide-kernel scratch layout the
 * Betti pass can choose (65..4,096 points, regular and capacity-retry at every growth level) has
 * positive power-of-two int32 table capacities. DGN_OK, or DGN_ERR_INTERNAL with *first_bad =
 * nmax * 64 + big * 16 + grow of the first layout that does not. */
int dgn_debug_check_wide_layouts(int64_t* first_bad);
const char* dgn_ctx_last_error(const dgn_ctx* ctx);

/* Per-kernel timing with hipEvents recorded on the launch stream around every launch. */
typedef struct {
    char name[48];
    int64_t launches;
    double total_ms;
    /* algorithmic bytes / flops the launches were accounted for */
    double bytes;
    double flops;
} dgn_kernel_time;
int dgn_ctx_enable_timing(dgn_ctx* ctx, int on);
/* Synchronizes, folds pending events, returns the number of kernel records (<= cap copied). */
int dgn_ctx_kernel_times(dgn_ctx* ctx, dgn_kernel_time* out, int cap);
int dgn_ctx_reset_timing(dgn_ctx* ctx);

/* ---- batched input (replaces crystal::Structure, src/crystal/structure.cpp:7-20) -------- */
typedef struct {
    int64_t num_structures;
    int64_t num_atoms;          /* total atoms over all structures                      */
    const double* lattice;      /* [B][3][3] row-major, rows = a, b, c (Structure::lattice)  */
    const double* positions;    /* [A][3] Cartesian (Atom::position = L^T * frac)       */
    const int32_t* species;     /* [A] species index (Atom::element, vasp_parser.cpp:66) */
    const int64_t* atom_offset; /* [B+1] first atom of each structure                   */
} dgn_batch;

/* ---- graph: NeighborList + gaussian_rbf + CrystalGraph edge part ----------------------
 * Replaces graph::NeighborList(structure, r_cutoff=10, max_neighbors=20, epsilon=1e-10)
 * (include/graph/neighbor_list.hpp:19-22, src/graph/neighbor_list.cpp:14-94), the per-edge
 * gaussian_rbf(distance, r_cutoff, dr) (src/graph/edge_features.cpp:7-24) and the edge loop of
 * CrystalGraph (src/graph/crystal_graph.cpp:23-40).
 * Output CSR: rows = atoms of the whole batch in order; row_ptr is global (int64); col_idx is
 * the neighbour's index WITHIN its structure (Neighbor::idx); edges of a row are sorted by
 * (distance, idx, image) and truncated to max_neighbors. */
enum { DGN_NONE = 0, DGN_F32 = 1, DGN_F64 = 2 };

typedef struct {
    double r_cutoff;        /* NeighborList r_cutoff (reference default 10.0)           */
    uint64_t max_neighbors; /* reference default 20; UINT64_MAX = unlimited           */
    double epsilon;         /* self-image skip threshold (1e-10): an image of the query atom
                               closer than epsilon is skipped (neighbor_list.cpp:47); epsilon <= 0
                               keeps the atom itself at distance 0, as the reference does */
    double rbf_cutoff;      /* CrystalGraph r_cutoff for the RBF (default 10.0)       */
    double rbf_dr;          /* CrystalGraph dr (default 0.1)                          */
    int32_t rbf_dtype;      /* DGN_F32 (default), DGN_F64, DGN_NONE                    */
    int32_t write_displacement; /* also emit Neighbor::displacement [E][3] f64         */
} dgn_graph_params;

void dgn_graph_params_default(dgn_graph_params* p);
int dgn_rbf_bins(double rbf_cutoff, double rbf_dr); /* floor(rc/dr), edge_features.cpp:13 */

typedef struct {
    int32_t* col_idx;      /* [E]                                                  */
    double* distance;      /* [E]                                                  */
    double* displacement;  /* [E][3] or NULL                                        */
    void* rbf;             /* [E][n_rbf] row-major f32/f64 or NULL                  */
} dgn_graph_out;

/* Phase 1 (device): per-atom counts and their scan are kept in the context; the total edge
 * count E is copied to *num_edges (this call synchronizes the stream once). */
int dgn_dev_graph_count(dgn_ctx* ctx, const dgn_batch* batch, const dgn_graph_params* p,
                        int64_t* num_edges);
/* Phase 2 (device, async): write row_ptr[A+1] and fill the CSR + edge features (capacity E from
 * phase 1). Must follow dgn_dev_graph_count on the same context with the same batch/params. */
int dgn_dev_graph_emit(dgn_ctx* ctx, const dgn_batch* batch, const dgn_graph_params* p,
                       int64_t* row_ptr, const dgn_graph_out* out);

/* Host-level convenience: the library owns the result; free with dgn_graph_result_free. */
typedef struct {
    int64_t num_atoms, num_edges;
    int32_t n_rbf, rbf_dtype;
    int64_t* row_ptr;
    int32_t* col_idx;
    double* distance;
    double* displacement; /* NULL unless requested */
    void* rbf;            /* NULL if DGN_NONE       */
} dgn_graph_result;
int dgn_host_graph(dgn_ctx* ctx, const dgn_batch* host_batch, const dgn_graph_params* p,
                   dgn_graph_result** out);
void dgn_graph_result_free(dgn_graph_result* r);

/* ---- topology: per-atom 35-d Betti statistics -------------------------------------------
 * Replaces topology::compute_structure_betti_features(structure, r_cutoff=10, threads=8)
 * (include/topology/betti_features.hpp:37-39, src/topology/betti_features.cpp:57-119), i.e.
 * NeighborList(rc, SIZE_MAX) + compute_persistence (src/topology/ripser_wrapper.cpp:11-70,
 * Ripser dim 2, Z/2, threshold rc) + compute_statistics (betti_features.cpp:24-55).
 * features: [A][35] f64 row-major (the facade transposes to the reference's column-major
 * per-structure MatrixXd). counts (optional): [A][4] int32 = #dim0 finite, #dim0 infinite,
 * #dim1, #dim2 pairs exactly as the reference emits them (death > birth; essential dim>=1
 * classes are not emitted). An isolated atom yields 35 zeros and counts (0,1,0,0)
 * (the reference segfaults, third_party/ripser/ripser.cpp:761). */
typedef struct {
    double r_cutoff; /* reference default 10.0 */
} dgn_betti_params;

/* dgn_dev_betti synchronizes once, after its own neighbour count (the local complexes' size sets the
 * kernel tier and workspaces); the Betti kernels then run asynchronously and their error status
 * (envelope, workspace overflow of a retried complex, a search/count disagreement) is returned by the
 * next synchronizing call on the context (dgn_ctx_synchronize, dgn_dev_graph_count, a dgn_host_*
 * call); the affected atoms' features are NaN and their counts -1 either way. */
int dgn_dev_betti(dgn_ctx* ctx, const dgn_batch* batch, const dgn_betti_params* p, double* features,
                  int32_t* counts);
int dgn_host_betti(dgn_ctx* ctx, const dgn_batch* host_batch, const dgn_betti_params* p,
                   double* features, int32_t* counts);

/* Fused step (device; no host synchronization while every local complex has at most kWideRegular
 * (512) points -- the 5 A path and the reference's 10 A default alike: the wide tier's rank-code
 * slices are sized from the count pass's census of wide complexes and take their lengths on the
 * device, and the capacity-retry launch is device-driven (a complex that outgrows its first level
 * is reported as DGN_ERR_CAPACITY here; dgn_host_betti grows the tables instead). Larger complexes
 * size the rank-coded retry from a host read. Errors are reported by the next synchronizing call
 * as for dgn_dev_betti): dgn_dev_graph_emit of a
 * preceding dgn_dev_graph_count, then dgn_dev_betti on the same batch. When the Betti cutoff equals
 * the graph cutoff (and epsilon is the default 1e-10) the Betti pass reuses the graph count's
 * per-atom neighbour counts and hit masks instead of searching a third time: CrystalGraph's
 * NeighborList(rc, K) and compute_structure_betti_features' NeighborList(rc, SIZE_MAX)
 * (betti_features.cpp:107) enumerate the same candidates. The positions must not change between
 * the count and this call (as for dgn_dev_graph_emit); the count's 1/count(species) Betti weights are
 * reused only when `batch->species` is the pointer the count saw, whose contents must not change in
 * between either (a different pointer: the Betti pass runs its own neighbour count). */
int dgn_dev_graph_betti(dgn_ctx* ctx, const dgn_batch* batch, const dgn_graph_params* p, int64_t* row_ptr,
                        const dgn_graph_out* out, const dgn_betti_params* bp, double* features, int32_t* counts);

/* ---- node features + topological block (CrystalGraph node_features) --------
 * Device pointers, asynchronous on the context's stream. out: [A][D + k] f64 row-major, row i =
 * embed[species[i]] (the species-keyed embedding gather of crystal_graph.cpp:19-21; embed is
 * [num_keys][D] f64 row-major, row s = atom_embeddings.at(s)) followed by k columns
 * (betti[i] - pca_mean) * pca_components (PCA::transform, pca.cpp:36-44; betti [A][35] f64 as
 * dgn_dev_betti writes it, pca_mean [35], pca_components [35][k] row-major, k <= 35): the
 * N x (D + k) concatenation add_topo_features (crystal_graph.cpp:65-67) names. betti may be NULL
 * (k must then be 0). The call waits for its stream (one flag read back) and returns DGN_ERR_ARG
 * if a species key is outside [0, num_keys): the reference's std::map::at throws out_of_range. */
int dgn_dev_node_features(dgn_ctx* ctx, const dgn_batch* batch, const double* embed, int32_t num_keys, int32_t D,
                          const double* betti, const double* pca_mean, const double* pca_components, int32_t k,
                          double* out);

/* ---- flat float32 edge arrays (WasmAPI graph accessors) ------------------
 * Replaces WasmAPI::num_edges / get_edge_sources / get_edge_targets / get_edge_distances /
 * get_edge_displacements (src/viz/wasm_bindings.cpp:206-294) for a whole batch: from a CSR written by
 * dgn_dev_graph_emit (row_ptr [A+1], col_idx [E], distance [E], displacement [E][3] when requested)
 * write sources[E] (the row atom's index within its structure), targets[E] (= col_idx),
 * distances_f32[E] and displacements_f32[E][3] (static_cast<float> of the f64 values). Device
 * pointers, asynchronous on the context's stream; any output may be NULL (its input may then be
 * NULL too). */
int dgn_dev_edge_arrays(dgn_ctx* ctx, const dgn_batch* batch, const int64_t* row_ptr, const int32_t* col_idx,
                        const double* distance, const double* displacement, int32_t* sources, int32_t* targets,
                        float* distances_f32, float* displacements_f32);
/* Host-level: NeighborList(r_cutoff, max_neighbors, epsilon) of a host batch on the device, then the
 * arrays above (WasmAPI::build_graph + the graph accessors). Free with dgn_edge_arrays_free. */
typedef struct {
    int64_t num_edges;
    int32_t* sources;
    int32_t* targets;
    float* distances;
    float* displacements; /* [E][3] */
} dgn_edge_arrays;
int dgn_host_edge_arrays(dgn_ctx* ctx, const dgn_batch* host_batch, double r_cutoff, uint64_t max_neighbors,
                         double epsilon, dgn_edge_arrays** out);
void dgn_edge_arrays_free(dgn_edge_arrays* a);

/* Local-complex persistence from point clouds (replaces topology::compute_persistence,
 * src/topology/ripser_wrapper.cpp:60-70). clouds: [C][max_points][3] f64 (host), npoints[C].
 * pairs: [C][3][cap][2] f32 (host) sorted ascending by (birth, death); counts [C][4].
 * Envelope: max_points <= 16,384; clouds above 2,048 points are reduced per connected component of
 * their threshold graph, each of at most 4,096 points and, above 2,048, fewer than 2^20 distances
 * within the threshold; outside it DGN_ERR_UNSUPPORTED, never a truncated result. */
int dgn_host_persistence(dgn_ctx* ctx, const double* clouds, const int32_t* npoints, int64_t num_clouds,
                         int32_t max_points, double threshold, float* pairs, int32_t cap, int32_t* counts);

/* Gaussian RBF of caller-given distances (replaces the per-edge gaussian_rbf calls of
 * CrystalGraph, src/graph/crystal_graph.cpp:32-40). Host arrays. layout 0 = row-major [E][n_rbf],
 * 1 = column-major (Eigen MatrixXd edge_attr: element (e,k) at k*E + e). dtype DGN_F32/DGN_F64. */
int dgn_host_rbf(dgn_ctx* ctx, const double* distances, int64_t num_edges, double rbf_cutoff,
                 double rbf_dr, int32_t dtype, int32_t layout, void* out);

/* Persistence from caller-given distance matrices (replaces
 * topology::compute_persistence_from_distances, src/topology/ripser_wrapper.cpp:11-58): lower:
 * [C][max_points*(max_points-1)/2] f32, the strict lower triangle row by row (i = 1..n-1, j < i)
 * exactly as ripser_wrapper.cpp:20-24 packs it; other arguments as dgn_host_persistence. */
int dgn_host_persistence_lower(dgn_ctx* ctx, const float* lower, const int32_t* npoints, int64_t num_clouds,
                               int32_t max_points, double threshold, float* pairs, int32_t cap,
                               int32_t* counts);

/* Diagnostics (parity tests): the local complexes of atoms [atom_first, atom_first + count) of a
 * host batch as the Betti pass's distance kernel builds them (NeighborList(rc, SIZE_MAX) search +
 * Gram distances, betti_features.cpp:67-73 / ripser_wrapper.cpp:20-24). lower: [count]
 * [max_points*(max_points-1)/2] f32 strict lower triangles in the kernel's cloud row order;
 * npoints[count]; keys (optional): [count][max_points] int64, row p >= 1 of the cloud is neighbour
 * key[p-1] = (j << 24) | (na+128) << 16 | (nb+128) << 8 | (nc+128) (atom j, lattice image
 * (na, nb, nc)), row 0 the centre. DGN_ERR_CAPACITY if a complex exceeds max_points. */
int dgn_debug_betti_clouds(dgn_ctx* ctx, const dgn_batch* host_batch, double r_cutoff, int64_t atom_first,
                           int64_t count, int32_t max_points, float* lower, int32_t* npoints, int64_t* keys);

/* ---- synthetic batches (bench/test inputs) -----------------------
 * kind 0 = simple cubic m^3 (s = 2.32 A), kind 1 = FCC m^3 cells (a = 3.684 A). Host arrays:
 * lattice [B][9], positions [B*n][3], species [B*n], atom_offset [B+1]. */
int64_t dgn_synth_atoms_per_structure(int kind, int m);
int dgn_synth_batch(int kind, int m, int64_t num_structures, int64_t first_id, double* lattice,
                    double* positions, int32_t* species, int64_t* atom_offset);

#ifdef __cplusplus
}
#endif
#endif /* DGN_H */
