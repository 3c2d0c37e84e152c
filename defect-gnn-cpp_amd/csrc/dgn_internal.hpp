// dgn_internal.hpp — host-side launchers shared between the C ABI (dgn_api.cpp) and the
// kernel translation units. Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "dgn_device.hpp"

namespace dgn {

constexpr int kGraphBlock = 256;          // 4 waves
constexpr int kQA = 64;                   // query atoms per block (16 per wave, round-robin)
constexpr int kStage = 512;               // structures up to this size are staged in LDS
constexpr int kStreamMaxK = 64;           // max_neighbors up to this: block-streamed RBF emit
constexpr int kCellMax = 4096;            // cells per structure (cell list, natoms > kStage)
constexpr int kScanThreads = 1024;
constexpr int kRing = 128;                // per-wave candidate ring (one-image prefilter)
constexpr int kMaskWords = kStage / 64;   // hit-mask words per query atom (staged structures)
constexpr int kFewMaskWords = 8;          // `few` structures of <= 64 atoms: a hit word per image combination
static_assert(kFewMaskWords <= kMaskWords, "few masks use the per-atom mask slots");

// graph error bits (Scalars::error_flag), decoded in dgn_api.cpp
constexpr uint32_t kGErrCap = 1u << 0;       // more candidates than the emit capacity
constexpr uint32_t kGErrMismatch = 1u << 1;  // emit / Betti search disagrees with the count pass
constexpr uint32_t kGErrFar = 1u << 2;       // a position more than 500 cells away from the origin
constexpr uint32_t kGErrMissedHit = 1u << 3; // a count-pass hit failed the emit's exact test

struct GraphLaunch {
    const StructMeta* meta;
    const int32_t* atom_struct;  // [A] structure of each atom (prep_structures_kernel)
    const int64_t* atom_offset;
    const double* pos;
    const int32_t* cell_start;   // cell list: [first_b + b + c], c <= ncells (structures with cells)
    const double4* cell_pos;     // cell-sorted atoms: x, y, z, packed (j, floor of fractional coords)
    const uint64_t* mask;        // [A][kMaskWords] exact hits of the count pass (staged one-image), or null
    int64_t num_structures, num_atoms;
    double rc2, eps;
    uint64_t kmax;
    int32_t qa;                  // query atoms per block of the count / emit (graph_tile_atoms)
};

struct RbfSpec {
    int32_t dtype;  // DGN_NONE / DGN_F32 / DGN_F64
    int32_t nbins;
    double dr, inv_sigma2, norm;
    double c2;      // -0.5 * log2(e) / sigma^2 (f32 path exponent scale)
    float inv_nbins, norm_f;
};

// Per structure: geometry + the reference image bound + search strategy (thread per structure),
// then (block per structure) the atom -> structure map, the far-position check, the cell list of
// structures above kStage atoms and (optional) the per-atom 1/count(species) Betti weight.
hipError_t launch_prep_structures(hipStream_t s, const double* lattice, const int64_t* atom_offset, const double* pos,
                                  const int32_t* species, int64_t num_structures, double rc, StructMeta* meta,
                                  int32_t* atom_struct, int32_t* cell_start, double4* cell_pos, double* weight,
                                  uint32_t* error_flag);
// per-atom hit counts m (every neighbour within rc; the emit keeps min(m, kmax)); per block:
// block_sums[b] = sum of min(m, kmax) and block_aux[kAux b] = max m, block_aux[kAux b+1] = sum over
// atoms of (m + 1)^2, block_aux[kAux b+2] = largest structure, block_aux[kAux b+3] = sum of m,
// block_aux[kAux b+4] = atoms with 64 < m + 1 <= kWideRegular (low word) / > kWideRegular (high);
// mask_out (optional) [A][kMaskWords]: exact hits of staged one-image structures.
// defer [nblocks] (optional, needs mask_out): the one-image count kernel runs first and flags the
// tiles it cannot count for the general kernel
constexpr int kAux = 5;                   // block_aux words per count tile
constexpr int64_t kCountListGrid = 2048;  // blocks of the general count launch over the flags
hipError_t launch_graph_count(hipStream_t s, const GraphLaunch& g, int32_t* counts, int64_t* block_sums,
                              uint64_t* block_aux, uint64_t* mask_out, uint8_t* defer = nullptr);
hipError_t launch_block_scan(hipStream_t s, int64_t* block_sums, const uint64_t* block_aux, int64_t nblocks,
                             int64_t* total, uint32_t* max_candidates, unsigned long long* sum_sq,
                             uint32_t* max_natoms, unsigned long long* sum_m, unsigned long long* wide_atoms);
// Fused emit: each block re-runs the search for its atoms, ranks, writes row_ptr / col / dist /
// disp and the RBF. cap = graph_emit_cap(max candidates of the count pass, kmax): 64..2048 (the
// per-wave hit lists in LDS) or kEmitGlobalKeys (rows of more candidates: key_rows, caller-owned,
// emit_key_rows_per_chunk(max_candidates) rows of emit_key_row_doubles(max_candidates) doubles); stage = atoms
// staged in LDS (max structure size if <= kStage, else 0).
constexpr int kEmitGlobalKeys = -1;
constexpr int64_t kEmitGkChunkBlocks = 2048;        // tiles per launch of the global-key emit, at most
constexpr int64_t kEmitGkChunkBytes = 256ll << 20;  // key-row bytes per launch, at most (>= one tile)
int64_t emit_key_row_doubles(uint32_t max_candidates);
int64_t emit_key_chunk_tiles(uint32_t max_candidates);
int64_t emit_key_rows_per_chunk(uint32_t max_candidates);
hipError_t launch_graph_emit(hipStream_t s, const GraphLaunch& g, int cap, int stage, const int32_t* counts,
                             const int64_t* block_offsets, int64_t* row_ptr, int32_t* col, double* dist,
                             double* disp, void* rbf, const RbfSpec& rbf_spec, uint32_t* error_flag,
                             double* key_rows = nullptr, uint32_t max_candidates = 0, int chunk_tiles = 0);

hipError_t launch_rbf(hipStream_t s, const double* d, int64_t E, const RbfSpec& rs, int layout, void* out);

inline int64_t graph_blocks(int64_t num_atoms, int qa = kQA) { return (num_atoms + qa - 1) / qa; }
// query atoms per count / emit block: kQA, halved (down to 4) until the launch has >= 8 blocks per
// CU, so small batches (BASELINE configs 2 and 5) spread one or a few atoms per wave over the chip
// instead of 16 per wave over a few CUs
inline int graph_tile_atoms(int64_t num_atoms, int cus) {
    int qa = kQA;
    while (qa > 4 && graph_blocks(num_atoms, qa) < 8 * (int64_t)cus) qa >>= 1;
    return qa;
}
int graph_emit_cap(uint32_t max_candidates, uint64_t kmax);  // LDS cap, or kEmitGlobalKeys

// ---- Betti ----
// Outputs of the workgroup-per-complex apparent pass (betti_walk_kernel, betti_wide.hip) for the
// u16-coded wide complexes (65..kC16MaxPoints points, the reference's 10 A default), per position
// wi of a wide-list slice; the per-wave wide kernel then only reduces (meta == null: the per-wave
// kernel runs the whole complex itself)
enum { kWmNa2 = 0, kWmThr = 1, kWmNa1 = 2, kWmCl = 3, kWmD0 = 4, kWmInf0 = 5 };  // WalkOut::meta words
struct WalkOut {
    uint16_t* dmat;     // [slice][dstride]: the complex's full n x n u16 code matrix, diagonal 0xFFFF
    uint32_t* meta;     // [slice][8]: kWm* (list lengths may exceed their caps: capacity retry)
    float* d0;          // [slice][d0stride]: dim-0 deaths != 0, in Prim's order
    uint16_t* mce;      // [slice][mstride]: dim-1 min-cofacet vertex per edge (packed index), 0xFFFF none
    // [slice][cap1] dim-1 columns not in an apparent pair: packed edge (18 bits) | cofacet vertex << 18
    // | cofacet diameter code << 27
    uint64_t* e1;
    uint32_t* cl;       // [slice][cap1] triangles cleared by the dim-1 apparent pairs (combinatorial index)
    // [slice][cap] dim-2 columns not in an apparent pair, with their F-minimal cofacet (initial
    // pivot): packed triangle (27 bits) | cofacet vertex << 27 | cofacet diameter code << 36
    uint64_t* ent;
    int64_t dstride, d0stride, mstride;
    int32_t cap1, cap;  // powers of two
    int32_t nmax;
};
struct BettiLaunch {
    int64_t num_atoms;        // complexes of this launch
    float thr;                // (float) r_cutoff
    double* features;         // [A][35]
    int32_t* counts;          // [A][4] or null
    uint32_t* error_flag;
    uint32_t* work_counter;   // persistent work queue (main launch)
    uint32_t* work_counter2;  // persistent work queue (overflow launch)
    // complexes larger than the main instantiation's NP are listed here by a bucket pass and
    // reduced by a second, wider launch (so one rare large complex does not put the whole batch
    // on the low-occupancy instantiation)
    int32_t* overflow_list;   // [num_atoms]
    uint32_t* overflow_len;
    // complexes of the main launch with more than 512 distances <= thr (its register sort holds
    // 512 keys): listed by the main kernel and reduced by an NP = 64 launch after it
    int32_t* dense_list;      // [num_atoms]
    uint32_t* dense_len;
    uint32_t* dense_queue;
    uint8_t* scratch;         // per-wave global scratch
    int64_t scratch_per_wave;
    // optional cloud-input mode (dgn_host_persistence): complex c = clouds[c][max_points][3]
    const double* clouds;
    // Betti pass input: lower[c][tri_stride] f32 strict lower triangles (from betti_dist_kernel
    // or caller-given, dgn_host_persistence_lower), npoints[c], optional weight[c]
    const float* lower;
    const int32_t* npoints;
    const double* weight;     // 1/count(species) per complex (null = 1)
    int64_t tri_stride;       // floats per complex in `lower`
    int32_t cloud_stride;     // max_points (cloud-input mode row stride)
    // optional raw pair output: [C][3][pair_cap][2] f32 (dim0 as (0, death)), unsorted
    float* pairs_out;
    int32_t pair_cap;
    // complexes above 64 points, listed by the bucket pass for betti_wide_kernel
    int32_t* wide_list;       // [num_atoms]
    uint32_t* wide_len;
    uint32_t* wide_queue;
    // set by launch_betti per launch
    const int32_t* work_list; // null = all complexes 0..num_atoms-1
    const uint32_t* work_len; // entries of work_list (device)
    uint32_t* queue;          // work counter of this launch
    int32_t skip_above;       // 1 = complexes above NP are left to the overflow launch
    // capacity retry: complexes whose reduction outgrew a kernel's workspace are appended here
    // (null = report DGN_ERR_CAPACITY) and reduced again by betti_wide_kernel with the big layout
    int32_t* retry_list;      // [num_atoms]
    uint32_t* retry_len;
    int32_t force_retry;      // tests (DGN_DEBUG_FORCE_RETRY): the host lists every complex for the retry launch
    uint32_t* retried;        // capacity-retry launches: +1 per complex reduced (diagnostics counter), or null
    // complexes above kWideRegular points (the retry launch's BIG wide instantiation): per retry
    // slot r, rank codes of the packed lower triangle and the sorted f32 distances (betti_rank_codes)
    const uint32_t* rank_codes;  // [slots][rank_stride]
    const uint32_t* rank_sorted; // [slots][rank_stride]
    int64_t rank_stride;
    WalkOut walk;                // u16-coded wide launch after the walk pass (walk.meta null: none)
};
// wide complexes (65..kWideMaxPoints points, betti_wide.hip): per-wave scratch layout. Up to
// kWideRegular points in the regular launch; above it (rank-coded: 10-bit vertices up to
// kWideBigPoints, 11-bit vertices and the adjacency in scratch above) in the retry launch after
// betti_rank_codes
constexpr int kWideMaxPoints = 2048;
// caller-given clouds / triangles (dgn_host_persistence[_lower], one connected component at a time):
// complexes of up to this many points whose distances within the threshold number below 2^20 (the
// GIANT instantiation, betti_wide.hip)
constexpr int kWideGiantPoints = 4096;
// dgn_host_persistence[_lower] above kWideMaxPoints points: split into the connected components of
// the threshold graph (betti_split.hip), each reduced by the ordinary tiers; the union-find keeps
// a complex's parents in LDS (4 B per point)
constexpr int kSplitMaxPoints = 16384;
constexpr int kWideBigPoints = 1024;
constexpr int kWideRegular = 512;
constexpr int kC16MaxPoints = 362;  // C(362, 2) < 2^16: u16 rank codes (wide launch)
constexpr int kWideMaxGrow = 3;     // capacity-retry layout levels: tables of 2^24 .. 2^30 entries
constexpr int64_t kWideMaxCols = int64_t(1) << 29;  // column / pivot / pair tables (pivot hash: 2x)
constexpr int kWideWaves = 2;       // waves per wide workgroup, sharing one LDS adjacency buffer
struct WideLayout {
    uint8_t* base;  // scratch of wave w at base + w * total
    int64_t total;
    int32_t nmax, na_cap, p_cap, h_cap, vs_cap, vl_cap;
    int32_t slots;  // scratch slots of the launch (set by launch_betti_wide)
    int64_t guard;  // column-addition limit per column (a runaway-loop backstop)
    int64_t D, mc_e, mc_t, edges, adj, na_key, na_tau, na_tv, na_col, cl_list, vstore, vlist, h_key, h_meta,
        h_used, p1, p2, d0;
    int64_t clb;     // prewalked layout: cleared-triangle bitmap [C(nmax, 3) bits] (mc_t and D empty)
    int32_t prewalked;
};
// cap_limit > 0 (tests, DGN_DEBUG_WIDE_CAP): the regular layout's column / pivot / pair tables
// hold at most cap_limit entries, so ordinary complexes overflow in the kernel and take the
// capacity-retry path
// grow (big only, 0..kWideMaxGrow): the capacity-retry level, tables of 2^(base_log2 + 2 grow) entries
WideLayout betti_wide_layout(int nmax, bool big = false, int64_t cap_limit = 0, int grow = 0, int base_log2 = 24,
                             bool prewalked = false);
// walk pass (betti_walk_kernel): one workgroup per complex of the slice list (bl.wide_list, its
// device length bl.wide_len, u16 rank codes bl.rank_codes), outputs in bl.walk; `count` = the
// slice's length bound (grid)
constexpr int kWalkCap = 1 << 16;  // columns / cleared triangles per complex the walk pass lists (more: retry)
WalkOut betti_walk_out_layout(int nmax);  // strides and cap (pointers null)
int64_t betti_walk_out_bytes(int nmax);   // per complex
hipError_t launch_betti_walk(hipStream_t s, const BettiLaunch& b, int64_t count, int nmax);
hipError_t launch_betti_wide(hipStream_t s, const BettiLaunch& b, const WideLayout& l, int waves);
int betti_wide_resident_waves(int device, int nmax, bool c16 = false, bool pre = false);  // device-wide resident waves (occupancy API)
// rank codes for the complexes list[0..count) (retry slots): codes[r][t] = index of the first
// occurrence of lower[list[r]][t] in the complex's sorted packed triangle (order- and
// equality-preserving), sorted[r][...] = that sorted triangle (f32 bits). temp: caller-owned,
// size from betti_rank_temp_bytes. dev_len (may be null): the list's length on the device when
// `count` is only an upper bound (slots at or past it are left empty).
size_t betti_rank_temp_bytes(int64_t count, int64_t stride);
hipError_t betti_rank_codes(hipStream_t s, const float* lower, int64_t tri_stride, const int32_t* npoints,
                            const int32_t* list, int64_t count, int64_t stride, uint32_t* codes, uint32_t* sorted,
                            void* temp, size_t temp_bytes, const uint32_t* dev_len = nullptr);
// per slice q < nsl of a list of *total entries (device): sl[2q] = min(slice, max(0, *total - q slice)),
// sl[2q + 1] = 0 (the slice launch's queue)
hipError_t launch_slice_lengths(hipStream_t s, const uint32_t* total, int64_t slice, int64_t nsl, uint32_t* sl);

// component split (betti_split.hip): f32 packed triangles of clouds [first, first + count) (VALU
// Gram, the reference's arithmetic), union-find roots labels[c][v] over d <= thr, and the packed
// sub-triangle of each listed component (map: ascending vertices at off[q], size[q], of complex src[q])
hipError_t launch_big_gram(hipStream_t s, const double* clouds, int64_t cloud_stride, const int32_t* npoints,
                           int64_t first, int64_t count, float* lower, int64_t tri_stride);
hipError_t launch_components(hipStream_t s, const float* lower, int64_t tri_stride, const int32_t* npoints,
                             int64_t first, int64_t count, float thr, int32_t* labels, int64_t label_stride);
hipError_t launch_gather_sub(hipStream_t s, const float* lower, int64_t tri_stride, const int32_t* src,
                             const int64_t* off, const int32_t* size, const int32_t* map, int64_t count,
                             float* sub, int64_t sub_stride);

// distance pass over complexes [first, first + count) of a BettiLaunch's cloud input
struct DistLaunch {
    int64_t first, count;
    float* lower;      // [count][tri_stride]
    int32_t* npoints;  // [count]
    double* weight;    // [count]
};
hipError_t launch_betti_dist(hipStream_t s, const BettiLaunch& b, const DistLaunch& d);
// distance pass with its own neighbour search (graph_kernels.hip): complex c = atom first + c,
// cloud = centre + every neighbour within rc (betti_features.cpp:67-73, NeighborList(rc, inf));
// writes the packed f32 lower triangle and npoints; counts = the count pass's per-atom m.
// keys_out (diagnostics, may be null): [count][key_stride] packed (j, image) of cloud rows 1..m
hipError_t launch_betti_dist_search(hipStream_t s, const GraphLaunch& g, int64_t first, int64_t count,
                                    int max_points, int64_t tri_stride, const int32_t* counts, float* lower,
                                    int32_t* npoints, uint32_t* error_flag, uint64_t* keys_out = nullptr,
                                    int key_stride = 0);
int betti_max_points();      // largest local complex (centre + neighbours) the kernel accepts
int64_t betti_scratch_bytes_per_wave();
// fresh per-wave scratch: every min-cofacet byte "no cofacet" (0xFF), never a clearing mark
hipError_t betti_init_scratch(hipStream_t s, uint8_t* base, int slots);
// fresh wide scratch layout: empty pivot hash tables, u16 min-cofacet tables "no cofacet"
hipError_t betti_wide_init_scratch(hipStream_t s, const WideLayout& l, int waves);
int betti_grid_waves(int device);
// side stream for the overflow tier: forked from the launch stream after the bucket pass, joined
// after the main launch; it owns `overflow_waves` scratch slots past the main grid's
struct BettiFork {
    hipStream_t side;
    hipEvent_t fork, join;
    int overflow_waves;
};
// main (<= 48 points) + overflow (49..64) + wide (65..512) launches; `wide` null if max_points <= 64;
// `fork` null: the overflow tier runs after the main launch on the same stream
hipError_t launch_betti(hipStream_t s, const BettiLaunch& b, int max_points, int grid_waves, const WideLayout* wide,
                        int wide_waves, const BettiFork* fork = nullptr);

// ---- node features (node_kernels.hip) ----
// out[A][D + k]: embed[species[i]] (D f64) then (betti[i] - mean) * comp (k f64; comp row-major
// 35 x k); error_flag bit 0: a species key outside [0, nkeys)
hipError_t launch_node_features(hipStream_t s, const int32_t* species, int64_t A, const double* embed, int32_t nkeys,
                                int32_t D, const double* betti, const double* mean, const double* comp, int32_t k,
                                double* out, uint32_t* error_flag);
// flat per-edge arrays of a CSR (WasmAPI graph accessors): src = row atom's in-structure index,
// tgt = col, f32 casts of dist and disp [E][3]; any output may be null
hipError_t launch_edge_arrays(hipStream_t s, const int64_t* row_ptr, const int64_t* atom_offset, int64_t B, int64_t A,
                              const int32_t* col, const double* dist, const double* disp, int32_t* src, int32_t* tgt,
                              float* dist32, float* disp32);

}  // namespace dgn
