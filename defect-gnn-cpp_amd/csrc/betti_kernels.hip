// betti_kernels.hip — per-atom Vietoris–Rips persistence (dim 0/1/2, Z/2) and the 35 Betti
// statistics, one wave64 per local complex, for gfx950.
//
// Replaces, per atom (src/topology/betti_features.cpp:57-101):
//   local cloud row0 = pos_i, row k+1 = pos_i + disp_k           (betti_features.cpp:67-73)
//   Gram distances -> float32 lower triangle                      (ripser_wrapper.cpp:60-70, 17-24)
//   ripser<sparse_distance_matrix>(dim 2, thr, ratio 1, mod 2)    (third_party/ripser/ripser.cpp)
//   7 x compute_statistics -> 35 doubles                           (betti_features.cpp:24-55, 87-98)
//
// Algorithm (MI355X-first; DESIGN.md "Betti kernel"):
//   * n <= NP points per complex (NP in {32, 48, 64}): one lane per vertex, 64-bit adjacency
//     masks, the distance matrix in LDS as u16 RANK CODES (code = index of the distance's first
//     occurrence among the complex's sorted distances <= thr; 0xFFFF above thr and on the
//     diagonal): order and equality are all the reduction ever asks of a distance
//     (ripser.cpp:318-324, 386-395), the f32 values come back from the sorted table only for
//     the emitted pairs. 2 B per entry keep a 48-point complex in 5 KB of LDS (eight waves per
//     SIMD instead of five with the f32 matrix);
//   * distance matrix (the distance kernels, dgn_device.hpp gram_triangle_*): the K = 3 Gram product
//     with every product rounded, summed in the reference's order ((p0+p1)+p2), then
//     sqrt(max(0,(sq_i+sq_j)-2p)) -> f32, bit-identical to the reference's Eigen/SSE2 arithmetic --
//     one packed pair per lane on the f64 VALU for n <= 64 (round 5: measured faster than 16x16
//     v_mfma_f64 tiles, 5.94 -> 4.20 ms per config-4 shard), matrix-core tiles above 64 points;
//   * dim 0: Prim on F-keys (diameter, then combinatorial index descending) == Kruskal's unique
//     minimum spanning forest in Ripser's order (ripser.cpp:725-762);
//   * dim 1 and dim 2: cohomology with clearing. One lane per column finds its pivot (F-minimal
//     cofacet) and settles apparent pairs (sigma youngest facet of tau, tau oldest cofacet of
//     sigma). The wave then walks the remaining columns in Ripser's column order. A column is
//     carried as its V list (the set of column simplices summed into it, Ripser's reduction
//     matrix) with a membership bitmap in LDS; its pivot is recomputed lane-parallel as the
//     F-minimal cofacet of odd multiplicity over the coboundaries of V (no sorting, no merging).
//     Owners are looked up in a pivot table (serially resolved columns) or re-derived on the fly
//     (apparent pairs). The persistence pairing of a total order is unique, so the emitted
//     (birth, death) multiset equals the lock-free Ripser's (death > birth only; essential
//     dim>=1 classes are not emitted, ripser.cpp:1209-1225).
//   * persistent grid, chunked dynamic dequeue; per-wave global scratch for reduced columns
//     and pair lists.
#include <atomic>

#include "dgn_internal.hpp"

namespace dgn {

constexpr int kVCap = 128;        // simplices in one column's V list (registers: 2 per lane)
constexpr int kVStoreCap = 65536; // stored V-list entries per dimension
constexpr int kNACap = 4096;      // non-apparent columns per dimension (scratch)
constexpr int kPivCap = 4096;     // serially resolved pivots per dimension
constexpr int kPairCap = 4096;    // pairs per dimension (scratch)
constexpr uint32_t kNoCode = 0xFFFFu;  // rank-code matrix: distance above thr, or the diagonal
#ifndef DGN_CHUNK
#define DGN_CHUNK 1
#endif
constexpr int kChunk = DGN_CHUNK;  // complexes per dequeue (1: the grid drains within one complex; A/B 227.6 vs 230.4 ms at 4)
#ifndef DGN_PV_UNROLL
#define DGN_PV_UNROLL 4
#endif
constexpr int kPvUnroll = DGN_PV_UNROLL;  // V entries per step of the pivot search
#ifndef DGN_APP_STEPS
#define DGN_APP_STEPS 1
#endif
constexpr int kAppSteps = DGN_APP_STEPS;  // walk steps of an apparent pass's first round

constexpr uint64_t kInf = ~0ull;
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kLazyBit = 0x80000000u;  // vmeta: V = {column simplex} (packed in the low bits)
// min-cofacet table entries (one byte per edge / triangle): the vertex k whose insertion gives
// the F-minimal cofacet, or one of these marks
constexpr uint8_t kMcNone = 0xFF;     // not a column, or no cofacet
constexpr uint8_t kMcCleared = 0xFE;  // triangle is the pivot of a dim-1 column (clearing)

// error bits (mirrored in dgn_api.cpp)
constexpr uint32_t kErrTooManyPoints = 1u << 0;
constexpr uint32_t kErrWorkCol = 1u << 1;
constexpr uint32_t kErrNA = 1u << 2;
constexpr uint32_t kErrPiv = 1u << 3;
constexpr uint32_t kErrPairs = 1u << 4;
constexpr uint32_t kErrR = 1u << 5;
constexpr uint32_t kErrCapacity = kErrWorkCol | kErrNA | kErrPiv | kErrPairs | kErrR;

// scratch layout per wave (bytes)
struct ScratchLayout {
    static constexpr int64_t na_key = 0;                             // uint64 [kNACap] (unsorted)
    static constexpr int64_t na_tau = na_key + 8 * kNACap;           // uint64 [kNACap]
    static constexpr int64_t sna_key = na_tau + 8 * kNACap;          // sorted copies
    static constexpr int64_t sna_tau = sna_key + 8 * kNACap;
    static constexpr int64_t vmeta = sna_tau + 8 * kNACap;           // uint32 [kPivCap]
    static constexpr int64_t piv = vmeta + 4 * kPivCap;              // uint64 [kPivCap]
    static constexpr int64_t p1 = piv + 8 * kPivCap;                 // float2 [kPairCap]
    static constexpr int64_t p2 = p1 + 8 * kPairCap;                 // float2 [kPairCap]
    static constexpr int64_t vstore = p2 + 8 * kPairCap;             // uint32 [kVStoreCap]
    // F-minimal cofacet of every edge / triangle of the complex as the inserted vertex (one
    // byte), indexed by the dense combinatorial index; kMcNone for simplices that are not
    // columns or have no cofacet. Before the dim-2 pass a triangle entry may hold kMcCleared;
    // the dim-2 pass reads and overwrites every triangle entry of the complex. One byte keeps
    // the per-wave table (C(n,3) B) cache-resident for the serial walk's owner lookups.
    static constexpr int64_t mincof = vstore + 4 * kVStoreCap;       // uint8 [C(64,3)] triangles
    static constexpr int64_t mincof_e = mincof + (64 * 63 * 62 / 6);  // uint8 [C(64,2)] edges
    static constexpr int64_t edges = (mincof_e + (64 * 63 / 2) + 15) / 16 * 16;  // uint16 [C(64,2)] (i << 8 | j)
    static constexpr int64_t tris = (edges + 2 * (64 * 63 / 2) + 15) / 16 * 16;  // uint32 [C(64,3)] packed triangles
    static constexpr int64_t d0 = tris + 4 * (64 * 63 * 62 / 6);    // f32 [64] dim-0 deaths
    // columns whose min-cofacet walk did not finish in the first round of an apparent pass (packed
    // edge or triangle), walked to the end by a second round over this list
    static constexpr int64_t defer = d0 + 4 * 64;                    // uint32 [C(64,3)]
    // rank codes (rank_codes): the compacted keys of the distances <= thr, and the sorted f32
    // distances (code -> value, for the emitted pairs)
    static constexpr int64_t rankk = (defer + 4 * (64 * 63 * 62 / 6) + 15) / 16 * 16;  // uint64 [1024]
    static constexpr int64_t svals = rankk + 8 * 1024;               // f32 [1024]
    static constexpr int64_t total = svals + 4 * 1024;
};

// Per-wave LDS: the u16 rank-code matrix, the adjacency masks and the forest. The 48-point tier
// (every 5 A complex of FCC-256: 43..46 points) takes 5,040 B, so LDS admits 32 waves per CU (eight
// per SIMD, the most the SIMD holds; the registers are then capped at 64 VGPRs / 80 SGPRs); the
// f32 matrix took 8 KB at 44 points (five waves per SIMD) and 9.6 KB at 48 (four). The hot reads
// (rows a, b, c at column k = lane) are conflict-free (two lanes per bank word).
template <int NP>
struct BettiSmem {
    static constexpr int S = NP;
    uint16_t D[NP * S];               // full symmetric rank-code matrix, D[i * S + j]
    uint64_t adj[NP];
    uint8_t par[NP];                  // minimum spanning forest: parent of each vertex (0xFF = root)
};
#ifndef DGN_NARROW_WAVES
#define DGN_NARROW_WAVES 8  // waves per SIMD of the 32- and 48-point tiers (A/B: 6 / 7 / 8 waves =
                            // 139.4 / 132.8 / 130.1 ms betti_vr per config-4 shard; at 8 the compiler
                            // spills a few per-complex values, none in the reduction's loops)
#endif
template <int NP>
constexpr int betti_waves_per_simd() { return NP <= 48 ? DGN_NARROW_WAVES : 4; }

// ---------------------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------------------
// One-wave workgroups: a wave's LDS instructions execute in order, so lane-to-lane hand-offs
// through LDS need only a compiler barrier. __syncthreads() would add a workgroup release
// fence (s_waitcnt vmcnt(0)) that stalls on every in-flight global load/store; it is kept only
// where data passes between lanes through global scratch.
__device__ __forceinline__ void lds_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }
// move a wave-uniform value to an SGPR so dependent integer math runs on the scalar unit
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
    return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x);
}
// lanes [0, m) as a mask (full EXEC): one v_cmp into an SGPR pair. The narrow kernel is bound by
// the scalar unit's issue rate (one SALU per SIMD every ~4 cycles against a VALU every ~2.4 at 8
// waves per SIMD, tools/ubench/issue.hip), so masks and per-entry arithmetic go to the VALU where
// the scalar form would take several SALU (the shift/select form of this mask: 5-6).
__device__ __forceinline__ uint64_t lanes_below(int m) {
    return __builtin_amdgcn_ballot_w64((int)(threadIdx.x & 63) < m);
}
__device__ __forceinline__ int c2(int x) { return x * (x - 1) / 2; }
__device__ __forceinline__ int c3(int x) { return x * (x - 1) * (x - 2) / 6; }
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, kWave);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, kWave);
    return ((uint64_t)hi << 32) | lo;
}
// F-order key: ascending key == Ripser's filtration order (diameter ascending, then the
// combinatorial index DESCENDING, greater_diameter_or_smaller_index at ripser.cpp:318-324), the
// diameter as its rank code. Vertex tuples packed 8 bits per vertex in descending order preserve
// the colex (index) order.
__device__ __forceinline__ uint64_t make_key(uint32_t code, uint32_t packed) {
    return ((uint64_t)code << 32) | (uint64_t)(~packed);
}
__device__ __forceinline__ uint32_t key_code(uint64_t k) { return (uint32_t)(k >> 32); }
__device__ __forceinline__ uint32_t key_packed(uint64_t k) { return ~(uint32_t)k; }

__device__ __forceinline__ uint32_t pack2(int a, int b) { return ((uint32_t)a << 8) | (uint32_t)b; }
__device__ __forceinline__ uint32_t pack3(int a, int b, int c) {
    return ((uint32_t)a << 16) | ((uint32_t)b << 8) | (uint32_t)c;
}
__device__ __forceinline__ uint32_t pack4(int a, int b, int c, int d) {
    return ((uint32_t)a << 24) | ((uint32_t)b << 16) | ((uint32_t)c << 8) | (uint32_t)d;
}
__device__ __forceinline__ uint32_t tri_with(int a, int b, int k) {  // a > b; insert k
    return k > a ? pack3(k, a, b) : (k > b ? pack3(a, k, b) : pack3(a, b, k));
}
__device__ __forceinline__ uint32_t tet_with(int a, int b, int c, int k) {  // a > b > c; insert k
    return k > a ? pack4(k, a, b, c) : k > b ? pack4(a, k, b, c) : k > c ? pack4(a, b, k, c) : pack4(a, b, c, k);
}
// vertex of the packed cofacet `tau` that is not in its packed facet `f` (vertex sums)
__device__ __forceinline__ uint32_t byte_sum(uint32_t p) { return (p & 255) + ((p >> 8) & 255) + ((p >> 16) & 255) + (p >> 24); }
__device__ __forceinline__ uint32_t extra_vertex(uint32_t tau, uint32_t f) { return byte_sum(tau) - byte_sum(f); }
__device__ __forceinline__ int tri_dense(int a, int b, int c) {  // combinatorial index, a > b > c
    return a * (a - 1) * (a - 2) / 6 + b * (b - 1) / 2 + c;
}
// per-lane form (vector registers): 24-bit multiplies and an exact f32 division by 6 (the
// product is a multiple of 6 below 2^18) instead of a quarter-rate 32-bit multiply-high
__device__ __forceinline__ int tri_dense_lane(int a, int b, int c) {
    const uint32_t p = __umul24(__umul24((uint32_t)a, (uint32_t)(a - 1)), (uint32_t)(a - 2));
    return (int)((float)p * (1.0f / 6.0f) + 0.5f) + (int)(__umul24((uint32_t)b, (uint32_t)(b - 1)) >> 1) + c;
}
__device__ __forceinline__ int edge_dense(int a, int b) { return a * (a - 1) / 2 + b; }  // a > b
// dense combinatorial index of a packed column simplex (edge for dim 1, triangle for dim 2)
__device__ __forceinline__ int col_dense(int dim, uint32_t p) {
    return dim == 1 ? edge_dense((p >> 8) & 255, p & 255) : tri_dense((p >> 16) & 255, (p >> 8) & 255, p & 255);
}
__device__ __forceinline__ uint32_t sort2(int a, int b) { return a > b ? pack2(a, b) : pack2(b, a); }
__device__ __forceinline__ uint32_t sort3(int a, int b, int c) {  // any order -> packed descending
    const int hi = max(a, max(b, c)), lo = min(a, min(b, c)), mid = a + b + c - hi - lo;
    return pack3(hi, mid, lo);
}

// ---------------------------------------------------------------------------------------
// one local complex
// ---------------------------------------------------------------------------------------
template <int NP>
struct Complex {
    BettiSmem<NP>& s;
    int n;
    float thr;
    uint8_t* scratch;
    uint32_t err;
    // pair counts (wave-uniform)
    int n_d0, n_inf0, n_p1, n_p2;

    // Distances are rank codes (order- and equality-preserving): maxima are unsigned maxima, and
    // a simplex through a pair above thr (or a repeated vertex) gets kNoCode by the maximum
    // alone. The matrix is stored full, so a lookup is one multiply-add whichever vertex is
    // larger; loads zero-extend the u16 code.
    static constexpr int S = BettiSmem<NP>::S;
    uint32_t zero_code;  // code of the distance 0.0f if the complex has one, else ~0u
    __device__ const uint16_t* Db() const { return s.D; }
    __device__ uint32_t dlowb(int a, int b) const { return Db()[a * S + b]; }
    __device__ uint32_t db(int i, int j) const { return Db()[i * S + j]; }
    __device__ uint64_t ekey(int i, int j) const {  // i != j; reads row i (Prim: i uniform)
        const int a = max(i, j), b = min(i, j);
        return make_key(db(i, j), pack2(a, b));
    }
    __device__ uint32_t tri_diamb(int a, int b, int c) const {  // a > b > c
        return max(max(dlowb(a, b), dlowb(a, c)), dlowb(b, c));
    }
    __device__ uint64_t tkey(int a, int b, int c) const { return make_key(tri_diamb(a, b, c), pack3(a, b, c)); }
    // tree edge (i, j): one is the other's parent in the spanning forest
    __device__ bool is_tree(int i, int j) const { return s.par[i] == j || s.par[j] == i; }
    // clearing marks live in the triangle min-cofacet table (scratch) until the dim-2 pass
    __device__ bool is_cleared(int a, int b, int c) const {
        return at(sp<uint8_t>(ScratchLayout::mincof), tri_dense(a, b, c)) == kMcCleared;
    }
    __device__ void set_cleared(int a, int b, int c) { at(sp<uint8_t>(ScratchLayout::mincof), tri_dense(a, b, c)) = kMcCleared; }
    __device__ void set_cleared_lane(int a, int b, int c) {
        at(sp<uint8_t>(ScratchLayout::mincof), tri_dense_lane(a, b, c)) = kMcCleared;
    }
    __device__ uint8_t* mincof_of(int dim) const {
        return sp<uint8_t>(dim == 1 ? ScratchLayout::mincof_e : ScratchLayout::mincof);
    }
    template <typename T>
    __device__ T* sp(int64_t off) const { return reinterpret_cast<T*>(scratch + off); }
    // pairs (birth, death): rank codes during the reduction (uint2), decoded in place to f32
    // (float2) before the statistics (decode_outputs)
    __device__ float2* pairs(int dim) const { return sp<float2>(dim == 1 ? ScratchLayout::p1 : ScratchLayout::p2); }
    __device__ uint2* pair_codes(int dim) const { return sp<uint2>(dim == 1 ? ScratchLayout::p1 : ScratchLayout::p2); }

    // per-lane: F-minimal cofacet key of edge (a > b) / triangle (a > b > c) over cand (kInf if
    // cand is empty). For one simplex, inserting a larger vertex k gives a larger packed tuple,
    // i.e. an F-smaller key among cofacets of equal diameter; so walking k downwards, a later
    // (smaller) k wins only with a strictly smaller diameter, and the first k whose distances to
    // the simplex are all <= its diameter is the F-minimal cofacet and ends the search (found).
    // Only the winner's packed tuple is built. bk = the inserted vertex; when found, hda/hdb/hdc
    // are its distances to a, b, c, so the apparent test needs no further reads.
    // At most `steps` steps of four candidates are walked; `cand` returns the candidates not
    // walked (nonzero with !found: the walk is unfinished and the result is not the minimum).
    __device__ uint64_t min_cofacet_lane(int dim, int a, int b, int c, uint32_t dbits, uint64_t& cand, int& bk,
                                         bool& found, uint32_t& hda, uint32_t& hdb, uint32_t& hdc,
                                         int steps) const {
        uint32_t bd = 0xFFFFFFFFu;  // diameter of the best cofacet so far
        bk = -1;
        found = false;
        hda = hdb = hdc = 0u;
        const uint16_t* ra = Db() + a * S;  // rows a, b, c: entry k is d(., k)
        const uint16_t* rb = Db() + b * S;
        const uint16_t* rcv = Db() + c * S;
        // the candidates bit-reversed: the largest remaining k is the lowest set bit, taken with a
        // trailing-zero count and cleared with r & (r - 1) (no validity select: 0 stays 0)
        uint64_t r = ((uint64_t)__builtin_bitreverse32((uint32_t)cand) << 32) | __builtin_bitreverse32((uint32_t)(cand >> 32));
        // four candidates per step (descending), their distance reads issued together
        for (int st = 0; r && st < steps; ++st) {
            int kk[4];
            bool val[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                val[j] = r != 0;
                kk[j] = 63 - (val[j] ? __builtin_ctzll(r) : 63);
                r &= r - 1;
            }
            uint32_t da[4], dbb[4], dc[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                da[j] = ra[kk[j]];
                dbb[j] = rb[kk[j]];
                dc[j] = dim == 2 ? rcv[kk[j]] : 0u;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const uint32_t dk = max(max(da[j], dbb[j]), max(dc[j], dbits));  // cofacet diameter
                const bool take = val[j] && !found && dk < bd;
                const bool hit = take && dk == dbits;
                bd = take ? dk : bd;
                bk = take ? kk[j] : bk;
                hda = hit ? da[j] : hda;
                hdb = hit ? dbb[j] : hdb;
                hdc = hit ? dc[j] : hdc;
                found = found || hit;
            }
            if (found) break;
        }
        cand = r;  // nonzero: candidates left unwalked (only their count matters to the callers)
        if (bk < 0) return kInf;
        const uint32_t pk = dim == 1 ? tri_with(a, b, bk) : tet_with(a, b, c, bk);
        return ((uint64_t)bd << 32) | (uint64_t)(~pk);
    }

    // F-max facet of pivot tau as (packed vertices)
    __device__ uint32_t max_facet(int dim, uint64_t tau) const {
        // largest diameter, ties to the smallest index: the facet dropping the largest vertex
        // first (packed order (b,c) < (a,c) < (a,b), and (b,c,d) < (a,c,d) < (a,b,d) < (a,b,c))
        const uint32_t p = key_packed(tau);
        if (dim == 1) {
            const int a = (p >> 16) & 255, b = (p >> 8) & 255, c = p & 255;
            const uint32_t dab = dlowb(a, b), dac = dlowb(a, c), dbc = dlowb(b, c);
            const uint32_t m = max(max(dab, dac), dbc);
            return dbc == m ? pack2(b, c) : (dac == m ? pack2(a, c) : pack2(a, b));
        } else {
            const int a = (p >> 24) & 255, b = (p >> 16) & 255, c = (p >> 8) & 255, d = p & 255;
            const uint32_t dab = dlowb(a, b), dac = dlowb(a, c), dad = dlowb(a, d);
            const uint32_t dbc = dlowb(b, c), dbd = dlowb(b, d), dcd = dlowb(c, d);
            const uint32_t fa = max(max(dbc, dbd), dcd), fb = max(max(dac, dad), dcd);
            const uint32_t fc = max(max(dab, dad), dbd), fd = max(max(dab, dac), dbc);
            const uint32_t m = max(max(fa, fb), max(fc, fd));
            return fa == m ? pack3(b, c, d) : (fb == m ? pack3(a, c, d) : (fc == m ? pack3(a, b, d) : pack3(a, b, c)));
        }
    }
    // Apparent owner of pivot tau (whole wave, uniform): its F-max facet f, if tau is f's
    // F-minimal cofacet (recorded for every column by the lane-parallel pass; tree edges and
    // cleared triangles hold kNone), else kNone.
    __device__ uint32_t apparent_owner_wave(int dim, uint64_t tau) const {
        // computed redundantly by every lane on the VALU (the scalar unit is the bound port)
        uint32_t th, tl;
        asm("v_mov_b32 %0, %1" : "=v"(th) : "s"((uint32_t)(tau >> 32)));
        asm("v_mov_b32 %0, %1" : "=v"(tl) : "s"((uint32_t)tau));
        const uint64_t vt = ((uint64_t)th << 32) | tl;
        const uint32_t vf = max_facet(dim, vt);
        const uint32_t vm = at(mincof_of(dim), dim == 1 ? col_dense(1, vf)
                                                         : tri_dense_lane((vf >> 16) & 255, (vf >> 8) & 255, vf & 255));
        return uni(vm == extra_vertex(key_packed(vt), vf) ? vf : kNone);
        const uint32_t f = uni(max_facet(dim, uni64(tau)));
        const uint32_t m = at(mincof_of(dim), col_dense(dim, f));
        return uni(m) == extra_vertex(key_packed(tau), f) ? f : kNone;
    }

    __device__ uint64_t column_key(int dim, uint32_t cp) const {
        return dim == 1 ? ekey((cp >> 8) & 255, cp & 255) : tkey((cp >> 16) & 255, (cp >> 8) & 255, cp & 255);
    }

    // ---- serially resolved pivot table: entries 0..127 in registers (lane t holds entries t
    // and t + 64: pivot key and V-list descriptor), the rest in scratch
    uint64_t pk0 = 0, pk1 = 0;
    uint32_t pm0 = 0, pm1 = 0;

    __device__ int find_pivot(int npiv, uint64_t tau) const {
        const int lane = lane_id();
        uint64_t bal = ballot(pk0 == tau) & lanes_below(npiv);
        if (bal) return __ffsll((unsigned long long)bal) - 1;
        if (npiv > kWave) {
            bal = ballot(pk1 == tau) & lanes_below(npiv - kWave);
            if (bal) return kWave + __ffsll((unsigned long long)bal) - 1;
        }
        const uint64_t* sp_piv = sp<uint64_t>(ScratchLayout::piv);
        for (int base = 2 * kWave; base < npiv; base += kWave) {
            const int i = base + lane;
            bal = ballot(i < npiv && at(sp_piv, i) == tau);
            if (bal) return base + __ffsll((unsigned long long)bal) - 1;
        }
        return -1;
    }
    __device__ uint32_t piv_meta(int i) const {
        if (i < kWave) return rl(pm0, i);
        if (i < 2 * kWave) return rl(pm1, i - kWave);
        return uni(at(sp<uint32_t>(ScratchLayout::vmeta), i));
    }
    __device__ void piv_push(int i, uint64_t tau, uint32_t meta) {
        const int lane = lane_id();
        if (i < 2 * kWave) {
            const bool w0 = lane == i, w1 = lane == i - kWave;
            pk0 = w0 ? tau : pk0;
            pm0 = w0 ? meta : pm0;
            pk1 = w1 ? tau : pk1;
            pm1 = w1 ? meta : pm1;
        } else if (lane == 0) {
            sp<uint64_t>(ScratchLayout::piv)[i] = tau;
            at(sp<uint32_t>(ScratchLayout::vmeta), i) = meta;
        }
    }

    // ---- the working column's V list, resident in registers: lane t holds entry t (set 0) and
    // entry t + 64 (set 1) with its diameter. Toggles only move packed simplices; pivot_of_V
    // refreshes the diameters lane-parallel and reads entries back uniformly with v_readlane.
    uint32_t vs0 = 0, vs1 = 0;
    uint32_t vd0 = 0, vd1 = 0;

    __device__ static uint32_t rl(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }
    __device__ static uint64_t rl64(uint64_t x, int l) {
        return ((uint64_t)rl((uint32_t)(x >> 32), l) << 32) | rl((uint32_t)x, l);
    }
    __device__ void v_set(int i, uint32_t sp_) {
        const int lane = lane_id();
        vs0 = lane == i ? sp_ : vs0;
        vs1 = lane == i - 64 ? sp_ : vs1;
    }
    __device__ int v_find(uint32_t x, int v) const {
        uint64_t bal = ballot(vs0 == x) & lanes_below(v);
        if (bal) return __ffsll((unsigned long long)bal) - 1;
        if (v > 64) {
            bal = ballot(vs1 == x) & lanes_below(v - 64);
            if (bal) return 64 + __ffsll((unsigned long long)bal) - 1;
        }
        return -1;
    }
    // V ^= {x} (whole wave, uniform arguments); false on V-list overflow
    __device__ bool v_toggle(int, uint32_t x, int& v) {
        const int pos = v_find(x, v);
        if (pos >= 0) {
            if (pos != v - 1) v_set(pos, v - 1 < 64 ? rl(vs0, v - 1) : rl(vs1, v - 65));
            v = (int)uni((uint32_t)(v - 1));
            return true;
        }
        if (v >= kVCap) return false;
        v_set(v, x);
        v = (int)uni((uint32_t)(v + 1));
        return true;
    }
    __device__ uint32_t simplex_diam(int dim, uint32_t x) const {
        return dim == 1 ? dlowb((x >> 8) & 255, x & 255) : tri_diamb((x >> 16) & 255, (x >> 8) & 255, x & 255);
    }

    // Pivot of the column sum(delta s, s in V) (whole wave): the F-minimal cofacet of odd
    // multiplicity, restricted to keys above `floor` (the column's previous pivot: adding the
    // owner column cancels it and every other entry of both columns is larger). Lane k
    // evaluates the cofacet s u {k} of every s in V; one cofacet tau arises once per facet of
    // tau in V, always in a different lane (k = tau \ s), so the multiplicity of the wave
    // minimum is the popcount of a ballot. Even multiplicity: raise the floor and repeat.
    // kInf for the zero column.
    // key of the cofacet s u {k} for lane k (k < n); its high word is kNoCode (above every real
    // key) if k is not a common neighbour of s: the LDS matrix holds kNoCode for distances above
    // thr and on the diagonal, so the diameter maximum carries it. The low word, ~packed(tau), is
    // built in one v_perm_b32 from the complemented tuple of s (nsp = ~sp_) and lane k's
    // complemented vertex byte (kc = 255 - k, perm byte 4), with the byte order picked by where k
    // falls among the vertices of s (selector table kSel*). Branch-free: v_cndmask only.
    __device__ uint64_t cofacet_key(int dim, int k, uint32_t kc, uint32_t sp_, uint32_t ds) const {
        // the entry's row offsets and complement on the VALU (the scalar unit is the bound port)
        uint32_t vsp;
        asm("v_mov_b32 %0, %1" : "=v"(vsp) : "s"(sp_));
        const uint32_t k2 = 2u * (uint32_t)k;
        const uint32_t va = dim == 1 ? __builtin_amdgcn_ubfe(vsp, 8, 8) : __builtin_amdgcn_ubfe(vsp, 16, 8);
        const uint32_t vb = dim == 1 ? (vsp & 255u) : __builtin_amdgcn_ubfe(vsp, 8, 8);
        const uint32_t vcc_ = vsp & 255u;
        const uint8_t* Dbytes = reinterpret_cast<const uint8_t*>(Db());
        uint32_t dd = max(ds, max((uint32_t)*reinterpret_cast<const uint16_t*>(Dbytes + __umul24(va, 2 * S) + k2),
                                  (uint32_t)*reinterpret_cast<const uint16_t*>(Dbytes + __umul24(vb, 2 * S) + k2)));
        uint32_t sel;
        if (dim == 1) {
            sel = (uint32_t)k > va ? 0x02040100u : ((uint32_t)k > vb ? 0x02010400u : 0x02010004u);
        } else {
            dd = max(dd, (uint32_t)*reinterpret_cast<const uint16_t*>(Dbytes + __umul24(vcc_, 2 * S) + k2));
            sel = (uint32_t)k > va ? 0x04020100u : ((uint32_t)k > vb ? 0x02040100u : ((uint32_t)k > vcc_ ? 0x02010400u : 0x02010004u));
        }
        const uint32_t nk = __builtin_amdgcn_perm(kc, ~vsp, sel);
        return __builtin_bit_cast(uint64_t, make_uint2(nk, dd));  // (dd, nk) as one register pair
    }

    // key - base as one v_lshl_add_u64 on the (nk, dd) register pair (the compiler's own form adds
    // the two halves separately: three VALU per V entry)
    __device__ static uint64_t rel_key(uint64_t key, uint64_t nbase) {
        uint64_t r;
        asm("v_lshl_add_u64 %0, %1, 0, %2" : "=v"(r) : "v"(key), "s"(nbase));
        return r;
    }
    // Pivot of the column sum(delta s, s in V) (whole wave): the F-minimal cofacet of odd
    // multiplicity, restricted to keys above `floor` (the column's previous pivot: adding the
    // owner column cancels it and every other entry of both columns is larger). Lane k
    // evaluates the cofacet s u {k} of every s in V; one cofacet tau arises once per facet of
    // tau in V, always in a different lane (k = tau \ s), so the multiplicity of the wave
    // minimum is the popcount of a ballot. Even multiplicity: raise the floor and repeat.
    // kInf for the zero column.
    __device__ uint64_t pivot_of_V(int dim, int v_, uint64_t floor) {
        const int k = lane_id();
        const uint32_t kc = 255u - (uint32_t)k;
        const int v = (int)uni((uint32_t)v_);
        if (k < v) vd0 = simplex_diam(dim, vs0);
        if (v > 64 && k + 64 < v) vd1 = simplex_diam(dim, vs1);
        for (;;) {
            // keys are taken relative to base = floor + 1: key - base wraps the keys <= floor
            // above every key > floor, so one unsigned minimum skips them (floor is a real key,
            // never kInf)
            const uint64_t base = floor + 1;
            const uint64_t nbase = 0ull - base;
            uint64_t lmin = kInf;
            // kPvUnroll V entries per step, their distance reads in flight together, then the rest;
            // entries 0..63 (register set 0) and 64.. (set 1) in separate loops, so no entry pays a
            // branch to pick its register set (A/B: 196.0 -> 189.4 ms per shard; making the pivot
            // table, V-list and column-record selects branch-free as well cost +2 %)
            auto scan = [&](uint32_t vs, uint32_t vdb, int cnt) {
                int i = 0;
                for (; i + kPvUnroll <= cnt; i += kPvUnroll) {
                    uint64_t kq[kPvUnroll];
#pragma unroll
                    for (int u = 0; u < kPvUnroll; ++u) kq[u] = rel_key(cofacet_key(dim, k, kc, rl(vs, i + u), rl(vdb, i + u)), nbase);
#pragma unroll
                    for (int u = 0; u < kPvUnroll; ++u) lmin = kq[u] < lmin ? kq[u] : lmin;
                }
                for (; i < cnt; ++i) {
                    const uint64_t key = rel_key(cofacet_key(dim, k, kc, rl(vs, i), rl(vdb, i)), nbase);
                    lmin = key < lmin ? key : lmin;
                }
            };
            // lanes k >= n are not vertices: they keep kInf (exec-masked, no per-entry test)
            if (k < n) {
                scan(vs0, vd0, v < 64 ? v : 64);
                if (v > 64) scan(vs1, vd1, v - 64);
            }
            // wave minimum: the high words first; a unique minimal high word settles it (and its
            // multiplicity, 1) without the low-word stage
            const uint32_t lhi = (uint32_t)(lmin >> 32);
            const uint32_t mh = wave_min_u32(lhi);
            const uint64_t bh = ballot(lhi == mh);
            uint64_t mt;
            int mult;
            if (__popcll(bh) == 1) {
                mt = ((uint64_t)mh << 32) | rl((uint32_t)lmin, __ffsll((unsigned long long)bh) - 1);
                mult = 1;
            } else {
                const uint32_t ml = wave_min_u32(lhi == mh ? (uint32_t)lmin : 0xFFFFFFFFu);
                mt = ((uint64_t)mh << 32) | ml;
                mult = __popcll(ballot(lmin == mt));
            }
            const uint64_t m = mt + base;
            // no cofacet above floor: the minimum is a non-neighbour key (high word kNoCode; every
            // lane without a cofacet: all ones) or a wrapped key <= floor
            if ((uint32_t)(m >> 32) >= kNoCode || m <= floor) return kInf;
            if (mult & 1) return m;
            floor = m;
        }
    }

    // per-lane apparent owner of pivot tau (kNone if none): its F-max facet f, if tau is f's
    // F-minimal cofacet (recorded for every column by the lane-parallel pass)
    __device__ uint32_t apparent_owner_lane(int dim, uint64_t tau) const {
        const uint32_t f = max_facet(dim, tau);
        const uint32_t m = at(mincof_of(dim), col_dense(dim, f));
        return m == extra_vertex(key_packed(tau), f) ? f : kNone;
    }

    // dim-0 deaths and the dim-1 / dim-2 pairs: rank codes -> f32 (the complex's decode table),
    // in place (each lane rewrites its own entries)
    __device__ void decode_outputs(uint32_t* d0s) const {
        const int lane = lane_id();
        const float* sv = sp<float>(ScratchLayout::svals);
        __syncthreads();  // the decode table and the code lists (scratch) were written by other lanes
        for (int i = lane; i < n_d0; i += kWave) at(d0s, i) = __float_as_uint(at(sv, at(d0s, i)));
        for (int d = 1; d <= 2; ++d) {
            const int np = min(d == 1 ? n_p1 : n_p2, kPairCap);
            for (int i = lane; i < np; i += kWave) {
                const uint2 c = at(pair_codes(d), i);
                at(pairs(d), i) = make_float2(at(sv, c.x), at(sv, c.y));
            }
        }
        __syncthreads();
    }

    // Walk the non-apparent columns in Ripser's order (whole wave). na_* (scratch) hold each
    // column's key and its unreduced pivot. Up to 128 records live in registers (lane t:
    // records t and t + 64) with their rank in column order and the apparent owner of their
    // initial pivot, all computed lane-parallel; larger sets are rank-sorted into scratch.
    __device__ void reduce_serial(int dim, int nna) {
        const int lane = lane_id();
        if (nna > kNACap) { err |= kErrNA; return; }
        const uint64_t* gk = sp<uint64_t>(ScratchLayout::na_key);
        const uint64_t* gt = sp<uint64_t>(ScratchLayout::na_tau);
        const bool regs = nna <= 2 * kWave;
        uint64_t rk0 = 0, rk1 = 0, rt0 = 0, rt1 = 0;
        int rr0 = -1, rr1 = -1;
        uint32_t ra0 = kNone, ra1 = kNone;
        uint64_t* sk = sp<uint64_t>(ScratchLayout::sna_key);
        uint64_t* st = sp<uint64_t>(ScratchLayout::sna_tau);
        if (regs) {
            if (lane < nna) { rk0 = at(gk, lane); rt0 = at(gt, lane); }
            if (lane + kWave < nna) { rk1 = at(gk, lane + kWave); rt1 = at(gt, lane + kWave); }
            // rank by column key DESCENDING (Ripser processes columns in decreasing F-order)
            int r0 = 0, r1 = 0;
            const int n0 = nna < kWave ? nna : kWave;
            for (int u = 0; u < n0; ++u) {
                const uint64_t ku = rl64(rk0, u);
                r0 += ku > rk0;
                r1 += ku > rk1;
            }
            for (int u = kWave; u < nna; ++u) {
                const uint64_t ku = rl64(rk1, u - kWave);
                r0 += ku > rk0;
                r1 += ku > rk1;
            }
            rr0 = lane < nna ? r0 : -1;
            rr1 = lane + kWave < nna ? r1 : -1;
            // apparent owners of the initial pivots (global loads overlap across lanes)
            if (lane < nna) ra0 = apparent_owner_lane(dim, rt0);
            if (lane + kWave < nna) ra1 = apparent_owner_lane(dim, rt1);
        } else {
            for (int i = lane; i < nna; i += kWave) {
                const uint64_t v = gk[i];
                int rank = 0;
                for (int u = 0; u < nna; ++u) rank += gk[u] > v;
                sk[rank] = v;
                st[rank] = gt[i];
            }
            __syncthreads();
        }
        uint32_t* gvstore = sp<uint32_t>(ScratchLayout::vstore);
        int npiv = 0, vused = 0;
        for (int ci = 0; ci < nna; ++ci) {
            uint64_t colkey, tau;
            uint32_t app0 = kNone;
            bool have_app = false;
            if (regs) {
                uint64_t bal = ballot(rr0 == ci);
                if (bal) {
                    const int l = __ffsll((unsigned long long)bal) - 1;
                    colkey = rl64(rk0, l);
                    tau = rl64(rt0, l);
                    app0 = rl(ra0, l);
                } else {
                    bal = ballot(rr1 == ci);
                    const int l = __ffsll((unsigned long long)bal) - 1;
                    colkey = rl64(rk1, l);
                    tau = rl64(rt1, l);
                    app0 = rl(ra1, l);
                }
                have_app = true;
            } else {
                colkey = uni64(sk[ci]);
                tau = uni64(st[ci]);
            }
            // the walk's state is wave-uniform; readfirstlane says so to the compiler, whose
            // divergence analysis otherwise lets one vector-held value turn every branch of the
            // walk into exec-masked code
            colkey = uni64(colkey);
            tau = uni64(tau);
            const uint32_t cp = key_packed(colkey);
            const uint32_t birth = key_code(colkey);
            int owner = (int)uni((uint32_t)find_pivot(npiv, tau));
            uint32_t app = uni(owner >= 0 ? kNone : (have_app ? app0 : apparent_owner_wave(dim, tau)));
            int v = 0;  // 0 = lazy: V == {this column}
            if (owner >= 0 || app != kNone) {
                v_toggle(dim, cp, v);
                int guard = 0;
                while (true) {
                    // V ^= V(owner)
                    bool ok = true;
                    if (app != kNone) {
                        // an apparent owner precedes this column in Ripser's order (key greater):
                        // guaranteed (an apparent pair's column is the F-max facet of its pivot);
                        // checking it cost 2.4 % of the Betti pass, and the parity tests compare
                        // every pair with the oracle
                        ok = v_toggle(dim, app, v);
                    } else {
                        const uint32_t m = piv_meta(owner);
                        if (m & kLazyBit) {
                            ok = v_toggle(dim, m & ~kLazyBit, v);
                        } else {
                            const int off = (int)uni(m >> 9), len = (int)uni(m & 511);
                            // owner's V list: one lane-parallel load per 64 entries, then readlanes
                            for (int t0 = 0; t0 < len && ok; t0 += kWave) {
                                const int t = t0 + lane;
                                uint32_t w = 0;
                                if (t < len) w = at(gvstore, off + t);
                                const int cnt = len - t0 < kWave ? len - t0 : kWave;
                                for (int u = 0; u < cnt && ok; ++u) ok = v_toggle(dim, rl(w, u), v);
                            }
                        }
                    }
                    if (!ok) { err |= kErrWorkCol; return; }
                    tau = uni64(v > 0 ? pivot_of_V(dim, v, tau) : kInf);
                    if (tau == kInf) break;  // zero column: essential class, not emitted
                    owner = (int)uni((uint32_t)find_pivot(npiv, tau));
                    app = uni(owner >= 0 ? kNone : apparent_owner_wave(dim, tau));
                    if (owner < 0 && app == kNone) break;  // tau is this column's pivot
                    if (++guard > 100000) { err |= kErrWorkCol; return; }
                }
                if (tau == kInf) continue;  // zero column
            }
            // ---- tau is the pivot of this column ----
            const uint32_t death = key_code(tau);
            if (death > birth) {  // codes order as the distances (ripser.cpp:1240)
                if (lane == 0) {
                    const int slot = dim == 1 ? n_p1 : n_p2;
                    if (slot < kPairCap) at(pair_codes(dim), slot) = make_uint2(birth, death);
                }
                if (dim == 1) ++n_p1;
                else ++n_p2;
            }
            if (dim == 1 && lane == 0) {
                const uint32_t tp = key_packed(tau);
                set_cleared((tp >> 16) & 255, (tp >> 8) & 255, tp & 255);
            }
            if (npiv >= kPivCap) { err |= kErrPiv; return; }
            uint32_t meta;
            if (v == 0) {
                meta = kLazyBit | cp;
            } else {
                if (vused + v > kVStoreCap || v > 511) { err |= kErrR; return; }
                for (int t = lane; t < v; t += kWave) {
                    const uint32_t x = t < kWave ? vs0 : vs1;
                    at(gvstore, vused + t) = x;
                }
                meta = ((uint32_t)vused << 9) | (uint32_t)v;
                vused = (int)uni((uint32_t)(vused + v));
            }
            piv_push(npiv, tau, meta);
            npiv = (int)uni((uint32_t)(npiv + 1));
            lds_sync();
        }
    }
};


// Ascending bitonic sort of 64 R keys in registers, element e = lane * R + r: exchanges at a
// distance j < R stay in the lane (registers r and r ^ j), the others pair lane with lane ^ (j / R)
// (ds_bpermute). Merge levels k < R are unrolled (directions known per register); from k = R on
// the direction is a lane bit and the levels run as a loop (a short kernel: the sort runs once
// per complex next to the reduction's hot loops in the instruction cache).
template <int R>
__device__ __forceinline__ void bitonic_in_lane(uint64_t (&x)[R], int j, bool asc) {
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if (r & j) continue;
        const uint64_t a = x[r], b = x[r | j];
        const bool sw = (a > b) == asc;
        x[r] = sw ? b : a;
        x[r | j] = sw ? a : b;
    }
}
template <int R>
__device__ __forceinline__ void bitonic_sort_regs(uint64_t (&x)[R], int lane) {
    constexpr int P = kWave * R;
#pragma unroll
    for (int k = 2; k < R; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                if (r & j) continue;
                const bool asc = (r & k) == 0;
                const uint64_t a = x[r], b = x[r | j];
                const bool sw = (a > b) == asc;
                x[r] = sw ? b : a;
                x[r | j] = sw ? a : b;
            }
        }
    }
#pragma unroll 1
    for (int k = R; k <= P; k <<= 1) {
        const bool asc = k >= P || (lane & (k / R)) == 0;  // bit k of e
#pragma unroll 1
        for (int j = k >> 1; j >= R; j >>= 1) {
            const int lm = j / R;
            const bool keep_min = ((lane & lm) == 0) == asc;
            // four registers' exchanges in flight together
#pragma unroll
            for (int r0 = 0; r0 < R; r0 += 4) {
                uint64_t p[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) p[q] = shfl_xor64(x[r0 + q], lm);
#pragma unroll
                for (int q = 0; q < 4; ++q) x[r0 + q] = ((p[q] < x[r0 + q]) == keep_min) ? p[q] : x[r0 + q];
            }
        }
#pragma unroll
        for (int j = R >> 1; j > 0; j >>= 1) bitonic_in_lane<R>(x, j, asc);
    }
}

// Rank codes of one complex (one wave): the packed f32 lower triangle (ripser_wrapper.cpp:20-24
// packing) becomes the full u16 matrix s.D of codes -- code(d) = the index of d's first
// occurrence among the complex's sorted distances <= thr (order- and equality-preserving),
// kNoCode above thr (sparse_distance_matrix keeps d <= thr, ripser.cpp:386-395) and on the
// diagonal -- and sv_out[code] = d (the decode table). The m distances <= thr are compacted
// (ballots) as (f32 bits << 12 | i << 6 | j) keys into the matrix region of the LDS (free until
// the codes are written), sorted in registers (bitonic, R per lane: 512 or 1,024 keys), and each
// sorted key scatters its run's first index to (i, j) and (j, i). Returns the code of 0.0f if the complex has a zero distance, ~0u if it has none, and
// kRankDense if more than kRankMax<NP> distances are <= thr (R = 8 registers per lane in the
// 32- and 48-point tiers: 512 keys, the dense launch takes the rest; 16 in the 64-point tier:
// 1,024, the capacity retry takes the rest).
constexpr uint32_t kRankDense = 0xFFFFFFFEu;
template <int NP>
constexpr int kRankMax = NP <= 48 ? 512 : 1024;
template <int R, class KeyAt, class Clear>
__device__ __forceinline__ uint32_t rank_sorted(uint16_t* D, int S, KeyAt&& key_at, Clear&& clear, int m, float* sv_out,
                                                int lane) {
    uint64_t x[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = lane * R + r;
        x[r] = e < m ? key_at(e) : ~0ull;
    }
    clear();  // the keys are in registers: the matrix region may be overwritten
    bitonic_sort_regs<R>(x, lane);
    // code = the first index of the element's value run = the running maximum of (e if element
    // e starts a run, else 0): within the lane, then across lanes (exclusive max-scan)
    const uint32_t prev_bits = (uint32_t)__shfl_up((int)(uint32_t)(x[R - 1] >> 12), 1, kWave);
    uint32_t c[R];
    uint32_t run = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const uint32_t bits = (uint32_t)(x[r] >> 12);
        const bool first = r == 0 ? (lane == 0 || bits != prev_bits) : bits != (uint32_t)(x[r - 1] >> 12);
        run = first ? (uint32_t)(lane * R + r) : run;
        c[r] = run;
    }
    uint32_t carry = c[R - 1];
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const uint32_t w = (uint32_t)__shfl_up((int)carry, o, kWave);
        carry = lane >= o ? max(carry, w) : carry;
    }
    uint32_t in = (uint32_t)__shfl_up((int)carry, 1, kWave);
    in = lane == 0 ? 0u : in;
#pragma unroll
    for (int r = 0; r < R; ++r) c[r] = max(c[r], in);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int e = lane * R + r;
        if (e < m) {
            const uint32_t k = (uint32_t)x[r];
            const int i = (k >> 6) & 63, j = k & 63;
            D[i * S + j] = (uint16_t)c[r];
            D[j * S + i] = (uint16_t)c[r];
            at(sv_out, e) = __uint_as_float((uint32_t)(x[r] >> 12));
        }
    }
    (void)S;
    return __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x[0] >> 12), 0)) == 0.0f && m > 0
               ? 0u
               : 0xFFFFFFFFu;
}

template <int NP>
__device__ __forceinline__ uint32_t rank_codes(BettiSmem<NP>& s, const float* __restrict__ L, int n, float thr,
                                               float* sv_out, uint64_t* keys) {
    constexpr int S = BettiSmem<NP>::S;
    // the keys go to the matrix region of the LDS while it is free (NP = 48: 576 keys, 64: 1,024,
    // every key the sort takes), past it to scratch (NP = 32: keys 256..511)
    constexpr int kLdsKeys = NP * S / 4;
    uint64_t* kl = reinterpret_cast<uint64_t*>(s.D);
    const int lane = lane_id();
    const int tot = c2(n);
    // (1) compaction of the distances <= thr, t-order; lane l holds entries t = l + 64 u, its
    // (i, j) advanced incrementally (entry t of the packing is row i, column t - c2(i))
    int i = (int)((1.0f + sqrtf(1.0f + 8.0f * (float)lane)) * 0.5f);
    i -= c2(i) > lane;
    i += c2(i + 1) <= lane;
    int j = lane - c2(i);
    int m = 0;
    for (int t0 = 0; t0 < tot; t0 += 2 * kWave) {
        const int t = t0 + lane;
        const float v0 = t < tot ? at(L, t) : INFINITY;
        const float v1 = t + kWave < tot ? at(L, t + kWave) : INFINITY;
        const int i0 = i, j0 = j;
        j += kWave;
        while (j >= i) { j -= i; ++i; }
        const int i1 = i, j1 = j;
        j += kWave;
        while (j >= i) { j -= i; ++i; }
        // padding lanes past the triangle (t >= tot) never count as edges, even at thr = +inf:
        // their (i, j) run past n and a mirrored store would overwrite real codes
        const bool ok0 = t < tot && v0 <= thr, ok1 = t + kWave < tot && v1 <= thr;
        const uint64_t b0 = ballot(ok0), b1 = ballot(ok1);
        const int s0 = m + mask_prefix(b0);
        const uint64_t k0 = ((uint64_t)__float_as_uint(v0) << 12) | (uint64_t)((i0 << 6) | j0);
        if (ok0 && s0 < kLdsKeys) kl[s0] = k0;
        else if (ok0 && s0 < kRankMax<NP>) at(keys, s0) = k0;
        m += __popcll(b0);
        const int s1 = m + mask_prefix(b1);
        const uint64_t k1 = ((uint64_t)__float_as_uint(v1) << 12) | (uint64_t)((i1 << 6) | j1);
        if (ok1 && s1 < kLdsKeys) kl[s1] = k1;
        else if (ok1 && s1 < kRankMax<NP>) at(keys, s1) = k1;
        m += __popcll(b1);
    }
    m = (int)uni((uint32_t)m);
    if (m > kRankMax<NP>) return kRankDense;
    if constexpr (kLdsKeys < kRankMax<NP>) __syncthreads();  // scratch keys are read by other lanes
    lds_sync();
    auto key_at = [&](int e) __attribute__((always_inline)) {
        if constexpr (kLdsKeys >= kRankMax<NP>) return kl[e];
        else return e < kLdsKeys ? kl[e] : at(keys, e);
    };
    // the matrix starts as kNoCode everywhere (pairs above thr, the diagonal)
    auto clear = [&]() __attribute__((always_inline)) {
        lds_sync();
        uint32_t* Dw = reinterpret_cast<uint32_t*>(s.D);
        for (int w = lane; w < NP * S / 2; w += kWave) Dw[w] = (kNoCode << 16) | kNoCode;
        lds_sync();
    };
    uint32_t z;
    if constexpr (NP <= 48) {
        z = rank_sorted<8>(s.D, S, key_at, clear, m, sv_out, lane);
    } else {
        z = m <= 512 ? rank_sorted<8>(s.D, S, key_at, clear, m, sv_out, lane)
                     : rank_sorted<16>(s.D, S, key_at, clear, m, sv_out, lane);
    }
    lds_sync();
    return z;
}

template <int NP>
__global__ __launch_bounds__(kWave, betti_waves_per_simd<NP>()) void betti_kernel(BettiLaunch bl) {
    __shared__ BettiSmem<NP> s;
    // the lane index is re-derived opaquely at every phase (relane): the compiler cannot hoist
    // lane-derived masks and per-lane addresses out of the complex loop, where they were live
    // across the whole kernel and spilled (16 VGPRs at the 96-VGPR budget of NP = 44)
    int lane = lane_id();
    auto relane = [&]() __attribute__((always_inline)) {
        lane = lane_id();
        asm volatile("" : "+v"(lane));
    };
    uint8_t* scratch = bl.scratch + (int64_t)blockIdx.x * bl.scratch_per_wave;
    const int64_t A = bl.num_atoms;

    // complexes of this launch: all of them, or the overflow list written by the bucket pass
    const int64_t total = bl.work_list ? (int64_t)*bl.work_len : A;
    for (;;) {
        // Wave-uniform dequeue without a branch on the lane: every lane adds (lane == 0) to the
        // queue (one atomic after the compiler's wave combine) and lane 0's ticket is read back
        // with v_readlane into an SGPR, so the loop exit and everything keyed on the complex (gi,
        // n) are scalar branches. Round 2 handed lane 0's ticket to the wave through an LDS slot
        // behind `if (lane == 0)`; a `continue` out of the loop then let the compiler thread a copy
        // of the loop head specialised for lanes 1..63 -- for them the atomic is skipped, so the
        // copy re-reads the unchanged slot (a `readlane` of the specialised ticket constant-folds
        // to the same effect) and spins while lane 0 waits in the exit guard: the gfx950 "hang"
        // (DESIGN.md 3.2).
        const uint32_t ticket = atomicAdd((unsigned int*)bl.queue, lane == 0 ? 1u : 0u);
        const int64_t chunk0 = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)ticket, 0) * kChunk;
        if (chunk0 >= total) break;
        for (int64_t wi = chunk0; wi < chunk0 + kChunk && wi < total; ++wi) {
            const int64_t gi = bl.work_list ? (int64_t)(int32_t)uni((uint32_t)bl.work_list[wi]) : wi;
            const int n = (int)uni((uint32_t)bl.npoints[gi]);
            double* feat = bl.features ? bl.features + 35 * gi : nullptr;
            if (n > NP) {
                if (bl.skip_above) continue;  // reduced by the overflow launch
                if (lane == 0) atomicOr(bl.error_flag, kErrTooManyPoints);
                if (feat && lane < 35) feat[lane] = __builtin_nan("");
                if (bl.counts && lane < 4) bl.counts[4 * gi + lane] = -1;
                continue;
            }
            // 1/count(species) weight (betti_features.cpp:62-63, 77), from the distance pass
            const double weight = bl.weight ? bl.weight[gi] : 1.0;

            // the scratch base re-enters through an empty asm (scalar constraint: still uniform)
            // per complex, so per-lane scratch addresses are formed at their uses as scalar base +
            // vector offset instead of being hoisted out of the dequeue loop as 64-bit vector
            // pointers, which the compiler then spills
            uint8_t* cscr = scratch;
            asm volatile("" : "+s"(cscr));
            Complex<NP> cx{s, n, bl.thr, cscr, 0u, 0, 0, 0, 0};
            cx.zero_code = 0xFFFFFFFFu;
            constexpr int S = BettiSmem<NP>::S;
            cx.zero_code = rank_codes<NP>(s, bl.lower + gi * bl.tri_stride, n, cx.thr,
                                          cx.template sp<float>(ScratchLayout::svals),
                                          cx.template sp<uint64_t>(ScratchLayout::rankk));
            if (cx.zero_code == kRankDense) {
                // more distances <= thr than this tier's register sort holds: the dense launch
                // (NP = 64, 1,024 keys) after this one, or beyond that the capacity-retry launch
                // (wide kernel, f32 matrix), reduces the complex and writes its outputs
                if (NP <= 48 && bl.dense_list) {
                    if (lane == 0) bl.dense_list[atomicAdd(bl.dense_len, 1u)] = (int32_t)gi;
                } else if (bl.retry_list) {
                    if (lane == 0) bl.retry_list[atomicAdd(bl.retry_len, 1u)] = (int32_t)gi;
                } else {
                    if (lane == 0) atomicOr(bl.error_flag, kErrWorkCol);
                    if (feat && lane < 35) feat[lane] = __builtin_nan("");
                    if (bl.counts && lane < 4) bl.counts[4 * gi + lane] = -1;
                }
                continue;
            }
            lds_sync();
            // ---- adjacency (sparse_distance_matrix: i != j and d <= thr, ripser.cpp:386-395) ----
            relane();
            uint64_t myadj = 0;  // this lane's row
            {
                for (int i = 0; i < n; ++i) {
                    // the kNoCode diagonal fails the test: no self loops
                    const uint64_t row = ballot(s.D[i * S + lane] != kNoCode) & lanes_below(n);
                    myadj = lane == i ? row : myadj;
                }
                if (lane < NP) s.adj[lane] = myadj;  // (lanes >= NP would write past adj)
            }
            uint32_t* d0s = cx.template sp<uint32_t>(ScratchLayout::d0);  // codes; f32 after decode_outputs
            const int dim_max = n - 2 < 2 ? n - 2 : 2;  // ripser.cpp:560
            cx.n_inf0 = 0;
            cx.n_d0 = 0;
            // ---- dim 0: Prim on F-keys == Kruskal's forest in Ripser order (ripser.cpp:725-762) ----
            relane();
            // best = the lane's F-minimal edge to the forest (kInf once the lane is in the forest,
            // and for lanes >= n); the wave minimum of its high word (the diameter) alone decides
            // unless two lanes tie on it. Deaths and forest parents stay in registers (lane t: death
            // t; each lane its own parent) and are written once after the loop.
            {
                bool in_tree = lane == 0, root = lane == 0;
                int parent = 0;
                uint32_t death = 0;  // rank code
                uint64_t best = kInf;
                if (lane < n && lane != 0 && (myadj & 1ull)) best = cx.ekey(0, lane);
                if (n >= 1) cx.n_inf0 = 1;
                uint64_t tree = 1;  // forest vertices (uniform)
                for (int added = 1; added < n; ++added) {
                    const uint32_t hi = (uint32_t)(best >> 32);
                    const uint32_t mh = wave_min_u32(hi);
                    int v;
                    bool newcomp = false;
                    if (mh == 0xFFFFFFFFu) {  // new component: lowest vertex outside the forest
                        v = __ffsll((unsigned long long)(~tree & lanes_below(n))) - 1;
                        cx.n_inf0 += 1;
                        newcomp = true;
                    } else {
                        uint64_t bal = ballot(hi == mh);
                        if (__popcll(bal) > 1) {  // equal diameters: the low words (F-order index) decide
                            const uint32_t ml = wave_min_u32(hi == mh ? (uint32_t)best : 0xFFFFFFFFu);
                            bal = ballot(best == (((uint64_t)mh << 32) | ml));
                        }
                        v = __ffsll((unsigned long long)bal) - 1;
                        if (mh != cx.zero_code) {  // (0, d) emitted only if d != 0 (ripser.cpp:741-748)
                            death = lane == cx.n_d0 ? mh : death;
                            cx.n_d0 += 1;
                        }
                    }
                    tree |= 1ull << v;
                    if (lane == v) {
                        in_tree = true;
                        root = newcomp;
                        best = kInf;
                    }
                    if (!in_tree && ((myadj >> v) & 1ull)) {
                        const uint64_t k = cx.ekey(v, lane);
                        if (k < best) { best = k; parent = v; }
                    }
                }
                if (lane < cx.n_d0) at(d0s, lane) = death;
                if (lane < NP) s.par[lane] = (lane < n && !root) ? (uint8_t)parent : (uint8_t)0xFF;
            }
            lds_sync();
            // ---- edge list (i > j, d <= thr), row-major ----
            relane();
            uint16_t* edges = cx.template sp<uint16_t>(ScratchLayout::edges);
            int n_edges = 0;
            {
                const uint64_t low = lane < n ? (s.adj[lane] & ((lane == 0) ? 0ull : ((1ull << lane) - 1ull))) : 0ull;
                const int c = __popcll(low);
                const int inc = wave_inclusive_sum(c);
                // readlane, not a shuffle: the count must be a scalar (a shuffle result is a
                // vector value to the compiler, and every loop over the edges would be exec-masked)
                n_edges = (int)uni((uint32_t)__builtin_amdgcn_readlane(inc, kWave - 1));
                int off = inc - c;
                uint64_t mm = low;
                while (mm) {
                    const int j = __ffsll((unsigned long long)mm) - 1;
                    mm &= mm - 1;
                    at(edges, off++) = (uint16_t)((lane << 8) | j);
                }
            }
            __syncthreads();  // edge list (global scratch) visible to every lane
            cx.n_p1 = 0;
            cx.n_p2 = 0;
            uint64_t* na_key = cx.template sp<uint64_t>(ScratchLayout::na_key);
            uint64_t* na_tau = cx.template sp<uint64_t>(ScratchLayout::na_tau);
            uint8_t* mincof = cx.template sp<uint8_t>(ScratchLayout::mincof);
            uint8_t* mincof_e = cx.template sp<uint8_t>(ScratchLayout::mincof_e);
                    // ---- dim 1: one lane per column (non-tree edge) ----
                    relane();
            uint32_t* defer = cx.template sp<uint32_t>(ScratchLayout::defer);
            if (dim_max >= 1) {
                int nna = 0, ndef = 0;
                // One lane per edge column. Round A walks at most kAppSteps steps of every column's
                // min-cofacet walk; columns not settled by then are listed and walked to the end by
                // round B, so a round-synchronous pass is not paced by its few long walks.
                auto edge_col = [&](bool active, uint32_t ed, int steps) {
                    bool na_col = false, dfr = false;
                    uint64_t colkey = 0, best = kInf;
                    if (active) {
                        const int i = ed >> 8, j = ed & 255;
                        uint32_t mc = kMcNone;
                        if (!cx.is_tree(i, j)) {
                            const uint32_t dij = cx.dlowb(i, j);
                            colkey = make_key(dij, pack2(i, j));
                            uint64_t cand = s.adj[i] & s.adj[j];
                            if (cand) {
                                int bk;
                                bool found;
                                uint32_t hda, hdb, hdc;
                                best = cx.min_cofacet_lane(1, i, j, 0, dij, cand, bk, found, hda, hdb, hdc, steps);
                                dfr = !found && cand != 0;
                                // apparent iff (i,j) is the F-max facet of its pivot triangle: a
                                // zero-persistence cofacet whose other facets (bk replacing i or j)
                                // are shorter, or as long with a larger index (bk above the
                                // replaced vertex). An apparent pair has zero persistence: no pair
                                // is emitted (death > birth only, ripser.cpp:1240).
                                const bool apparent = found && (bk > i || hdb < dij) && (bk > j || hda < dij);
                                if (apparent) {
                                    const uint32_t tp = key_packed(best);
                                    cx.set_cleared_lane((tp >> 16) & 255, (tp >> 8) & 255, tp & 255);
                                } else {
                                    na_col = !dfr;
                                }
                                mc = (uint32_t)bk;
                            }
                        }
                        if (!dfr) at(mincof_e, edge_dense(i, j)) = (uint8_t)mc;
                    }
                    const uint64_t bal = ballot(na_col);
                    if (na_col) {
                        const int slot = nna + mask_prefix(bal);
                        if (slot < kNACap) {
                            at(na_key, slot) = colkey;
                            at(na_tau, slot) = best;
                        }
                    }
                    nna += __popcll(bal);
                    const uint64_t bd = ballot(dfr);
                    if (dfr) at(defer, ndef + mask_prefix(bd)) = ed;
                    ndef += __popcll(bd);
                };
                for (int base = 0; base < n_edges; base += kWave) {
                    const int e = base + lane;
                    edge_col(e < n_edges, e < n_edges ? (uint32_t)at(edges, e) : 0u, kAppSteps);
                }
                if (ndef) {
                    __syncthreads();  // the deferred list (scratch) is read by other lanes
                    const int nd = ndef;
                    for (int base = 0; base < nd; base += kWave) {
                        const int e = base + lane;
                        edge_col(e < nd, e < nd ? at(defer, e) : 0u, 1 << 20);
                    }
                }
                __syncthreads();
                cx.reduce_serial(1, nna);
                __syncthreads();  // clearing marks (scratch stores) complete before the dim-2 pass
            }
            if (!(dim_max >= 2 && cx.err == 0) && n >= 3) {
                // no dim-2 pass to consume them: erase every triangle entry (clearing marks)
                for (int t = lane; t < c3(n); t += kWave) at(mincof, t) = kMcNone;
                __syncthreads();
            }
            // ---- dim 2: one lane per column (uncleared triangle) ----
            relane();
            if (dim_max >= 2 && cx.err == 0) {
                int nna = 0;
                // (2a) stream the complex's triangles into a scratch list: each lane owns an edge
                // (a > b) and walks c < b in adj[a] & adj[b]; lanes refill from the edge list
                uint32_t* tl = cx.template sp<uint32_t>(ScratchLayout::tris);
                int ntri = 0;
                {
                    int next_edge = 0;
                    int ea = 0, eb = 0;
                    uint64_t tmask = 0;
                    // the edge list is read through a register window: lane t holds edges wbase + t
                    // (win) and wbase + 64 + t (win_next, loaded one window ahead), so a refill is a
                    // lane shuffle instead of a dependent scratch load (edges without a c < b in
                    // common refill again at once)
                    int wbase = 0;
                    uint32_t win = lane < n_edges ? (uint32_t)at(edges, lane) : 0u;
                    uint32_t win_next = kWave + lane < n_edges ? (uint32_t)at(edges, kWave + lane) : 0u;
                    while (true) {
                        while (true) {  // refill lanes with empty masks
                            const bool need = tmask == 0;
                            const uint64_t bal = ballot(need);
                            if (!bal || next_edge >= n_edges) break;
                            const int e = next_edge + mask_prefix(bal);
                            const int off = e - wbase;  // < 128: next_edge - wbase < 64
                            const uint32_t v0 = (uint32_t)__shfl((int)win, off & (kWave - 1), kWave);
                            const uint32_t v1 = (uint32_t)__shfl((int)win_next, off & (kWave - 1), kWave);
                            if (need && e < n_edges) {
                                const uint32_t ed = off < kWave ? v0 : v1;
                                ea = ed >> 8;
                                eb = ed & 255;
                                tmask = s.adj[ea] & s.adj[eb] & ((1ull << eb) - 1ull);
                            }
                            next_edge += __popcll(bal);
                            if (next_edge - wbase >= kWave) {  // window consumed: slide by 64
                                wbase += kWave;
                                win = win_next;
                                const int t = wbase + kWave + lane;
                                win_next = t < n_edges ? (uint32_t)at(edges, t) : 0u;
                            }
                            if (ballot(tmask == 0) == 0) break;
                        }
                        const bool active = tmask != 0;
                        const uint64_t bal = ballot(active);
                        if (!bal) break;
                        if (active) {
                            const int c = __ffsll((unsigned long long)tmask) - 1;
                            tmask &= tmask - 1;
                            at(tl, ntri + mask_prefix(bal)) = pack3(ea, eb, c);
                        }
                        ntri += __popcll(bal);
                    }
                }
                __syncthreads();  // the list (scratch) is read by other lanes
                // (2b) one lane per column (uncleared triangle), in two rounds as in the dim-1
                // pass: round A walks at most kAppSteps steps per column and lists the unsettled
                // ones, round B walks those to the end. Global reads leave the per-round dependency
                // chain: list entries are fetched two rounds ahead, their clearing bytes one round
                // ahead.
                int ndef = 0;
                auto tri_col = [&](bool active, uint32_t tp, uint32_t clb, int steps) {
                    bool na_col = false, dfr = false;
                    uint64_t colkey = 0, best = kInf;
                    if (active) {
                        const int a = (tp >> 16) & 255, b = (tp >> 8) & 255, c = tp & 255;
                        uint32_t mc = kMcNone;
                        if (clb != kMcCleared) {
                            const uint32_t dab = cx.dlowb(a, b), dac = cx.dlowb(a, c), dbc = cx.dlowb(b, c);
                            const uint32_t ds = max(max(dab, dac), dbc);
                            colkey = make_key(ds, tp);
                            uint64_t cand = s.adj[a] & s.adj[b] & s.adj[c];
                            if (cand) {
                                int bk;
                                bool found;
                                uint32_t hda, hdb, hdc;
                                best = cx.min_cofacet_lane(2, a, b, c, ds, cand, bk, found, hda, hdb, hdc, steps);
                                dfr = !found && cand != 0;
                                // apparent iff (a,b,c) is the F-max facet of its pivot tetrahedron
                                // (the dim-1 facet test, one facet per replaced vertex); zero
                                // persistence, so no pair is emitted
                                const bool apparent = found && (bk > a || max(max(hdb, hdc), dbc) < ds) &&
                                                      (bk > b || max(max(hda, hdc), dac) < ds) &&
                                                      (bk > c || max(max(hda, hdb), dab) < ds);
                                na_col = !apparent && !dfr;
                                mc = (uint32_t)bk;
                            }
                        }
                        if (!dfr) at(mincof, tri_dense_lane(a, b, c)) = (uint8_t)mc;
                    }
                    const uint64_t bal = ballot(na_col);
                    if (na_col) {
                        const int slot = nna + mask_prefix(bal);
                        if (slot < kNACap) {
                            at(na_key, slot) = colkey;
                            at(na_tau, slot) = best;
                        }
                    }
                    nna += __popcll(bal);
                    const uint64_t bd = ballot(dfr);
                    if (dfr) at(defer, ndef + mask_prefix(bd)) = tp;
                    ndef += __popcll(bd);
                };
                uint32_t tp1 = lane < ntri ? at(tl, lane) : 0u;
                uint32_t cl1 = lane < ntri ? (uint32_t)at(mincof, tri_dense_lane((tp1 >> 16) & 255, (tp1 >> 8) & 255, tp1 & 255)) : 0u;
                uint32_t tp2 = kWave + lane < ntri ? at(tl, kWave + lane) : 0u;
                for (int base = 0; base < ntri; base += kWave) {
                    const uint32_t tp = tp1, clb = cl1;
                    const bool active = base + lane < ntri;
                    tp1 = tp2;
                    cl1 = base + kWave + lane < ntri
                              ? (uint32_t)at(mincof, tri_dense_lane((tp2 >> 16) & 255, (tp2 >> 8) & 255, tp2 & 255))
                              : 0u;
                    tp2 = base + 2 * kWave + lane < ntri ? at(tl, base + 2 * kWave + lane) : 0u;
                    tri_col(active, tp, clb, kAppSteps);
                }
                if (ndef) {
                    __syncthreads();  // the deferred list (scratch) is read by other lanes
                    const int nd = ndef;
                    uint32_t tq = lane < nd ? at(defer, lane) : 0u;
                    for (int base = 0; base < nd; base += kWave) {
                        const uint32_t tp = tq;
                        tq = base + kWave + lane < nd ? at(defer, base + kWave + lane) : 0u;
                        // deferred columns are never cleared
                        tri_col(base + lane < nd, tp, 0u, 1 << 20);
                    }
                }
                __syncthreads();
                cx.reduce_serial(2, nna);
                lds_sync();
            }
            __syncthreads();
            if (cx.n_p1 > kPairCap || cx.n_p2 > kPairCap) cx.err |= kErrPairs;
            const uint32_t err = uni(cx.err);
            if (err && bl.retry_list && (err & kErrCapacity) == err) {
                // workspace overflow: the capacity-retry launch (betti_wide_kernel, big layout)
                // reduces this complex again and writes its outputs
                if (lane == 0) bl.retry_list[atomicAdd(bl.retry_len, 1u)] = (int32_t)gi;
            } else if (err) {
                if (lane == 0) atomicOr(bl.error_flag, err);
                if (feat && lane < 35) at(feat, lane) = __builtin_nan("");
                if (bl.counts && lane < 4) at(bl.counts + 4 * gi, lane) = -1;
            } else {
                // ---- statistics (betti_features.cpp:24-55, 87-98; utils/math.hpp:9-28) ----
                relane();
                cx.decode_outputs(d0s);
                const float* d0f = reinterpret_cast<const float*>(d0s);
                const double myval = betti_stats35(d0f, cx.n_d0, cx.pairs(1), cx.n_p1, cx.pairs(2), cx.n_p2, weight);
                if (feat && lane < 35) at(feat, lane) = myval;
                if (bl.pairs_out) {
                    float2* po = reinterpret_cast<float2*>(bl.pairs_out) + (int64_t)gi * 3 * bl.pair_cap;
                    for (int i = lane; i < cx.n_d0 && i < bl.pair_cap; i += kWave) at(po, i) = make_float2(0.0f, at(d0f, i));
                    for (int i = lane; i < cx.n_p1 && i < bl.pair_cap; i += kWave) at(po, bl.pair_cap + i) = at(cx.pairs(1), i);
                    for (int i = lane; i < cx.n_p2 && i < bl.pair_cap; i += kWave) at(po, 2 * bl.pair_cap + i) = at(cx.pairs(2), i);
                }
                if (bl.counts && lane < 4)  // #dim0 finite, #dim0 infinite, #dim1, #dim2
                    at(bl.counts + 4 * gi, lane) = lane == 0 ? cx.n_d0 : (lane == 1 ? cx.n_inf0 : (lane == 2 ? cx.n_p1 : cx.n_p2));
            }
            lds_sync();
        }
    }
}

// ---------------------------------------------------------------------------------------
// Local distance matrices of caller-given clouds (dgn_host_persistence: compute_persistence,
// ripser_wrapper.cpp:60-70): gram_triangle_* (dgn_device.hpp; VALU pairs up to 64 points, matrix-
// core Gram tiles above). One wave per
// complex. The atom-centred clouds of dgn_*_betti come from betti_dist_search_kernel
// (graph_kernels.hip), which finds the neighbours itself.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void betti_dist_kernel(BettiLaunch bl, DistLaunch dl) {
    __shared__ double sq_s[4][kWideMaxPoints];
    const int lane = lane_id(), w = threadIdx.x >> 6;
    double* sq = sq_s[w];
    for (int64_t c = (int64_t)blockIdx.x * 4 + w; c < dl.count; c += (int64_t)gridDim.x * 4) {
        const int64_t gi = dl.first + c;
        const int n = bl.npoints[gi];
        if (lane == 0) {
            dl.npoints[c] = n;
            dl.weight[c] = 1.0;
        }
        if (n > kWideMaxPoints) continue;  // the Betti pass flags it
        const double* cloud = bl.clouds + (int64_t)gi * bl.cloud_stride * 3;
        float* L = dl.lower + c * bl.tri_stride;
        if (n > 64) {
            gram_triangle_wide(n, sq, L, [&](int p, double x[3]) {
                x[0] = cloud[3 * p];
                x[1] = cloud[3 * p + 1];
                x[2] = cloud[3 * p + 2];
            }, bl.tri_stride);
            continue;
        }
        const int pl = lane < n ? lane : n - 1;
        const double px[3] = {cloud[3 * pl], cloud[3 * pl + 1], cloud[3 * pl + 2]};
        gram_triangle_narrow(px, n, sq, L, bl.tri_stride);
    }
}

hipError_t launch_betti_dist(hipStream_t st, const BettiLaunch& b, const DistLaunch& d) {
    if (d.count <= 0) return hipSuccess;
    int64_t blocks = (d.count + 3) / 4;
    if (blocks > 256 * 64) blocks = 256 * 64;
    hipLaunchKernelGGL(betti_dist_kernel, dim3((unsigned)blocks), dim3(256), 0, st, b, d);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------------------
int betti_max_points() { return kWideMaxPoints; }
int64_t betti_scratch_bytes_per_wave() { return ScratchLayout::total; }

hipError_t betti_init_scratch(hipStream_t s, uint8_t* base, int slots) {
    // the triangle table and the edge table are adjacent: one 2D memset over all slots
    const size_t width = (size_t)(ScratchLayout::mincof_e + 64 * 63 / 2 - ScratchLayout::mincof);
    return hipMemset2DAsync(base + ScratchLayout::mincof, (size_t)ScratchLayout::total, kMcNone, width, (size_t)slots, s);
}

static int np_for(int max_points) { return max_points <= 32 ? 32 : (max_points <= 48 ? 48 : 64); }

int betti_grid_waves(int device) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 1024;
    // occupancy of the smallest instantiation bounds the slots we allocate scratch for
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, betti_kernel<32>, kWave, 0) != hipSuccess || per_cu <= 0)
        per_cu = 8;
    return prop.multiProcessorCount * per_cu;
}

// route complexes above np_small points: up to 64 to the overflow list (NP = 64 launch), above 64
// to the wide list (betti_wide_kernel), above kWideRegular to the retry list; wave-aggregated appends
__device__ __forceinline__ void bucket_append(bool take, int32_t* list, uint32_t* len, int64_t gi) {
    const uint64_t b = ballot(take);
    if (!b) return;
    const int leader = __ffsll((unsigned long long)b) - 1;
    uint32_t base = 0;
    if (lane_id() == leader) base = atomicAdd(len, (uint32_t)__popcll(b));
    base = (uint32_t)__shfl((int)base, leader, kWave);
    if (take) list[base + mask_prefix(b)] = (int32_t)gi;
}
__global__ __launch_bounds__(256) void betti_bucket_kernel(BettiLaunch bl, int np_small) {
    const int64_t gi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int n = gi < bl.num_atoms ? bl.npoints[gi] : 0;
    const bool mid = gi < bl.num_atoms && n > np_small && n <= 64;
    // above kWideRegular points: straight to the retry list (rank-coded BIG launch)
    const bool huge = gi < bl.num_atoms && n > kWideRegular && bl.retry_list;
    const bool wide = gi < bl.num_atoms && n > 64 && !huge;
    bucket_append(huge, bl.retry_list, bl.retry_len, gi);
    bucket_append(mid, bl.overflow_list, bl.overflow_len, gi);
    bucket_append(wide, bl.wide_list, bl.wide_len, gi);
}

// device facts for the persistent grids, queried once per device (hipGetDeviceProperties is a
// slow host call and every Betti call launches up to three grids)
// (relaxed atomics: contexts on different host threads may fill a slot concurrently; every
// writer stores the same value)
static int cu_count(int dev) {
    static std::atomic<int> cus[64];
    if (dev < 0 || dev >= 64) return 256;
    int v = cus[dev].load(std::memory_order_relaxed);
    if (v == 0) {
        hipDeviceProp_t prop;
        v = hipGetDeviceProperties(&prop, dev) == hipSuccess ? prop.multiProcessorCount : 256;
        cus[dev].store(v, std::memory_order_relaxed);
    }
    return v;
}

#ifndef DGN_PAD_LDS
#define DGN_PAD_LDS 0  // A/B builds only: extra dynamic LDS per wave (lower residency)
#endif
template <int NP>
static int grid_np(int grid_waves, int64_t max_items) {
    int dev = 0, per_cu = 0;
    (void)hipGetDevice(&dev);
    static std::atomic<int> occ[64];
    if (dev >= 0 && dev < 64 && occ[dev].load(std::memory_order_relaxed) > 0) {
        per_cu = occ[dev].load(std::memory_order_relaxed);
    } else {
        hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, betti_kernel<NP>, kWave, DGN_PAD_LDS);
        if (e != hipSuccess || per_cu <= 0) per_cu = 4;
        if (dev >= 0 && dev < 64) occ[dev].store(per_cu, std::memory_order_relaxed);
    }
    int grid = cu_count(dev) * per_cu;
    if (grid > grid_waves) grid = grid_waves;
    const int64_t chunks = (max_items + kChunk - 1) / kChunk;
    if (grid > chunks) grid = (int)(chunks > 0 ? chunks : 1);
    return grid;
}

static int grid_for(int np, int grid_waves, int64_t max_items) {
    if (np == 32) return grid_np<32>(grid_waves, max_items);
    if (np == 48) return grid_np<48>(grid_waves, max_items);
    return grid_np<64>(grid_waves, max_items);
}

template <int NP>
static hipError_t launch_np(hipStream_t st, const BettiLaunch& b, int grid) {
    hipLaunchKernelGGL(betti_kernel<NP>, dim3(grid), dim3(kWave), DGN_PAD_LDS, st, b);
    return hipGetLastError();
}

static hipError_t launch_for(int np, hipStream_t st, const BettiLaunch& b, int grid) {
    if (np == 32) return launch_np<32>(st, b, grid);
    if (np == 48) return launch_np<48>(st, b, grid);
    return launch_np<64>(st, b, grid);
}

// Tiered dispatch: the main launch uses the instantiation sized for typical complexes (NP = 48:
// 32 resident waves per CU); complexes above it are listed by betti_bucket_kernel and reduced by
// an NP = 64 launch (49..64 points) forked beside the main one and betti_wide_kernel (65..512
// points). Counters and list lengths live on the device, so nothing synchronizes with the host in
// between.
hipError_t launch_betti(hipStream_t st, const BettiLaunch& b, int max_points, int grid_waves, const WideLayout* wide,
                        int wide_waves, const BettiFork* fork) {
    const int np_big = np_for(max_points < 64 ? max_points : 64);
    const int np_main = np_big > 48 ? 48 : np_big;
    BettiLaunch m = b;
    m.work_list = nullptr;
    m.queue = b.work_counter;
    m.skip_above = max_points > np_main ? 1 : 0;
    if (m.skip_above) {
        const int64_t blocks = (b.num_atoms + 255) / 256;
        hipLaunchKernelGGL(betti_bucket_kernel, dim3((unsigned)blocks), dim3(256), 0, st, b, np_main);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    // scratch slots [0, main_grid) belong to the main launch (and then to the mid launch)
    const int main_grid = grid_for(np_main, fork ? grid_waves - fork->overflow_waves : grid_waves, b.num_atoms);
    const bool overflow = m.skip_above && np_big > 48;
    BettiLaunch o = b;
    o.work_list = b.overflow_list;
    o.work_len = b.overflow_len;
    o.queue = b.work_counter2;
    o.skip_above = 0;
    hipError_t e;
    if (overflow && fork) {
        // The few complexes of the overflow tier are the slowest ones: reduced after the main
        // launch they would add one heavy complex's latency to the pass. Instead they run on a
        // forked stream beside the main launch, on scratch slots past the main grid's.
        o.scratch = b.scratch + (int64_t)main_grid * b.scratch_per_wave;
        const int og = grid_for(64, fork->overflow_waves, b.num_atoms);
        if ((e = hipEventRecord(fork->fork, st)) != hipSuccess) return e;
        if ((e = hipStreamWaitEvent(fork->side, fork->fork, 0)) != hipSuccess) return e;
        if ((e = launch_for(64, fork->side, o, og)) != hipSuccess) return e;
        if ((e = hipEventRecord(fork->join, fork->side)) != hipSuccess) return e;
    }
    e = launch_for(np_main, st, m, main_grid);
    if (e != hipSuccess) return e;
    {
        // complexes the main launch listed as dense (more than 512 distances <= thr): NP = 64
        // launch on the main grid's scratch slots; its waves leave at once when the list is empty
        BettiLaunch d = b;
        d.work_list = b.dense_list;
        d.work_len = b.dense_len;
        d.queue = b.dense_queue;
        d.skip_above = 0;
        d.dense_list = nullptr;
        if ((e = launch_for(64, st, d, grid_for(64, main_grid, b.num_atoms))) != hipSuccess) return e;
    }
    if (!m.skip_above) return e;
    if (overflow) {
        if (fork) {
            if ((e = hipStreamWaitEvent(st, fork->join, 0)) != hipSuccess) return e;
        } else {
            e = launch_for(64, st, o, grid_for(64, grid_waves, b.num_atoms));
            if (e != hipSuccess) return e;
        }
    }
    if (max_points > 64 && wide) e = launch_betti_wide(st, b, *wide, wide_waves);
    return e;
}

}  // namespace dgn
