// betti_wide.hip — Vietoris–Rips persistence (dim 0/1/2, Z/2) and the 35 Betti statistics for
// local complexes of 65..512 points, one wave64 per complex, for gfx950.
//
// The reference's default cutoff is 10 A (compute_structure_betti_features,
// include/topology/betti_features.hpp:37-39; preprocess_betti.cpp:32,117): FCC-256 complexes
// then have ~340 points. betti_kernels.hip covers n <= 64 with
// one lane per vertex and the complex in LDS; this kernel runs the same algorithm with the
// same output contract on larger complexes:
//   * vertex sets are multi-word bitsets in LDS (W = ceil(n / 64) 64-bit words per vertex; the
//     dynamic LDS block is sized by the launch's largest complex, so smaller cutoffs keep more
//     waves resident); lane k handles vertices k, k + 64, ...;
//   * the f32 distance matrix is stored full and row-major in per-wave scratch, so the
//     lane-per-vertex reads of one row are coalesced;
//   * simplices are named by their combinatorial index (Ripser's colex numbering,
//     ripser.cpp:181-201): a key is (diameter bits << 32) | ~index, so ascending keys are
//     Ripser's filtration order (greater_diameter_or_smaller_index, ripser.cpp:318-324);
//     vertices travel packed 9 bits per vertex, descending;
//   * the non-apparent columns are bitonic-sorted in scratch, the serially resolved pivots live
//     in an open-addressing hash table in scratch, the min-cofacet tables hold u16 vertices.
// Pairing semantics as betti_kernels.hip: dim 0 by Prim on F-keys (Kruskal's forest in Ripser's
// order, ripser.cpp:725-762); dim 1/2 cohomology with clearing, apparent pairs settled
// lane-parallel, the rest reduced in Ripser's column order (decreasing F-key); death > birth
// only, essential dim >= 1 classes are not emitted (ripser.cpp:1209-1225, 1240). The pairing
// of a total order is unique, so the emitted multiset equals Ripser's.
#include <algorithm>
#include <cstdlib>

#include "dgn_internal.hpp"

#ifndef DGN_PV_UNROLL
#define DGN_PV_UNROLL 2  // V entries evaluated together in the pivot search
#endif
#ifndef DGN_WIDE_STEP
#define DGN_WIDE_STEP 4
#endif

namespace dgn {
namespace {

constexpr uint64_t kInfW = ~0ull;
constexpr uint16_t kMcNoneW = 0xFFFF;     // not a column, or no cofacet
constexpr uint16_t kMcClearedW = 0xFFFE;  // triangle is the pivot of a dim-1 column (clearing)
constexpr uint64_t kLazyW = 1ull << 63;    // pivot meta: V = {column simplex} (packed, low bits)
constexpr uint64_t kNoMetaW = ~0ull;       // pivot not in the table
constexpr int kMetaLenBits = 24;           // pivot meta: (V-store offset << 24) | V length
// error bits (decoded in dgn_api.cpp)
constexpr uint32_t kEPoints = 1u << 0, kEWork = 1u << 1, kENA = 1u << 2, kEPiv = 1u << 3, kEPairs = 1u << 4,
                   kER = 1u << 5, kEGuard = 1u << 7;
constexpr uint32_t kECapacity = kEWork | kENA | kEPiv | kEPairs | kER | kEGuard;

__device__ __forceinline__ uint64_t bin2(uint64_t v) { return v * (v - 1) / 2; }
__device__ __forceinline__ uint64_t bin3(uint64_t v) { return v * (v - 1) * (v - 2) / 6; }
__device__ __forceinline__ uint64_t bin4(uint64_t v) { return v * (v - 1) * (v - 2) * (v - 3) / 24; }
__device__ __forceinline__ uint32_t rlw(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }
__device__ __forceinline__ uint64_t rlw64(uint64_t x, int l) {
    return ((uint64_t)rlw((uint32_t)(x >> 32), l) << 32) | rlw((uint32_t)x, l);
}
// lanes 0 .. m - 1 (m in 0..64)
__device__ __forceinline__ uint64_t lanes_below_w(int m) { return m >= 64 ? ~0ull : (1ull << m) - 1ull; }
__device__ __forceinline__ uint32_t uniw(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t uniw64(uint64_t x) {
    return ((uint64_t)uniw((uint32_t)(x >> 32)) << 32) | uniw((uint32_t)x);
}
__device__ __forceinline__ void wave_lds_order() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }
// lane-to-lane hand-off through this wave's global scratch (V list, pivot table, V store, lists):
// a workgroup-scope fence, which waits for every outstanding memory access of the wave
// (vmcnt(0) lgkmcnt(0)) without a barrier -- the two waves of a workgroup run different phases
// of different complexes (betti_wide_body)
__device__ __forceinline__ void wave_scratch_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

// combinatorial index of a packed simplex with nv vertices
// insert vertex x (not in p) into a packed simplex of nv vertices
__device__ __forceinline__ int c2i(int x) { return x * (x - 1) / 2; }

// KW: bitset words per vertex the instantiation handles (complexes of up to 64 KW points).
// BIG (complexes of 513..1024 points): vertices packed in 10 bits, distances replaced by their
// rank codes in the complex (order- and equality-preserving, < 2^20; betti_rank_codes) so a
// simplex key (code << 36) | ~index fits 64 bits (C(1024, 4) < 2^36); code -> f32 via the
// complex's sorted distances. HUGE (1025..2048 points): 11-bit vertices, codes < 2^22 and keys
// (code << 40) | ~index (C(2048, 4) < 2^40); a packed triangle (33 bits) travels as a u64 and the
// adjacency bitsets (n x 32 words) move from LDS to the wave's scratch. Otherwise 9-bit vertices
// and (f32 bits << 32) | ~index keys.
// MODE: kF32 (distances as f32 bits), kC16 (u16 rank codes: 4-byte -> 2-byte matrix for
// complexes of <= 362 points, C(362, 2) < 2^16), kBig, kHuge (above).
// kGiant (2,049..kWideGiantPoints points, one connected component of a caller-given cloud or triangle):
// 12-bit vertices, keys (code << 44) | ~index (C(4096, 4) < 2^44) with the codes of the distances
// <= thr below 2^20 (larger codes, all above thr, clamp to kGiantCodeMax; a complex with 2^20 or more
// distances within thr is outside the envelope); HUGE's scratch bitsets, and no min-cofacet table
// (C(n, 3) entries): clearing marks in a bitmap, the dim-2 apparent owners decided from the matrix
// rows as in the prewalked path
constexpr int kF32 = 0, kC16 = 1, kBig = 2, kHuge = 3, kGiant = 4;
constexpr uint32_t kGiantCodeMax = (1u << 20) - 1;
template <int KW, int MODE, bool PRE = false>
struct WideCx {
    static constexpr bool BIG = MODE == kBig;
    static constexpr bool GIANT = MODE == kGiant;
    static constexpr bool HUGE = MODE == kHuge || GIANT;  // bitsets in scratch, u64 packed triangles
    static constexpr bool NOMCT = PRE || GIANT;            // no dim-2 min-cofacet table
    using CLT = std::conditional_t<GIANT, uint64_t, uint32_t>;  // a clearing-list entry (triangle index)
    static constexpr bool CODED = MODE != kF32;
    static constexpr int kWW = KW;
    static constexpr int VB = GIANT ? 12 : (HUGE ? 11 : (BIG ? 10 : 9));  // bits per packed vertex
    static constexpr uint64_t VM = (1ull << VB) - 1;
    static constexpr int KS = GIANT ? 44 : (HUGE ? 40 : (BIG ? 36 : 32));  // key: (distance code << KS) | ~index
    // a packed column simplex / V entry (edge or triangle, 3 VB bits)
    using PT = std::conditional_t<HUGE, uint64_t, uint32_t>;
    static constexpr PT kNoneP = ~PT(0);
    __device__ static PT rlp(PT x, int l) {
        if constexpr (HUGE) return rlw64(x, l);
        else return rlw(x, l);
    }
    __device__ static PT unip(PT x) {
        if constexpr (HUGE) return uniw64(x);
        else return uniw(x);
    }
    __device__ static int pv(uint64_t p, int field) { return (int)((p >> (VB * field)) & VM); }
    __device__ static uint64_t pidx(int nv, uint64_t p) {
        if (nv == 2) return bin2(pv(p, 1)) + pv(p, 0);
        if (nv == 3) return bin3(pv(p, 2)) + bin2(pv(p, 1)) + pv(p, 0);
        return bin4(pv(p, 3)) + bin3(pv(p, 2)) + bin2(pv(p, 1)) + pv(p, 0);
    }
    __device__ static uint64_t pinsert(int nv, uint64_t p, int x) {
        int below = 0;
        for (int t = 0; t < nv; ++t) below += pv(p, t) < x;
        const uint64_t mask = (1ull << (VB * below)) - 1;
        return ((p & ~mask) << VB) | ((uint64_t)x << (VB * below)) | (p & mask);
    }
    __device__ static uint64_t wkey(uint32_t dc, uint64_t idx) {
        return ((uint64_t)dc << KS) | (~idx & ((1ull << KS) - 1));
    }
    __device__ static uint32_t kdiam(uint64_t key) { return (uint32_t)(key >> KS); }
    __device__ static uint32_t pack_edge(int i, int j) { return ((uint32_t)i << VB) | (uint32_t)j; }
    // PRE (u16 codes after the walk pass, betti_walk_kernel): the matrix, the bitsets, the threshold
    // code and the dim-2 column list come from bl.walk; clearing marks live in a bitmap (ly.clb)
    // and the dim-2 apparent owners are decided from the matrix (lookup) -- no min-cofacet table
    static_assert(!PRE || MODE == kC16, "the walk pass covers the u16-coded complexes");
    // NOMCT without PRE (GIANT): the kernel's own passes keep their clearing marks in the bitmap too
    const BettiLaunch& bl;
    const WideLayout& ly;
    uint64_t* adj;  // LDS [n][W]: row v = the neighbours of vertex v, W words
    uint16_t* par;  // LDS [n]: spanning-forest parent, 0xFFFF = root
    uint8_t* scr;
    int n, W;
    float thr;
    uint32_t err;
    int n_d0, n_inf0, n_p1, n_p2;
    const uint32_t* vals = nullptr;  // CODED: the complex's sorted f32 distances (code -> value)
    // the working column's V list: in registers (lane i holds entry i) while it has <= 64 entries,
    // else (vspill, uniform) in scratch (vlist); scratch only for the 8-word instantiation (its
    // registers are spent: the register list there spilled 150 VGPRs)
    static constexpr bool VREG = KW <= 6 || KW > 8;
    PT vreg = 0;
    bool vspill = false;
    // the threshold in distance-code space (largest code of a distance <= thr; f32 bits in kF32
    // mode): the reduction tests common neighbours from the distances alone (no adjacency), with
    // an all-ones diagonal excluding the simplex's own vertices
    uint32_t thrc = 0;

    const uint8_t* dm = nullptr;  // the distance matrix: this wave's scratch (ly.D) or PRE the walk pass's
    int ns = 0;                   // its row stride in elements (n; PRE: n rounded up to 4, 8-byte rows)
    int64_t wslot = 0;            // the complex's slice position (PRE: its walk-pass outputs)
    uint16_t* mce = nullptr;      // dim-1 min-cofacet table: scratch (ly.mc_e) or PRE the walk pass's
    float* d0p = nullptr;         // dim-0 deaths: scratch (ly.d0) or PRE the walk pass's

    __device__ float value(uint32_t dc) const { return CODED ? __uint_as_float(vals[dc]) : __uint_as_float(dc); }
    // cleared-triangle bitmap (PRE): set / test bit t
    __device__ uint32_t* clbits() const { return sp<uint32_t>(ly.clb); }
    __device__ void clear_mark(uint64_t t) const { atomicOr(clbits() + (t >> 5), 1u << (t & 31)); }
    // (the marks are L2 atomics: read past the CU's L1, which may hold a stale copy of the word)
    __device__ bool is_cleared(uint64_t t) const {
        return (__hip_atomic_load(clbits() + (t >> 5), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (t & 31)) & 1u;
    }

    template <class T>
    __device__ T* sp(int64_t off) const { return reinterpret_cast<T*>(scr + off); }
    // d(i, j) at a per-lane (i, j): scalar matrix base + 32-bit element offset (i n + j < 2^22), not
    // a 64-bit vector address built from a 64-bit product per read
    __device__ uint32_t d(int i, int j) const {
        const uint32_t ix = (uint32_t)i * (uint32_t)ns + (uint32_t)j;
        if (MODE == kC16) return at(reinterpret_cast<const uint16_t*>(dm), ix);
        return at(reinterpret_cast<const uint32_t*>(dm), ix);
    }
    __device__ uint64_t aw(int v, int w) const { return adj[v * W + w]; }
    // d(a, x) for a wave-uniform row a: scalar row base + 32-bit lane offset
    __device__ uint32_t drow(int a, uint32_t x) const {
        const uint32_t ra = (uint32_t)a * (uint32_t)ns;
        if (MODE == kC16) return at(reinterpret_cast<const uint16_t*>(dm) + ra, x);
        return at(reinterpret_cast<const uint32_t*>(dm) + ra, x);
    }
    // u16 codes (n <= 362, 9-bit vertices): the pivot search compares cofacets by the packed-tuple
    // key (code << 36) | ~tuple, order-isomorphic to (code << 32) | ~index (a tuple packed
    // descending compares as its colex index), so a candidate costs no binomials; the winner's
    // index is computed once
    static constexpr bool PACKKEY = MODE == kC16;
    static constexpr int PKS = 36;
    __device__ static uint64_t pkey(uint32_t dc, uint64_t tuple) {
        return ((uint64_t)dc << PKS) | (~tuple & ((1ull << PKS) - 1));
    }
    __device__ bool is_tree(int i, int j) const { return par[i] == j || par[j] == i; }
    __device__ uint32_t sdiam(int dim, uint64_t p) const {  // dim 1: edge, dim 2: triangle
        if (dim == 1) return d(pv(p, 1), pv(p, 0));
        return max(max(d(pv(p, 2), pv(p, 1)), d(pv(p, 2), pv(p, 0))), d(pv(p, 1), pv(p, 0)));
    }

    // ---- distance matrix (mirrored from the packed lower triangle) + adjacency bitsets ----
    __device__ void load(int64_t gi, int64_t slot) {
        const int lane = lane_id();
        if constexpr (PRE) {  // the walk pass built the matrix and the threshold code
            (void)gi;
            (void)lane;
            thrc = uniw(bl.walk.meta[8 * slot + kWmThr]);
            return;
        }
        const float* L = bl.lower + gi * bl.tri_stride;
        uint32_t* D = sp<uint32_t>(ly.D);
        uint16_t* D16 = sp<uint16_t>(ly.D);
        const uint32_t* Lc = CODED ? bl.rank_codes + slot * bl.rank_stride : nullptr;
        for (int i = lane; i < n * W; i += kWave) adj[i] = 0ull;
        for (int i = lane; i < n; i += kWave) {  // all-ones diagonal: no vertex is its own neighbour
            if (MODE == kC16) D16[(int64_t)i * n + i] = 0xFFFF;
            else D[(int64_t)i * n + i] = 0xFFFFFFFFu;
        }
        uint32_t tmax = 0;
        if constexpr (HUGE) wave_scratch_sync();  // the zeroed bitsets (scratch) before the atomics
        else wave_lds_order();
        for (int i = 1; i < n; ++i) {
            for (int j0 = 0; j0 < i; j0 += kWave) {
                const int j = j0 + lane;
                bool e = false;
                if (j < i) {
                    const float v = L[c2i(i) + j];
                    uint32_t dv = CODED ? Lc[c2i(i) + j] : __float_as_uint(v);
                    if (GIANT) dv = min(dv, kGiantCodeMax);  // the codes above thr saturate
                    if (MODE == kC16) {
                        D16[(int64_t)i * n + j] = (uint16_t)dv;
                        D16[(int64_t)j * n + i] = (uint16_t)dv;
                    } else {
                        D[(int64_t)i * n + j] = dv;
                        D[(int64_t)j * n + i] = dv;
                    }
                    e = v <= thr;  // sparse_distance_matrix keeps d <= threshold (ripser.cpp:386-395)
                    if (e) tmax = max(tmax, dv);
                }
                const uint64_t b = ballot(e);
                if (lane == 0) {  // row i, columns j < i
                    if constexpr (HUGE) atomicOr((unsigned long long*)&adj[i * W + (j0 >> 6)], b);
                    else adj[i * W + (j0 >> 6)] = b;
                }
                if (e) atomicOr((unsigned long long*)&adj[j * W + (i >> 6)], 1ull << (i & 63));
            }
        }
        thrc = ~wave_min_u32(~tmax);
        if (GIANT && thrc >= kGiantCodeMax) err |= kEPoints;  // 2^20 or more distances within thr
        // HUGE: the bitsets were built by L2 atomics; the agent-scope fence drops the CU's L1 copies
        if constexpr (HUGE) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
        wave_scratch_sync();
    }

    // ---- dim 0: Prim on F-keys == Kruskal's forest in Ripser's order (ripser.cpp:725-762) ----
    __device__ void prim() {
        const int lane = lane_id();
        float* d0s = sp<float>(ly.d0);
        uint64_t best[kWW];
        int bp[kWW];
        // bit t: vertex 64 t + lane is in the forest (64 words for GIANT)
        using MT = std::conditional_t<(kWW > 32), uint64_t, uint32_t>;
        MT intree = lane == 0 ? MT(1) : MT(0);
        for (int i = lane; i < n; i += kWave) par[i] = 0xFFFF;
#pragma unroll
        for (int t = 0; t < kWW; ++t) {
            const int v = 64 * t + lane;
            best[t] = kInfW;
            bp[t] = 0;
            if (t < W && v < n && v != 0 && ((aw(0, t) >> lane) & 1ull)) best[t] = wkey(d(0, v), bin2(v));
        }
        wave_lds_order();
        n_inf0 = 1;
        n_d0 = 0;
        for (int added = 1; added < n; ++added) {
            uint64_t lmin = kInfW;
            int lt = 0, lp = 0, lfree = 1 << 30;
#pragma unroll
            for (int t = 0; t < kWW; ++t) {
                const int v = 64 * t + lane;
                const bool out = t < W && v < n && !((intree >> t) & MT(1));
                if (out && best[t] < lmin) {
                    lmin = best[t];
                    lt = t;
                    lp = bp[t];
                }
                if (out && v < lfree) lfree = v;
            }
            const uint64_t m = wave_min_u64(lmin);
            int v;
            if (m == kInfW) {  // new component: lowest vertex outside the forest
                v = (int)wave_min_u32((uint32_t)lfree);
                ++n_inf0;
            } else {
                const int l = __ffsll((unsigned long long)ballot(lmin == m)) - 1;
                v = 64 * (int)rlw((uint32_t)lt, l) + l;
                const int u = (int)rlw((uint32_t)lp, l);
                const uint32_t dd = kdiam(m);
                if (value(dd) != 0.0f) {  // (0, d) emitted only if d != 0 (ripser.cpp:741-748)
                    if (lane == 0) d0s[n_d0] = value(dd);
                    ++n_d0;
                }
                if (lane == 0) par[v] = (uint16_t)u;
            }
            if (lane == (v & 63)) intree |= MT(1) << (v >> 6);
            wave_lds_order();
#pragma unroll
            for (int t = 0; t < kWW; ++t) {
                const int w = 64 * t + lane;
                if (t < W && w < n && !((intree >> t) & MT(1)) && ((aw(v, t) >> lane) & 1ull)) {
                    const uint64_t k = wkey(d(v, w), v > w ? bin2(v) + w : bin2(w) + v);
                    if (k < best[t]) {
                        best[t] = k;
                        bp[t] = v;
                    }
                }
            }
        }
        wave_lds_order();
    }

    // ---- edges (i > j, d <= thr) in index order ----
    __device__ int edge_list() {
        const int lane = lane_id();
        uint32_t* edges = sp<uint32_t>(ly.edges);
        int off = 0;
        for (int i = 1; i < n; ++i)
            for (int w = 0; 64 * w < i; ++w) {
                uint64_t bits = uniw64(aw(i, w));  // one LDS word: uniform (scalar count below)
                const int lim = i - 64 * w;
                if (lim < 64) bits &= (1ull << lim) - 1ull;
                if ((bits >> lane) & 1ull) edges[off + mask_prefix(bits)] = pack_edge(i, 64 * w + lane);
                off += __popcll(bits);
            }
        wave_scratch_sync();
        return off;
    }

    // F-minimal cofacet of sigma (dim 1: edge a > b; dim 2: triangle a > b > c, packed sp_) over
    // the common-neighbour bitset cand: its key (kInf if none), packed vertices and added vertex.
    // Walking k downwards, the first k with all distances <= diam is the F-minimal cofacet
    // (largest index at the smallest diameter) and ends the walk (found); its distances to
    // a, b, c are returned for the apparent test.
    __device__ uint64_t min_cofacet(int dim, int a, int b, int c, uint32_t dsig, uint64_t sp_, const uint64_t* cand,
                                    uint64_t& bestp, int& bk, bool& found, uint32_t& hda, uint32_t& hdb,
                                    uint32_t& hdc, int* steps = nullptr) const {
        uint64_t best = kInfW;
        uint32_t bd = 0xFFFFFFFFu;
        found = false;
        bk = -1;
        bestp = 0;
        // candidates popped highest first, four per step so their distance reads are in flight
        // together (scratch reads: the latency, not the bandwidth, is what a lane waits for)
        int w = W - 1;
        uint64_t m = cand[W - 1];
        for (;;) {
            int kk[4];
            bool val[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                while (m == 0ull && w > 0) {
                    --w;
#pragma unroll
                    for (int u = 0; u < kWW; ++u)
                        if (u == w) m = cand[u];
                }
                val[j] = m != 0ull;
                const int bit = val[j] ? 63 - __clzll((long long)m) : 0;
                kk[j] = 64 * w + bit;
                if (val[j]) m &= ~(1ull << bit);
            }
            if (!val[0]) break;
            if (steps) ++*steps;
            uint32_t da[4], dbv[4], dc[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int k = val[j] ? kk[j] : kk[0];
                da[j] = d(a, k);
                dbv[j] = d(b, k);
                dc[j] = dim == 2 ? d(c, k) : 0u;
            }
            // walking k downwards, a later (smaller) k wins only with a strictly smaller diameter
            // (inserting a larger vertex gives the larger combinatorial index, i.e. the F-smaller
            // key at equal diameter): only (diameter, k) are tracked, the winner's key is built once
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                if (!val[j] || found) continue;
                const int k = kk[j];
                const uint32_t dk = max(max(da[j], dbv[j]), dc[j]);
                if (dk <= dsig) {
                    bd = dsig;
                    bk = k;
                    found = true;
                    hda = da[j];
                    hdb = dbv[j];
                    hdc = dc[j];
                } else if (dk < bd) {
                    bd = dk;
                    bk = k;
                }
            }
            if (found || !val[3]) break;
        }
        if (bk < 0) return kInfW;
        bestp = pinsert(dim + 1, sp_, bk);
        best = wkey(bd, pidx(dim + 2, bestp));
        return best;
    }

    // append a non-apparent column (lanes with `na`) to the scratch list
    // (the dim-1 list starts at entry 0, the dim-2 list at `base`: both are built before either
    // dimension is reduced)
    __device__ void na_append(int base, bool na, int& nna, uint64_t colkey, uint64_t tau, uint64_t tv, PT colp) {
        const uint64_t bal = ballot(na);
        if (na) {
            const int slot = base + nna + mask_prefix(bal);
            if (slot < ly.na_cap) {
                sp<uint64_t>(ly.na_key)[slot] = colkey;
                sp<uint64_t>(ly.na_tau)[slot] = tau;
                sp<uint64_t>(ly.na_tv)[slot] = tv;
                sp<PT>(ly.na_col)[slot] = colp;
            }
        }
        nna += __popcll(bal);
    }

    // ---- dim 1: one lane per column (non-tree edge) ----
    __device__ int pass_dim1(int n_edges) {
        const int lane = lane_id();
        const uint32_t* edges = sp<uint32_t>(ly.edges);
        uint16_t* mc_e = sp<uint16_t>(ly.mc_e);
        uint16_t* mc_t = sp<uint16_t>(ly.mc_t);
        int nna = 0;
        for (int base = 0; base < n_edges; base += kWave) {
            const int e = base + lane;
            bool na = false;
            uint64_t colkey = 0, best = kInfW, bestp = 0;
            PT colp = 0;
            uint64_t clr = ~0ull;  // NOMCT: the triangle this apparent pair clears
            if (e < n_edges) {
                const uint32_t ed = edges[e];
                const int i = (int)(ed >> VB), j = (int)(ed & VM);
                uint16_t mc = kMcNoneW;
                if (!is_tree(i, j)) {
                    const uint32_t dij = d(i, j);
                    colp = ed;
                    colkey = wkey(dij, bin2(i) + j);
                    uint64_t cand[kWW];
#pragma unroll
                    for (int w = 0; w < kWW; ++w) cand[w] = w < W ? (aw(i, w) & aw(j, w)) : 0ull;
                    bool found;
                    int bk;
                    uint32_t hda = 0, hdb = 0, hdc = 0;
                    best = min_cofacet(1, i, j, 0, dij, ed, cand, bestp, bk, found, hda, hdb, hdc);
                    if (best != kInfW) {
                        // apparent iff (i, j) is the F-max facet of its zero-persistence cofacet:
                        // the facets with k replacing a larger vertex must be strictly shorter
                        const bool app = found && (bk > i || hdb < dij) && (bk > j || hda < dij);
                        if (app) {
                            if constexpr (NOMCT) clr = pidx(3, bestp);
                            else at(mc_t, (uint32_t)pidx(3, bestp)) = kMcClearedW;  // clearing for dim 2
                        } else {
                            na = true;
                        }
                        mc = (uint16_t)bk;
                    }
                }
                at(mc_e, (uint32_t)(bin2(i) + j)) = mc;
            }
            if constexpr (NOMCT) {  // bitmap mark + its list entry (reset after the reductions)
                const uint64_t cbal = ballot(clr != ~0ull);
                if (clr != ~0ull) {
                    clear_mark(clr);
                    const int q = ncl + mask_prefix(cbal);
                    if (q < ly.na_cap) sp<CLT>(ly.cl_list)[q] = (CLT)clr;  // (reset: see reduce_finish)
                }
                ncl += __popcll(cbal);
            }
            // apparent pairs have zero persistence: nothing to emit
            na_append(0, na, nna, colkey, best, bestp, colp);
        }
        wave_scratch_sync();
        return nna;
    }

    // ---- dim 2: one lane per column (uncleared triangle), a per-lane work queue ----
    static constexpr int kStep = DGN_WIDE_STEP;  // candidates per walk step (distance reads in flight)
    // position of the r-th (0-based) set bit of x (r < popcount(x))
    __device__ static int select_bit(uint64_t x, int r) {
        int pos = 0;
#pragma unroll
        for (int sh = 32; sh >= 1; sh >>= 1) {
            const int cnt = __popcll(x & ((1ull << sh) - 1ull));
            const bool up = r >= cnt;
            r = up ? r - cnt : r;
            x = up ? x >> sh : x;
            pos += up ? sh : 0;
        }
        return pos;
    }
    // The triangles (a, b, c), c < b a common neighbour of the edge a > b, are dealt in edge-list
    // order from a wave-uniform cursor: a lane whose walk ended (zero-persistence cofacet found,
    // or candidates exhausted) takes the next triangle at once, so lanes never wait for the
    // longest walk of a round (10 A: 2.1 steps per column on average, 11 for the longest lane of
    // a 64-column round), and at any time the wave's lanes hold consecutive triangles -- mostly of
    // one or two edges, so their reads of rows a and b fall in a few lines (round 3 gave each
    // lane its own edge: 64 different rows a, b per load). A fresh triangle's clearing mark and
    // edge lengths are loaded together with its first candidates.
    __device__ int pass_dim2(int n_edges, int base) {
        [[maybe_unused]] const int lane = lane_id();
        const uint32_t* edges = sp<uint32_t>(ly.edges);
        uint16_t* mc_t = sp<uint16_t>(ly.mc_t);
        int nna = 0;
        // the cursor (uniform): edge ce = (ca > cb), word cw of its c < cb, the c's not yet dealt;
        // the edge list is read 64 entries at a time (lane i: entry eb0 + i) and the next batch
        // is prefetched when the cursor enters the current one, so advancing to an edge is a
        // readlane, not a dependent scratch load
        int ce = -1, ca = 0, cb = 0, cw = 0;
        uint64_t cm = 0;
        int eb0 = 0;
        uint32_t ebuf = lane < n_edges ? edges[lane] : 0u;
        uint32_t enext = kWave + lane < n_edges ? edges[kWave + lane] : 0u;
        int ea = 0, eb = 0;  // the lane's triangle's edge
        bool act = false, fresh = false;
        int c = 0, w = 0, bk = 0;
        uint64_t m = 0, tidx = 0;
        uint32_t bd = 0xFFFFFFFFu;  // diameter of the best cofacet of the lane's triangle so far
        uint32_t ds = 0, dab = 0, dac = 0, dbc = 0, hda = 0, hdb = 0, hdc = 0;
        PT colp = 0;
        bool found = false;
        for (;;) {
            // (1) lanes without a triangle take the next ones from the cursor, in order
            for (;;) {
                uint64_t need = ballot(!act);
                if (!need) break;
                while (cm == 0ull && ce < n_edges) {  // advance the cursor to the next word with a c
                    if (ce >= 0 && 64 * (cw + 1) < cb) {
                        ++cw;
                    } else {
                        if (++ce >= n_edges) break;
                        if (ce >= eb0 + kWave) {  // next batch (already in flight), prefetch the one after
                            eb0 += kWave;
                            ebuf = enext;
                            enext = eb0 + kWave + lane < n_edges ? edges[eb0 + kWave + lane] : 0u;
                        }
                        const uint32_t ed = rlw(ebuf, ce - eb0);
                        ca = (int)(ed >> VB);
                        cb = (int)(ed & VM);
                        cw = 0;
                    }
                    uint64_t mm = uniw64(aw(ca, cw) & aw(cb, cw));
                    const int lim = cb - 64 * cw;
                    if (lim < 64) mm &= (1ull << lim) - 1ull;
                    cm = mm;
                }
                if (cm == 0ull) break;  // every triangle dealt
                const int p = __popcll(cm), q = __popcll(need);
                const int r = mask_prefix(need);  // this lane's rank among the lanes to fill
                if (!act && r < p) {
                    c = 64 * cw + select_bit(cm, r);
                    ea = ca;
                    eb = cb;
                    act = fresh = true;
                }
                // drop the dealt c's (the lowest min(p, q) bits)
                cm = q >= p ? 0ull : cm & ~((1ull << select_bit(cm, q)) - 1ull);
            }
            if (fresh) {
                tidx = bin3(ea) + bin2(eb) + c;
                colp = ((PT)ea << (2 * VB)) | ((PT)eb << VB) | (PT)c;
                w = W - 1;
                m = aw(ea, w) & aw(eb, w) & aw(c, w);
                bd = 0xFFFFFFFFu;
                bk = -1;
                found = false;
            }
            if (!ballot(act)) break;
            bool na = false;
            uint64_t colkey = 0, ntau = kInfW, ntv = 0;
            PT ncolp = 0;
            if (act) {
                const int a = ea, b = eb;
                // (2) one step: up to kStep candidates, highest first
                int kk[kStep];
                bool val[kStep];
#pragma unroll
                for (int j = 0; j < kStep; ++j) {
                    while (m == 0ull && w > 0) {
                        --w;
                        m = aw(a, w) & aw(b, w) & aw(c, w);
                    }
                    val[j] = m != 0ull;
                    const int bit = val[j] ? 63 - __clzll((long long)m) : 0;
                    kk[j] = 64 * w + bit;
                    if (val[j]) m &= ~(1ull << bit);
                }
                uint32_t da[kStep], dbv[kStep], dc[kStep];
#pragma unroll
                for (int j = 0; j < kStep; ++j) {
                    const int k = val[j] ? kk[j] : c;
                    da[j] = d(a, k);
                    dbv[j] = d(b, k);
                    dc[j] = d(c, k);
                }
                bool cleared = false;
                if (fresh) {
                    if constexpr (NOMCT) cleared = is_cleared(tidx);
                    else cleared = at(mc_t, (uint32_t)tidx) == kMcClearedW;
                    dab = d(a, b);
                    dac = d(a, c);
                    dbc = d(b, c);
                    ds = max(max(dab, dac), dbc);
                    fresh = false;
                }
                bool done;
                if (cleared) {
                    // consumed: the entry leaves the complex non-cleared (NOMCT: the bitmap is reset
                    // from the clearing list after the reductions)
                    if constexpr (!NOMCT) at(mc_t, (uint32_t)tidx) = kMcNoneW;
                    done = true;
                } else {
                    // (diameter, k) only, as in min_cofacet: a smaller k wins only with a strictly
                    // smaller diameter; the winner's key is built when the walk ends
#pragma unroll
                    for (int j = 0; j < kStep; ++j) {
                        if (!val[j] || found) continue;
                        const int k = kk[j];
                        const uint32_t dk = max(max(da[j], dbv[j]), dc[j]);
                        if (dk <= ds) {
                            bd = ds;
                            bk = k;
                            found = true;
                            hda = da[j];
                            hdb = dbv[j];
                            hdc = dc[j];
                        } else if (dk < bd) {
                            bd = dk;
                            bk = k;
                        }
                    }
                    done = found || !val[kStep - 1];
                    if (done) {
                        // apparent iff (a, b, c) is the F-max facet of its zero-persistence cofacet
                        uint16_t mc = kMcNoneW;
                        uint64_t best = kInfW, bestp = 0;
                        if (bk >= 0) {
                            bestp = pinsert(3, colp, bk);
                            best = wkey(bd, pidx(4, bestp));
                            const bool app = found && (bk > a || max(max(hdb, hdc), dbc) < ds) &&
                                             (bk > b || max(max(hda, hdc), dac) < ds) &&
                                             (bk > c || max(max(hda, hdb), dab) < ds);
                            na = !app;
                            mc = (uint16_t)bk;
                        }
                        if constexpr (!NOMCT) at(mc_t, (uint32_t)tidx) = mc;
                        (void)mc;
                        colkey = wkey(ds, tidx);
                        ntau = best;
                        ntv = bestp;
                        ncolp = colp;
                    }
                }
                if (done) act = false;
            }
            na_append(base, na, nna, colkey, ntau, ntv, ncolp);
        }
        wave_scratch_sync();
        return nna;
    }

    // ---- non-apparent columns in Ripser's order: bitonic sort, key descending ----
    // dim 2 (`cleared`): columns whose triangle is the pivot of a reduced dim-1 column (clearing
    // marks, set after this list was built) get key 0 and sort last; returns the columns kept
    // the column arrays of one dimension (this wave's scratch from `base`)
    __device__ void na_arrays(int dim, int base, uint64_t*& K, uint64_t*& T, uint64_t*& V, PT*& Cc) const {
        (void)dim;
        K = sp<uint64_t>(ly.na_key) + base;
        T = sp<uint64_t>(ly.na_tau) + base;
        V = sp<uint64_t>(ly.na_tv) + base;
        Cc = sp<PT>(ly.na_col) + base;
    }
    __device__ int sort_na(int base, int cnt, bool cleared) {
        const int lane = lane_id();
        int N = 1;
        while (N < cnt) N <<= 1;
        uint64_t *K, *T, *V;
        PT* Cc;
        na_arrays(cleared ? 2 : 1, base, K, T, V, Cc);
        for (int i = cnt + lane; i < N; i += kWave) K[i] = 0ull;  // padding sorts last
        int kept = cnt;
        if (cleared) {
            const uint16_t* mc_t = sp<uint16_t>(ly.mc_t);
            for (int i0 = 0; i0 < cnt; i0 += kWave) {
                const int i = i0 + lane;
                bool cl = false;
                if (i < cnt) {
                    const uint64_t idx = ~K[i] & ((1ull << KS) - 1);
                    if constexpr (NOMCT) cl = is_cleared(idx);
                    else cl = at(mc_t, (uint32_t)idx) == kMcClearedW;
                    if (cl) K[i] = 0ull;
                }
                kept -= __popcll(ballot(cl));
            }
        }
        wave_scratch_sync();
        for (int k = 2; k <= N; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                for (int i = lane; i < N; i += kWave) {
                    const int l = i ^ j;
                    if (l > i) {
                        const uint64_t x = K[i], y = K[l];
                        if (((i & k) == 0) ? (x < y) : (x > y)) {
                            K[i] = y;
                            K[l] = x;
                            const uint64_t t0 = T[i], v0 = V[i];
                            const PT c0 = Cc[i];
                            T[i] = T[l];
                            V[i] = V[l];
                            Cc[i] = Cc[l];
                            T[l] = t0;
                            V[l] = v0;
                            Cc[l] = c0;
                        }
                    }
                }
                wave_scratch_sync();
            }
        return kept;
    }

    // ---- serially resolved pivots: open-addressing hash table (key 0 = empty) ----
    __device__ static uint32_t hmix(uint64_t k) {
        k ^= k >> 33;
        k *= 0xff51afd7ed558ccdull;
        k ^= k >> 33;
        return (uint32_t)k;
    }
    __device__ uint64_t hfind(uint64_t k) const {
        const int lane = lane_id();
        const uint64_t* HK = sp<uint64_t>(ly.h_key);
        const uint64_t* HM = sp<uint64_t>(ly.h_meta);
        const uint32_t mask = (uint32_t)ly.h_cap - 1u;
        const uint32_t base = hmix(k) & mask;
        for (int probe = 0; probe < ly.h_cap; probe += kWave) {
            const uint64_t x = HK[(base + (uint32_t)(probe + lane)) & mask];
            const uint64_t hit = ballot(x == k), emp = ballot(x == 0ull);
            const int fh = hit ? __ffsll((unsigned long long)hit) - 1 : kWave;
            const int fe = emp ? __ffsll((unsigned long long)emp) - 1 : kWave;
            if (fh < fe) return uniw64(HM[(base + (uint32_t)(probe + fh)) & mask]);
            if (fe < kWave) return kNoMetaW;
        }
        return kNoMetaW;
    }
    // insert k at `fslot`, the first empty slot of k's probe window as the column's last lookup
    // saw it (nothing was inserted since), or probe for one (fslot = ~0: that window was full). No
    // fence here: the caller's one fence covers this and the column's other stores
    __device__ bool hinsert(uint64_t k, uint64_t meta, int npiv, uint32_t fslot) {
        const int lane = lane_id();
        uint64_t* HK = sp<uint64_t>(ly.h_key);
        uint64_t* HM = sp<uint64_t>(ly.h_meta);
        const uint32_t mask = (uint32_t)ly.h_cap - 1u;
        const uint32_t base = hmix(k) & mask;
        if (npiv >= ly.na_cap) return false;
        uint32_t slot = fslot;
        for (int probe = 0; slot == ~0u && probe < ly.h_cap; probe += kWave) {
            const uint64_t x = HK[(base + (uint32_t)(probe + lane)) & mask];
            const uint64_t emp = ballot(x == 0ull);
            if (emp) slot = (base + (uint32_t)(probe + __ffsll((unsigned long long)emp) - 1)) & mask;
        }
        if (slot == ~0u) return false;
        if (lane == 0) {
            HK[slot] = k;
            HM[slot] = meta;
            sp<uint32_t>(ly.h_used)[npiv] = slot;
        }
        return true;
    }

    // Owner of the pivot tau in one round trip where possible: the first 64-slot window of the
    // pivot table (keys and metadata) and tau's edge lengths (lane p loads edge p) are loaded
    // together; a table hit returns its metadata (app = kNone). Otherwise the apparent owner: tau's
    // F-max facet f if tau is f's F-minimal cofacet (recorded by the lane-parallel pass; tree edges
    // and cleared triangles hold kMcNone), decided from the edge lengths already in registers and
    // one min-cofacet table read. Returns kNoMetaW when tau is not in the table.
    __device__ uint64_t lookup(int dim, uint64_t tau, uint64_t tv, PT& app, uint32_t& fslot) const {
        const int lane = lane_id();
        const uint64_t* HK = sp<uint64_t>(ly.h_key);
        const uint64_t* HM = sp<uint64_t>(ly.h_meta);
        const uint32_t mask = (uint32_t)ly.h_cap - 1u;
        const uint32_t slot = (hmix(tau) + (uint32_t)lane) & mask;
        const uint64_t hk = HK[slot];
        const uint64_t hm = HM[slot];
        const int nv = dim + 2;
        const int v0 = pv(tv, nv - 1), v1 = pv(tv, nv - 2), v2 = pv(tv, nv - 3), v3 = nv == 4 ? pv(tv, 0) : 0;
        // edge p of tau (vertices descending v0 > v1 > ...): (s, t) from nibble tables
        const int np = nv == 4 ? 6 : 3;
        const int lp = lane < np ? lane : 0;
        const int ps = (int)(((nv == 4 ? 0x211000u : 0x100u) >> (4 * lp)) & 0xFu);
        const int pt = (int)(((nv == 4 ? 0x332321u : 0x221u) >> (4 * lp)) & 0xFu);
        const int va = ps == 0 ? v0 : (ps == 1 ? v1 : v2);
        const int vb = pt == 1 ? v1 : (pt == 2 ? v2 : v3);
        const uint32_t dl = d(va, vb);
        const uint64_t hit = ballot(hk == tau), emp = ballot(hk == 0ull);
        const int fh = hit ? __ffsll((unsigned long long)hit) - 1 : kWave;
        const int fe = emp ? __ffsll((unsigned long long)emp) - 1 : kWave;
        app = kNoneP;
        fslot = ~0u;
        if (fh < fe) return rlw64(hm, fh);
        if (fe == kWave) {  // the window was full: probe on (rare at load factor <= 1/2)
            const uint64_t m = hfind(tau);
            if (m != kNoMetaW) return m;
        } else {
            fslot = (hmix(tau) + (uint32_t)fe) & mask;
        }
        uint32_t dd[4][4];
        if (nv == 4) {
            dd[0][1] = rlw(dl, 0);
            dd[0][2] = rlw(dl, 1);
            dd[0][3] = rlw(dl, 2);
            dd[1][2] = rlw(dl, 3);
            dd[1][3] = rlw(dl, 4);
            dd[2][3] = rlw(dl, 5);
        } else {
            dd[0][1] = rlw(dl, 0);
            dd[0][2] = rlw(dl, 1);
            dd[1][2] = rlw(dl, 2);
        }
        const int v[4] = {v0, v1, v2, v3};
        uint64_t bestk = 0, bestf = 0;
        int drop = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {  // facet without v[t]
            if (t >= nv) break;
            uint32_t diam = 0;
            uint64_t f = 0;
#pragma unroll
            for (int s2 = 0; s2 < 4; ++s2) {
                if (s2 >= nv || s2 == t) continue;
                f = (f << VB) | (uint64_t)v[s2];
#pragma unroll
                for (int u = s2 + 1; u < 4; ++u)
                    if (u < nv && u != t) diam = max(diam, dd[s2][u]);
            }
            const uint64_t kk = wkey(diam, pidx(nv - 1, f));
            if (kk > bestk) {
                bestk = kk;
                bestf = f;
                drop = t;
            }
        }
        const int vd = drop == 0 ? v0 : (drop == 1 ? v1 : (drop == 2 ? v2 : v3));
        if constexpr (NOMCT) {
            if (dim == 2) {
                // tau = f u {vd} with diam f = diam tau (f is its F-max facet), so vd is a
                // zero-persistence cofacet vertex of f, and tau is f's F-minimal cofacet -- the
                // pass_dim2 walk's winner -- iff no vertex x > vd, x not in f, has every distance
                // to f within diam f (the all-ones diagonal excludes f's vertices). Decided from
                // f's three rows (coalesced), words from vd's on; such a pair is always apparent
                // (diam tau = diam f and f its F-max facet), and a cleared f (a dim-1 pivot) is
                // never in one, so no min-cofacet table or clearing state is needed. (Loading the
                // four rows of tau together with the table window instead -- one round trip less
                // -- measured slower: 24 loads and 51 spilled VGPRs per lookup)
                const int fa = pv(bestf, 2), fb = pv(bestf, 1), fc = pv(bestf, 0);
                const uint32_t fd = kdiam(bestk);
                const int t0 = vd >> 6;
                uint32_t ra[KW], rb[KW], rc[KW];
                bool later = false;
                if constexpr (PRE) {  // 8-byte rows: packed vectors (prow)
                    prow(fa, ra);
                    prow(fb, rb);
                    prow(fc, rc);
#pragma unroll
                    for (int t = 0; t < KW; ++t) {
                        const int x = slot_x(t, lane);
                        later |= x > vd && x < n && max(max(ra[t], rb[t]), rc[t]) <= fd;
                    }
                } else {
#pragma unroll
                    for (int t = 0; t < KW; ++t) {
                        if (t < t0 || t >= W) continue;
                        const uint32_t x = (uint32_t)min(64 * t + lane, n - 1);
                        ra[t] = drow(fa, x);
                        rb[t] = drow(fb, x);
                        rc[t] = drow(fc, x);
                    }
#pragma unroll
                    for (int t = 0; t < KW; ++t) {
                        if (t < t0 || t >= W) continue;
                        const int x = 64 * t + lane;
                        later |= x > vd && x < n && max(max(ra[t], rb[t]), rc[t]) <= fd;
                    }
                }
                if (!ballot(later)) app = (PT)bestf;
                return kNoMetaW;
            }
        }
        const uint16_t m = dim == 1 ? at(mce, (uint32_t)pidx(2, bestf))
                                     : at(sp<uint16_t>(ly.mc_t), (uint32_t)pidx(3, bestf));
        if (uniw(m) == (uint32_t)vd) app = (PT)bestf;
        return kNoMetaW;
    }

    // ---- the working column's V list: registers up to 64 entries, then scratch (vlist[0..v),
    // packed simplices, no small cap) ----
    __device__ int v_find(PT x, int v) const {
        const int lane = lane_id();
        const PT* VL = sp<PT>(ly.vlist);
        for (int base = 0; base < v; base += kWave) {
            const PT y = base + lane < v ? VL[base + lane] : kNoneP;
            const uint64_t bal = ballot(y == x);
            if (bal) return base + __ffsll((unsigned long long)bal) - 1;
        }
        return -1;
    }
    __device__ bool v_toggle(PT x, int& v) {  // V ^= {x}; false on overflow
        const int lane = lane_id();
        if (VREG && !vspill) {
            // register list: no memory round trip (find by ballot, remove by moving the last entry)
            const uint64_t hit = ballot(vreg == x) & lanes_below_w(v);
            if (hit) {
                const int pos = __ffsll((unsigned long long)hit) - 1;
                const PT last = rlp(vreg, v - 1);
                if (lane == pos) vreg = last;
                v = v - 1;
                return true;
            }
            if (v < kWave) {
                if (lane == v) vreg = x;
                v = v + 1;
                return true;
            }
            // a 65th entry: the list moves to scratch
            sp<PT>(ly.vlist)[lane] = vreg;
            vspill = true;
            wave_scratch_sync();
        }
        PT* VL = sp<PT>(ly.vlist);
        const int pos = v_find(x, v);
        if (pos >= 0) {
            if (pos != v - 1) {
                const PT last = unip(VL[v - 1]);
                if (lane == 0) VL[pos] = last;
            }
            v = v - 1;
        } else {
            if (v >= ly.vl_cap) return false;
            if (lane == 0) VL[v] = x;
            v = v + 1;
        }
        wave_scratch_sync();  // the list (scratch) is read by every lane next
        return true;
    }

    // PRE rows as packed u16 vectors (row stride ns, a multiple of 4): KW 2 -- one dword per lane,
    // vertices 2k, 2k + 1; KW 4 -- one dwordx2, 4k .. 4k + 3; KW 6 -- a dwordx2 (4k .. 4k + 3) and a
    // dword (256 + 2k, 256 + 2k + 1). Lanes past n read the next row or the complex's padding.
    __device__ static int slot_x(int t, int k) {
        if constexpr (KW == 2) return 2 * k + t;
        else if constexpr (KW == 4) return 4 * k + t;
        else return t < 4 ? 4 * k + t : 256 + 2 * k + (t - 4);
    }
    __device__ void prow(int a, uint32_t (&out)[KW]) const {
        static_assert(!PRE || KW == 2 || KW == 4 || KW == 6, "prewalked instantiations: 2, 4, 6 words");
        const int k = lane_id();
        const uint16_t* R = reinterpret_cast<const uint16_t*>(dm) + (uint32_t)a * (uint32_t)ns;
        if constexpr (KW == 2) {
            const uint32_t w = at(reinterpret_cast<const uint32_t*>(R), (uint32_t)k);
            out[0] = w & 0xFFFFu;
            out[1] = w >> 16;
        } else {
            const uint64_t w = at(reinterpret_cast<const uint64_t*>(R), (uint32_t)k);
#pragma unroll
            for (int q = 0; q < 4; ++q) out[q] = (uint32_t)(w >> (16 * q)) & 0xFFFFu;
            if constexpr (KW == 6) {
                const uint32_t w2 = at(reinterpret_cast<const uint32_t*>(R), 128u + (uint32_t)k);
                out[4] = w2 & 0xFFFFu;
                out[5] = w2 >> 16;
            }
        }
    }

    // Pivot of sum(delta s, s in V) above `floor` (the previous pivot): lane k evaluates the
    // cofacets s u {x}, x = 64 t + k; a cofacet arises once per facet in V; the multiplicity of
    // the minimum is summed over lanes (a lane can meet it from several words). Even: raise the
    // floor and repeat. Returns kInf for the zero column; tv = packed pivot (in: the floor's).
    __device__ uint64_t pivot_of_V(int dim, int v, uint64_t floor, uint64_t& tv) {
        const int k = lane_id();
        if constexpr (PACKKEY) floor = pkey(kdiam(floor), tv);  // tv: the floor's packed tuple
        const PT* VL = sp<PT>(ly.vlist);
        // V entries and their diameters live in registers (lane i: entry base + i), read back with
        // readlane, so an entry costs no dependent load; the first 64 stay across floor rounds
        const PT vl0 = k < v ? ((VREG && !vspill) ? vreg : VL[k]) : PT(0);
        const uint32_t vd0 = k < v ? sdiam(dim, vl0) : 0u;
        for (;;) {
            uint64_t lmin = kInfW, lp = 0;
            int lcnt = 0;
            auto eval = [&](PT s, uint32_t ds) {
                const int a = dim == 1 ? pv(s, 1) : pv(s, 2);
                const int b = dim == 1 ? pv(s, 0) : pv(s, 1);
                const int c = pv(s, 0);
                // every word's row reads issued before any is used (coalesced rows a, b, c)
                uint32_t da[KW], db[KW], dc[KW];
                if constexpr (PRE) {
                    // PRE (8-byte rows): packed u16 vectors, slot t of lane k is vertex slot_x(t, k)
                    // -- a third of the per-word u16 loads
                    prow(a, da);
                    prow(b, db);
                    if (dim == 2) prow(c, dc);
                    else
#pragma unroll
                        for (int t = 0; t < KW; ++t) dc[t] = 0u;
                } else
#pragma unroll
                for (int t = 0; t < KW; ++t) {
                    const int x = min(64 * t + k, n - 1);
                    if constexpr (PACKKEY) {
                        da[t] = drow(a, (uint32_t)x);
                        db[t] = drow(b, (uint32_t)x);
                        dc[t] = dim == 2 ? drow(c, (uint32_t)x) : 0u;
                    } else {
                        da[t] = d(a, x);
                        db[t] = d(b, x);
                        dc[t] = dim == 2 ? d(c, x) : 0u;
                    }
                }
#pragma unroll
                for (int t = 0; t < KW; ++t) {
                    if (!PRE && t >= W) break;
                    const int x = PRE ? slot_x(t, k) : 64 * t + k;
                    const uint32_t dd = max(max(ds, dc[t]), max(da[t], db[t]));
                    const uint64_t p = pinsert(dim + 1, s, x);
                    const uint64_t kk = PACKKEY ? pkey(dd, p) : wkey(dd, pidx(dim + 2, p));
                    // x is a common neighbour iff every distance to s is within the threshold (the
                    // all-ones diagonal rules out s's own vertices; lanes past n read row n - 1)
                    if (x < n && dd <= thrc && kk > floor) {
                        if (kk < lmin) {
                            lmin = kk;
                            lcnt = 1;
                            lp = p;
                        } else if (kk == lmin) {
                            ++lcnt;
                        }
                    }
                }
            };
            for (int base = 0; base < v; base += kWave) {
                PT vl = vl0;
                uint32_t vd = vd0;
                if (base > 0) {
                    vl = base + k < v ? VL[base + k] : PT(0);
                    vd = base + k < v ? sdiam(dim, vl) : 0u;
                }
                const int cnt = v - base < kWave ? v - base : kWave;
                int i = 0;
#if DGN_PV_UNROLL >= 4
                for (; i + 3 < cnt; i += 4) {  // four entries' distance reads in flight together
                    eval(rlp(vl, i), rlw(vd, i));
                    eval(rlp(vl, i + 1), rlw(vd, i + 1));
                    eval(rlp(vl, i + 2), rlw(vd, i + 2));
                    eval(rlp(vl, i + 3), rlw(vd, i + 3));
                }
#endif
                for (; i + 1 < cnt; i += 2) {  // two entries' distance reads in flight together
                    eval(rlp(vl, i), rlw(vd, i));
                    eval(rlp(vl, i + 1), rlw(vd, i + 1));
                }
                if (i < cnt) eval(rlp(vl, i), rlw(vd, i));
            }
            const uint64_t m = wave_min_u64(lmin);
            if (m == kInfW) return kInfW;
            const int cnt = (int)wave_sum_u32(lmin == m ? (uint32_t)lcnt : 0u);
            if (cnt & 1) {
                const int l = __ffsll((unsigned long long)ballot(lmin == m)) - 1;
                tv = rlw64(lp, l);
                if constexpr (PACKKEY) return wkey((uint32_t)(m >> PKS), pidx(dim + 2, tv));
                return m;
            }
            floor = m;
        }
    }

    // ---- the non-apparent columns of one dimension, in Ripser's order ----
    // the next power of two >= x (the bitonic sort's padded length)
    __device__ static int pow2ceil(int x) {
        int N = 1;
        while (N < x) N <<= 1;
        return N;
    }
    __device__ void reduce(int dim, int nna, int base) {
        const int lane = lane_id();
        if (base + pow2ceil(nna) > ly.na_cap) {
            err |= kENA;
            return;
        }
        nna = sort_na(base, nna, dim == 2);
        uint64_t *K, *T, *V;
        PT* Cc;
        na_arrays(dim, base, K, T, V, Cc);
        PT* vstore = sp<PT>(ly.vstore);
        float2* pairs = sp<float2>(dim == 1 ? ly.p1 : ly.p2);
        int& np = dim == 1 ? n_p1 : n_p2;
        int npiv = 0;
        int64_t vused = 0;
        // the next column's record is loaded while this one is reduced (its load is not on the chain)
        uint64_t nK = 0, nT = 0, nV = 0;
        PT nC = 0;
        if (nna > 0) {
            nK = K[0];
            nT = T[0];
            nV = V[0];
            nC = Cc[0];
        }
        for (int ci = 0; ci < nna && err == 0u; ++ci) {
            const uint64_t colkey = uniw64(nK);
            uint64_t tau = uniw64(nT);
            uint64_t tv = uniw64(nV);
            const PT cp = unip(nC);
            if (ci + 1 < nna) {
                nK = K[ci + 1];
                nT = T[ci + 1];
                nV = V[ci + 1];
                nC = Cc[ci + 1];
            }
            const uint32_t birth = kdiam(colkey);
            PT app;
            uint32_t fslot;
            uint64_t meta = lookup(dim, tau, tv, app, fslot);
            int v = 0;  // 0 = lazy: V == {this column}
            vspill = !VREG;
            if (meta != kNoMetaW || app != kNoneP) {
                v_toggle(cp, v);
                int64_t guard = 0;
                for (;;) {
                    bool ok = true;
                    if (app != kNoneP) {
                        ok = v_toggle(app, v);
                    } else if (meta & kLazyW) {
                        ok = v_toggle((PT)(meta & ~kLazyW), v);
                    } else {
                        const int64_t off = (int64_t)(meta >> kMetaLenBits);
                        const int len = (int)(meta & ((1ull << kMetaLenBits) - 1));
                        for (int t0 = 0; t0 < len && ok; t0 += kWave) {
                            const PT w = t0 + lane < len ? vstore[off + t0 + lane] : PT(0);
                            const int cnt = len - t0 < kWave ? len - t0 : kWave;
                            for (int u = 0; u < cnt && ok; ++u) ok = v_toggle(rlp(w, u), v);
                        }
                    }
                    if (!ok) {
                        err |= kEWork;
                        break;
                    }
                    tau = v > 0 ? pivot_of_V(dim, v, tau, tv) : kInfW;
                    if (tau == kInfW) break;  // zero column: essential class, not emitted
                    meta = lookup(dim, tau, tv, app, fslot);
                    if (meta == kNoMetaW && app == kNoneP) break;  // tau is this column's pivot
                    if (++guard > ly.guard) {
                        err |= kEGuard;
                        break;
                    }
                }
                if (err || tau == kInfW) continue;
            }
            const uint32_t death = kdiam(tau);
            if (value(death) > value(birth)) {
                if (lane == 0 && np < ly.p_cap) pairs[np] = make_float2(value(birth), value(death));
                ++np;
            }
            if (dim == 1) {  // clearing: tau's column is zero in dim 2 (reset after the dim-2 sort)
                const uint64_t ti = pidx(3, tv);
                if (lane == 0) {
                    if constexpr (NOMCT) clear_mark(ti);
                    else at(sp<uint16_t>(ly.mc_t), (uint32_t)ti) = kMcClearedW;
                    if (!PRE || ncl < ly.na_cap) sp<CLT>(ly.cl_list)[ncl] = (CLT)ti;
                }
                ++ncl;
            }
            uint64_t m;
            if (v == 0) {
                m = kLazyW | cp;
            } else {
                if ((int64_t)vused + v > ly.vs_cap) {
                    err |= kER;
                    break;
                }
                if (!VREG || vspill) {
                    const PT* VL = sp<PT>(ly.vlist);
                    for (int t = lane; t < v; t += kWave) vstore[vused + t] = VL[t];
                } else if (lane < v) {
                    vstore[vused + lane] = vreg;
                }
                m = ((uint64_t)vused << kMetaLenBits) | (uint64_t)v;
                vused += v;
            }
            if (!hinsert(tau, m, npiv, fslot)) {
                err |= kEPiv;
                break;
            }
            ++npiv;
            // one fence for the column's stores (V store, pivot table, pair, clearing mark): the next
            // lookups and owner toggles (other lanes) read them
            wave_scratch_sync();
        }
        wave_scratch_sync();
        // empty the pivot table for the next dimension / complex
        uint64_t* HK = sp<uint64_t>(ly.h_key);
        const uint32_t* used = sp<uint32_t>(ly.h_used);
        for (int i = lane; i < npiv; i += kWave) HK[used[i]] = 0ull;
        wave_scratch_sync();
    }

    // ---- statistics (betti_features.cpp:24-55, 87-98; utils/math.hpp:9-28) + outputs ----
    // true when the complex's outputs were written (false: listed for the retry launch, or an
    // error with NaN outputs)
    __device__ bool finish(int64_t gi, double weight) {
        const int lane = lane_id();
        double* feat = bl.features ? bl.features + 35 * gi : nullptr;
        if (n_p1 > ly.p_cap || n_p2 > ly.p_cap) err |= kEPairs;
        if (err && bl.retry_list && (err & kECapacity) == err) {
            // workspace overflow: listed for the capacity-retry launch (betti_wide_layout big),
            // which writes this complex's outputs
            if (lane == 0) bl.retry_list[atomicAdd(bl.retry_len, 1u)] = (int32_t)gi;
            return false;
        }
        if (err) {
            if (lane == 0) atomicOr(bl.error_flag, err);
            if (feat && lane < 35) feat[lane] = __builtin_nan("");
            if (bl.counts && lane < 4) bl.counts[4 * gi + lane] = -1;
            return false;
        }
        const float* d0s = d0p;
        const float2* P1 = sp<float2>(ly.p1);
        const float2* P2 = sp<float2>(ly.p2);
        const double myval = betti_stats35(d0s, n_d0, P1, n_p1, P2, n_p2, weight);
        if (feat && lane < 35) feat[lane] = myval;
        if (bl.pairs_out) {
            float2* po = reinterpret_cast<float2*>(bl.pairs_out) + gi * 3 * bl.pair_cap;
            for (int i = lane; i < n_d0 && i < bl.pair_cap; i += kWave) po[i] = make_float2(0.0f, d0s[i]);
            for (int i = lane; i < n_p1 && i < bl.pair_cap; i += kWave) po[bl.pair_cap + i] = P1[i];
            for (int i = lane; i < n_p2 && i < bl.pair_cap; i += kWave) po[2 * bl.pair_cap + i] = P2[i];
        }
        if (bl.counts && lane == 0) {
            bl.counts[4 * gi + 0] = n_d0;
            bl.counts[4 * gi + 1] = n_inf0;
            bl.counts[4 * gi + 2] = n_p1;
            bl.counts[4 * gi + 3] = n_p2;
        }
        return true;
    }

    // Phase 1, with the workgroup's adjacency buffer held (betti_wide_body): the matrix and the
    // bitsets, the forest, the edge list and both lane-parallel (apparent) passes; the dim-2 pass
    // runs before the dim-1 reduction, so the columns the latter clears (their triangles are dim-1
    // pivots) are dropped from the dim-2 list when it is sorted
    int nna1 = 0, nna2 = 0, base2 = 0, ncl = 0;
    __device__ void apparent(int64_t gi, int64_t slot) {
        load(gi, slot);
        if (GIANT && err) return;  // outside the envelope: NaN outputs and the flag (finish)
        if constexpr (PRE) {
            apparent_from_walk(slot);
            return;
        }
        prim();
        const int n_edges = edge_list();
        nna1 = pass_dim1(n_edges);
        base2 = pow2ceil(nna1);
        nna2 = pass_dim2(n_edges, base2);
    }
    // PRE: the walk pass's lists into this wave's column arrays (dim 1 at 0, dim 2 at base2) with
    // their keys, initial pivots and cofacet tuples (the diameters from the matrix); the triangles the
    // dim-1 apparent pairs clear marked in the bitmap first, and dropped from the dim-2 list (most of
    // it at 10 A) instead of being sorted
    __device__ void apparent_from_walk(int64_t slot) {
        const int lane = lane_id();
        const WalkOut& wo = bl.walk;
        const uint32_t* meta = wo.meta + 8 * slot;
        n_d0 = (int)uniw(meta[kWmD0]);
        n_inf0 = (int)uniw(meta[kWmInf0]);
        const int n1 = (int)uniw(meta[kWmNa1]), ncw = (int)uniw(meta[kWmCl]), nw = (int)uniw(meta[kWmNa2]);
        if (n1 > wo.cap1 || ncw > wo.cap1 || nw > wo.cap || pow2ceil(n1) + pow2ceil(nw) > ly.na_cap) {
            err |= kENA;  // a list that overflowed: capacity retry
            return;
        }
        const uint32_t* CL = wo.cl + slot * (int64_t)wo.cap1;
        for (int i = lane; i < ncw; i += kWave) clear_mark(CL[i]);
        uint64_t* K = sp<uint64_t>(ly.na_key);
        uint64_t* T = sp<uint64_t>(ly.na_tau);
        uint64_t* V = sp<uint64_t>(ly.na_tv);
        PT* Cc = sp<PT>(ly.na_col);
        const uint64_t* E1 = wo.e1 + slot * (int64_t)wo.cap1;
        for (int i = lane; i < n1; i += kWave) {
            const uint64_t e = E1[i];
            const uint32_t ed = (uint32_t)(e & ((1u << 18) - 1u));
            const int bk = (int)((e >> 18) & VM);
            const uint32_t bd = (uint32_t)(e >> 27);
            const int a = (int)(ed >> VB), b = (int)(ed & VM);
            const uint64_t bestp = pinsert(2, ed, bk);
            K[i] = wkey(d(a, b), bin2(a) + b);
            T[i] = wkey(bd, pidx(3, bestp));
            V[i] = bestp;
            Cc[i] = (PT)ed;
        }
        nna1 = n1;
        base2 = pow2ceil(n1);
        wave_scratch_sync();  // the marks (L2 atomics) before the tests below
        const uint64_t* E = wo.ent + slot * (int64_t)wo.cap;
        nna2 = 0;
        for (int i0 = 0; i0 < nw; i0 += kWave) {
            const int i = i0 + lane;
            const uint64_t e = i < nw ? E[i] : 0ull;
            const uint32_t colp = (uint32_t)(e & ((1u << 27) - 1u));
            const uint32_t ti = (uint32_t)pidx(3, colp);
            const bool keep = i < nw && !is_cleared(ti);
            const uint64_t kb = ballot(keep);
            if (keep) {
                const int q = base2 + nna2 + mask_prefix(kb);
                const int bk = (int)((e >> 27) & VM);
                const uint32_t bd = (uint32_t)(e >> 36);
                const uint64_t bestp = pinsert(3, colp, bk);
                K[q] = wkey(sdiam(2, colp), ti);
                T[q] = wkey(bd, pidx(4, bestp));
                V[q] = bestp;
                Cc[q] = (PT)colp;
            }
            nna2 += __popcll(kb);
        }
        wave_scratch_sync();
    }
    // Phase 2, from scratch alone (no LDS): the two reductions, the statistics and the outputs.
    // True when the complex's outputs were written.
    __device__ bool reduce_finish(int64_t gi, double weight) {
        reduce(1, nna1, 0);
        if (err == 0u) reduce(2, nna2, base2);
        // the dim-1 clearing marks were read by the dim-2 sort; reset them for the next complex
        // (every other min-cofacet entry a later complex reads is rewritten by its dim-2 pass)
        const CLT* cl = sp<CLT>(ly.cl_list);
        if constexpr (GIANT) {
            // every set bit of the bitmap is listed (ncl <= the edges < 2^20 <= na_cap)
            for (int i = lane_id(); i < ncl && i < ly.na_cap; i += kWave) clbits()[cl[i] >> 5] = 0u;
        } else if constexpr (PRE) {
            // every set bit of the bitmap is listed (a word shared by two entries is zeroed twice)
            const int64_t words = ((int64_t)c2i(n) * (n - 2) / 3 + 31) / 32 + 1;
            const int ncw = (int)uniw(bl.walk.meta[8 * wslot + kWmCl]);
            if (ncl > ly.na_cap || ncw > bl.walk.cap1) {
                for (int64_t i = lane_id(); i < words; i += kWave) at(clbits(), (uint32_t)i) = 0u;
            } else {
                const uint32_t* CL = bl.walk.cl + wslot * (int64_t)bl.walk.cap1;
                for (int i = lane_id(); i < ncl; i += kWave) at(clbits(), cl[i] >> 5) = 0u;
                for (int i = lane_id(); i < ncw; i += kWave) at(clbits(), CL[i] >> 5) = 0u;
            }
        } else {
            uint16_t* mc_t = sp<uint16_t>(ly.mc_t);
            for (int i = lane_id(); i < ncl; i += kWave) at(mc_t, cl[i]) = kMcNoneW;
        }
        wave_scratch_sync();
        const bool ok = finish(gi, weight);
        wave_scratch_sync();
        return ok;
    }
};

template <int KW, int MODE, bool PRE = false>
__device__ __forceinline__ void betti_wide_body(const BettiLaunch& bl, const WideLayout& ly) {
    // dynamic LDS (wide_lds_bytes), one buffer per workgroup of kWideWaves waves: the buffer token
    // (u64), the adjacency [nmax][ceil(nmax / 64)] u64 and the forest parents [nmax] u16 (HUGE:
    // the parents only; the adjacency lives in each wave's scratch at ly.adj). A wave holds the
    // buffer from its complex's load through the two apparent passes, then reduces from scratch
    // alone while the other wave loads its next complex: twice the waves per CU for the LDS of one
    // complex (the reductions, about half of a 10 A complex's time, read no LDS).
    extern __shared__ uint64_t wide_lds[];
    constexpr bool kHugeMode = MODE == kHuge || MODE == kGiant;
    const int64_t ww = (ly.nmax + 63) / 64;
    const int lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
    const int64_t slot = (int64_t)blockIdx.x * kWideWaves + w;
    uint32_t* tok = reinterpret_cast<uint32_t*>(wide_lds);
    if (threadIdx.x == 0) *tok = 0u;  // the buffer starts free (the one workgroup barrier)
    __syncthreads();
    if (slot >= ly.slots) return;  // the last workgroup of an odd wave count
    uint64_t* lds = wide_lds + 1;
    uint8_t* scr = ly.base + slot * ly.total;
    uint64_t* adj = kHugeMode ? reinterpret_cast<uint64_t*>(scr + ly.adj) : lds;
    uint16_t* par = reinterpret_cast<uint16_t*>(kHugeMode ? lds : lds + ly.nmax * ww);
    const int64_t total = (int64_t)*bl.wide_len;
    for (;;) {
        // wave-uniform dequeue without a branch on the lane (see betti_kernels.hip): every lane adds
        // (lane == 0), lane 0's ticket goes to an SGPR
        const uint32_t ticket = atomicAdd(bl.wide_queue, lane == 0 ? 1u : 0u);
        const int64_t wi = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)ticket, 0);
        if (wi >= total) break;
        const int64_t gi = (int64_t)(int32_t)uniw((uint32_t)bl.wide_list[wi]);
        const int n = (int)uniw((uint32_t)bl.npoints[gi]);
        // complexes above kWideRegular points never reach the regular launch (the bucket pass lists
        // them for the rank-coded retry launch); a larger one here is outside the layout
        if (n > ly.nmax) {
            if (lane == 0) atomicOr(bl.error_flag, kEPoints);
            if (bl.features && lane < 35) bl.features[35 * gi + lane] = __builtin_nan("");
            if (bl.counts && lane < 4) bl.counts[4 * gi + lane] = -1;
        } else {
            WideCx<KW, MODE, PRE> cx{bl, ly, adj, par, scr, n, (n + 63) / 64, bl.thr, 0u, 0, 0, 0, 0};
            if (MODE != kF32) cx.vals = bl.rank_sorted + wi * bl.rank_stride;
            cx.wslot = wi;
            cx.dm = scr + ly.D;
            cx.ns = n;
            cx.mce = reinterpret_cast<uint16_t*>(scr + ly.mc_e);
            cx.d0p = reinterpret_cast<float*>(scr + ly.d0);
            // take the buffer: every lane tries the same compare-and-swap, the wave holds it when one
            // of its lanes won (a uniform ballot; no branch on the lane, see the dequeue)
            for (;;) {
                const uint32_t prev = atomicCAS(tok, 0u, 1u);
                if (ballot(prev == 0u)) break;
                __builtin_amdgcn_s_sleep(4);
            }
            cx.apparent(gi, wi);
            wave_scratch_sync();  // every LDS access of the apparent phase done
            *tok = 0u;            // release (every lane stores the same word)
            // dgn_debug_retry_count counts the complexes a retry launch reduced successfully
            const bool ok = cx.reduce_finish(gi, bl.weight ? bl.weight[gi] : 1.0);
            if (ok && bl.retried && lane == 0) atomicAdd(bl.retried, 1u);
        }
    }
}

template <int KW, int MODE>
__global__ __launch_bounds__(kWave * kWideWaves) void betti_wide_kernel(BettiLaunch bl, WideLayout ly) {
    betti_wide_body<KW, MODE>(bl, ly);
}
#ifndef DGN_WIDE_C16_WAVES
#define DGN_WIDE_C16_WAVES 5  // waves per SIMD the u16-code instantiations are compiled for
#endif
// the u16-code instantiations (the 10 A path) with a register budget for DGN_WIDE_C16_WAVES waves
// per SIMD: resident waves are what this latency-bound kernel scales with
// After the walk pass (u16 codes): the reductions, the statistics and the outputs only, from the
// walk pass's per-complex outputs and this wave's scratch -- no LDS, so residency is set by registers
template <int KW>
__device__ __forceinline__ void betti_reduce_body(const BettiLaunch& bl, const WideLayout& ly) {
    const int lane = lane_id();
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
    const int64_t slot = (int64_t)blockIdx.x * kWideWaves + w;
    if (slot >= ly.slots) return;
    uint8_t* scr = ly.base + slot * ly.total;
    const int64_t total = (int64_t)*bl.wide_len;
    for (;;) {
        const uint32_t ticket = atomicAdd(bl.wide_queue, lane == 0 ? 1u : 0u);  // as betti_wide_body
        const int64_t wi = (int64_t)(uint32_t)__builtin_amdgcn_readlane((int)ticket, 0);
        if (wi >= total) break;
        const int64_t gi = (int64_t)(int32_t)uniw((uint32_t)bl.wide_list[wi]);
        const int n = (int)uniw((uint32_t)bl.npoints[gi]);
        if (n > ly.nmax) {
            if (lane == 0) atomicOr(bl.error_flag, kEPoints);
            if (bl.features && lane < 35) bl.features[35 * gi + lane] = __builtin_nan("");
            if (bl.counts && lane < 4) bl.counts[4 * gi + lane] = -1;
            continue;
        }
        WideCx<KW, kC16, true> cx{bl, ly, nullptr, nullptr, scr, n, (n + 63) / 64, bl.thr, 0u, 0, 0, 0, 0};
        cx.vals = bl.rank_sorted + wi * bl.rank_stride;
        cx.wslot = wi;
        cx.dm = reinterpret_cast<const uint8_t*>(bl.walk.dmat + wi * bl.walk.dstride);
        cx.ns = (n + 3) & ~3;
        cx.mce = bl.walk.mce + wi * bl.walk.mstride;
        cx.d0p = bl.walk.d0 + wi * bl.walk.d0stride;
        cx.apparent(gi, wi);
        const bool ok = cx.reduce_finish(gi, bl.weight ? bl.weight[gi] : 1.0);
        if (ok && bl.retried && lane == 0) atomicAdd(bl.retried, 1u);
    }
}
#ifndef DGN_WIDE_PRE_WAVES
#define DGN_WIDE_PRE_WAVES 8  // waves per SIMD of the reduction-only (prewalked) instantiations (A/B at 10 A, 128 structures: 5 / 6 / 8 = 48.9 / 51.7 / 50.4; with packed rows 6 / 7 / 8 = 53.6-53.9 / 53.3-54.0 / 55.2-55.4 structures/s)
#endif
template <int KW, bool PRE>
__global__ __launch_bounds__(kWave * kWideWaves) __attribute__((amdgpu_waves_per_eu(PRE ? DGN_WIDE_PRE_WAVES : DGN_WIDE_C16_WAVES)))
void betti_wide_kernel_c16(BettiLaunch bl, WideLayout ly) {
    if constexpr (PRE) betti_reduce_body<KW>(bl, ly);
    else betti_wide_body<KW, kC16, false>(bl, ly);
}

// ---- the apparent phase as a workgroup-per-complex pass (u16-coded complexes, the 10 A path) ----
// The per-wave wide kernel spent about 65 % of a 10 A complex in its dim-2 apparent walk (DESIGN.md
// 3.2): every triangle's walk reads d(a, k), d(b, k), d(c, k) for its candidates k, scattered 2-byte
// reads of a 232 KB per-wave scratch matrix, ~1.95 M vector-memory instructions per complex, bound
// by the texture path's per-lane address rate. Here the complex's packed u16 code triangle (<= 128 KB
// at 362 points) and its adjacency bitsets (<= 17 KB) sit in the LDS of one CU, and 16 waves run
// every phase that needs them from there (ds_read_u16, 32 lanes per LDS cycle): the spanning forest
// (dim 0, one wave), the dim-1 apparent pass and the dim-2 apparent walk of its ~10^6 triangles. The
// pass writes per complex what the reductions read (betti_wide_kernel_c16<KW, true>, which then needs
// no LDS): the full n x n code matrix (coalesced rows), the dim-0 deaths, the dim-1 min-cofacet
// table, the dim-1 columns and the dim-2 columns not in an apparent pair with their F-minimal
// cofacet (their initial pivot), and the triangles the dim-1 apparent pairs clear. These are exactly
// what the per-wave kernel's own passes build (the dim-2 walk covers every triangle; the cleared ones
// are dropped when the reduction kernel reads the list). No dim-2 min-cofacet table: the reduction
// decides apparent owners from the matrix (lookup, PRE form).
constexpr int kWalkWaves = 16;
#ifndef DGN_WALK_STEP
#define DGN_WALK_STEP 4  // candidates per step of the walk pass's dim-2 walk
#endif
constexpr int kWalkRing = 128;  // queued triangles per wave (refilled below 64: at most 63 + 64 held)
__device__ __forceinline__ uint32_t c2u(int x) { return ((uint32_t)x * (uint32_t)(x - 1)) >> 1; }
__device__ __forceinline__ uint32_t walk_ticket(uint32_t* ctr) {  // wave-uniform, no branch on the lane
    const uint32_t t = atomicAdd(ctr, lane_id() == 0 ? 1u : 0u);
    return (uint32_t)__builtin_amdgcn_readlane((int)t, 0);
}
// LDS counters of the walk pass
enum { kWcWalk = 0, kWcN2 = 1, kWcTmax = 2, kWcRow = 3, kWcN1 = 4, kWcCl = 5, kWcD0 = 6, kWcInf0 = 7 };
// append the lanes with `p` to a per-complex list whose length is LDS counter *ctr (one LDS atomic
// per wave); returns this lane's slot
__device__ __forceinline__ uint32_t walk_append(uint32_t* ctr, bool p) {
    const uint64_t bal = ballot(p);
    if (!bal) return 0u;
    const uint32_t base =
        (uint32_t)__builtin_amdgcn_readlane((int)atomicAdd(ctr, lane_id() == 0 ? (uint32_t)__popcll(bal) : 0u), 0);
    return base + (uint32_t)mask_prefix(bal);
}
__global__ __launch_bounds__(kWave * kWalkWaves) void betti_walk_kernel(BettiLaunch bl) {
    using H = WideCx<2, kC16>;  // packing helpers (9-bit vertices, keys (code << 32) | ~index)
    extern __shared__ uint64_t walk_lds[];
    const WalkOut& wo = bl.walk;
    const int64_t wi = blockIdx.x;
    if (wi >= (int64_t)*bl.wide_len) return;  // past the slice's device-side length: the whole block
    const int lane = lane_id();
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
    const int64_t gi = bl.wide_list[wi];
    const int n = bl.npoints[gi];
    const int W = (n + 63) / 64;
    const int wmax = (wo.nmax + 63) / 64;
    const int np4 = (wo.nmax + 3) & ~3;
    // LDS: the packed codes at offset 0 (row i at c2(i)), then the bitsets, counters, forest
    // parents, dim-0 death codes and the per-wave triangle rings
    uint16_t* T = reinterpret_cast<uint16_t*>(walk_lds);
    uint64_t* adj = walk_lds + ((int64_t)wo.nmax * (wo.nmax - 1) / 2 + 3) / 4;  // [n][W]
    uint32_t* ctr = reinterpret_cast<uint32_t*>(adj + wo.nmax * wmax);          // kWc* counters
    uint16_t* par = reinterpret_cast<uint16_t*>(ctr + 8);                      // forest parents, 0xFFFF = root
    uint16_t* d0c = par + np4;                                                 // dim-0 death codes
    uint32_t* rings = reinterpret_cast<uint32_t*>(d0c + np4);                  // [kWalkWaves][kWalkRing]
    const uint32_t* vals = bl.rank_sorted + wi * bl.rank_stride;           // code -> f32 bits
    for (int i = threadIdx.x; i < n * W; i += kWave * kWalkWaves) adj[i] = 0ull;
    if (threadIdx.x < 8) ctr[threadIdx.x] = 0u;
    __syncthreads();
    // (1) codes into LDS; adjacency d <= thr (ripser.cpp:386-395) by row ballots, mirrored bits by
    // LDS atomics (rows are shared between waves); the threshold code = the largest code <= thr
    {
        const float* L = bl.lower + gi * bl.tri_stride;
        const uint32_t* Lc = bl.rank_codes + wi * bl.rank_stride;
        uint32_t tmax = 0;
        for (int i = 1 + wv; i < n; i += kWalkWaves) {
            const int ci = c2i(i);
            for (int j0 = 0; j0 < i; j0 += kWave) {
                const int j = j0 + lane;
                bool e = false;
                if (j < i) {
                    const uint32_t code = Lc[ci + j];
                    T[ci + j] = (uint16_t)code;
                    e = L[ci + j] <= bl.thr;
                    if (e) tmax = max(tmax, code);
                }
                const uint64_t b = ballot(e);
                if (lane == 0 && b) atomicOr((unsigned long long*)&adj[i * W + (j0 >> 6)], b);
                if (e) atomicOr((unsigned long long*)&adj[j * W + (i >> 6)], 1ull << (i & 63));
            }
        }
        tmax = ~wave_min_u32(~tmax);
        if (lane == 0) atomicMax(&ctr[kWcTmax], tmax);
    }
    __syncthreads();
    const uint32_t thrc = ctr[kWcTmax];
    auto aw = [&](int v, int w) __attribute__((always_inline)) { return adj[v * W + w]; };
    // d(x, k), x != k, from the packed triangle: cx = c2(x), ck = c2(k)
    auto dd = [&](int x, int cx, int k, int ck) __attribute__((always_inline)) -> uint32_t {
        return T[k < x ? cx + k : ck + x];
    };
    // (2) the full matrix (row-major, coalesced rows) for the reductions; wave 0: dim 0, Prim on
    // F-keys == Kruskal's forest in Ripser's order (ripser.cpp:725-762), as WideCx::prim
    if (wv == 0) {
        constexpr int KWM = (kC16MaxPoints + 63) / 64;
        uint64_t best[KWM];
        int bp[KWM];
        uint32_t intree = lane == 0 ? 1u : 0u;  // bit t: vertex 64 t + lane is in the forest
        for (int i = lane; i < n; i += kWave) par[i] = 0xFFFF;
#pragma unroll
        for (int t = 0; t < KWM; ++t) {
            const int v = 64 * t + lane;
            best[t] = kInfW;
            bp[t] = 0;
            if (t < W && v < n && v != 0 && ((aw(0, t) >> lane) & 1ull)) best[t] = H::wkey(T[c2i(v)], bin2(v));
        }
        // a death's value is 0 iff its code is 0 and the complex's smallest distance is 0 (codes are
        // first indices of value runs in the sorted triangle)
        const bool zero0 = __uint_as_float(vals[0]) == 0.0f;
        wave_lds_order();
        int nd0 = 0, ninf = 1;
        for (int added = 1; added < n; ++added) {
            uint64_t lmin = kInfW;
            int lt = 0, lp = 0, lfree = 1 << 30;
#pragma unroll
            for (int t = 0; t < KWM; ++t) {
                const int v = 64 * t + lane;
                const bool out = t < W && v < n && !((intree >> t) & 1u);
                if (out && best[t] < lmin) {
                    lmin = best[t];
                    lt = t;
                    lp = bp[t];
                }
                if (out && v < lfree) lfree = v;
            }
            const uint64_t m = wave_min_u64(lmin);
            int v;
            if (m == kInfW) {  // new component: lowest vertex outside the forest
                v = (int)wave_min_u32((uint32_t)lfree);
                ++ninf;
            } else {
                const int l = __ffsll((unsigned long long)ballot(lmin == m)) - 1;
                v = 64 * (int)rlw((uint32_t)lt, l) + l;
                const int u = (int)rlw((uint32_t)lp, l);
                const uint32_t dc = H::kdiam(m);
                if (!(dc == 0u && zero0)) {  // (0, d) emitted only if d != 0 (ripser.cpp:741-748)
                    if (lane == 0) d0c[nd0] = (uint16_t)dc;
                    ++nd0;
                }
                if (lane == 0) par[v] = (uint16_t)u;
            }
            if (lane == (v & 63)) intree |= 1u << (v >> 6);
            wave_lds_order();
            const int cv = c2i(v);
#pragma unroll
            for (int t = 0; t < KWM; ++t) {
                const int x = 64 * t + lane;
                if (t < W && x < n && !((intree >> t) & 1u) && ((aw(v, t) >> lane) & 1ull)) {
                    const uint64_t k = H::wkey(dd(v, cv, x, c2i(x)), v > x ? bin2(v) + x : bin2(x) + v);
                    if (k < best[t]) {
                        best[t] = k;
                        bp[t] = v;
                    }
                }
            }
        }
        wave_lds_order();
        float* d0s = wo.d0 + wi * wo.d0stride;
        for (int i = lane; i < nd0; i += kWave) d0s[i] = __uint_as_float(vals[d0c[i]]);
        if (lane == 0) {
            ctr[kWcD0] = (uint32_t)nd0;
            ctr[kWcInf0] = (uint32_t)ninf;
        }
    } else {
        uint16_t* D = wo.dmat + wi * wo.dstride;
        const int ns = (n + 3) & ~3;  // 8-byte rows (the reductions read them as packed vectors)
        for (int i = wv - 1; i < n; i += kWalkWaves - 1) {
            const int ci = c2i(i);
            for (int x = lane; x < ns; x += kWave)
                D[i * ns + x] = x == i || x >= n ? (uint16_t)0xFFFF : (x < i ? T[ci + x] : T[c2i(x) + i]);
        }
    }
    __syncthreads();  // the forest (is a dim-1 column a tree edge?)
    // (3) dim 1, one lane per edge (i, j), j < i, rows dealt from an LDS cursor (WideCx::pass_dim1):
    // the F-minimal cofacet of every non-tree edge (walking k downwards, the first k with both
    // distances within d(i, j) ends the walk; a smaller k wins only with a strictly smaller
    // diameter), the min-cofacet table, the apparent pairs' triangles (cleared in dim 2) and the
    // other columns
    {
        uint16_t* mce = wo.mce + wi * wo.mstride;
        uint64_t* oe1 = wo.e1 + wi * (int64_t)wo.cap1;
        uint32_t* ocl = wo.cl + wi * (int64_t)wo.cap1;
        for (;;) {
            const int i = 1 + (int)walk_ticket(&ctr[kWcRow]);
            if (i >= n) break;
            const int ci = c2i(i);
            for (int w0 = 0; 64 * w0 < i; ++w0) {
                uint64_t bits = uniw64(aw(i, w0));
                const int lim = i - 64 * w0;
                if (lim < 64) bits &= (1ull << lim) - 1ull;
                if (!bits) continue;
                const int j = 64 * w0 + lane;
                bool app = false, na = false;
                uint32_t clr = 0;
                uint64_t ent = 0;
                if ((bits >> lane) & 1ull) {
                    uint16_t mc = kMcNoneW;
                    if (!(par[i] == j || par[j] == i)) {
                        const uint32_t dij = T[ci + j];
                        const int cj = c2i(j);
                        int bk = -1;
                        bool found = false;
                        uint32_t bdd = 0xFFFFFFFFu, hda = 0, hdb = 0;
                        for (int w = W - 1; w >= 0 && !found; --w) {
                            uint64_t m = aw(i, w) & aw(j, w);
                            while (m != 0ull && !found) {
                                const int bit = 63 - __clzll((long long)m);
                                m &= ~(1ull << bit);
                                const int k = 64 * w + bit;
                                const int ck = c2i(k);
                                const uint32_t da = dd(i, ci, k, ck), db = dd(j, cj, k, ck);
                                const uint32_t dk = max(da, db);
                                if (dk <= dij) {
                                    bdd = dij;
                                    bk = k;
                                    found = true;
                                    hda = da;
                                    hdb = db;
                                } else if (dk < bdd) {
                                    bdd = dk;
                                    bk = k;
                                }
                            }
                        }
                        if (bk >= 0) {
                            const uint32_t ed = ((uint32_t)i << 9) | (uint32_t)j;
                            app = found && (bk > i || hdb < dij) && (bk > j || hda < dij);
                            if (app) clr = (uint32_t)H::pidx(3, H::pinsert(2, ed, bk));
                            else {
                                na = true;
                                ent = (uint64_t)ed | ((uint64_t)bk << 18) | ((uint64_t)bdd << 27);
                            }
                            mc = (uint16_t)bk;
                        }
                    }
                    mce[ci + j] = mc;
                }
                const uint32_t q1 = walk_append(&ctr[kWcN1], na);
                if (na && q1 < (uint32_t)wo.cap1) oe1[q1] = ent;
                const uint32_t q2 = walk_append(&ctr[kWcCl], app);
                if (app && q2 < (uint32_t)wo.cap1) ocl[q2] = clr;
            }
        }
    }
    // (4) the dim-2 walk. Each wave takes top vertices a (descending: the largest share of triangles
    // first) from an LDS cursor and queues the triangles (a, b, c), c < b < a, of a's edges in a
    // per-wave LDS ring (one common-neighbour word of an edge per refill step: the lanes holding its
    // set bits store them at their prefix count); a lane whose walk ended takes the next queued
    // triangle at once (pass_dim2's dealing, without its per-lane bit selects).
    uint64_t* oent = wo.ent + wi * (int64_t)wo.cap;
    uint32_t* ring = rings + wv * kWalkRing;
    int ca = -1, cb = 0, cw = 0, bw = 0;  // cursor (uniform): edge (ca, cb), word cw of its c's
    uint64_t bm = 0;                      // b's of row ca word bw not yet taken
    bool exhausted = false;
    int head = 0, tail = 0;               // the ring's uniform read / write counts
    int ea = 0, eb = 0, c = 0, w = 0, bk = -1;
    uint32_t ra = 0, rb = 0, rcc = 0;     // c2 of the lane's triangle's vertices
    bool act = false, fresh = false, found = false;
    uint64_t m = 0;
    uint32_t bd = 0xFFFFFFFFu, ds = 0, dab = 0, dac = 0, dbc = 0, hda = 0, hdb = 0, hdc = 0;
    for (;;) {
        while (tail - head < kWave && !exhausted) {  // refill: the next edge word with a common neighbour
            uint64_t mm = 0;
            for (;;) {
                if (cb > 0 && 64 * (cw + 1) < cb) {
                    ++cw;
                } else {
                    while (bm == 0ull) {  // the next b of row ca, or the next top vertex
                        if (ca >= 0 && 64 * (bw + 1) < ca) {
                            ++bw;
                        } else {
                            ca = n - 1 - (int)walk_ticket(&ctr[kWcWalk]);
                            if (ca < 2) {
                                exhausted = true;
                                break;
                            }
                            bw = 0;
                        }
                        uint64_t r = uniw64(aw(ca, bw));
                        const int lim = ca - 64 * bw;
                        if (lim < 64) r &= (1ull << lim) - 1ull;
                        bm = r;
                    }
                    if (exhausted) break;
                    cb = 64 * bw + __ffsll((unsigned long long)bm) - 1;
                    bm &= bm - 1ull;
                    cw = 0;
                }
                mm = uniw64(aw(ca, cw) & aw(cb, cw));
                const int lim = cb - 64 * cw;
                if (lim < 64) mm &= (1ull << lim) - 1ull;
                if (mm) break;
            }
            if (exhausted) break;
            if ((mm >> lane) & 1ull)
                ring[(tail + mask_prefix(mm)) & (kWalkRing - 1)] =
                    ((uint32_t)ca << 18) | ((uint32_t)cb << 9) | (uint32_t)(64 * cw + lane);
            tail += __popcll(mm);
        }
        wave_lds_order();
        {  // idle lanes take queued triangles, in order
            const uint64_t need = ballot(!act);
            const int avail = tail - head;
            const int r = mask_prefix(need);
            if (!act && r < avail) {
                const uint32_t t = ring[(head + r) & (kWalkRing - 1)];
                ea = (int)(t >> 18);
                eb = (int)((t >> 9) & 511u);
                c = (int)(t & 511u);
                act = fresh = true;
            }
            head += min(__popcll(need), avail);
        }
        if (!ballot(act)) break;  // nothing queued, nothing left to queue
        bool na = false;
        uint64_t ent = 0;
        if (act) {
            if (fresh) {
                ra = c2u(ea);
                rb = c2u(eb);
                rcc = c2u(c);
                dab = T[ra + eb];
                dac = T[ra + c];
                dbc = T[rb + c];
                ds = max(max(dab, dac), dbc);
                w = W - 1;
                m = aw(ea, w) & aw(eb, w) & aw(c, w);
                bd = 0xFFFFFFFFu;
                bk = -1;
                found = false;
                fresh = false;
            }
            while (m == 0ull && w > 0) {  // the next word with a common neighbour of a, b, c
                --w;
                m = aw(ea, w) & aw(eb, w) & aw(c, w);
            }
            // up to kS candidates of this word, highest first
            constexpr int kS = DGN_WALK_STEP;
            int kk[kS];
            bool val[kS];
#pragma unroll
            for (int j = 0; j < kS; ++j) {
                val[j] = m != 0ull;
                const int bit = 63 - __clzll((long long)(m | 1ull));
                kk[j] = val[j] ? 64 * w + bit : c;  // d(c, c) reads a harmless in-range entry
                m &= ~(1ull << bit);
            }
            uint32_t da[kS], dbv[kS], dc[kS];
#pragma unroll
            for (int j = 0; j < kS; ++j) {
                const int k = kk[j];
                const uint32_t ck = c2u(k);
                da[j] = T[k < ea ? ra + k : ck + ea];
                dbv[j] = T[k < eb ? rb + k : ck + eb];
                dc[j] = T[k < c ? rcc + k : ck + c];
            }
            // (diameter, k) only: walking k downwards a smaller k wins only with a strictly smaller
            // diameter (pass_dim2)
#pragma unroll
            for (int j = 0; j < kS; ++j) {
                const uint32_t dk = max(max(da[j], dbv[j]), dc[j]);
                const bool z = val[j] && !found && dk <= ds;
                const bool lt = val[j] && !found && dk < bd;
                hda = z ? da[j] : hda;
                hdb = z ? dbv[j] : hdb;
                hdc = z ? dc[j] : hdc;
                bk = z || lt ? kk[j] : bk;
                bd = z ? ds : (lt ? dk : bd);
                found = found || z;
            }
            if (found || (m == 0ull && w == 0)) {
                act = false;
                if (bk >= 0) {
                    const uint32_t colp = ((uint32_t)ea << 18) | ((uint32_t)eb << 9) | (uint32_t)c;
                    const bool app = found && (bk > ea || max(max(hdb, hdc), dbc) < ds) &&
                                     (bk > eb || max(max(hda, hdc), dac) < ds) &&
                                     (bk > c || max(max(hda, hdb), dab) < ds);
                    if (!app) {  // the column, its cofacet vertex, the cofacet's diameter (WalkOut::ent)
                        na = true;
                        ent = (uint64_t)colp | ((uint64_t)bk << 27) | ((uint64_t)bd << 36);
                    }
                }
            }
        }
        const uint32_t q = walk_append(&ctr[kWcN2], na);
        if (na && q < (uint32_t)wo.cap) oent[q] = ent;
    }
    (void)thrc;
    __syncthreads();
    if (threadIdx.x < 8) {
        const int t = threadIdx.x;
        const uint32_t v = t == kWmNa2 ? ctr[kWcN2] : t == kWmThr ? thrc : t == kWmNa1 ? ctr[kWcN1]
                         : t == kWmCl ? ctr[kWcCl] : t == kWmD0 ? ctr[kWcD0] : t == kWmInf0 ? ctr[kWcInf0] : 0u;
        wo.meta[8 * wi + t] = v;
    }
}

size_t walk_lds_bytes(int nmax) {
    const int64_t wmax = (nmax + 63) / 64, np4 = (nmax + 3) & ~3;
    return (size_t)(8 * (((int64_t)nmax * (nmax - 1) / 2 + 3) / 4) + 8 * nmax * wmax + 32 + 2 * 2 * np4 +
                    4 * kWalkWaves * kWalkRing);
}

int64_t align256(int64_t x) { return (x + 255) / 256 * 256; }

// the instantiation for complexes of up to nmax points: 2, 4, 6 or 8 bitset words per vertex
using WideKernel = void (*)(BettiLaunch, WideLayout);
WideKernel wide_kernel_for(int nmax, bool c16, bool pre = false) {
    const int w = (nmax + 63) / 64;
    if (c16 && nmax <= kC16MaxPoints) {  // u16 rank codes (betti_rank_codes before the launch)
        if (pre) {  // after the walk pass (betti_walk_kernel)
            if (w <= 2) return betti_wide_kernel_c16<2, true>;
            if (w <= 4) return betti_wide_kernel_c16<4, true>;
            return betti_wide_kernel_c16<6, true>;
        }
        if (w <= 2) return betti_wide_kernel_c16<2, false>;
        if (w <= 4) return betti_wide_kernel_c16<4, false>;
        return betti_wide_kernel_c16<6, false>;
    }
    if (w <= 2) return betti_wide_kernel<2, kF32>;
    if (w <= 4) return betti_wide_kernel<4, kF32>;
    if (w <= 6) return betti_wide_kernel<6, kF32>;
    if (w <= 8) return betti_wide_kernel<8, kF32>;
    if (w <= 16) return betti_wide_kernel<16, kBig>;  // 513..1024 points: rank-coded distances (BIG)
    if (w <= 32) return betti_wide_kernel<32, kHuge>; // 1025..2048 points: HUGE
    return betti_wide_kernel<64, kGiant>;             // 2049..4096 points (caller-given clouds): GIANT
}

size_t wide_lds_bytes(int nmax, bool pre = false) {  // per workgroup: token, adjacency, parents
    if (pre) return 0;  // the reduction-only launch after the walk pass
    const int64_t ww = (nmax + 63) / 64;
    if (nmax > kWideBigPoints) return (size_t)(8 * (1 + (nmax + 3) / 4));  // parents only
    return (size_t)(8 * (1 + nmax * ww + (nmax + 3) / 4));
}

}  // namespace

// Scratch layout of one wave for complexes of up to nmax points (all offsets 256-B aligned).
// big = the capacity-retry layout (complexes whose reduction outgrew the regular caps): column,
// pivot and pair tables of 2^(base_log2 + 2 grow) entries (base_log2 = 24 but for tests), never
// more than every simplex of the complex needs (C(nmax, 3) columns), and a V store of as many
// entries. The host raises `grow` while complexes still overflow (kWideMaxGrow levels): a complex
// outgrows the last level only when it needs more than kWideMaxCols (2^29) columns, pivots or pairs
// or a V store above 2^(base_log2 + 6) entries.
WideLayout betti_wide_layout(int nmax, bool big, int64_t cap_limit, int grow, int base_log2, bool prewalked) {
    WideLayout l{};
    const int64_t n = nmax;
    const int64_t e = n * (n - 1) / 2, t = n * (n - 1) * (n - 2) / 6;
    const bool huge = nmax > kWideBigPoints;
    const bool giant = nmax > kWideMaxPoints;  // no dim-2 min-cofacet table: a clearing bitmap
    const int64_t pt = huge ? 8 : 4;  // bytes of a packed column simplex (HUGE: 33-bit triangles)
    int64_t cap_max = big ? (int64_t(1) << (base_log2 + 2 * grow)) : (int64_t(1) << 17);
    // the pivot hash holds 2 cap entries and is probed with 32-bit masks: columns stop at 2^29
    // (hash 2^30) so every int32 cap below stays a positive power of two at the last level
    cap_max = std::min<int64_t>(cap_max, kWideMaxCols);
    if (!big && cap_limit > 0) {
        cap_max = 64;
        while (cap_max < cap_limit) cap_max <<= 1;
    }
    int64_t cap = std::min<int64_t>(1024, cap_max);
    while ((cap < t || cap < e) && cap < cap_max) cap <<= 1;
    l.nmax = nmax;
    l.na_cap = (int32_t)cap;
    l.p_cap = (int32_t)cap;
    l.h_cap = (int32_t)(2 * cap);
    l.vs_cap = big ? (int32_t)(int64_t(1) << (base_log2 + 2 * grow)) : (1 << 20);
    l.vl_cap = big ? (int32_t)std::min<int64_t>(cap, 1 << 22) : (1 << 16);
    l.guard = big ? (int64_t(1) << 32) : (int64_t(1) << 20);
    int64_t o = 0;
    auto take = [&](int64_t bytes) {
        const int64_t at = o;
        o = align256(o + bytes);
        return at;
    };
    l.prewalked = prewalked ? 1 : 0;
    l.D = take(prewalked ? 0 : 4 * n * n);  // prewalked: the walk pass's per-complex matrix
    l.mc_e = take(prewalked ? 0 : 2 * e);   // prewalked: the walk pass's per-complex table
    l.mc_t = take(prewalked || giant ? 0 : 2 * t);   // prewalked / giant: no dim-2 min-cofacet table
    l.clb = take(prewalked || giant ? 4 * (t / 32 + 2) : 0);
    l.edges = take(prewalked ? 0 : 4 * e);
    l.adj = take(huge ? 8 * n * ((n + 63) / 64) : 0);
    l.na_key = take(8 * cap);
    l.na_tau = take(8 * cap);
    l.na_tv = take(8 * cap);
    l.na_col = take(pt * cap);
    l.cl_list = take((giant ? 8 : 4) * cap);  // triangle indices of the dim-1 clearing marks
    l.vstore = take(pt * (int64_t)l.vs_cap);
    l.vlist = take(pt * (int64_t)l.vl_cap);
    l.h_key = take(8 * 2 * cap);
    l.h_meta = take(8 * 2 * cap);
    l.h_used = take(4 * cap);
    l.p1 = take(8 * cap);
    l.p2 = take(8 * cap);
    l.d0 = take(prewalked ? 0 : 4 * n);
    l.total = o;
    return l;
}

hipError_t betti_wide_init_scratch(hipStream_t s, const WideLayout& l, int waves) {
    hipError_t e = hipMemset2DAsync(l.base + l.h_key, (size_t)l.total, 0, 8 * (size_t)l.h_cap, (size_t)waves, s);
    if (e != hipSuccess) return e;
    // mc_e and mc_t (with their alignment padding) lie between l.mc_e and l.clb
    if (l.clb > l.mc_e) e = hipMemset2DAsync(l.base + l.mc_e, (size_t)l.total, 0xFF, (size_t)(l.clb - l.mc_e), (size_t)waves, s);
    if (e != hipSuccess || l.edges == l.clb) return e;  // the clearing bitmap (prewalked / giant) starts empty
    return hipMemset2DAsync(l.base + l.clb, (size_t)l.total, 0, (size_t)(l.edges - l.clb), (size_t)waves, s);
}

// waves of betti_wide_kernel resident on the whole device for complexes of up to nmax points
int betti_wide_resident_waves(int device, int nmax, bool c16, bool pre) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 512;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, wide_kernel_for(nmax, c16, pre), kWave * kWideWaves,
                                                     wide_lds_bytes(nmax, pre)) != hipSuccess ||
        per_cu <= 0)
        per_cu = 1;
    return prop.multiProcessorCount * per_cu * kWideWaves;
}

WalkOut betti_walk_out_layout(int nmax) {
    WalkOut w{};
    w.nmax = nmax;
    // u16, rows of (n + 3) & ~3 elements, + 512 of padding for the packed reads past the last row
    w.dstride = ((int64_t)nmax * ((nmax + 3) & ~3) + 512 + 127) / 128 * 128;
    w.d0stride = ((int64_t)nmax + 63) / 64 * 64;                   // f32
    w.mstride = ((int64_t)nmax * (nmax - 1) / 2 + 127) / 128 * 128;  // u16
    w.cap1 = kWalkCap;
    w.cap = kWalkCap;
    return w;
}
int64_t betti_walk_out_bytes(int nmax) {
    const WalkOut w = betti_walk_out_layout(nmax);
    return 2 * w.dstride + 32 + 4 * w.d0stride + 2 * w.mstride + (8 + 4) * (int64_t)w.cap1 + 8 * (int64_t)w.cap;
}
hipError_t launch_betti_walk(hipStream_t st, const BettiLaunch& b, int64_t count, int nmax) {
    if (count <= 0) return hipSuccess;
    if (nmax > kC16MaxPoints || nmax < 3) return hipErrorInvalidValue;
    hipLaunchKernelGGL(betti_walk_kernel, dim3((unsigned)count), dim3(kWave * kWalkWaves), walk_lds_bytes(nmax), st, b);
    return hipGetLastError();
}

hipError_t launch_betti_wide(hipStream_t st, const BettiLaunch& b, const WideLayout& l, int waves) {
    if (waves <= 0) return hipSuccess;
    WideLayout lw = l;
    lw.slots = waves;  // scratch slots allocated: a wave past them leaves at once
    hipLaunchKernelGGL(wide_kernel_for(l.nmax, b.rank_codes != nullptr && l.nmax <= kC16MaxPoints, l.prewalked != 0),
                       dim3((unsigned)((waves + kWideWaves - 1) / kWideWaves)), dim3(kWave * kWideWaves),
                       wide_lds_bytes(l.nmax, l.prewalked != 0), st, b, lw);
    return hipGetLastError();
}

}  // namespace dgn
