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
//     masks, the f32 distance matrix in LDS (stride NP+1, conflict-free row and column reads);
//   * distance matrix: the K=3 Gram product is built on the matrix cores with
//     v_mfma_f64_16x16x4_f64 as three rank-1 products (exactly round(x_ik*x_jk) each), summed on
//     the VALU in the reference's order ((p0+p1)+p2), then sqrt(max(0,(sq_i+sq_j)-2p)) -> f32:
//     bit-identical to the reference's Eigen/SSE2 arithmetic;
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
#include "dgn_internal.hpp"

namespace dgn {

constexpr int kVCap = 128;        // simplices in one column's V list (registers: 2 per lane)
constexpr int kVStoreLds = 128;   // stored V-list entries kept in LDS (rest in scratch)
constexpr int kVStoreCap = 65536; // stored V-list entries per dimension
constexpr int kNACap = 4096;      // non-apparent columns per dimension (scratch)
constexpr int kPivCap = 4096;     // serially resolved pivots per dimension
constexpr int kPairCap = 4096;    // pairs per dimension (scratch)
constexpr int kChunk = 4;         // complexes per dequeue

constexpr uint64_t kInf = ~0ull;
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kLazyBit = 0x80000000u;  // vmeta: V = {column simplex} (packed in the low bits)

// error bits (mirrored in dgn_api.cpp)
constexpr uint32_t kErrTooManyPoints = 1u << 0;
constexpr uint32_t kErrWorkCol = 1u << 1;
constexpr uint32_t kErrNA = 1u << 2;
constexpr uint32_t kErrPiv = 1u << 3;
constexpr uint32_t kErrPairs = 1u << 4;
constexpr uint32_t kErrR = 1u << 5;
constexpr uint32_t kErrOrder = 1u << 6;

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
    // F-minimal cofacet (packed) of every edge / triangle of the complex, indexed by its dense
    // combinatorial index; kNone for simplices that are not columns or have no cofacet
    static constexpr int64_t mincof = vstore + 4 * kVStoreCap;       // uint32 [C(64,3)]
    static constexpr int64_t total = mincof + 4 * (64 * 63 * 62 / 6);
};

template <int NP>
struct BettiSmem {
    float Dt[NP * (NP - 1) / 2];  // f32 distances, strict lower triangle: (i > j) at i(i-1)/2 + j
    uint64_t adj[NP];
    uint64_t tree[NP];
    uint16_t edges[NP * (NP - 1) / 2];
    uint32_t cleared[(NP * (NP - 1) * (NP - 2) / 6 + 31) / 32];
    union {
        struct {
            double X[NP][3];
            double sq[NP];
        } cloud;
    } u;
    uint32_t vstore[kVStoreLds];
    float d0[NP];
};

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
// materialize a value in a VGPR here (stops the compiler from sinking select arms into
// divergent branches; the arms below are cheap and computed unconditionally)
__device__ __forceinline__ uint32_t pin(uint32_t x) {
    asm volatile("" : "+v"(x));
    return x;
}
__device__ __forceinline__ int pin(int x) {
    asm volatile("" : "+v"(x));
    return x;
}
__device__ __forceinline__ int c2(int x) { return x * (x - 1) / 2; }
__device__ __forceinline__ int c3(int x) { return x * (x - 1) * (x - 2) / 6; }
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, kWave);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, kWave);
    return ((uint64_t)hi << 32) | lo;
}
// min over the wave of a 64-bit key, DPP row rotations (VALU latency) + 4 readlanes
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
    uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
#define DGN_MIN_STEP(ctrl)                                                          \
    {                                                                               \
        const uint32_t l2 = (uint32_t)__builtin_amdgcn_update_dpp((int)lo, (int)lo, ctrl, 0xf, 0xf, false); \
        const uint32_t h2 = (uint32_t)__builtin_amdgcn_update_dpp((int)hi, (int)hi, ctrl, 0xf, 0xf, false); \
        const bool take = (h2 < hi) || (h2 == hi && l2 < lo);                       \
        lo = take ? l2 : lo;                                                        \
        hi = take ? h2 : hi;                                                        \
    }
    DGN_MIN_STEP(0x121)  // row_ror:1
    DGN_MIN_STEP(0x122)  // row_ror:2
    DGN_MIN_STEP(0x124)  // row_ror:4
    DGN_MIN_STEP(0x128)  // row_ror:8
#undef DGN_MIN_STEP
    uint64_t best = kInf;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint64_t x = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, 16 * r) << 32) |
                           (uint32_t)__builtin_amdgcn_readlane((int)lo, 16 * r);
        best = x < best ? x : best;
    }
    return best;
}

// F-order key: ascending key == Ripser's filtration order (diameter ascending, then the
// combinatorial index DESCENDING, greater_diameter_or_smaller_index at ripser.cpp:318-324).
// Vertex tuples packed 8 bits per vertex in descending order preserve the colex (index) order.
__device__ __forceinline__ uint64_t make_key(float diam, uint32_t packed) {
    return ((uint64_t)__float_as_uint(diam) << 32) | (uint64_t)(~packed);
}
__device__ __forceinline__ float key_diam(uint64_t k) { return __uint_as_float((uint32_t)(k >> 32)); }
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
__device__ __forceinline__ int tri_dense(int a, int b, int c) {  // combinatorial index, a > b > c
    return a * (a - 1) * (a - 2) / 6 + b * (b - 1) / 2 + c;
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
    int n_adds, n_spills;  // diagnostics
#ifdef DGN_PHASE_TIMING
    uint64_t* ph = nullptr;
    uint64_t* tprev = nullptr;
    __device__ void stamp(int k) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        ph[k] += t - *tprev;
        *tprev = t;
    }
#define DGN_SUB(k) stamp(k)
#else
#define DGN_SUB(k) \
    do {           \
    } while (0)
#endif

    __device__ float dlow(int a, int b) const { return s.Dt[c2(a) + b]; }  // a > b
    __device__ float dist(int i, int j) const {                              // i != j
        const int a = i > j ? i : j, b = i > j ? j : i;
        return s.Dt[c2(a) + b];
    }
    __device__ uint64_t ekey(int i, int j) const {  // i != j
        const int a = i > j ? i : j, b = i > j ? j : i;
        return make_key(s.Dt[c2(a) + b], pack2(a, b));
    }
    __device__ float tri_diam(int a, int b, int c) const {  // a > b > c
        return fmaxf(fmaxf(dlow(a, b), dlow(a, c)), dlow(b, c));
    }
    __device__ uint64_t tkey(int a, int b, int c) const { return make_key(tri_diam(a, b, c), pack3(a, b, c)); }
    __device__ bool is_cleared(int a, int b, int c) const {
        const int t = tri_dense(a, b, c);
        return (s.cleared[t >> 5] >> (t & 31)) & 1u;
    }
    __device__ void set_cleared(int a, int b, int c) {
        const int t = tri_dense(a, b, c);
        atomicOr(&s.cleared[t >> 5], 1u << (t & 31));
    }
    template <typename T>
    __device__ T* sp(int64_t off) const { return reinterpret_cast<T*>(scratch + off); }
    __device__ float2* pairs(int dim) const { return sp<float2>(dim == 1 ? ScratchLayout::p1 : ScratchLayout::p2); }

    // wave-uniform: append pairs (birth, death) for lanes with `emit`
    __device__ void append_pairs(int dim, bool emit, float birth, float death) {
        const uint64_t bal = ballot(emit);
        int& np = dim == 1 ? n_p1 : n_p2;
        if (emit) {
            const int slot = np + mask_prefix(bal);
            if (slot < kPairCap) pairs(dim)[slot] = make_float2(birth, death);
        }
        np += __popcll(bal);
    }

    // per-lane: F-minimal cofacet key of edge (a > b) / triangle (a > b > c) over cand.
    // Inserting a larger vertex k gives a larger packed tuple, i.e. an F-smaller key among
    // cofacets of equal diameter; so walking k downwards, the first k whose distances to the
    // simplex are all <= diam yields the F-minimal cofacet (diameter diam, largest index)
    // and ends the search. Cofacets seen before it have larger diameters.
    __device__ uint64_t min_cofacet_lane(int dim, int a, int b, int c, float diam, uint64_t cand) const {
        uint64_t best = kInf;
        while (cand) {
            const int k = 63 - __clzll((long long)cand);
            cand &= ~(1ull << k);
            float dk = fmaxf(dist(a, k), dist(b, k));
            if (dim == 2) dk = fmaxf(dk, dist(c, k));
            const uint32_t pk = dim == 1 ? tri_with(a, b, k) : tet_with(a, b, c, k);
            if (dk <= diam) {
                best = make_key(diam, pk);
                break;
            }
            const uint64_t key = make_key(dk, pk);
            best = key < best ? key : best;
        }
        return best;
    }

    // whole wave: F-minimal cofacet, lane k evaluates vertex k
    __device__ uint64_t min_cofacet_wave(int dim, int a, int b, int c, float diam, uint64_t cand) const {
        const int k = lane_id();
        uint64_t key = kInf;
        if ((cand >> k) & 1ull) {
            if (dim == 1) key = make_key(fmaxf(diam, fmaxf(dist(a, k), dist(b, k))), tri_with(a, b, k));
            else key = make_key(fmaxf(diam, fmaxf(fmaxf(dist(a, k), dist(b, k)), dist(c, k))), tet_with(a, b, c, k));
        }
        return wave_min_u64(key);
    }

    // F-max facet of pivot tau as (packed vertices); owner iff it is a column (not a tree edge,
    // not cleared) whose F-min cofacet is tau (apparent pair)
    __device__ uint32_t max_facet(int dim, uint64_t tau, bool& is_column) const {
        const uint32_t p = key_packed(tau);
        if (dim == 1) {
            const int a = (p >> 16) & 255, b = (p >> 8) & 255, c = p & 255;
            uint64_t best = ekey(a, b);
            int fa = a, fb = b;
            uint64_t k = ekey(a, c);
            if (k > best) { best = k; fa = a; fb = c; }
            k = ekey(b, c);
            if (k > best) { best = k; fa = b; fb = c; }
            is_column = !((s.tree[fa] >> fb) & 1ull);
            return pack2(fa, fb);
        } else {
            const int a = (p >> 24) & 255, b = (p >> 16) & 255, c = (p >> 8) & 255, d = p & 255;
            uint64_t best = tkey(a, b, c);
            int fa = a, fb = b, fc = c;
            uint64_t k = tkey(a, b, d);
            if (k > best) { best = k; fa = a; fb = b; fc = d; }
            k = tkey(a, c, d);
            if (k > best) { best = k; fa = a; fb = c; fc = d; }
            k = tkey(b, c, d);
            if (k > best) { best = k; fa = b; fb = c; fc = d; }
            is_column = !is_cleared(fa, fb, fc);
            return pack3(fa, fb, fc);
        }
    }
    // Apparent owner of pivot tau (whole wave, uniform): its F-max facet f, if tau is f's
    // F-minimal cofacet (recorded for every column by the lane-parallel pass), else kNone.
    __device__ uint32_t apparent_owner_wave(int dim, uint64_t tau) const {
        bool col;
        const uint32_t f = uni(max_facet(dim, uni64(tau), col));
#ifdef DGN_APP_FLY
        if (!uni(col)) return kNone;
        const int a = (f >> 16) & 255, b = (f >> 8) & 255, c = f & 255;
        uint64_t mk;
        if (dim == 1) mk = min_cofacet_wave(1, b, c, 0, dlow(b, c), uni64(s.adj[b]) & uni64(s.adj[c]));
        else mk = min_cofacet_wave(2, a, b, c, tri_diam(a, b, c), uni64(s.adj[a]) & uni64(s.adj[b]) & uni64(s.adj[c]));
        return mk == uni64(tau) ? f : kNone;
#else
        const uint32_t m = sp<uint32_t>(ScratchLayout::mincof)[col_dense(dim, f)];
        return uni(m) == key_packed(tau) ? f : kNone;
#endif
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
        uint64_t bal = ballot(lane < npiv && pk0 == tau);
        if (bal) return __ffsll((unsigned long long)bal) - 1;
        if (npiv > kWave) {
            bal = ballot(lane + kWave < npiv && pk1 == tau);
            if (bal) return kWave + __ffsll((unsigned long long)bal) - 1;
        }
        const uint64_t* sp_piv = sp<uint64_t>(ScratchLayout::piv);
        for (int base = 2 * kWave; base < npiv; base += kWave) {
            const int i = base + lane;
            bal = ballot(i < npiv && sp_piv[i] == tau);
            if (bal) return base + __ffsll((unsigned long long)bal) - 1;
        }
        return -1;
    }
    __device__ uint32_t piv_meta(int i) const {
        if (i < kWave) return rl(pm0, i);
        if (i < 2 * kWave) return rl(pm1, i - kWave);
        return uni(sp<uint32_t>(ScratchLayout::vmeta)[i]);
    }
    __device__ void piv_push(int i, uint64_t tau, uint32_t meta) {
        const int lane = lane_id();
        if (i < kWave) {
            if (lane == i) { pk0 = tau; pm0 = meta; }
        } else if (i < 2 * kWave) {
            if (lane == i - kWave) { pk1 = tau; pm1 = meta; }
        } else if (lane == 0) {
            sp<uint64_t>(ScratchLayout::piv)[i] = tau;
            sp<uint32_t>(ScratchLayout::vmeta)[i] = meta;
        }
    }

    // ---- the working column's V list, resident in registers: lane t holds entry t (set 0) and
    // entry t + 64 (set 1) with its diameter. Toggles only move packed simplices; pivot_of_V
    // refreshes the diameters lane-parallel and reads entries back uniformly with v_readlane.
    uint32_t vs0 = 0, vs1 = 0;
    float vd0 = 0.f, vd1 = 0.f;
    uint64_t myadj = 0;  // lane k: adjacency row of vertex k (cofacet candidates test bits of it)

    __device__ static uint32_t rl(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }
    __device__ static uint64_t rl64(uint64_t x, int l) {
        return ((uint64_t)rl((uint32_t)(x >> 32), l) << 32) | rl((uint32_t)x, l);
    }
    __device__ void v_set(int i, uint32_t sp_) {
        const int lane = lane_id();
        if (i < 64) {
            if (lane == i) vs0 = sp_;
        } else if (lane == i - 64) {
            vs1 = sp_;
        }
    }
    __device__ int v_find(uint32_t x, int v) const {
        const int lane = lane_id();
        uint64_t bal = ballot(lane < v && vs0 == x);
        if (bal) return __ffsll((unsigned long long)bal) - 1;
        if (v > 64) {
            bal = ballot(lane + 64 < v && vs1 == x);
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
    __device__ float simplex_diam(int dim, uint32_t x) const {
        return dim == 1 ? dlow((x >> 8) & 255, x & 255) : tri_diam((x >> 16) & 255, (x >> 8) & 255, x & 255);
    }

    // Pivot of the column sum(delta s, s in V) (whole wave): the F-minimal cofacet of odd
    // multiplicity, restricted to keys above `floor` (the column's previous pivot: adding the
    // owner column cancels it and every other entry of both columns is larger). Lane k
    // evaluates the cofacet s u {k} of every s in V; one cofacet tau arises once per facet of
    // tau in V, always in a different lane (k = tau \ s), so the multiplicity of the wave
    // minimum is the popcount of a ballot. Even multiplicity: raise the floor and repeat.
    // kInf for the zero column.
    // key of the cofacet s u {k} for lane k (kInf if k is not a common neighbour of s or the
    // key is not above floor). Branch-free: the lower-triangle index of (k, x) is
    // c2(max) + min, so no lane-divergent selects between scalar and vector arms.
    __device__ uint64_t cofacet_key_above(int dim, int k, uint32_t sp_, float diam, uint64_t floor) const {
        const int a = dim == 1 ? (int)((sp_ >> 8) & 255) : (int)((sp_ >> 16) & 255);
        const int b = dim == 1 ? (int)(sp_ & 255) : (int)((sp_ >> 8) & 255);
        const int c = (int)(sp_ & 255);
        const bool on = dim == 1 ? ((myadj >> a) & (myadj >> b) & 1ull) != 0
                                 : ((myadj >> a) & (myadj >> b) & (myadj >> c) & 1ull) != 0;
        // every arm is materialized (pin) so the selects stay v_cndmask, never exec branches
        const int msk = -(int)on;
        const int ha = max(k, a), la = min(k, a), hb = max(k, b), lb = min(k, b);
        const int ia = pin(((ha * (ha - 1)) >> 1) + la) & msk;
        const int ib = pin(((hb * (hb - 1)) >> 1) + lb) & msk;
        float dd = fmaxf(diam, fmaxf(s.Dt[ia], s.Dt[ib]));
        uint32_t pk;
        const uint32_t uk = (uint32_t)k;
        if (dim == 1) {
            // insert k into (a > b): k > a -> (k,a,b); a > k > b -> (a,k,b); else (a,b,k)
            const uint32_t ab = sp_ & 0xFFFFu;
            const uint32_t p1 = pin((uk << 16) | ab);
            const uint32_t p2 = pin(((uint32_t)a << 16) | (uk << 8) | (uint32_t)b);
            const uint32_t p3 = pin((ab << 8) | uk);
            pk = k > a ? p1 : (k > b ? p2 : p3);
        } else {
            const int hc = max(k, c), lc = min(k, c);
            const int ic = pin(((hc * (hc - 1)) >> 1) + lc) & msk;
            dd = fmaxf(dd, s.Dt[ic]);
            const uint32_t abc = sp_ & 0xFFFFFFu;
            const uint32_t p1 = pin((uk << 24) | abc);
            const uint32_t p2 = pin(((uint32_t)a << 24) | (uk << 16) | (abc & 0xFFFFu));
            const uint32_t p3 = pin(((abc >> 8) << 16) | (uk << 8) | (uint32_t)c);
            const uint32_t p4 = pin((abc << 8) | uk);
            pk = k > a ? p1 : (k > b ? p2 : (k > c ? p3 : p4));
        }
        const uint64_t key = make_key(dd, pk);
        return (on && key > floor) ? key : kInf;
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
        const int v = (int)uni((uint32_t)v_);
        const int v0 = v < 64 ? v : 64;
        if (k < v) vd0 = simplex_diam(dim, vs0);
        if (v > 64 && k + 64 < v) vd1 = simplex_diam(dim, vs1);
        for (;;) {
            uint64_t lmin = kInf;
            for (int i = 0; i < v0; ++i) {
                const uint64_t key = cofacet_key_above(dim, k, rl(vs0, i), __uint_as_float(rl(__float_as_uint(vd0), i)), floor);
                lmin = key < lmin ? key : lmin;
            }
            for (int i = 64; i < v; ++i) {
                const uint64_t key =
                    cofacet_key_above(dim, k, rl(vs1, i - 64), __uint_as_float(rl(__float_as_uint(vd1), i - 64)), floor);
                lmin = key < lmin ? key : lmin;
            }
            const uint64_t m = wave_min_u64(lmin);
#ifdef DGN_PHASE_TIMING
            ph[24] += 1;
            ph[25] += (uint64_t)v;
#endif
            if (m == kInf) return kInf;
            if (__popcll(ballot(lmin == m)) & 1) return m;
            floor = m;
        }
    }

    // per-lane apparent owner of pivot tau (kNone if none): its F-max facet f, if tau is f's
    // F-minimal cofacet (recorded for every column by the lane-parallel pass)
    __device__ uint32_t apparent_owner_lane(int dim, uint64_t tau) const {
        bool col;
        const uint32_t f = max_facet(dim, tau, col);
        const uint32_t m = sp<uint32_t>(ScratchLayout::mincof)[col_dense(dim, f)];
        return m == key_packed(tau) ? f : kNone;
    }

    // Walk the non-apparent columns in Ripser's order (whole wave). na_* (scratch) hold each
    // column's key and its unreduced pivot. Up to 128 records live in registers (lane t:
    // records t and t + 64) with their rank in column order and the apparent owner of their
    // initial pivot, all computed lane-parallel; larger sets are rank-sorted into scratch.
    __device__ void reduce_serial(int dim, int nna) {
        const int lane = lane_id();
        if (nna > kNACap) { err |= kErrNA; return; }
        myadj = lane < n ? s.adj[lane] : 0ull;
        const uint64_t* gk = sp<uint64_t>(ScratchLayout::na_key);
        const uint64_t* gt = sp<uint64_t>(ScratchLayout::na_tau);
        const bool regs = nna <= 2 * kWave;
        uint64_t rk0 = 0, rk1 = 0, rt0 = 0, rt1 = 0;
        int rr0 = -1, rr1 = -1;
        uint32_t ra0 = kNone, ra1 = kNone;
        uint64_t* sk = sp<uint64_t>(ScratchLayout::sna_key);
        uint64_t* st = sp<uint64_t>(ScratchLayout::sna_tau);
        if (regs) {
            if (lane < nna) { rk0 = gk[lane]; rt0 = gt[lane]; }
            if (lane + kWave < nna) { rk1 = gk[lane + kWave]; rt1 = gt[lane + kWave]; }
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
        DGN_SUB(16);
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
            const uint32_t cp = key_packed(colkey);
            const float birth = key_diam(colkey);
            DGN_SUB(17);
            int owner = find_pivot(npiv, tau);
            DGN_SUB(18);
            uint32_t app = owner >= 0 ? kNone : (have_app ? app0 : apparent_owner_wave(dim, tau));
            DGN_SUB(19);
            int v = 0;  // 0 = lazy: V == {this column}
            if (owner >= 0 || app != kNone) {
                v_toggle(dim, cp, v);
                int guard = 0;
                while (true) {
                    // V ^= V(owner)
                    bool ok = true;
                    if (app != kNone) {
                        // an apparent owner precedes this column in Ripser's order (key greater)
                        if (!(column_key(dim, app) > colkey)) { err |= kErrOrder; return; }
                        ok = v_toggle(dim, app, v);
                    } else {
                        const uint32_t m = piv_meta(owner);
                        if (m & kLazyBit) {
                            ok = v_toggle(dim, m & ~kLazyBit, v);
                        } else {
                            const int off = (int)uni(m >> 9), len = (int)uni(m & 511);
                            for (int t = 0; t < len && ok; ++t) {
                                const uint32_t x = uni(off + t < kVStoreLds ? s.vstore[off + t] : gvstore[off + t]);
                                ok = v_toggle(dim, x, v);
                            }
                        }
                    }
                    if (!ok) { err |= kErrWorkCol; return; }
                    ++n_adds;
                    DGN_SUB(20);
#ifdef DGN_PHASE_TIMING
                    ph[14] += (uint64_t)v;
                    ph[15] += (uint64_t)v * (uint64_t)v;
                    ph[23] = (uint64_t)v > ph[23] ? (uint64_t)v : ph[23];
#endif
                    tau = v > 0 ? pivot_of_V(dim, v, tau) : kInf;
                    DGN_SUB(21);
                    if (tau == kInf) break;  // zero column: essential class, not emitted
                    owner = find_pivot(npiv, tau);
                    DGN_SUB(18);
                    app = owner >= 0 ? kNone : apparent_owner_wave(dim, tau);
                    DGN_SUB(19);
                    if (owner < 0 && app == kNone) break;  // tau is this column's pivot
                    if (++guard > 100000) { err |= kErrWorkCol; return; }
                }
                if (tau == kInf) continue;  // zero column
            }
            // ---- tau is the pivot of this column ----
            const float death = key_diam(tau);
            if (death > birth) {
                if (lane == 0) {
                    const int slot = dim == 1 ? n_p1 : n_p2;
                    if (slot < kPairCap) pairs(dim)[slot] = make_float2(birth, death);
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
                    if (vused + t < kVStoreLds) s.vstore[vused + t] = x;
                    else gvstore[vused + t] = x;
                }
                meta = ((uint32_t)vused << 9) | (uint32_t)v;
                vused = (int)uni((uint32_t)(vused + v));
            }
            piv_push(npiv, tau, meta);
            npiv = (int)uni((uint32_t)(npiv + 1));
            lds_sync();
            DGN_SUB(22);
        }
    }
};

#ifdef DGN_PHASE_TIMING
#define DGN_PHASE(k)                                          \
    do {                                                      \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();     \
        ph[k] += t_ - t_prev;                                 \
        t_prev = t_;                                          \
    } while (0)
#else
#define DGN_PHASE(k) \
    do {             \
    } while (0)
#endif

template <int NP>
__global__ __launch_bounds__(kWave, 3) void betti_kernel(BettiLaunch bl) {
    __shared__ BettiSmem<NP> s;
    __shared__ int64_t chunk_s;
#ifdef DGN_PHASE_TIMING
    uint64_t ph[32] = {0};
    uint64_t t_prev = __builtin_amdgcn_s_memtime();
#endif
    const int lane = lane_id();
    uint8_t* scratch = bl.scratch + (int64_t)blockIdx.x * bl.scratch_per_wave;
    const int64_t A = bl.num_atoms;

    // complexes of this launch: all of them, or the overflow list written by the bucket pass
    const int64_t total = bl.work_list ? (int64_t)*bl.overflow_len : A;
    for (;;) {
        if (lane == 0) chunk_s = (int64_t)atomicAdd((unsigned int*)bl.queue, 1u) * kChunk;
        __syncthreads();
        const int64_t chunk0 = chunk_s;
        __syncthreads();
        if (chunk0 >= total) break;
        for (int64_t wi = chunk0; wi < chunk0 + kChunk && wi < total; ++wi) {
            const int64_t gi = bl.work_list ? (int64_t)bl.work_list[wi] : wi;
            int64_t r0 = 0;
            int n;
            if (bl.clouds || bl.lower) {
                n = bl.npoints[gi];
            } else {
                r0 = bl.row_ptr[gi];
                n = (int)(bl.row_ptr[gi + 1] - r0) + 1;
            }
            double* feat = bl.features ? bl.features + 35 * gi : nullptr;
            if (n > NP) {
                if (bl.skip_above) continue;  // reduced by the overflow launch
                if (lane == 0) atomicOr(bl.error_flag, kErrTooManyPoints);
                if (feat && lane < 35) feat[lane] = __builtin_nan("");
                if (bl.counts && lane < 4) bl.counts[4 * gi + lane] = -1;
                continue;
            }
            // structure of gi and the 1/count weight (betti_features.cpp:62-63, 77)
            double weight = 1.0;
            if (bl.species) {
                int64_t lo = 0, hi = bl.num_structures - 1;
                while (lo < hi) {
                    const int64_t mid = (lo + hi + 1) >> 1;
                    if (bl.atom_offset[mid] <= gi) lo = mid;
                    else hi = mid - 1;
                }
                const int64_t s0 = bl.atom_offset[lo], s1 = bl.atom_offset[lo + 1];
                const int spc = bl.species[gi];
                int cnt = 0;
                for (int64_t j = s0 + lane; j < s1; j += kWave) cnt += (bl.species[j] == spc);
                cnt = wave_sum(cnt);
                weight = 1.0 / (double)cnt;
            }

            Complex<NP> cx{s, n, bl.thr, scratch, 0u, 0, 0, 0, 0, 0, 0};
#ifdef DGN_PHASE_TIMING
            cx.ph = ph;
            cx.tprev = &t_prev;
#endif
            DGN_PHASE(7);
            // ---- load the local cloud (betti_features.cpp:67-73) ----
            if (lane < n && bl.clouds) {
                const double* xc = bl.clouds + ((int64_t)gi * bl.cloud_stride + lane) * 3;
                s.u.cloud.X[lane][0] = xc[0];
                s.u.cloud.X[lane][1] = xc[1];
                s.u.cloud.X[lane][2] = xc[2];
                s.u.cloud.sq[lane] = (xc[0] * xc[0] + xc[1] * xc[1]) + xc[2] * xc[2];
            } else if (lane < n && !bl.lower) {
                const double* q = bl.pos + 3 * gi;
                double x[3];
                if (lane == 0) {
                    x[0] = q[0]; x[1] = q[1]; x[2] = q[2];
                } else {
                    const double* dv = bl.disp + 3 * (r0 + lane - 1);
                    x[0] = q[0] + dv[0]; x[1] = q[1] + dv[1]; x[2] = q[2] + dv[2];
                }
                s.u.cloud.X[lane][0] = x[0];
                s.u.cloud.X[lane][1] = x[1];
                s.u.cloud.X[lane][2] = x[2];
                // rowwise().squaredNorm(): (x0^2 + x1^2) + x2^2
                s.u.cloud.sq[lane] = (x[0] * x[0] + x[1] * x[1]) + x[2] * x[2];
            }
            lds_sync();
            // ---- distance matrix on the matrix cores (ripser_wrapper.cpp:64-67) ----
            if (bl.lower) {
                // given f32 lower triangle (ripser_wrapper.cpp:20-24 packing)
                const float* L = bl.lower + (int64_t)gi * ((int64_t)bl.cloud_stride * (bl.cloud_stride - 1) / 2);
                const int tot = n * (n - 1) / 2;
                for (int t = lane; t < tot; t += kWave) s.Dt[t] = L[t];  // same packing
            } else {
                typedef double double4_t __attribute__((ext_vector_type(4)));
                const int T = (n + 15) / 16;
                const int kk = lane >> 4;
                for (int I = 0; I < T; ++I) {
                    for (int J = 0; J <= I; ++J) {
                        const int ra = 16 * I + (lane & 15);
                        const int cb = 16 * J + (lane & 15);
                        const double xa = (ra < n && kk < 3) ? s.u.cloud.X[ra][kk] : 0.0;
                        const double xb = (cb < n && kk < 3) ? s.u.cloud.X[cb][kk] : 0.0;
                        const double4_t z = {0.0, 0.0, 0.0, 0.0};
                        // rank-1 products: operand k' nonzero only for k' == k -> round(x_ik * x_jk)
                        const double4_t p0 = __builtin_amdgcn_mfma_f64_16x16x4f64(kk == 0 ? xa : 0.0, kk == 0 ? xb : 0.0, z, 0, 0, 0);
                        const double4_t p1 = __builtin_amdgcn_mfma_f64_16x16x4f64(kk == 1 ? xa : 0.0, kk == 1 ? xb : 0.0, z, 0, 0, 0);
                        const double4_t p2 = __builtin_amdgcn_mfma_f64_16x16x4f64(kk == 2 ? xa : 0.0, kk == 2 ? xb : 0.0, z, 0, 0, 0);
                        const int col = 16 * J + (lane & 15);
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int row = 16 * I + (lane >> 4) + 4 * r;
                            if (row < n && col < row) {  // strict lower triangle (ripser_wrapper.cpp:20-24)
                                const double dot = (p0[r] + p1[r]) + p2[r];  // GEBP k order, no FMA
                                const double d2 = (s.u.cloud.sq[row] + s.u.cloud.sq[col]) - 2.0 * dot;
                                s.Dt[c2(row) + col] = (float)sqrt(fmax(d2, 0.0));
                            }
                        }
                    }
                }
            }
            lds_sync();
            DGN_PHASE(0);
            // ---- adjacency (sparse_distance_matrix: i != j and d <= thr, ripser.cpp:386-395) ----
            {
                uint64_t m = 0;
                if (lane < n) {
                    for (int w2 = 0; w2 < n; ++w2)
                        if (w2 != lane && cx.dist(lane, w2) <= cx.thr) m |= 1ull << w2;
                }
                s.adj[lane] = lane < n ? m : 0ull;
                s.tree[lane] = 0ull;
            }
            for (int i = lane; i < (int)(sizeof(s.cleared) / 4); i += kWave) s.cleared[i] = 0u;
            lds_sync();
            const int dim_max = n - 2 < 2 ? n - 2 : 2;  // ripser.cpp:560
            cx.n_inf0 = 0;
            cx.n_d0 = 0;
            // ---- dim 0: Prim on F-keys == Kruskal's forest in Ripser order (ripser.cpp:725-762) ----
            {
                bool in_tree = lane == 0;
                int parent = 0;
                uint64_t best = kInf;
                if (lane < n && lane != 0 && ((s.adj[0] >> lane) & 1ull)) best = cx.ekey(0, lane);
                if (n >= 1) cx.n_inf0 = 1;
                int added = 1;
                while (added < n) {
                    const uint64_t cand = (lane < n && !in_tree) ? best : kInf;
                    const uint64_t kmin = wave_min_u64(cand);
                    int v;
                    if (kmin == kInf) {  // new component: lowest vertex outside the forest
                        const uint64_t out = ballot(lane < n && !in_tree);
                        v = __ffsll((unsigned long long)out) - 1;
                        cx.n_inf0 += 1;
                    } else {
                        const uint64_t bal = ballot(cand == kmin);
                        v = __ffsll((unsigned long long)bal) - 1;
                        const int u = __shfl(parent, v, kWave);
                        const float dd = key_diam(kmin);
                        if (dd != 0.0f) {  // (0, d) emitted only if d != 0 (ripser.cpp:741-748)
                            if (lane == 0) s.d0[cx.n_d0] = dd;
                            cx.n_d0 += 1;
                        }
                        if (lane == 0) {
                            s.tree[u] |= 1ull << v;
                            s.tree[v] |= 1ull << u;
                        }
                    }
                    if (lane == v) in_tree = true;
                    ++added;
                    if (lane < n && !in_tree && ((s.adj[v] >> lane) & 1ull)) {
                        const uint64_t k = cx.ekey(v, lane);
                        if (k < best) { best = k; parent = v; }
                    }
                }
            }
            lds_sync();
            // ---- edge list (i > j, d <= thr), row-major ----
            int n_edges = 0;
            {
                const uint64_t low = lane < n ? (s.adj[lane] & ((lane == 0) ? 0ull : ((1ull << lane) - 1ull))) : 0ull;
                const int c = __popcll(low);
                const int inc = wave_inclusive_sum(c);
                n_edges = __shfl(inc, kWave - 1, kWave);
                int off = inc - c;
                uint64_t mm = low;
                while (mm) {
                    const int j = __ffsll((unsigned long long)mm) - 1;
                    mm &= mm - 1;
                    s.edges[off++] = (uint16_t)((lane << 8) | j);
                }
            }
            lds_sync();
            cx.n_p1 = 0;
            cx.n_p2 = 0;
            DGN_PHASE(1);
            uint64_t* na_key = cx.template sp<uint64_t>(ScratchLayout::na_key);
            uint64_t* na_tau = cx.template sp<uint64_t>(ScratchLayout::na_tau);
            uint32_t* mincof = cx.template sp<uint32_t>(ScratchLayout::mincof);
                    // ---- dim 1: one lane per column (non-tree edge) ----
            if (dim_max >= 1) {
                int nna = 0;
                for (int base = 0; base < n_edges; base += kWave) {
                    const int e = base + lane;
                    bool apparent = false, na_col = false;
                    float birth = 0.f, death = 0.f;
                    uint64_t colkey = 0, best = kInf;
                    if (e < n_edges) {
                        const int i = s.edges[e] >> 8, j = s.edges[e] & 255;
                        uint32_t mc = kNone;
                        if (!((s.tree[i] >> j) & 1ull)) {
                            birth = cx.dlow(i, j);
                            colkey = make_key(birth, pack2(i, j));
                            const uint64_t cand = s.adj[i] & s.adj[j];
                            if (cand) {
                                best = cx.min_cofacet_lane(1, i, j, 0, birth, cand);
                                death = key_diam(best);
                                bool col_unused;
                                // apparent iff (i,j) is the F-max facet of its pivot triangle
                                apparent = cx.max_facet(1, best, col_unused) == pack2(i, j);
                                if (apparent) {
                                    const uint32_t tp = key_packed(best);
                                    cx.set_cleared((tp >> 16) & 255, (tp >> 8) & 255, tp & 255);
                                } else {
                                    na_col = true;
                                }
                                mc = key_packed(best);
                            }
                        }
                        mincof[edge_dense(i, j)] = mc;
                    }
                    cx.append_pairs(1, apparent && death > birth, birth, death);
                    const uint64_t bal = ballot(na_col);
                    if (na_col) {
                        const int slot = nna + mask_prefix(bal);
                        if (slot < kNACap) {
                            na_key[slot] = colkey;
                            na_tau[slot] = best;
                        }
                    }
                    nna += __popcll(bal);
                }
                __syncthreads();
                DGN_PHASE(2);
#ifdef DGN_PHASE_TIMING
                ph[8] += nna;
                const int a0 = cx.n_adds;
#endif
                cx.reduce_serial(1, nna);
                lds_sync();
                DGN_PHASE(3);
#ifdef DGN_PHASE_TIMING
                ph[10] += cx.n_adds - a0;
#endif
            }
            // ---- dim 2: one lane per column (uncleared triangle) ----
            if (dim_max >= 2 && cx.err == 0) {
                int nna = 0;
                // stream triangles: each lane owns an edge (a > b) and walks c < b in adj[a] & adj[b]
                int next_edge = 0;
                int ea = 0, eb = 0;
                uint64_t tmask = 0;
                while (true) {
                    while (true) {  // refill lanes with empty masks
                        const bool need = tmask == 0;
                        const uint64_t bal = ballot(need);
                        if (!bal || next_edge >= n_edges) break;
                        const int e = next_edge + mask_prefix(bal);
                        if (need && e < n_edges) {
                            ea = s.edges[e] >> 8;
                            eb = s.edges[e] & 255;
                            tmask = s.adj[ea] & s.adj[eb] & ((1ull << eb) - 1ull);
                        }
                        next_edge += __popcll(bal);
                        if (ballot(tmask == 0) == 0) break;
                    }
                    const bool active = tmask != 0;
                    if (!ballot(active)) break;
                    bool apparent = false, na_col = false;
                    float birth = 0.f, death = 0.f;
                    uint64_t colkey = 0, best = kInf;
                    if (active) {
                        const int a = ea, b = eb;
                        const int c = __ffsll((unsigned long long)tmask) - 1;
                        tmask &= tmask - 1;
                        uint32_t mc = kNone;
                        if (!cx.is_cleared(a, b, c)) {
                            birth = cx.tri_diam(a, b, c);
                            colkey = make_key(birth, pack3(a, b, c));
                            const uint64_t cand = s.adj[a] & s.adj[b] & s.adj[c];
                            if (cand) {
                                best = cx.min_cofacet_lane(2, a, b, c, birth, cand);
                                death = key_diam(best);
                                bool col_unused;
                                // apparent iff (a,b,c) is the F-max facet of its pivot tetrahedron
                                apparent = cx.max_facet(2, best, col_unused) == pack3(a, b, c);
                                na_col = !apparent;
                                mc = key_packed(best);
                            }
                        }
                        mincof[tri_dense(a, b, c)] = mc;
                    }
                    cx.append_pairs(2, apparent && death > birth, birth, death);
                    const uint64_t bal = ballot(na_col);
                    if (na_col) {
                        const int slot = nna + mask_prefix(bal);
                        if (slot < kNACap) {
                            na_key[slot] = colkey;
                            na_tau[slot] = best;
                        }
                    }
                    nna += __popcll(bal);
                }
                __syncthreads();
                DGN_PHASE(4);
#ifdef DGN_PHASE_TIMING
                ph[9] += nna;
                const int a0 = cx.n_adds;
#endif
                cx.reduce_serial(2, nna);
                lds_sync();
                DGN_PHASE(5);
#ifdef DGN_PHASE_TIMING
                ph[11] += cx.n_adds - a0;
                ph[12] += cx.n_spills;
                ph[13] += 1;
#endif
            }
            __syncthreads();
            if (cx.n_p1 > kPairCap || cx.n_p2 > kPairCap) cx.err |= kErrPairs;
            if (cx.err) {
                if (lane == 0) atomicOr(bl.error_flag, cx.err);
                if (feat && lane < 35) feat[lane] = __builtin_nan("");
                if (bl.counts && lane < 4) bl.counts[4 * gi + lane] = -1;
                continue;
            }
            // ---- statistics (betti_features.cpp:24-55, 87-98; utils/math.hpp:9-28) ----
            // group g: 0 d0 death | 1..3 d1 pers, birth, death | 4..6 d2 pers, birth, death
            double myval = 0.0;
            for (int g = 0; g < 7; ++g) {
                const int m = g == 0 ? cx.n_d0 : (g <= 3 ? cx.n_p1 : cx.n_p2);
                double st[5] = {0, 0, 0, 0, 0};
                if (m > 0) {
                    const float2* P = g == 0 ? nullptr : cx.pairs(g <= 3 ? 1 : 2);
                    const int which = g == 0 ? 1 : ((g - 1) % 3 == 0 ? 2 : ((g - 1) % 3 == 1 ? 0 : 1));
                    double sum = 0.0, mx = -INFINITY, mn = INFINITY;
                    for (int i = lane; i < m; i += kWave) {
                        double v;
                        if (g == 0) v = (double)s.d0[i];
                        else {
                            const float2 pr = P[i];
                            const double bb = pr.x, dd = pr.y;
                            v = which == 0 ? bb : (which == 1 ? dd : dd - bb);
                        }
                        sum += v;
                        mx = fmax(mx, v);
                        mn = fmin(mn, v);
                    }
                    sum = wave_sum(sum);
                    mx = wave_max(mx);
                    mn = wave_min(mn);
                    const double mean = sum / (double)m;
                    double ss = 0.0;
                    for (int i = lane; i < m; i += kWave) {
                        double v;
                        if (g == 0) v = (double)s.d0[i];
                        else {
                            const float2 pr = P[i];
                            const double bb = pr.x, dd = pr.y;
                            v = which == 0 ? bb : (which == 1 ? dd : dd - bb);
                        }
                        ss += (v - mean) * (v - mean);
                    }
                    ss = wave_sum(ss);
                    st[0] = mean;
                    st[1] = sqrt(ss / (double)m);  // population std (math.hpp:13-16)
                    st[2] = mx;
                    st[3] = mn;
                    st[4] = sum * weight;  // weighted_sum = sum * weight (math.hpp:26-28)
                }
                const int r = lane - 5 * g;
                if (r == 0) myval = st[0];
                if (r == 1) myval = st[1];
                if (r == 2) myval = st[2];
                if (r == 3) myval = st[3];
                if (r == 4) myval = st[4];
            }
            if (feat && lane < 35) feat[lane] = myval;
            if (bl.pairs_out) {
                float2* po = reinterpret_cast<float2*>(bl.pairs_out) + (int64_t)gi * 3 * bl.pair_cap;
                for (int i = lane; i < cx.n_d0 && i < bl.pair_cap; i += kWave) po[i] = make_float2(0.0f, s.d0[i]);
                for (int i = lane; i < cx.n_p1 && i < bl.pair_cap; i += kWave) po[bl.pair_cap + i] = cx.pairs(1)[i];
                for (int i = lane; i < cx.n_p2 && i < bl.pair_cap; i += kWave) po[2 * bl.pair_cap + i] = cx.pairs(2)[i];
            }
            if (bl.counts && lane == 0) {
                bl.counts[4 * gi + 0] = cx.n_d0;
                bl.counts[4 * gi + 1] = cx.n_inf0;
                bl.counts[4 * gi + 2] = cx.n_p1;
                bl.counts[4 * gi + 3] = cx.n_p2;
            }
            lds_sync();
            DGN_PHASE(6);
        }
    }
#ifdef DGN_PHASE_TIMING
    if (lane == 0 && bl.phase_cycles)
        for (int k = 0; k < 32; ++k) if (k != 23) atomicAdd(&bl.phase_cycles[k], (unsigned long long)ph[k]);
    if (lane == 0 && bl.phase_cycles) atomicMax(&bl.phase_cycles[23], (unsigned long long)ph[23]);
#endif
}

// ---------------------------------------------------------------------------------------
int betti_max_points() { return 64; }
int64_t betti_scratch_bytes_per_wave() { return ScratchLayout::total; }

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

// route complexes with more than np_small points to the overflow list (wave-aggregated append)
__global__ __launch_bounds__(256) void betti_bucket_kernel(BettiLaunch bl, int np_small) {
    const int64_t gi = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int n = 0;
    if (gi < bl.num_atoms)
        n = (bl.clouds || bl.lower) ? bl.npoints[gi] : (int)(bl.row_ptr[gi + 1] - bl.row_ptr[gi]) + 1;
    const bool big = gi < bl.num_atoms && n > np_small;
    const uint64_t bal = ballot(big);
    if (!bal) return;
    const int leader = __ffsll((unsigned long long)bal) - 1;
    uint32_t base = 0;
    if (lane_id() == leader) base = atomicAdd(bl.overflow_len, (uint32_t)__popcll(bal));
    base = (uint32_t)__shfl((int)base, leader, kWave);
    if (big) bl.overflow_list[base + mask_prefix(bal)] = (int32_t)gi;
}

template <int NP>
static hipError_t launch_np(hipStream_t st, const BettiLaunch& b, int grid_waves, int64_t max_items) {
    int dev = 0, per_cu = 0;
    hipError_t e;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, dev)) != hipSuccess) return e;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, betti_kernel<NP>, kWave, 0);
    if (e != hipSuccess || per_cu <= 0) per_cu = 4;
    int grid = prop.multiProcessorCount * per_cu;
    if (grid > grid_waves) grid = grid_waves;
    const int64_t chunks = (max_items + kChunk - 1) / kChunk;
    if (grid > chunks) grid = (int)(chunks > 0 ? chunks : 1);
    hipLaunchKernelGGL(betti_kernel<NP>, dim3(grid), dim3(kWave), 0, st, b);
    return hipGetLastError();
}

static hipError_t launch_for(int np, hipStream_t st, const BettiLaunch& b, int grid_waves, int64_t max_items) {
    if (np == 32) return launch_np<32>(st, b, grid_waves, max_items);
    if (np == 48) return launch_np<48>(st, b, grid_waves, max_items);
    return launch_np<64>(st, b, grid_waves, max_items);
}

// Two-level dispatch: the main launch uses the instantiation sized for typical complexes
// (NP <= 48: about half the LDS of NP = 64, so twice the resident waves); complexes above it
// are listed by betti_bucket_kernel and reduced by an NP = 64 launch. Counters and the list
// length live on the device, so nothing synchronizes with the host in between.
hipError_t launch_betti(hipStream_t st, const BettiLaunch& b, int max_points, int grid_waves) {
    const int np_big = np_for(max_points);
    const int np_main = np_big > 48 ? 48 : np_big;
    BettiLaunch m = b;
    m.work_list = nullptr;
    m.queue = b.work_counter;
    m.skip_above = np_big > np_main ? 1 : 0;
    if (m.skip_above) {
        const int64_t blocks = (b.num_atoms + 255) / 256;
        hipLaunchKernelGGL(betti_bucket_kernel, dim3((unsigned)blocks), dim3(256), 0, st, b, np_main);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
    }
    hipError_t e = launch_for(np_main, st, m, grid_waves, b.num_atoms);
    if (e != hipSuccess || !m.skip_above) return e;
    BettiLaunch o = b;
    o.work_list = b.overflow_list;
    o.queue = b.work_counter2;
    o.skip_above = 0;
    return launch_for(np_big, st, o, grid_waves, b.num_atoms);
}

}  // namespace dgn
