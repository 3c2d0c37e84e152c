// betti_wg.hip — Vietoris–Rips persistence (dim 0/1/2, Z/2) and the 35 Betti statistics for
// local complexes of 129..362 points, ONE WORKGROUP (kNW waves) PER COMPLEX with the complex's
// distance matrix resident in LDS, for gfx950.
//
// The reference's default cutoff is 10 A (preprocess_betti.cpp:32,117; betti_features.hpp:37-39):
// FCC-256 complexes then have ~340 points. betti_wide.hip reduces them one wave per complex with
// the distance matrix in per-wave scratch; at ~2,000 resident waves those matrices (~230 KB each)
// overflow L2 and the Infinity Cache, and every walk step waits for HBM. Here the
// complex's u16 rank codes (betti_rank_codes: order- and equality-preserving, C(362, 2) < 2^16)
// sit in LDS as the packed lower triangle (<= 128 KB) next to the adjacency bitsets (<= 17 KB),
// so every distance read is an LDS read, and no per-simplex table lives in memory at all:
//   * load, adjacency: all waves;  Prim (wave 0) beside the edge list (wave 1);
//   * dim-1 / dim-2 apparent passes: lane per column, the edges dealt to the lanes from an LDS
//     counter, each lane's next edge prefetched (dim 2: a per-lane work queue over the edges'
//     triangles, as betti_wide.hip). No min-cofacet
//     tables: the reduction re-derives an apparent owner from the LDS matrix when it needs one
//     (lane-parallel, a few hundred cycles instead of a scattered HBM read);
//   * clearing: the dim-1 pivots (apparent and reduced) set a bit per triangle in a scratch bitset;
//     the dim-2 pass does not consult it (a cleared triangle is a dim-1 death, so never apparent in
//     dim 2 — each simplex is in at most one persistence pair) and the cleared columns are dropped
//     from the dim-2 column list before the sort, then the listed bits are reset;
//   * the reduction, in Ripser's column order, is driven by wave 0 alone (column records, pivot
//     table, V list in LDS, V store); the other waves sleep at a barrier and wake only for the pivot
//     searches — the reduction's hot loop — whose (V entry, bitset word) pairs they share, their
//     minima combined through LDS (two barriers per floor round, none per column);
//   * the pivot table (scratch) is sized by the column count, so it stays cache-resident, and an
//     insert reuses the empty slot its last lookup found.
// Same algorithm and output contract as betti_wide.hip (pairing of a total order: the emitted
// multiset equals Ripser's, ripser.cpp:514-1269; death > birth only, essential dim >= 1 classes
// not emitted, ripser.cpp:1209-1225, 1240). Capacity overflows list the complex for the
// capacity-retry launch (betti_wide.hip big layout).
#include "dgn_internal.hpp"

#ifndef DGN_WG_WAVES
#define DGN_WG_WAVES 8
#endif

namespace dgn {
namespace {

#define WG_LDS __attribute__((address_space(3)))

constexpr int kNW = DGN_WG_WAVES;          // waves per workgroup (per complex)
static_assert(kNW >= 2, "Prim and the edge list run on two waves");
constexpr int kWgThreads = kNW * kWave;
constexpr int kVlCap = 512;                // V list entries (LDS); more: capacity retry
constexpr uint64_t kInf = ~0ull;
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint64_t kLazy = 1ull << 63;    // pivot meta: V = {column simplex}
constexpr uint64_t kNoMeta = ~0ull;
constexpr int kMetaLenBits = 24;
// error bits: the same as betti_wide.hip (decoded in dgn_api.cpp)
constexpr uint32_t kEPoints = 1u << 0, kEWork = 1u << 1, kENA = 1u << 2, kEPiv = 1u << 3, kEPairs = 1u << 4,
                   kER = 1u << 5, kEGuard = 1u << 7;
constexpr uint32_t kECapacity = kEWork | kENA | kEPiv | kEPairs | kER | kEGuard;
constexpr int VB = 9;  // bits per packed vertex (n <= 362 < 512)
constexpr uint64_t VM = (1ull << VB) - 1;

// control block (static LDS)
struct WgCtl {
    uint32_t ticket[2];  // complex dequeue (double-buffered by iteration parity)
    uint32_t ctr[6];     // dim-1 edge chunks, dim-2 edges, dim-1 / dim-2 columns, clear list
    int32_t nedges;
    uint32_t err;        // wave 0's error bits after a reduction
    // pivot-search request (wave 0 -> helper waves) and the per-wave results
    uint64_t rq_floor;
    int32_t rq_v, rq_dim, rq_stop, npiv;
    uint64_t smin[kNW];
    uint64_t spk[kNW];
    uint32_t scnt[kNW];
    uint32_t vl[kVlCap];  // V list (packed simplices) and their diameters
    uint32_t vd[kVlCap];
};
__shared__ WgCtl wg_ctl;
extern __shared__ uint64_t wg_dyn[];

__device__ __forceinline__ uint32_t b2(uint32_t v) { return v * (v - 1u) / 2u; }
__device__ __forceinline__ uint32_t b3(uint32_t v) { return b2(v) * (v - 2u) / 3u; }
__device__ __forceinline__ uint32_t b4(uint32_t v) { return b3(v) * (v - 3u) / 4u; }  // < 2^32 for v <= 362
__device__ __forceinline__ uint32_t rl(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }
__device__ __forceinline__ uint64_t rl64(uint64_t x, int l) {
    return ((uint64_t)rl((uint32_t)(x >> 32), l) << 32) | rl((uint32_t)x, l);
}
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) { return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x); }
__device__ __forceinline__ int pv(uint64_t p, int field) { return (int)((p >> (VB * field)) & VM); }
// combinatorial index (Ripser's colex numbering, ripser.cpp:181-201), 32-bit: C(362, 4) < 2^32
__device__ __forceinline__ uint32_t pidx(int nv, uint64_t p) {
    if (nv == 2) return b2(pv(p, 1)) + pv(p, 0);
    if (nv == 3) return b3(pv(p, 2)) + b2(pv(p, 1)) + pv(p, 0);
    return b4(pv(p, 3)) + b3(pv(p, 2)) + b2(pv(p, 1)) + pv(p, 0);
}
__device__ __forceinline__ uint64_t pinsert(int nv, uint64_t p, int x) {
    int below = 0;
    for (int t = 0; t < nv; ++t) below += pv(p, t) < x;
    const uint64_t mask = (1ull << (VB * below)) - 1;
    return ((p & ~mask) << VB) | ((uint64_t)x << (VB * below)) | (p & mask);
}
// key: (distance code << 32) | ~index — ascending keys are Ripser's filtration order
// (greater_diameter_or_smaller_index, ripser.cpp:318-324)
__device__ __forceinline__ uint64_t wkey(uint32_t dc, uint32_t idx) { return ((uint64_t)dc << 32) | (uint64_t)(~idx); }
__device__ __forceinline__ uint32_t kdiam(uint64_t key) { return (uint32_t)(key >> 32); }
__device__ __forceinline__ int c2i(int x) { return x * (x - 1) / 2; }
// workgroup-scope LDS add of `v` by lane 0 (every lane executes the atomic: no branch on the
// lane, see betti_kernels.hip's dequeue); the old value, wave-uniform
__device__ __forceinline__ uint32_t lds_add_uniform(uint32_t* p, uint32_t v) {
    const uint32_t old = __hip_atomic_fetch_add(p, lane_id() == 0 ? v : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return rl(old, 0);
}
// Workgroup barrier that orders LDS only: waits for this wave's LDS operations (lgkmcnt), not
// for its outstanding global loads and stores as __syncthreads' workgroup fence does (vmcnt(0):
// wave 0's table inserts and V-store writes would stall every pivot-search round)
__device__ __forceinline__ void sync_lds() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
// min over the wave of a u32 (DPP row rotations + 4 readlanes)
__device__ __forceinline__ uint32_t wave_min32(uint32_t x) {
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x121, 0xf, 0xf, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x122, 0xf, 0xf, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x124, 0xf, 0xf, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp((int)x, (int)x, 0x128, 0xf, 0xf, false));
    return min(min(rl(x, 0), rl(x, 16)), min(rl(x, 32), rl(x, 48)));
}

template <int KW>
struct WgCx {
    const BettiLaunch& bl;
    const WideLayout& ly;
    WG_LDS uint64_t* adj;  // [n][KW]: row v = the neighbours of vertex v
    WG_LDS uint16_t* par;  // [n]: spanning-forest parent, 0xFFFF = root
    WG_LDS uint16_t* Dm;   // packed lower triangle of rank codes: (i > j) at i(i-1)/2 + j
    uint8_t* scr;
    int n, W, wv, lane;
    uint32_t ub;           // codes below ub are edges (distance <= threshold)
    bool zero0;            // code 0 is the distance 0
    uint32_t err;
    int n_d0, n_inf0, n_p1, n_p2;
    const uint32_t* vals;  // the complex's sorted f32 distances (code -> value)
    uint32_t hmask;        // pivot table slots in use - 1 (sized per reduction)
    int ins_slot;          // the empty table slot the last lookup found (-1: probe on insert)

    template <class T>
    __device__ T* sp(int64_t off) const { return reinterpret_cast<T*>(scr + off); }
    __device__ uint32_t d(int i, int j) const {
        const uint32_t hi = (uint32_t)max(i, j), lo = (uint32_t)min(i, j);
        return Dm[((hi * (hi - 1u)) >> 1) + lo];
    }
    __device__ uint64_t aw(int v, int w) const { return adj[v * KW + w]; }
    __device__ bool is_tree(int i, int j) const { return par[i] == j || par[j] == i; }
    __device__ uint32_t sdiam(int dim, uint64_t p) const {
        if (dim == 1) return d(pv(p, 1), pv(p, 0));
        return max(max(d(pv(p, 2), pv(p, 1)), d(pv(p, 2), pv(p, 0))), d(pv(p, 1), pv(p, 0)));
    }
#ifdef DGN_PHASE_TIMING
    // diagnostics build: wave 0's s_memtime cycles per phase / reduction sub-phase, and counters,
    // into bl.phase_cycles (the slots tools/diag_wide.py reads)
    uint64_t tq = 0;
    __device__ void dg_add(int k, uint64_t v) const {
        if (wv == 0 && lane == 0 && bl.phase_cycles) atomicAdd(&bl.phase_cycles[k], (unsigned long long)v);
    }
    __device__ void dg_mark(int k) {
        const uint64_t t = __builtin_amdgcn_s_memtime();
        if (k >= 0) dg_add(k, t - tq);
        tq = t;
    }
#define WG_MARK(k) dg_mark(k)
#define WG_COUNT(k, v) dg_add(k, (uint64_t)(v))
#else
#define WG_MARK(k) \
    do {           \
    } while (0)
#define WG_COUNT(k, v) \
    do {               \
    } while (0)
#endif

    // ---- rank codes -> LDS, threshold code, adjacency bitsets ----
    __device__ void load(int64_t slot) {
        const int tid = threadIdx.x;
        const int m = c2i(n);
        const uint32_t* Lc = bl.rank_codes + slot * bl.rank_stride;  // rank_stride: multiple of 64
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
        for (int t = 4 * tid; t < m; t += 4 * kWgThreads) {
            if (t + 4 <= m) {
                const u32x4 c = *reinterpret_cast<const u32x4*>(Lc + t);
                const u16x4 h = {(uint16_t)c.x, (uint16_t)c.y, (uint16_t)c.z, (uint16_t)c.w};
                *reinterpret_cast<WG_LDS u16x4*>(Dm + t) = h;
            } else {
                for (int k = t; k < m; ++k) Dm[k] = (uint16_t)Lc[k];
            }
        }
        // ub = #{sorted distances <= thr} (sparse_distance_matrix keeps d <= threshold,
        // ripser.cpp:386-395): two rounds of parallel probes of the sorted triangle (m >= 2016
        // for the > 64-point complexes of the wide list, so every first-round probe is >= 0)
        const uint32_t tb = __float_as_uint(bl.thr);
        const int64_t pr = ((int64_t)(tid + 1) * m) / kWgThreads - 1;
        const int k1 = __syncthreads_count(pr >= 0 && vals[pr] <= tb);
        const int64_t lo = k1 == 0 ? 0 : ((int64_t)k1 * m) / kWgThreads;  // probe k1 - 1 is true
        const int64_t hi = k1 == kWgThreads ? m : ((int64_t)(k1 + 1) * m) / kWgThreads - 1;  // probe k1 false
        const int k2 = __syncthreads_count(lo + tid < hi && vals[lo + tid] <= tb);
        ub = (uint32_t)(lo + k2);
        zero0 = vals[0] == 0u;
        // Dm complete (the barriers above); adjacency rows, one ballot per (row, word)
        for (int p = wv; p < n * W; p += kNW) {
            const int i = p / W, w = p - i * W;
            const int j = 64 * w + lane;
            const bool e = j < n && j != i && d(i, j) < ub;
            const uint64_t b = ballot(e);
            if (lane == 0) adj[i * KW + w] = b;
        }
        __syncthreads();
    }

    // ---- dim 0 (wave 0): Prim on F-keys == Kruskal's forest in Ripser's order (ripser.cpp:725-762)
    __device__ void prim() {
        uint32_t* d0s = sp<uint32_t>(ly.d0);  // death codes (values in finish)
        uint64_t best[KW];
        int bp[KW];
        uint32_t intree = lane == 0 ? 1u : 0u;  // bit t: vertex 64 t + lane is in the forest
        for (int i = lane; i < n; i += kWave) par[i] = 0xFFFF;
#pragma unroll
        for (int t = 0; t < KW; ++t) {
            const int v = 64 * t + lane;
            best[t] = kInf;
            bp[t] = 0;
            if (t < W && v < n && v != 0 && ((aw(0, t) >> lane) & 1ull)) best[t] = wkey(d(0, v), b2(v));
        }
        n_inf0 = 1;
        n_d0 = 0;
        for (int added = 1; added < n; ++added) {
            uint64_t lmin = kInf;
            int lt = 0, lp = 0, lfree = 1 << 30;
#pragma unroll
            for (int t = 0; t < KW; ++t) {
                const int v = 64 * t + lane;
                const bool out = t < W && v < n && !((intree >> t) & 1u);
                if (out && best[t] < lmin) {
                    lmin = best[t];
                    lt = t;
                    lp = bp[t];
                }
                if (out && v < lfree) lfree = v;
            }
            const uint64_t m = wave_min(lmin);
            int v;
            if (m == kInf) {  // new component: lowest vertex outside the forest
                v = wave_min(lfree);
                ++n_inf0;
            } else {
                const int l = __ffsll((unsigned long long)ballot(lmin == m)) - 1;
                v = 64 * (int)rl((uint32_t)lt, l) + l;
                const int u = (int)rl((uint32_t)lp, l);
                const uint32_t dd = kdiam(m);
                if (!(dd == 0u && zero0)) {  // (0, d) emitted only if d != 0 (ripser.cpp:741-748)
                    if (lane == 0) d0s[n_d0] = dd;
                    ++n_d0;
                }
                if (lane == 0) par[v] = (uint16_t)u;
            }
            if (lane == (v & 63)) intree |= 1u << (v >> 6);
#pragma unroll
            for (int t = 0; t < KW; ++t) {
                const int w = 64 * t + lane;
                if (t < W && w < n && !((intree >> t) & 1u) && ((aw(v, t) >> lane) & 1ull)) {
                    const uint64_t k = wkey(d(v, w), v > w ? b2(v) + w : b2(w) + v);
                    if (k < best[t]) {
                        best[t] = k;
                        bp[t] = v;
                    }
                }
            }
        }
    }

    // ---- edges (i > j, d <= thr) in index order (wave 1, beside Prim) ----
    __device__ int edge_list() {
        uint32_t* edges = sp<uint32_t>(ly.edges);
        int off = 0;
        for (int i = 1; i < n; ++i)
            for (int w = 0; 64 * w < i; ++w) {
                uint64_t bits = aw(i, w);
                const int lim = i - 64 * w;
                if (lim < 64) bits &= (1ull << lim) - 1ull;
                if ((bits >> lane) & 1ull) edges[off + mask_prefix(bits)] = ((uint32_t)i << VB) | (uint32_t)(64 * w + lane);
                off += __popcll(bits);
            }
        return off;
    }

    // append the lanes' non-apparent columns (lanes with `na`) through the LDS column counter
    __device__ void na_append(bool na, uint32_t* ctr, uint64_t colkey, uint64_t tau, uint64_t tv, uint32_t colp) {
        const uint64_t bal = ballot(na);
        if (!bal) return;
        const uint32_t base = lds_add_uniform(ctr, (uint32_t)__popcll(bal));
        if (na) {
            const uint32_t slot = base + (uint32_t)mask_prefix(bal);
            if (slot < (uint32_t)ly.na_cap) {
                sp<uint64_t>(ly.na_key)[slot] = colkey;
                sp<uint64_t>(ly.na_tau)[slot] = tau;
                sp<uint64_t>(ly.na_tv)[slot] = tv;
                sp<uint32_t>(ly.na_col)[slot] = colp;
            }
        }
    }
    // clearing (dim-1 pivot triangles): a bit per triangle index in the bitset (layout mc_t), each
    // set bit's word listed (layout mc_e) for the reset at the end of the complex
    __device__ void clear_mark(bool on, uint32_t tidx) {
        const uint64_t bal = ballot(on);
        if (!bal) return;
        const uint32_t base = lds_add_uniform(&wg_ctl.ctr[4], (uint32_t)__popcll(bal));
        if (on) {
            atomicOr(sp<uint32_t>(ly.mc_t) + (tidx >> 5), 1u << (tidx & 31));
            sp<uint32_t>(ly.mc_e)[base + (uint32_t)mask_prefix(bal)] = tidx >> 5;
        }
    }

    // ---- dim 1: lane per column (non-tree edge), 64-edge chunks dealt from an LDS counter; the
    // next chunk's edge words are loaded while this one is walked ----
    __device__ void pass_dim1(int n_edges) {
        const uint32_t* edges = sp<uint32_t>(ly.edges);
        int base = (int)lds_add_uniform(&wg_ctl.ctr[0], kWave);
        uint32_t ed = base + lane < n_edges ? edges[base + lane] : 0u;
        while (base < n_edges) {
            const int e = base + lane;
            const uint32_t cur = ed;
            base = (int)lds_add_uniform(&wg_ctl.ctr[0], kWave);
            ed = base + lane < n_edges ? edges[base + lane] : 0u;
            bool na = false, app = false;
            uint64_t colkey = 0, best = kInf, bestp = 0;
            uint32_t colp = 0;
            const int i = (int)(cur >> VB), j = (int)(cur & VM);
            if (e < n_edges && !is_tree(i, j)) {
                const uint32_t dij = d(i, j);
                colp = cur;
                colkey = wkey(dij, b2(i) + j);
                // F-minimal cofacet: walking k downwards over the common neighbours, the first k
                // with both distances <= d(i, j) ends the walk; before it, a smaller k wins only
                // with a strictly smaller diameter
                uint32_t bd = 0xFFFFFFFFu, hda = 0, hdb = 0;
                int bk = -1;
                bool found = false;
                for (int w = W - 1; w >= 0 && !found; --w) {
                    uint64_t m = aw(i, w) & aw(j, w);
                    while (m != 0ull && !found) {
                        const int bit = 63 - __clzll((long long)m);
                        m &= ~(1ull << bit);
                        const int k = 64 * w + bit;
                        const uint32_t da = d(i, k), db = d(j, k);
                        const uint32_t dk = max(da, db);
                        if (dk <= dij) {
                            bd = dij;
                            bk = k;
                            found = true;
                            hda = da;
                            hdb = db;
                        } else if (dk < bd) {
                            bd = dk;
                            bk = k;
                        }
                    }
                }
                if (bk >= 0) {
                    bestp = pinsert(2, cur, bk);
                    best = wkey(bd, pidx(3, bestp));
                    // apparent iff (i, j) is the F-max facet of its zero-persistence cofacet
                    app = found && (bk > i || hdb < dij) && (bk > j || hda < dij);
                    na = !app;
                }
            }
            clear_mark(app, app ? pidx(3, bestp) : 0u);  // clearing for dim 2
            na_append(na, &wg_ctl.ctr[2], colkey, best, bestp, colp);
        }
    }

    // ---- dim 2: lane per column (triangle), a per-lane work queue over the edges, edges dealt
    // from an LDS counter (see betti_wide.hip pass_dim2). Cleared triangles are walked too (they are
    // never apparent) and dropped from the column list by the sort's filter ----
    static constexpr int kStep = 4;
    __device__ void pass_dim2(int n_edges) {
        const uint32_t* edges = sp<uint32_t>(ly.edges);
        // each lane's next edge word is prefetched when it takes an edge (kNone: none left)
        uint32_t nxt;
        {
            const int e0 = (int)lds_add_uniform(&wg_ctl.ctr[1], kWave) + lane;
            nxt = e0 < n_edges ? edges[e0] : kNone;
        }
        int ea = 0, eb = 0, tw = -1;
        uint64_t tm = 0;
        bool act = false, fresh = false;
        int c = 0, w = 0, bk = 0;
        uint64_t m = 0;
        uint32_t tidx = 0;
        uint32_t bd = 0xFFFFFFFFu;
        uint32_t ds = 0, dab = 0, dac = 0, dbc = 0, colp = 0, hda = 0, hdb = 0, hdc = 0;
        bool found = false;
        for (;;) {
            for (;;) {
                while (!act && tm == 0ull && tw >= 0) {
                    ++tw;
                    if (64 * tw >= eb) {
                        tw = -1;
                        break;
                    }
                    tm = aw(ea, tw) & aw(eb, tw);
                    const int lim = eb - 64 * tw;
                    if (lim < 64) tm &= (1ull << lim) - 1ull;
                }
                const bool need = !act && tm == 0ull && nxt != kNone;
                const uint64_t bal = ballot(need);
                if (!bal) break;
                const int base = (int)lds_add_uniform(&wg_ctl.ctr[1], (uint32_t)__popcll(bal));
                if (need) {
                    ea = (int)(nxt >> VB);
                    eb = (int)(nxt & VM);
                    tw = 0;
                    tm = aw(ea, 0) & aw(eb, 0);
                    if (eb < 64) tm &= (1ull << eb) - 1ull;
                    const int e = base + mask_prefix(bal);
                    nxt = e < n_edges ? edges[e] : kNone;
                }
            }
            if (!act && tm != 0ull) {
                c = 64 * tw + __ffsll((unsigned long long)tm) - 1;
                tm &= tm - 1ull;
                act = fresh = true;
                tidx = b3(ea) + b2(eb) + c;
                colp = ((uint32_t)ea << (2 * VB)) | ((uint32_t)eb << VB) | (uint32_t)c;
                w = W - 1;
                m = aw(ea, w) & aw(eb, w) & aw(c, w);
                bd = 0xFFFFFFFFu;
                bk = -1;
                found = false;
            }
            if (!ballot(act)) break;
            bool na = false;
            uint64_t colkey = 0, ntau = kInf, ntv = 0;
            uint32_t ncolp = 0;
            if (act) {
                const int a = ea, b = eb;
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
                if (fresh) {
                    dab = d(a, b);
                    dac = d(a, c);
                    dbc = d(b, c);
                    ds = max(max(dab, dac), dbc);
                    fresh = false;
                }
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
                if (found || !val[kStep - 1]) {
                    if (bk >= 0) {  // no cofacet: zero coboundary, not a column
                        const uint64_t bestp = pinsert(3, colp, bk);
                        const bool app = found && (bk > a || max(max(hdb, hdc), dbc) < ds) &&
                                         (bk > b || max(max(hda, hdc), dac) < ds) &&
                                         (bk > c || max(max(hda, hdb), dab) < ds);
                        na = !app;
                        colkey = wkey(ds, tidx);
                        ntau = wkey(bd, pidx(4, bestp));
                        ntv = bestp;
                        ncolp = colp;
                    }
                    act = false;
                }
            }
            na_append(na, &wg_ctl.ctr[3], colkey, ntau, ntv, ncolp);
        }
    }

    // sum of one int per thread over the workgroup (LDS: the pivot-search result slots)
    __device__ int block_sum(int x) {
        const int s = wave_sum(x);
        if (lane == 0) wg_ctl.scnt[wv] = (uint32_t)s;
        __syncthreads();
        int t = 0;
#pragma unroll
        for (int q = 0; q < kNW; ++q) t += (int)wg_ctl.scnt[q];
        __syncthreads();
        return (int)uni((uint32_t)t);
    }

    // ---- non-apparent columns in Ripser's order: bitonic sort (key descending) of (key, slot)
    // pairs in scratch by all threads, 4 compare-exchanges per thread per step with their loads
    // issued together; dim 2 first drops the cleared columns (key 0 sorts last, like the
    // padding). Returns the number of columns to reduce. ----
    __device__ int sort_na(int dim, int cnt) {
        const int tid = threadIdx.x;
        int N = 1;
        while (N < cnt) N <<= 1;
        uint64_t* K = sp<uint64_t>(ly.na_key);
        uint32_t* P = sp<uint32_t>(ly.na_perm);
        const uint32_t* Cc = sp<uint32_t>(ly.na_col);
        const uint32_t* clr = sp<uint32_t>(ly.mc_t);
        int drop = 0;
        for (int i = tid; i < N; i += kWgThreads) {
            bool gone = i >= cnt;
            if (dim == 2 && !gone) {
                const uint32_t cp = Cc[i];
                const uint32_t t = b3(cp >> (2 * VB)) + b2((cp >> VB) & VM) + (cp & VM);
                // the bits were set by L2 atomics: an L1-bypassing (agent-scope) load
                const uint32_t word = __hip_atomic_load(clr + (t >> 5), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                gone = (word >> (t & 31)) & 1u;
                drop += gone ? 1 : 0;
            }
            if (gone) K[i] = 0ull;
            P[i] = (uint32_t)i;
        }
        const int dropped = dim == 2 ? block_sum(drop) : 0;
        if (dim != 2) __syncthreads();
        const int half = N >> 1;
        for (int k = 2; k <= N; k <<= 1)
            for (int j = k >> 1; j > 0; j >>= 1) {
                const int lj = __ffs(j) - 1;
                for (int p0 = tid; p0 < half; p0 += 4 * kWgThreads) {
                    int ii[4];
                    uint64_t x[4], y[4];
                    uint32_t px[4], py[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int p = p0 + u * kWgThreads;
                        const int pc = p < half ? p : 0;
                        ii[u] = ((pc >> lj) << (lj + 1)) | (pc & (j - 1));
                        x[u] = K[ii[u]];
                        y[u] = K[ii[u] | j];
                        px[u] = P[ii[u]];
                        py[u] = P[ii[u] | j];
                    }
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        if (p0 + u * kWgThreads >= half) continue;
                        const int i = ii[u];
                        if (((i & k) == 0) ? (x[u] < y[u]) : (x[u] > y[u])) {
                            K[i] = y[u];
                            K[i | j] = x[u];
                            P[i] = py[u];
                            P[i | j] = px[u];
                        }
                    }
                }
                __syncthreads();
            }
        return cnt - dropped;
    }

    // ---- pivot table: open addressing in scratch (key 0 = empty), wave 0 only ----
    __device__ static uint32_t hmix(uint64_t k) {
        k ^= k >> 33;
        k *= 0xff51afd7ed558ccdull;
        k ^= k >> 33;
        return (uint32_t)k;
    }
    __device__ uint64_t hfind(uint64_t k) {
        const uint64_t* HK = sp<uint64_t>(ly.h_key);
        const uint64_t* HM = sp<uint64_t>(ly.h_meta);
        const uint32_t base = hmix(k) & hmask;
        for (uint32_t probe = 0; probe <= hmask; probe += kWave) {
            const uint64_t x = HK[(base + probe + (uint32_t)lane) & hmask];
            const uint64_t hit = ballot(x == k), emp = ballot(x == 0ull);
            const int fh = hit ? __ffsll((unsigned long long)hit) - 1 : kWave;
            const int fe = emp ? __ffsll((unsigned long long)emp) - 1 : kWave;
            if (fh < fe) return uni64(HM[(base + probe + (uint32_t)fh) & hmask]);
            if (fe < kWave) {
                ins_slot = (int)((base + probe + (uint32_t)fe) & hmask);
                return kNoMeta;
            }
        }
        ins_slot = -1;
        return kNoMeta;
    }
    __device__ bool hinsert(uint64_t k, uint64_t meta, int npiv) {
        if (npiv >= ly.na_cap) return false;
        uint64_t* HK = sp<uint64_t>(ly.h_key);
        uint64_t* HM = sp<uint64_t>(ly.h_meta);
        int slot = ins_slot;
        if (slot < 0) {  // the lookup saw no empty slot: probe
            const uint32_t base = hmix(k) & hmask;
            for (uint32_t probe = 0; probe <= hmask && slot < 0; probe += kWave) {
                const uint64_t emp = ballot(HK[(base + probe + (uint32_t)lane) & hmask] == 0ull);
                if (emp) slot = (int)((base + probe + (uint32_t)(__ffsll((unsigned long long)emp) - 1)) & hmask);
            }
            if (slot < 0) return false;
        }
        if (lane == 0) {
            HK[slot] = k;
            HM[slot] = meta;
            sp<uint32_t>(ly.h_used)[npiv] = (uint32_t)slot;
        }
        return true;
    }

    // Inserted vertex of the F-minimal cofacet of f (dim 1: edge, dim 2: triangle; packed) over
    // the common neighbours of f's vertices, lane-parallel from the LDS matrix: the minimal
    // (diameter, -vertex) — the walk's result in pass_dim1 / pass_dim2 (the first k walking
    // downwards with the smallest diameter). kNone if f has no cofacet.
    __device__ uint32_t min_cofacet_vertex(int dim, uint64_t f) const {
        const int a = dim == 1 ? pv(f, 1) : pv(f, 2);
        const int b = dim == 1 ? pv(f, 0) : pv(f, 1);
        const int c = pv(f, 0);
        const uint32_t ds = sdiam(dim, f);
        uint32_t best = kNone;
#pragma unroll
        for (int t = 0; t < KW; ++t) {
            if (t >= W) break;
            uint64_t am = aw(a, t) & aw(b, t);
            if (dim == 2) am &= aw(c, t);
            const int x = min(64 * t + lane, n - 1);
            const uint32_t dd = max(max(ds, dim == 2 ? d(c, x) : 0u), max(d(a, x), d(b, x)));
            const uint32_t key = (dd << 16) | (uint32_t)(511 - (64 * t + lane));
            if ((am >> lane) & 1ull) best = min(best, key);
        }
        const uint32_t m = wave_min32(best);
        return m == kNone ? kNone : (uint32_t)(511 - (int)(m & 0xFFFFu));
    }

    // Owner of the pivot tau (wave 0): the pivot table's first 64-slot window (a hit returns its
    // metadata), else the apparent owner — tau's F-max facet f, if tau is f's F-minimal cofacet —
    // re-derived from the LDS matrix (app = f's packed vertices), else kNoMeta / kNone. A miss
    // leaves the window's first empty slot in ins_slot for the insert.
    __device__ uint64_t lookup(int dim, uint64_t tau, uint64_t tv, uint32_t& app) {
        const uint64_t* HK = sp<uint64_t>(ly.h_key);
        const uint64_t* HM = sp<uint64_t>(ly.h_meta);
        const uint32_t base = hmix(tau) & hmask;
        const uint32_t slot = (base + (uint32_t)lane) & hmask;
        const uint64_t hk = HK[slot];
        const uint64_t hm = HM[slot];
        const int nv = dim + 2;
        const int v0 = pv(tv, nv - 1), v1 = pv(tv, nv - 2), v2 = pv(tv, nv - 3), v3 = nv == 4 ? pv(tv, 0) : 0;
        // F-max facet of tau from its edge lengths (the largest key: largest diameter, then the
        // smallest index), computed while the table window is in flight
        uint32_t dd[4][4];
        dd[0][1] = d(v0, v1);
        dd[0][2] = d(v0, v2);
        dd[1][2] = d(v1, v2);
        if (nv == 4) {
            dd[0][3] = d(v0, v3);
            dd[1][3] = d(v1, v3);
            dd[2][3] = d(v2, v3);
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
        const uint64_t hit = ballot(hk == tau), emp = ballot(hk == 0ull);
        const int fh = hit ? __ffsll((unsigned long long)hit) - 1 : kWave;
        const int fe = emp ? __ffsll((unsigned long long)emp) - 1 : kWave;
        app = kNone;
        if (fh < fe) return rl64(hm, fh);
        if (fe < kWave) {
            ins_slot = (int)((base + (uint32_t)fe) & hmask);
        } else {  // the window was full: probe on (rare at load factor <= 1/2)
            const uint64_t mm = hfind(tau);
            if (mm != kNoMeta) return mm;
        }
        const int vd = drop == 0 ? v0 : (drop == 1 ? v1 : (drop == 2 ? v2 : v3));
        if (min_cofacet_vertex(dim, bestf) == (uint32_t)vd) app = (uint32_t)bestf;
        return kNoMeta;
    }

    // ---- V list (wave 0, LDS) ----
    __device__ int v_find(uint32_t x, int v) const {
        for (int base = 0; base < v; base += kWave) {
            const uint32_t y = base + lane < v ? wg_ctl.vl[base + lane] : kNone;
            const uint64_t bal = ballot(y == x);
            if (bal) return base + __ffsll((unsigned long long)bal) - 1;
        }
        return -1;
    }
    __device__ bool v_toggle(int dim, uint32_t x, int& v) {
        const int pos = v_find(x, v);
        if (pos >= 0) {
            if (pos != v - 1) {
                const uint32_t last = uni(wg_ctl.vl[v - 1]), lastd = uni(wg_ctl.vd[v - 1]);
                if (lane == 0) {
                    wg_ctl.vl[pos] = last;
                    wg_ctl.vd[pos] = lastd;
                }
            }
            v = v - 1;
        } else {
            if (v >= kVlCap) return false;
            const uint32_t dx = sdiam(dim, x);
            if (lane == 0) {
                wg_ctl.vl[v] = x;
                wg_ctl.vd[v] = dx;
            }
            v = v + 1;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        return true;
    }

    // One wave's share of a pivot search (every wave): the (V entry, bitset word) pairs p = e W + t,
    // p = wv, wv + kNW, ...; lane k of a pair (s, t) evaluates the cofacet s u {64 t + k} (32-bit
    // combinatorial index: the partial sums of s's vertices plus x's binomial at its position; the
    // packed cofacet is built once, for the winning lane). Writes the wave's minimum above
    // `floor`, its multiplicity and the packed cofacet to the wave's LDS slot.
    __device__ void search_share(int dim, int v, uint64_t floor) {
        const int k = lane;
        uint64_t lmin = kInf;
        int lcnt = 0, lx = 0;
        uint32_t ls = 0;
        auto eval = [&](uint32_t s, uint32_t ds, int t) __attribute__((always_inline)) {
            const int a = dim == 1 ? pv(s, 1) : pv(s, 2);
            const int b = dim == 1 ? pv(s, 0) : pv(s, 1);
            const int c = pv(s, 0);
            const int x = 64 * t + k;
            const int xr = min(x, n - 1);
            const uint32_t da = d(a, xr), db = d(b, xr), dc = dim == 2 ? d(c, xr) : 0u;
            uint64_t am = aw(a, t) & aw(b, t);
            if (dim == 2) am &= aw(c, t);
            const uint32_t dd = max(max(ds, dc), max(da, db));
            const uint32_t ux = (uint32_t)x;
            const uint32_t ua = (uint32_t)a, ubb = (uint32_t)b, uc = (uint32_t)c;
            uint32_t idx;
            if (dim == 1) {  // triangle (a, b) u {x}
                idx = x > a ? b3(ux) + b2(ua) + ubb : (x > b ? b3(ua) + b2(ux) + ubb : b3(ua) + b2(ubb) + ux);
            } else {  // tetrahedron (a, b, c) u {x}
                const uint32_t a4 = b4(ua), a3 = b3(ua), bb3 = b3(ubb), bb2 = b2(ubb);
                idx = x > a ? b4(ux) + a3 + bb2 + uc
                            : (x > b ? a4 + b3(ux) + bb2 + uc
                                     : (x > c ? a4 + bb3 + b2(ux) + uc : a4 + bb3 + b2(uc) + ux));
            }
            const uint64_t kk = wkey(dd, idx);
            if (((am >> k) & 1ull) && kk > floor) {
                if (kk < lmin) {
                    lmin = kk;
                    lcnt = 1;
                    ls = s;
                    lx = x;
                } else if (kk == lmin) {
                    ++lcnt;
                }
            }
        };
        int e = 0, t = wv;
        while (t >= W) {
            t -= W;
            ++e;
        }
        while (e < v) {
            const uint32_t s = wg_ctl.vl[e], ds = wg_ctl.vd[e];
            int e2 = e, t2 = t + kNW;
            while (t2 >= W) {
                t2 -= W;
                ++e2;
            }
            if (e2 < v) {  // two pairs' reads in flight together
                const uint32_t s2 = wg_ctl.vl[e2], ds2 = wg_ctl.vd[e2];
                eval(s, ds, t);
                eval(s2, ds2, t2);
                e = e2;
                t = t2 + kNW;
                while (t >= W) {
                    t -= W;
                    ++e;
                }
            } else {
                eval(s, ds, t);
                e = e2;
                t = t2;
            }
        }
        const uint64_t m = wave_min(lmin);
        const int cnt = wave_sum(lmin == m ? lcnt : 0);
        uint64_t pk = 0;
        if (m != kInf) {
            const int wl = __ffsll((unsigned long long)ballot(lmin == m)) - 1;
            pk = pinsert(dim + 1, rl(ls, wl), (int)rl((uint32_t)lx, wl));
        }
        wg_ctl.smin[wv] = m;  // every lane stores the same (uniform) values
        wg_ctl.scnt[wv] = (uint32_t)cnt;
        wg_ctl.spk[wv] = pk;
    }

    // helper waves (1..kNW-1) during a reduction: wake at barrier A for a search request posted by
    // wave 0, evaluate their share, post it before barrier B; leave on the stop request
    __device__ void helper_loop() {
        for (;;) {
            sync_lds();  // A
            if (uni((uint32_t)wg_ctl.rq_stop)) break;
            const int dim = (int)uni((uint32_t)wg_ctl.rq_dim), v = (int)uni((uint32_t)wg_ctl.rq_v);
            const uint64_t floor = uni64(wg_ctl.rq_floor);
            search_share(dim, v, floor);
            sync_lds();  // B
        }
    }

    // Pivot of sum(delta s, s in V) above `floor` (wave 0 with the helpers): the combined minimum
    // with odd multiplicity; even: raise the floor and repeat. kInf for the zero column.
    __device__ uint64_t pivot_of_V(int dim, int v, uint64_t floor, uint64_t& tv) {
        WG_COUNT(29, 1);
        for (;;) {
            if (lane == 0) {
                wg_ctl.rq_floor = floor;
                wg_ctl.rq_v = v;
                wg_ctl.rq_dim = dim;
                wg_ctl.rq_stop = 0;
            }
            sync_lds();  // A
            search_share(dim, v, floor);
            sync_lds();  // B
            uint64_t M = kInf, PK = 0;
            uint32_t C = 0;
#pragma unroll
            for (int q = 0; q < kNW; ++q) {
                const uint64_t mq = wg_ctl.smin[q];
                if (mq < M) {
                    M = mq;
                    C = 0;
                    PK = wg_ctl.spk[q];
                }
                if (mq == M) C += wg_ctl.scnt[q];
            }
            M = uni64(M);
            WG_COUNT(30, 1);
            if (M == kInf) return kInf;
            if (uni(C) & 1u) {
                tv = uni64(PK);
                return M;
            }
            floor = M;
        }
    }

    // ---- the non-apparent columns of one dimension, in Ripser's order ----
    __device__ void reduce(int dim, int cnt) {
        if (cnt > ly.na_cap) {  // uniform: the column counter is shared
            err |= kENA;
            return;
        }
        WG_MARK(-1);
        const int nna = sort_na(dim, cnt);
        WG_MARK(16);
        // pivot table slots for this reduction: >= 2 nna (load factor <= 1/2), >= one window
        uint32_t hc = 64;
        while (hc < 2u * (uint32_t)nna && hc < (uint32_t)ly.h_cap) hc <<= 1;
        hmask = hc - 1u;
        if (wv != 0) {
            helper_loop();
        } else {
            reduce_driver(dim, nna);
            if (lane == 0) {
                wg_ctl.rq_stop = 1;
                wg_ctl.err = err;
            }
            sync_lds();  // A: the helpers leave
        }
        __syncthreads();
        err = uni(wg_ctl.err);
        // empty the pivot table for the next dimension / complex
        uint64_t* HK = sp<uint64_t>(ly.h_key);
        const uint32_t* used = sp<uint32_t>(ly.h_used);
        const int npiv = (int)uni((uint32_t)wg_ctl.npiv);
        for (int i = threadIdx.x; i < npiv; i += kWgThreads) HK[used[i]] = 0ull;
        __syncthreads();
    }

    __device__ void reduce_driver(int dim, int nna) {
        const uint64_t* K = sp<uint64_t>(ly.na_key);
        const uint32_t* P = sp<uint32_t>(ly.na_perm);
        const uint64_t* T = sp<uint64_t>(ly.na_tau);
        const uint64_t* V = sp<uint64_t>(ly.na_tv);
        const uint32_t* Cc = sp<uint32_t>(ly.na_col);
        uint32_t* vstore = sp<uint32_t>(ly.vstore);
        uint2* pairs = sp<uint2>(dim == 1 ? ly.p1 : ly.p2);  // (birth, death) codes
        int& np = dim == 1 ? n_p1 : n_p2;
        int npiv = 0;
        int64_t vused = 0;
        // column records, 64 at a time: lane i holds column cb + i
        uint64_t rk = 0, rt = 0, rv = 0;
        uint32_t rc = 0;
        for (int ci = 0; ci < nna && err == 0u; ++ci) {
            const int li = ci & 63;
            if (li == 0) {
                const int cc = ci + lane;
                if (cc < nna) {
                    const uint32_t p = P[cc];
                    rk = K[cc];
                    rt = T[p];
                    rv = V[p];
                    rc = Cc[p];
                }
            }
            const uint64_t colkey = rl64(rk, li);
            uint64_t tau = rl64(rt, li);
            uint64_t tv = rl64(rv, li);
            const uint32_t cp = rl(rc, li);
            uint32_t app;
            WG_MARK(21);
            uint64_t meta = lookup(dim, tau, tv, app);
            WG_MARK(17);
            int v = 0;  // 0 = lazy: V == {this column}
            if (meta != kNoMeta || app != kNone) {
                WG_COUNT(22, 1);  // columns that need a reduction
                bool ok = v_toggle(dim, cp, v);
                int64_t guard = 0;
                for (;;) {
                    if (app != kNone) {
                        ok = ok && v_toggle(dim, app, v);
                    } else if (meta & kLazy) {
                        ok = ok && v_toggle(dim, (uint32_t)(meta & ~kLazy), v);
                    } else {
                        const int64_t off = (int64_t)(meta >> kMetaLenBits);
                        const int len = (int)(meta & ((1ull << kMetaLenBits) - 1));
                        for (int t0 = 0; t0 < len && ok; t0 += kWave) {
                            const uint32_t w = t0 + lane < len ? vstore[off + t0 + lane] : 0u;
                            const int c = len - t0 < kWave ? len - t0 : kWave;
                            for (int u = 0; u < c && ok; ++u) ok = v_toggle(dim, rl(w, u), v);
                        }
                    }
                    if (!ok) {
                        err |= kEWork;
                        break;
                    }
                    WG_MARK(19);
                    WG_COUNT(24, 1);
                    WG_COUNT(25, v);
                    tau = v > 0 ? pivot_of_V(dim, v, tau, tv) : kInf;
                    WG_MARK(20);
                    if (tau == kInf) break;  // zero column: essential class, not emitted
                    meta = lookup(dim, tau, tv, app);
                    WG_MARK(17);
                    if (meta == kNoMeta && app == kNone) break;  // tau is this column's pivot
                    if (++guard > ly.guard) {
                        err |= kEGuard;
                        break;
                    }
                }
                if (err || tau == kInf) continue;
            }
            const uint32_t death = kdiam(tau), birth = kdiam(colkey);
            if (death > birth) {  // codes preserve order: value(death) > value(birth)
                if (lane == 0 && np < ly.p_cap) pairs[np] = make_uint2(birth, death);
                ++np;
            }
            if (dim == 1) clear_mark(lane == 0, pidx(3, tv));  // clearing for dim 2
            uint64_t mt;
            if (v == 0) {
                mt = kLazy | cp;
            } else {
                if (vused + v > ly.vs_cap) {
                    err |= kER;
                    break;
                }
                for (int t = lane; t < v; t += kWave) vstore[vused + t] = wg_ctl.vl[t];
                mt = ((uint64_t)vused << kMetaLenBits) | (uint64_t)v;
                vused += v;
            }
            if (!hinsert(tau, mt, npiv)) {
                err |= kEPiv;
                break;
            }
            ++npiv;
        }
        if (lane == 0) wg_ctl.npiv = npiv;
    }

    // ---- statistics (betti_features.cpp:24-55, 87-98; utils/math.hpp:9-28) + outputs (wave 0) ----
    __device__ void finish(int64_t gi, double weight) {
        double* feat = bl.features ? bl.features + 35 * gi : nullptr;
        if (n_p1 > ly.p_cap || n_p2 > ly.p_cap) err |= kEPairs;
        if (err && bl.retry_list && (err & kECapacity) == err) {
            // workspace overflow: listed for the capacity-retry launch, which writes the outputs
            if (lane == 0) bl.retry_list[atomicAdd(bl.retry_len, 1u)] = (int32_t)gi;
            return;
        }
        if (err) {
            if (lane == 0) atomicOr(bl.error_flag, err);
            if (feat && lane < 35) feat[lane] = __builtin_nan("");
            if (bl.counts && lane < 4) bl.counts[4 * gi + lane] = -1;
            return;
        }
        // codes -> f32 values, in place (each lane converts its own entries)
        uint32_t* d0c = sp<uint32_t>(ly.d0);
        for (int i = lane; i < n_d0; i += kWave) d0c[i] = vals[d0c[i]];
        uint2* q1 = sp<uint2>(ly.p1);
        uint2* q2 = sp<uint2>(ly.p2);
        for (int i = lane; i < n_p1; i += kWave) q1[i] = make_uint2(vals[q1[i].x], vals[q1[i].y]);
        for (int i = lane; i < n_p2; i += kWave) q2[i] = make_uint2(vals[q2[i].x], vals[q2[i].y]);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        const float* d0s = sp<float>(ly.d0);
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
    }

    // reset the clearing bits this complex set (their words are listed): every complex starts with
    // an all-zero bitset
    __device__ void clear_reset() {
        __syncthreads();
        const int nl = (int)uni(wg_ctl.ctr[4]);
        uint32_t* clr = sp<uint32_t>(ly.mc_t);
        const uint32_t* lst = sp<uint32_t>(ly.mc_e);
        for (int i = threadIdx.x; i < nl; i += kWgThreads) clr[lst[i]] = 0u;
    }

    __device__ void run(int64_t gi, int64_t slot, double weight) {
        WG_MARK(-1);
        load(slot);
        WG_MARK(0);
        if (threadIdx.x < 6) wg_ctl.ctr[threadIdx.x] = 0u;
        if (wv == 0) {
            prim();
        } else if (wv == 1) {
            const int ne = edge_list();
            wg_ctl.nedges = ne;  // every lane stores the same value
        }
        __syncthreads();
        const int n_edges = (int)uni((uint32_t)wg_ctl.nedges);
        WG_MARK(1);
        WG_COUNT(10, n_edges);
        pass_dim1(n_edges);
        __syncthreads();
        WG_MARK(2);
        WG_COUNT(8, uni(wg_ctl.ctr[2]));
        reduce(1, (int)uni(wg_ctl.ctr[2]));
        WG_MARK(3);
        // the reduction ends with a barrier: the clearing marks are complete before the filter
        if (err == 0u) {
            pass_dim2(n_edges);
            __syncthreads();
            WG_MARK(4);
            WG_COUNT(9, uni(wg_ctl.ctr[3]));
            reduce(2, (int)uni(wg_ctl.ctr[3]));
            WG_MARK(5);
        }
        clear_reset();
        if (wv == 0) finish(gi, weight);
        __syncthreads();
        WG_MARK(6);
    }
};

template <int KW>
__global__ __launch_bounds__(kWgThreads) void betti_wg_kernel(BettiLaunch bl, WideLayout ly) {
    // dynamic LDS (wg_lds_bytes): adjacency [nmax][KW] u64, forest parents [nmax] u16 (padded to
    // 8 bytes), the packed u16 code triangle [C(nmax, 2)]
    WG_LDS uint64_t* adj = (WG_LDS uint64_t*)wg_dyn;
    WG_LDS uint16_t* par = reinterpret_cast<WG_LDS uint16_t*>(adj + ly.nmax * KW);
    WG_LDS uint16_t* Dm = par + (ly.nmax + 3) / 4 * 4;
    const int wv = (int)uni(threadIdx.x / kWave);
    const int lane = lane_id();
    uint8_t* scr = ly.base + (int64_t)blockIdx.x * ly.total;
    const int64_t total = (int64_t)*bl.wide_len;
    for (int it = 0;; ++it) {
        // dequeue: wave 0's lanes all execute the atomic (lane 0 adds 1), the ticket goes through LDS
        if (wv == 0) {
            const uint32_t t = atomicAdd(bl.wide_queue, lane == 0 ? 1u : 0u);
            wg_ctl.ticket[it & 1] = rl(t, 0);
        }
        __syncthreads();
        const int64_t wi = (int64_t)uni(wg_ctl.ticket[it & 1]);
        if (wi >= total) break;
        const int64_t gi = (int64_t)(int32_t)uni((uint32_t)bl.wide_list[wi]);
        const int n = (int)uni((uint32_t)bl.npoints[gi]);
        if (n > ly.nmax) {  // outside the layout (never listed here by the host; defensive)
            if (wv == 0) {
                if (lane == 0) atomicOr(bl.error_flag, kEPoints);
                if (bl.features && lane < 35) bl.features[35 * gi + lane] = __builtin_nan("");
                if (bl.counts && lane < 4) bl.counts[4 * gi + lane] = -1;
            }
            continue;
        }
        WgCx<KW> cx{bl, ly, adj, par, Dm, scr, n, (n + 63) / 64, wv, lane, 0u, false, 0u, 0, 0, 0, 0,
                    bl.rank_sorted + wi * bl.rank_stride, 63u, -1};
        cx.run(gi, wi, bl.weight ? bl.weight[gi] : 1.0);
        if (bl.retried && wv == 0 && lane == 0) atomicAdd(bl.retried, 1u);
    }
}

using WgKernel = void (*)(BettiLaunch, WideLayout);
WgKernel wg_kernel_for(int nmax) {
    const int w = (nmax + 63) / 64;
    if (w <= 4) return betti_wg_kernel<4>;
    return betti_wg_kernel<6>;
}

}  // namespace

size_t betti_wg_lds_bytes(int nmax) {
    const int kw = (nmax + 63) / 64 <= 4 ? 4 : 6;
    return (size_t)(8 * nmax * kw + 2 * ((nmax + 3) / 4 * 4) + (2 * ((int64_t)nmax * (nmax - 1) / 2) + 7) / 8 * 8);
}

bool betti_wg_supported(int nmax) { return nmax > 128 && nmax <= kC16MaxPoints; }

int betti_wg_resident_blocks(int device, int nmax) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 256;
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, wg_kernel_for(nmax), kWgThreads, betti_wg_lds_bytes(nmax)) !=
            hipSuccess ||
        per_cu <= 0)
        per_cu = 1;
    return prop.multiProcessorCount * per_cu;
}

hipError_t launch_betti_wg(hipStream_t st, const BettiLaunch& b, const WideLayout& l, int blocks) {
    if (blocks <= 0) return hipSuccess;
    if (!b.rank_codes || !b.rank_sorted || !betti_wg_supported(l.nmax) || !l.wg) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wg_kernel_for(l.nmax), dim3((unsigned)blocks), dim3(kWgThreads), betti_wg_lds_bytes(l.nmax), st,
                       b, l);
    return hipGetLastError();
}

}  // namespace dgn
