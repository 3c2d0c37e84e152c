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
// so every distance read of the walks and of the pivot searches is an LDS read, and the
// workgroup's waves share the work:
//   * load, adjacency: all waves;  Prim (wave 0) beside the edge list (wave 1);
//   * dim-1 / dim-2 apparent passes: lane per column, the columns dealt to the waves from LDS
//     counters (dim 2: a per-lane work queue over the edges, as betti_wide.hip);
//   * the non-apparent columns: bitonic-sorted in scratch by all threads;
//   * the reduction, column by column in Ripser's order: every wave follows the same control
//     flow (the same uniform values from the same reads); the V list lives in LDS and only wave 0
//     changes it; the pivot search — the reduction's hot loop — deals its (V entry, bitset word)
//     pairs to the waves and combines their minima through LDS (one barrier per floor round);
//     scratch writes (pivot table, V store, pairs, clearing marks) are wave 0's, published by the
//     barrier that ends the column.
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
constexpr int kWgThreads = kNW * kWave;
constexpr int kVlCap = 512;                // V list entries (LDS); more: capacity retry
constexpr uint64_t kInf = ~0ull;
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint16_t kMcNone = 0xFFFF;     // not a column, or no cofacet
constexpr uint16_t kMcCleared = 0xFFFE;  // triangle is the pivot of a dim-1 column (clearing)
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
    uint32_t ticket[2];             // complex dequeue (double-buffered by iteration parity)
    uint32_t ctr[4];                // pass counters: dim-1 edges, dim-2 edges, dim-1 / dim-2 columns
    int32_t nedges;
    uint32_t cnt;                   // threshold search
    int32_t vv[2];                  // V length after wave 0's toggles (double-buffered by round)
    uint32_t vok[2];
    uint64_t smin[2][kNW];          // pivot search: per-wave minimum, multiplicity, packed cofacet
    uint64_t spk[2][kNW];
    uint32_t scnt[2][kNW];
    uint32_t vl[kVlCap];            // V list (packed simplices) and their diameters
    uint32_t vd[kVlCap];
};
__shared__ WgCtl wg_ctl;
extern __shared__ uint64_t wg_dyn[];

__device__ __forceinline__ uint64_t bin2(uint64_t v) { return v * (v - 1) / 2; }
__device__ __forceinline__ uint64_t bin3(uint64_t v) { return v * (v - 1) * (v - 2) / 6; }
__device__ __forceinline__ uint64_t bin4(uint64_t v) { return v * (v - 1) * (v - 2) * (v - 3) / 24; }
__device__ __forceinline__ uint32_t rl(uint32_t x, int l) { return (uint32_t)__builtin_amdgcn_readlane((int)x, l); }
__device__ __forceinline__ uint64_t rl64(uint64_t x, int l) {
    return ((uint64_t)rl((uint32_t)(x >> 32), l) << 32) | rl((uint32_t)x, l);
}
__device__ __forceinline__ uint32_t uni(uint32_t x) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) { return ((uint64_t)uni((uint32_t)(x >> 32)) << 32) | uni((uint32_t)x); }
__device__ __forceinline__ int pv(uint64_t p, int field) { return (int)((p >> (VB * field)) & VM); }
__device__ __forceinline__ uint64_t pidx(int nv, uint64_t p) {
    if (nv == 2) return bin2(pv(p, 1)) + pv(p, 0);
    if (nv == 3) return bin3(pv(p, 2)) + bin2(pv(p, 1)) + pv(p, 0);
    return bin4(pv(p, 3)) + bin3(pv(p, 2)) + bin2(pv(p, 1)) + pv(p, 0);
}
__device__ __forceinline__ uint64_t pinsert(int nv, uint64_t p, int x) {
    int below = 0;
    for (int t = 0; t < nv; ++t) below += pv(p, t) < x;
    const uint64_t mask = (1ull << (VB * below)) - 1;
    return ((p & ~mask) << VB) | ((uint64_t)x << (VB * below)) | (p & mask);
}
// key: (distance code << 32) | ~index — ascending keys are Ripser's filtration order
__device__ __forceinline__ uint64_t wkey(uint32_t dc, uint64_t idx) { return ((uint64_t)dc << 32) | (~idx & 0xFFFFFFFFull); }
__device__ __forceinline__ uint32_t kdiam(uint64_t key) { return (uint32_t)(key >> 32); }
__device__ __forceinline__ int c2i(int x) { return x * (x - 1) / 2; }
// workgroup-scope LDS add of `v` by lane 0 (every lane executes the atomic: no branch on the
// lane, see betti_kernels.hip's dequeue); the old value, wave-uniform
__device__ __forceinline__ uint32_t lds_add_uniform(uint32_t* p, uint32_t v) {
    const uint32_t old = __hip_atomic_fetch_add(p, lane_id() == 0 ? v : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return rl(old, 0);
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
    uint32_t rnd;          // LDS publish rounds (slot parity), identical in every wave
    const uint32_t* vals;  // the complex's sorted f32 distances (code -> value)

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
    __device__ float value(uint32_t dc) const { return __uint_as_float(vals[dc]); }
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
        // ripser.cpp:386-395): two rounds of 512 parallel probes of the sorted triangle
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
            if (t < W && v < n && v != 0 && ((aw(0, t) >> lane) & 1ull)) best[t] = wkey(d(0, v), bin2(v));
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
                    const uint64_t k = wkey(d(v, w), v > w ? bin2(v) + w : bin2(w) + v);
                    if (k < best[t]) {
                        best[t] = k;
                        bp[t] = v;
                    }
                }
            }
        }
    }

    // ---- edges (i > j, d <= thr) in index order (wave 1) ----
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

    // ---- dim 1: lane per column (non-tree edge), 64-edge chunks dealt from an LDS counter ----
    __device__ void pass_dim1(int n_edges) {
        const uint32_t* edges = sp<uint32_t>(ly.edges);
        uint16_t* mc_e = sp<uint16_t>(ly.mc_e);
        uint16_t* mc_t = sp<uint16_t>(ly.mc_t);
        for (;;) {
            const int base = (int)lds_add_uniform(&wg_ctl.ctr[0], kWave);
            if (base >= n_edges) break;
            const int e = base + lane;
            bool na = false;
            uint64_t colkey = 0, best = kInf, bestp = 0;
            uint32_t colp = 0;
            if (e < n_edges) {
                const uint32_t ed = edges[e];
                const int i = (int)(ed >> VB), j = (int)(ed & VM);
                uint16_t mc = kMcNone;
                if (!is_tree(i, j)) {
                    const uint32_t dij = d(i, j);
                    colp = ed;
                    colkey = wkey(dij, bin2(i) + j);
                    // F-minimal cofacet: walking k downwards over the common neighbours, the
                    // first k with both distances <= d(i, j) ends the walk; before it, a smaller k
                    // wins only with a strictly smaller diameter
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
                        bestp = pinsert(2, ed, bk);
                        best = wkey(bd, pidx(3, bestp));
                        // apparent iff (i, j) is the F-max facet of its zero-persistence cofacet
                        const bool app = found && (bk > i || hdb < dij) && (bk > j || hda < dij);
                        if (app) mc_t[pidx(3, bestp)] = kMcCleared;  // clearing for dim 2
                        else na = true;
                        mc = (uint16_t)bk;
                    }
                }
                mc_e[bin2(i) + j] = mc;
            }
            na_append(na, &wg_ctl.ctr[2], colkey, best, bestp, colp);
        }
    }

    // ---- dim 2: lane per column (uncleared triangle), a per-lane work queue over the edges,
    // edges dealt from an LDS counter (see betti_wide.hip pass_dim2) ----
    static constexpr int kStep = 4;
    __device__ void pass_dim2(int n_edges) {
        const uint32_t* edges = sp<uint32_t>(ly.edges);
        uint16_t* mc_t = sp<uint16_t>(ly.mc_t);
        int ea = 0, eb = 0, tw = -1;
        uint64_t tm = 0;
        bool act = false, fresh = false, drained = false;
        int c = 0, w = 0, bk = 0;
        uint64_t m = 0, tidx = 0;
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
                const bool need = !act && tm == 0ull;
                const uint64_t bal = ballot(need);
                if (!bal || drained) break;
                const int base = (int)lds_add_uniform(&wg_ctl.ctr[1], (uint32_t)__popcll(bal));
                if (base >= n_edges) {
                    drained = true;
                    break;
                }
                const int e = base + mask_prefix(bal);
                if (need && e < n_edges) {
                    const uint32_t ed = edges[e];
                    ea = (int)(ed >> VB);
                    eb = (int)(ed & VM);
                    tw = 0;
                    tm = aw(ea, 0) & aw(eb, 0);
                    if (eb < 64) tm &= (1ull << eb) - 1ull;
                }
            }
            if (!act && tm != 0ull) {
                c = 64 * tw + __ffsll((unsigned long long)tm) - 1;
                tm &= tm - 1ull;
                act = fresh = true;
                tidx = bin3(ea) + bin2(eb) + c;
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
                bool cleared = false;
                if (fresh) {
                    cleared = mc_t[tidx] == kMcCleared;
                    dab = d(a, b);
                    dac = d(a, c);
                    dbc = d(b, c);
                    ds = max(max(dab, dac), dbc);
                    fresh = false;
                }
                bool done;
                if (cleared) {
                    mc_t[tidx] = kMcNone;  // consumed: the entry leaves the complex non-cleared
                    done = true;
                } else {
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
                        uint16_t mc = kMcNone;
                        uint64_t best = kInf, bestp = 0;
                        if (bk >= 0) {
                            bestp = pinsert(3, colp, bk);
                            best = wkey(bd, pidx(4, bestp));
                            const bool app = found && (bk > a || max(max(hdb, hdc), dbc) < ds) &&
                                             (bk > b || max(max(hda, hdc), dac) < ds) &&
                                             (bk > c || max(max(hda, hdb), dab) < ds);
                            na = !app;
                            mc = (uint16_t)bk;
                        }
                        mc_t[tidx] = mc;
                        colkey = wkey(ds, tidx);
                        ntau = best;
                        ntv = bestp;
                        ncolp = colp;
                    }
                }
                if (done) act = false;
            }
            na_append(na, &wg_ctl.ctr[3], colkey, ntau, ntv, ncolp);
        }
    }

    // ---- non-apparent columns in Ripser's order: bitonic sort (key descending) of (key, slot)
    // pairs in scratch by all threads; 4 compare-exchanges per thread per step with their loads
    // issued together ----
    __device__ void sort_na(int cnt) {
        const int tid = threadIdx.x;
        int N = 1;
        while (N < cnt) N <<= 1;
        uint64_t* K = sp<uint64_t>(ly.na_key);
        uint32_t* P = sp<uint32_t>(ly.na_perm);
        for (int i = tid; i < N; i += kWgThreads) {
            if (i >= cnt) K[i] = 0ull;  // padding sorts last
            P[i] = (uint32_t)i;
        }
        __syncthreads();
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
    }

    // ---- pivot table: open addressing in scratch (key 0 = empty), written by wave 0 ----
    __device__ static uint32_t hmix(uint64_t k) {
        k ^= k >> 33;
        k *= 0xff51afd7ed558ccdull;
        k ^= k >> 33;
        return (uint32_t)k;
    }
    __device__ uint64_t hfind(uint64_t k) const {
        const uint64_t* HK = sp<uint64_t>(ly.h_key);
        const uint64_t* HM = sp<uint64_t>(ly.h_meta);
        const uint32_t mask = (uint32_t)ly.h_cap - 1u;
        const uint32_t base = hmix(k) & mask;
        for (int probe = 0; probe < ly.h_cap; probe += kWave) {
            const uint64_t x = HK[(base + (uint32_t)(probe + lane)) & mask];
            const uint64_t hit = ballot(x == k), emp = ballot(x == 0ull);
            const int fh = hit ? __ffsll((unsigned long long)hit) - 1 : kWave;
            const int fe = emp ? __ffsll((unsigned long long)emp) - 1 : kWave;
            if (fh < fe) return uni64(HM[(base + (uint32_t)(probe + fh)) & mask]);
            if (fe < kWave) return kNoMeta;
        }
        return kNoMeta;
    }
    // wave 0 writes; every wave gets the same answer (the table has 2 na_cap slots)
    __device__ bool hinsert(uint64_t k, uint64_t meta, int npiv) {
        if (npiv >= ly.na_cap) return false;
        if (wv != 0) return true;
        uint64_t* HK = sp<uint64_t>(ly.h_key);
        uint64_t* HM = sp<uint64_t>(ly.h_meta);
        const uint32_t mask = (uint32_t)ly.h_cap - 1u;
        const uint32_t base = hmix(k) & mask;
        for (int probe = 0; probe < ly.h_cap; probe += kWave) {
            const uint64_t x = HK[(base + (uint32_t)(probe + lane)) & mask];
            const uint64_t emp = ballot(x == 0ull);
            if (emp) {
                const uint32_t slot = (base + (uint32_t)(probe + __ffsll((unsigned long long)emp) - 1)) & mask;
                if (lane == 0) {
                    HK[slot] = k;
                    HM[slot] = meta;
                    sp<uint32_t>(ly.h_used)[npiv] = slot;
                }
                return true;
            }
        }
        return true;
    }

    // Owner of the pivot tau (see betti_wide.hip lookup): the pivot table's first 64-slot window
    // and tau's edge lengths loaded together; a table hit returns its metadata, otherwise the
    // apparent owner (tau's F-max facet f if tau is f's minimal cofacet) from the edge lengths in
    // registers and one min-cofacet table read. kNoMeta if tau is not in the table.
    __device__ uint64_t lookup(int dim, uint64_t tau, uint64_t tv, uint32_t& app) const {
        const uint64_t* HK = sp<uint64_t>(ly.h_key);
        const uint64_t* HM = sp<uint64_t>(ly.h_meta);
        const uint32_t mask = (uint32_t)ly.h_cap - 1u;
        const uint32_t slot = (hmix(tau) + (uint32_t)lane) & mask;
        const uint64_t hk = HK[slot];
        const uint64_t hm = HM[slot];
        const int nv = dim + 2;
        const int v0 = pv(tv, nv - 1), v1 = pv(tv, nv - 2), v2 = pv(tv, nv - 3), v3 = nv == 4 ? pv(tv, 0) : 0;
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
        app = kNone;
        if (fh < fe) return rl64(hm, fh);
        if (fe == kWave) {
            const uint64_t mm = hfind(tau);
            if (mm != kNoMeta) return mm;
        }
        uint32_t dd[4][4];
        if (nv == 4) {
            dd[0][1] = rl(dl, 0);
            dd[0][2] = rl(dl, 1);
            dd[0][3] = rl(dl, 2);
            dd[1][2] = rl(dl, 3);
            dd[1][3] = rl(dl, 4);
            dd[2][3] = rl(dl, 5);
        } else {
            dd[0][1] = rl(dl, 0);
            dd[0][2] = rl(dl, 1);
            dd[1][2] = rl(dl, 2);
        }
        const int v[4] = {v0, v1, v2, v3};
        uint64_t bestk = 0, bestf = 0;
        int drop = 0;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
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
        const uint16_t mcv = dim == 1 ? sp<uint16_t>(ly.mc_e)[pidx(2, bestf)] : sp<uint16_t>(ly.mc_t)[pidx(3, bestf)];
        const int vd = drop == 0 ? v0 : (drop == 1 ? v1 : (drop == 2 ? v2 : v3));
        if (uni(mcv) == (uint32_t)vd) app = (uint32_t)bestf;
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

    // Pivot of sum(delta s, s in V) above `floor`: the (V entry, bitset word) pairs are dealt to
    // the waves; lane k of a pair (s, t) evaluates the cofacet s u {64 t + k}; each wave's minimum
    // and its multiplicity go through LDS; the combined minimum with odd multiplicity is the pivot,
    // even: raise the floor and repeat. kInf for the zero column.
    __device__ uint64_t pivot_of_V(int dim, int v, uint64_t floor, uint64_t& tv) {
        const int k = lane;
        WG_COUNT(29, 1);  // pivot searches
        for (;;) {
            uint64_t lmin = kInf, lp = 0;
            int lcnt = 0;
#ifdef DGN_WG_FASTKEY
            // 32-bit combinatorial index of s u {x} (C(362, 4) < 2^32): the uniform partial sums of
            // s's vertices plus x's binomial at its position; the packed cofacet is built once,
            // for the winning lane (its entry s and vertex x are tracked instead)
            uint32_t ls = 0;
            int lx = 0;
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
                const uint32_t x2 = ux * (ux - 1u) / 2u, x3 = x2 * (ux - 2u) / 3u, x4 = x3 * (ux - 3u) / 4u;
                const uint32_t ua = (uint32_t)a, ub_ = (uint32_t)b, uc = (uint32_t)c;
                const uint32_t a2 = ua * (ua - 1u) / 2u, a3 = a2 * (ua - 2u) / 3u;
                const uint32_t b2 = ub_ * (ub_ - 1u) / 2u;
                uint32_t idx;
                if (dim == 1) {  // triangle (a, b) u {x}
                    idx = x > a ? x3 + a2 + ub_ : (x > b ? a3 + x2 + ub_ : a3 + b2 + ux);
                } else {  // tetrahedron (a, b, c) u {x}
                    const uint32_t a4 = a3 * (ua - 3u) / 4u, b3 = b2 * (ub_ - 2u) / 3u;
                    const uint32_t c2 = uc * (uc - 1u) / 2u;
                    idx = x > a ? x4 + a3 + b2 + uc
                                : (x > b ? a4 + x3 + b2 + uc : (x > c ? a4 + b3 + x2 + uc : a4 + b3 + c2 + ux));
                }
                const uint64_t kk = ((uint64_t)dd << 32) | (uint64_t)(~idx);
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
#else
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
                const uint64_t p = pinsert(dim + 1, s, x);
                const uint64_t kk = wkey(dd, pidx(dim + 2, p));
                if (((am >> k) & 1ull) && kk > floor) {
                    if (kk < lmin) {
                        lmin = kk;
                        lcnt = 1;
                        lp = p;
                    } else if (kk == lmin) {
                        ++lcnt;
                    }
                }
            };
#endif
            // pairs p = e W + t, p = wv, wv + kNW, ...: (e, t) stepped without division
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
#ifdef DGN_WG_FASTKEY
            if (m != kInf) {
                const int wl = __ffsll((unsigned long long)ballot(lmin == m)) - 1;
                pk = pinsert(dim + 1, rl(ls, wl), (int)rl((uint32_t)lx, wl));
            }
            (void)lp;
#else
            if (m != kInf) pk = rl64(lp, __ffsll((unsigned long long)ballot(lmin == m)) - 1);
#endif
            const int r = rnd & 1;
            wg_ctl.smin[r][wv] = m;  // every lane stores the same (uniform) values
            wg_ctl.scnt[r][wv] = (uint32_t)cnt;
            wg_ctl.spk[r][wv] = pk;
            __syncthreads();
            ++rnd;
            uint64_t M = kInf, PK = 0;
            uint32_t C = 0;
#pragma unroll
            for (int q = 0; q < kNW; ++q) {
                const uint64_t mq = wg_ctl.smin[r][q];
                if (mq < M) {
                    M = mq;
                    C = 0;
                    PK = wg_ctl.spk[r][q];
                }
                if (mq == M) C += wg_ctl.scnt[r][q];
            }
            M = uni64(M);
            WG_COUNT(30, 1);  // floor rounds
            if (M == kInf) return kInf;
            if (uni(C) & 1u) {
                tv = uni64(PK);
                return M;
            }
            floor = M;
        }
    }

    // ---- the non-apparent columns of one dimension, in Ripser's order (every wave) ----
    __device__ void reduce(int dim, int nna) {
        if (nna > ly.na_cap) {
            err |= kENA;
            return;
        }
        WG_MARK(-1);
        sort_na(nna);
        WG_MARK(16);
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
                bool first = true;
                int64_t guard = 0;
                for (;;) {
                    const int r = rnd & 1;
                    if (wv == 0) {
                        bool ok = true;
                        int vv = v;
                        if (first) {
                            vv = 0;
                            ok = v_toggle(dim, cp, vv);
                        }
                        if (app != kNone) {
                            ok = ok && v_toggle(dim, app, vv);
                        } else if (meta & kLazy) {
                            ok = ok && v_toggle(dim, (uint32_t)(meta & ~kLazy), vv);
                        } else {
                            const int64_t off = (int64_t)(meta >> kMetaLenBits);
                            const int len = (int)(meta & ((1ull << kMetaLenBits) - 1));
                            for (int t0 = 0; t0 < len && ok; t0 += kWave) {
                                const uint32_t w = t0 + lane < len ? vstore[off + t0 + lane] : 0u;
                                const int cnt = len - t0 < kWave ? len - t0 : kWave;
                                for (int u = 0; u < cnt && ok; ++u) ok = v_toggle(dim, rl(w, u), vv);
                            }
                        }
                        wg_ctl.vv[r] = vv;
                        wg_ctl.vok[r] = ok ? 1u : 0u;
                    }
                    __syncthreads();
                    ++rnd;
                    first = false;
                    v = (int)uni((uint32_t)wg_ctl.vv[r]);
                    if (!uni(wg_ctl.vok[r])) {
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
                if (wv == 0 && lane == 0 && np < ly.p_cap) pairs[np] = make_uint2(birth, death);
                ++np;
            }
            if (dim == 1 && wv == 0 && lane == 0) sp<uint16_t>(ly.mc_t)[pidx(3, tv)] = kMcCleared;  // clearing
            uint64_t mt;
            if (v == 0) {
                mt = kLazy | cp;
            } else {
                if (vused + v > ly.vs_cap) {
                    err |= kER;
                    break;
                }
                if (wv == 0)
                    for (int t = lane; t < v; t += kWave) vstore[vused + t] = wg_ctl.vl[t];
                mt = ((uint64_t)vused << kMetaLenBits) | (uint64_t)v;
                vused += v;
            }
            WG_MARK(-1);
            // every wave's last lookup of this column reads the table before wave 0 inserts tau (a
            // lagging wave that saw tau's own entry would take another reduction round alone)
            __syncthreads();
            if (!hinsert(tau, mt, npiv)) {
                err |= kEPiv;
                break;
            }
            ++npiv;
            __syncthreads();  // wave 0's table insert, V store and clearing mark before the next column
        }
        __syncthreads();
        // empty the pivot table for the next dimension / complex
        uint64_t* HK = sp<uint64_t>(ly.h_key);
        const uint32_t* used = sp<uint32_t>(ly.h_used);
        for (int i = threadIdx.x; i < npiv; i += kWgThreads) HK[used[i]] = 0ull;
        __syncthreads();
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

    __device__ void run(int64_t gi, int64_t slot, double weight) {
        WG_MARK(-1);
        load(slot);
        WG_MARK(0);
        if (threadIdx.x < 4) wg_ctl.ctr[threadIdx.x] = 0u;
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
        // reduce ends with a barrier: the clearing marks are complete before the dim-2 pass
        if (err == 0u) {
            pass_dim2(n_edges);
            __syncthreads();
            WG_MARK(4);
            WG_COUNT(9, uni(wg_ctl.ctr[3]));
            reduce(2, (int)uni(wg_ctl.ctr[3]));
            WG_MARK(5);
        } else {
            // no dim-2 pass consumes the clearing marks: erase every triangle entry
            uint16_t* mc_t = sp<uint16_t>(ly.mc_t);
            const int64_t nt = (int64_t)bin3((uint64_t)n);
            for (int64_t t = threadIdx.x; t < nt; t += kWgThreads) mc_t[t] = kMcNone;
            __syncthreads();
        }
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
    uint32_t rnd = 0;
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
        WgCx<KW> cx{bl, ly, adj, par, Dm, scr, n, (n + 63) / 64, wv, lane, 0u, false, 0u, 0, 0, 0, 0, rnd,
                    bl.rank_sorted + wi * bl.rank_stride};
        cx.run(gi, wi, bl.weight ? bl.weight[gi] : 1.0);
        rnd = cx.rnd;
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
    if (!b.rank_codes || !b.rank_sorted || !betti_wg_supported(l.nmax)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(wg_kernel_for(l.nmax), dim3((unsigned)blocks), dim3(kWgThreads), betti_wg_lds_bytes(l.nmax), st,
                       b, l);
    return hipGetLastError();
}

}  // namespace dgn
