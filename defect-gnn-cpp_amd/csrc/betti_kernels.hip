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
//   * dim 1 and dim 2: cohomology with clearing. Every column's pivot is found lane-parallel and
//     apparent pairs (sigma youngest facet of tau, tau oldest cofacet of sigma) are settled in
//     one pass; the few remaining columns are reduced in Ripser's column order by the whole
//     wave, with Z/2 column additions as sorted-key symmetric differences (binary-search merge
//     in LDS) and owner lookups that re-derive apparent owners on the fly. The persistence
//     pairing of a total order is unique, so the emitted (birth, death) multiset equals the
//     lock-free Ripser's (death > birth only; essential dim>=1 classes not emitted).
//   * persistent grid, chunked dynamic dequeue; per-wave global scratch for reduced columns
//     and pair lists.
#include "dgn_internal.hpp"

namespace dgn {

constexpr int kWCap = 256;        // working-column keys (LDS)
constexpr int kNACap = 512;       // non-apparent columns per dimension (scratch)
constexpr int kPivCap = 256;      // serially reduced pivots per dimension (LDS keys)
constexpr int kPairCap = 1024;    // pairs per dimension (scratch)
constexpr int kRCap = 8192;       // reduced-column keys per dimension (scratch)
constexpr int kChunk = 4;         // complexes per dequeue

constexpr uint64_t kInf = ~0ull;

// error bits
constexpr uint32_t kErrTooManyPoints = 1u << 0;
constexpr uint32_t kErrWorkCol = 1u << 1;
constexpr uint32_t kErrNA = 1u << 2;
constexpr uint32_t kErrPiv = 1u << 3;
constexpr uint32_t kErrPairs = 1u << 4;
constexpr uint32_t kErrR = 1u << 5;
constexpr uint32_t kErrOrder = 1u << 6;

// scratch layout per wave (bytes)
struct ScratchLayout {
    static constexpr int64_t na = 0;                                  // uint64 [kNACap]
    static constexpr int64_t rmeta = na + 8 * kNACap;                // uint32 [kPivCap] (off<<12|len)
    static constexpr int64_t p1 = rmeta + 4 * kPivCap;               // float2 [kPairCap]
    static constexpr int64_t p2 = p1 + 8 * kPairCap;                 // float2 [kPairCap]
    static constexpr int64_t r = p2 + 8 * kPairCap;                  // uint64 [kRCap]
    static constexpr int64_t total = r + 8 * kRCap;
};

template <int NP>
struct BettiSmem {
    float D[NP][NP + 1];
    uint64_t adj[NP];
    uint64_t tree[NP];
    uint16_t edges[NP * (NP - 1) / 2];
    uint32_t cleared[(NP * (NP - 1) * (NP - 2) / 6 + 31) / 32];
    union {
        struct {
            double X[NP][3];
            double sq[NP];
        } cloud;
        struct {
            uint64_t A[kWCap];  // working column / merge buffers
            uint64_t B[kWCap];
            uint64_t C[kWCap];
        } col;
    } u;
    uint64_t piv[kPivCap];
    float d0[NP];
};

// ---------------------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, kWave);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, kWave);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, int m) {
    const uint32_t lo = (uint32_t)__shfl_xor((int)(uint32_t)v, m, kWave);
    const uint32_t hi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), m, kWave);
    return ((uint64_t)hi << 32) | lo;
}
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        const uint64_t w = shfl_xor64(v, o);
        v = w < v ? w : v;
    }
    return v;
}
// ascending bitonic sort of one key per lane (kInf pads)
__device__ __forceinline__ uint64_t wave_sort_u64(uint64_t key) {
    const int lane = lane_id();
#pragma unroll
    for (int k = 2; k <= kWave; k <<= 1) {
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const uint64_t other = shfl_xor64(key, j);
            const bool keep_min = ((lane & j) == 0) == ((lane & k) == 0);
            const uint64_t mn = other < key ? other : key;
            const uint64_t mx = other < key ? key : other;
            key = keep_min ? mn : mx;
        }
    }
    return key;
}
__device__ __forceinline__ uint32_t readlane_u32(uint32_t v, int l) { return (uint32_t)__shfl((int)v, l, kWave); }

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
// insert k into descending (a,b) -> packed descending triple
__device__ __forceinline__ uint32_t tri_with(int a, int b, int k) {
    return k > a ? pack3(k, a, b) : (k > b ? pack3(a, k, b) : pack3(a, b, k));
}
__device__ __forceinline__ uint32_t tet_with(int a, int b, int c, int k) {
    return k > a ? pack4(k, a, b, c) : k > b ? pack4(a, k, b, c) : k > c ? pack4(a, b, k, c) : pack4(a, b, c, k);
}
__device__ __forceinline__ int tri_dense(int a, int b, int c) {  // combinatorial index, a > b > c
    return a * (a - 1) * (a - 2) / 6 + b * (b - 1) / 2 + c;
}

// number of elements < key in sorted arr[0..n)
__device__ __forceinline__ int lower_bound_u64(const uint64_t* arr, int n, uint64_t key) {
    int lo = 0, len = n;
    while (len > 0) {
        const int half = len >> 1;
        if (arr[lo + half] < key) {
            lo += half + 1;
            len -= half + 1;
        } else {
            len = half;
        }
    }
    return lo;
}

// out = A xor B (sorted symmetric difference), returns length (or -1 on overflow).
__device__ int merge_xor(const uint64_t* A, int na, const uint64_t* B, int nb, uint64_t* out) {
    const int lane = lane_id();
    int survA = 0, survB = 0;
    // first count survivors of both to know the output length
    int outlen = 0;
    for (int pass = 0; pass < 2; ++pass) {
        const uint64_t* S = pass == 0 ? A : B;
        const uint64_t* O = pass == 0 ? B : A;
        const int ns = pass == 0 ? na : nb, no = pass == 0 ? nb : na;
        int carry = 0;
        for (int base = 0; base < ns; base += kWave) {
            const int i = base + lane;
            bool surv = false;
            int lb = 0;
            uint64_t v = 0;
            if (i < ns) {
                v = S[i];
                lb = lower_bound_u64(O, no, v);
                surv = !(lb < no && O[lb] == v);
            }
            const uint64_t bal = ballot(surv);
            const int sp = carry + mask_prefix(bal);  // survivors of S before i
            if (surv) {
                const int pos = sp + lb - (i - sp);
                if (pos < kWCap) out[pos] = v;
            }
            carry += __popcll(bal);
        }
        if (pass == 0) survA = carry;
        else survB = carry;
    }
    outlen = survA + survB;
    return outlen <= kWCap ? outlen : -1;
}

// ---------------------------------------------------------------------------------------
// the kernel
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

    __device__ float dist(int a, int b) const { return s.D[a][b]; }
    __device__ uint64_t ekey(int i, int j) const {  // i != j
        const int a = i > j ? i : j, b = i > j ? j : i;
        return make_key(s.D[a][b], pack2(a, b));
    }
    __device__ float tri_diam(int a, int b, int c) const {
        return fmaxf(fmaxf(s.D[a][b], s.D[a][c]), s.D[b][c]);
    }
    __device__ uint64_t tkey(int a, int b, int c) const {  // a > b > c
        return make_key(tri_diam(a, b, c), pack3(a, b, c));
    }
    __device__ bool is_cleared(int a, int b, int c) const {
        const int t = tri_dense(a, b, c);
        return (s.cleared[t >> 5] >> (t & 31)) & 1u;
    }
    __device__ void set_cleared(int a, int b, int c) {
        const int t = tri_dense(a, b, c);
        atomicOr(&s.cleared[t >> 5], 1u << (t & 31));
    }
    __device__ uint64_t* na_list() { return reinterpret_cast<uint64_t*>(scratch + ScratchLayout::na); }
    __device__ uint32_t* rmeta() { return reinterpret_cast<uint32_t*>(scratch + ScratchLayout::rmeta); }
    __device__ float2* pairs(int dim) {
        return reinterpret_cast<float2*>(scratch + (dim == 1 ? ScratchLayout::p1 : ScratchLayout::p2));
    }
    __device__ uint64_t* rstore() { return reinterpret_cast<uint64_t*>(scratch + ScratchLayout::r); }

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

    // F-min cofacet (key) of the simplex with vertex tuple v (dim = 1 edge, 2 triangle) over
    // candidate mask cand, whole wave: lane k evaluates vertex k.
    __device__ uint64_t min_cofacet_wave(int dim, int a, int b, int c, float diam, uint64_t cand) const {
        const int k = lane_id();
        uint64_t key = kInf;
        if ((cand >> k) & 1ull) {
            if (dim == 1) {
                const float dd = fmaxf(diam, fmaxf(s.D[a][k], s.D[b][k]));
                key = make_key(dd, tri_with(a, b, k));
            } else {
                const float dd = fmaxf(diam, fmaxf(fmaxf(s.D[a][k], s.D[b][k]), s.D[c][k]));
                key = make_key(dd, tet_with(a, b, c, k));
            }
        }
        return wave_min_u64(key);
    }

    // Sorted coboundary of a column simplex into out (whole wave); returns length.
    __device__ int coboundary_sorted(int dim, int a, int b, int c, uint64_t* out) const {
        const int k = lane_id();
        uint64_t cand;
        float diam;
        if (dim == 1) {
            cand = s.adj[a] & s.adj[b];
            diam = s.D[a][b];
        } else {
            cand = s.adj[a] & s.adj[b] & s.adj[c];
            diam = tri_diam(a, b, c);
        }
        uint64_t key = kInf;
        if ((cand >> k) & 1ull) {
            if (dim == 1) key = make_key(fmaxf(diam, fmaxf(s.D[a][k], s.D[b][k])), tri_with(a, b, k));
            else key = make_key(fmaxf(diam, fmaxf(fmaxf(s.D[a][k], s.D[b][k]), s.D[c][k])), tet_with(a, b, c, k));
        }
        key = wave_sort_u64(key);
        const int len = __popcll(cand);
        if (k < len) out[k] = key;
        return len;
    }

    // If the pivot simplex tau (dim+1) is the pivot of an apparent pair, return the owner's
    // packed column vertices (dim simplex) else 0xFFFFFFFF. Whole wave.
    __device__ uint32_t apparent_owner(int dim, uint64_t tau) const {
        const uint32_t p = key_packed(tau);
        if (dim == 1) {
            const int a = (p >> 16) & 255, b = (p >> 8) & 255, c = p & 255;
            // F-max facet among (a,b), (a,c), (b,c)
            uint64_t k0 = ekey(a, b), k1 = ekey(a, c), k2 = ekey(b, c);
            int fa = a, fb = b;
            uint64_t best = k0;
            if (k1 > best) { best = k1; fa = a; fb = c; }
            if (k2 > best) { best = k2; fa = b; fb = c; }
            if ((s.tree[fa] >> fb) & 1ull) return 0xFFFFFFFFu;  // tree edges are not columns
            const uint64_t m = min_cofacet_wave(1, fa, fb, 0, s.D[fa][fb], s.adj[fa] & s.adj[fb]);
            return m == tau ? pack2(fa, fb) : 0xFFFFFFFFu;
        } else {
            const int a = (p >> 24) & 255, b = (p >> 16) & 255, c = (p >> 8) & 255, d = p & 255;
            uint64_t best = tkey(a, b, c);
            int fa = a, fb = b, fc = c;
            uint64_t k;
            k = tkey(a, b, d); if (k > best) { best = k; fa = a; fb = b; fc = d; }
            k = tkey(a, c, d); if (k > best) { best = k; fa = a; fb = c; fc = d; }
            k = tkey(b, c, d); if (k > best) { best = k; fa = b; fb = c; fc = d; }
            if (is_cleared(fa, fb, fc)) return 0xFFFFFFFFu;
            const uint64_t m = min_cofacet_wave(2, fa, fb, fc, tri_diam(fa, fb, fc), s.adj[fa] & s.adj[fb] & s.adj[fc]);
            return m == tau ? pack3(fa, fb, fc) : 0xFFFFFFFFu;
        }
    }

    // Serial reduction of the non-apparent columns of one dimension (whole wave).
    __device__ void reduce_serial(int dim, int nna) {
        const int lane = lane_id();
        uint64_t* na = na_list();
        // sort non-apparent columns by key DESCENDING (Ripser column order): rank sort
        if (nna > kNACap) { err |= kErrNA; return; }
        // rank sort into the B buffer region of LDS is too small for kNACap; sort in scratch:
        // simple odd-even pass over chunks is avoided — use rank counting over global memory.
        uint64_t* sorted = rstore();  // temporarily use the R store head, then shift R below
        for (int base = 0; base < nna; base += kWave) {
            const int i = base + lane;
            if (i < nna) {
                const uint64_t v = na[i];
                int rank = 0;
                for (int u = 0; u < nna; ++u) rank += (na[u] > v);
                sorted[rank] = v;
            }
        }
        __syncthreads();
        for (int base = 0; base < nna; base += kWave) {
            const int i = base + lane;
            if (i < nna) na[i] = sorted[i];
        }
        __syncthreads();
        int npiv = 0;
        int rused = 0;
        uint64_t* W = s.u.col.A;
        uint64_t* T = s.u.col.B;
        uint64_t* X = s.u.col.C;
        for (int ci = 0; ci < nna; ++ci) {
            const uint64_t colkey = na[ci];
            const uint32_t cp = key_packed(colkey);
            const float birth = key_diam(colkey);
            int ca, cb, cc = 0;
            if (dim == 1) { ca = (cp >> 8) & 255; cb = cp & 255; }
            else { ca = (cp >> 16) & 255; cb = (cp >> 8) & 255; cc = cp & 255; }
            int nw = coboundary_sorted(dim, ca, cb, cc, W);
            __syncthreads();
            int guard = 0;
            while (true) {
                if (nw == 0) break;  // essential class: not emitted (ripser.cpp:1209-1225)
                const uint64_t tau = W[0];
                // owner among serially reduced columns (LDS keys)
                int owner = -1;
                for (int base = 0; base < npiv; base += kWave) {
                    const int i = base + lane;
                    const bool hit = i < npiv && s.piv[i] == tau;
                    const uint64_t bal = ballot(hit);
                    if (bal) { owner = base + __ffsll((unsigned long long)bal) - 1; break; }
                }
                int nx = 0;
                if (owner >= 0) {
                    const uint32_t meta = rmeta()[owner];
                    const int off = (int)(meta >> 12), len = (int)(meta & 4095);
                    for (int i = lane; i < len; i += kWave) X[i] = rstore()[off + i];
                    nx = len;
                } else {
                    const uint32_t ow = apparent_owner(dim, tau);
                    if (ow == 0xFFFFFFFFu) {
                        // tau is unowned: pivot of this column
                        const float death = key_diam(tau);
                        if (lane == 0 && death > birth) {
                            const int slot = dim == 1 ? n_p1 : n_p2;
                            if (slot < kPairCap) pairs(dim)[slot] = make_float2(birth, death);
                        }
                        if (death > birth) { if (dim == 1) ++n_p1; else ++n_p2; }
                        if (dim == 1 && lane == 0) {
                            const uint32_t tp = key_packed(tau);
                            set_cleared((tp >> 16) & 255, (tp >> 8) & 255, tp & 255);
                        }
                        if (npiv >= kPivCap || rused + nw > kRCap) { err |= (npiv >= kPivCap ? kErrPiv : kErrR); return; }
                        for (int i = lane; i < nw; i += kWave) rstore()[rused + i] = W[i];
                        if (lane == 0) {
                            s.piv[npiv] = tau;
                            rmeta()[npiv] = ((uint32_t)rused << 12) | (uint32_t)nw;
                        }
                        rused += nw;
                        ++npiv;
                        __syncthreads();
                        break;
                    }
                    // owner must precede this column in Ripser's order (key greater)
                    const uint64_t okey = dim == 1 ? ekey((ow >> 8) & 255, ow & 255)
                                                   : tkey((ow >> 16) & 255, (ow >> 8) & 255, ow & 255);
                    if (!(okey > colkey)) { err |= kErrOrder; return; }
                    if (dim == 1) nx = coboundary_sorted(1, (ow >> 8) & 255, ow & 255, 0, X);
                    else nx = coboundary_sorted(2, (ow >> 16) & 255, (ow >> 8) & 255, ow & 255, X);
                }
                __syncthreads();
                const int nt = merge_xor(W, nw, X, nx, T);
                __syncthreads();
                if (nt < 0) { err |= kErrWorkCol; return; }
                uint64_t* tmp = W; W = T; T = tmp;
                nw = nt;
                if (++guard > 100000) { err |= kErrWorkCol; return; }
            }
        }
    }
};

template <int NP>
__global__ __launch_bounds__(kWave) void betti_kernel(BettiLaunch bl) {
    __shared__ BettiSmem<NP> s;
    __shared__ int64_t chunk_s;
    const int lane = lane_id();
    uint8_t* scratch = bl.scratch + (int64_t)blockIdx.x * bl.scratch_per_wave;
    const int64_t A = bl.num_atoms;

    for (;;) {
        if (lane == 0) chunk_s = (int64_t)atomicAdd((unsigned int*)bl.work_counter, 1u) * kChunk;
        __syncthreads();
        const int64_t chunk0 = chunk_s;
        __syncthreads();
        if (chunk0 >= A) break;
        for (int64_t gi = chunk0; gi < chunk0 + kChunk && gi < A; ++gi) {
            int64_t r0 = 0;
            int n;
            if (bl.clouds) {
                n = bl.npoints[gi];
            } else {
                r0 = bl.row_ptr[gi];
                n = (int)(bl.row_ptr[gi + 1] - r0) + 1;
            }
            double* feat = bl.features ? bl.features + 35 * gi : nullptr;
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
                const int sp = bl.species[gi];
                int cnt = 0;
                for (int64_t j = s0 + lane; j < s1; j += kWave) cnt += (bl.species[j] == sp);
                cnt = wave_sum(cnt);
                weight = 1.0 / (double)cnt;
            }

            if (n > NP) {
                if (lane == 0) atomicOr(bl.error_flag, kErrTooManyPoints);
                if (feat && lane < 35) feat[lane] = __builtin_nan("");
                if (bl.counts && lane < 4) bl.counts[4 * gi + lane] = -1;
                continue;
            }
            Complex<NP> cx{s, n, bl.thr, scratch, 0u, 0, 0, 0, 0};
            // ---- load the local cloud (betti_features.cpp:67-73) ----
            if (lane < n && bl.clouds) {
                const double* xc = bl.clouds + ((int64_t)gi * bl.cloud_stride + lane) * 3;
                s.u.cloud.X[lane][0] = xc[0];
                s.u.cloud.X[lane][1] = xc[1];
                s.u.cloud.X[lane][2] = xc[2];
                s.u.cloud.sq[lane] = (xc[0] * xc[0] + xc[1] * xc[1]) + xc[2] * xc[2];
            } else if (lane < n) {
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
            __syncthreads();
            // ---- distance matrix on the matrix cores (ripser_wrapper.cpp:64-67) ----
            {
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
                            if (row < n && col < n) {
                                const double dot = (p0[r] + p1[r]) + p2[r];  // GEBP k order, no FMA
                                const double d2 = (s.u.cloud.sq[row] + s.u.cloud.sq[col]) - 2.0 * dot;
                                const float d = row == col ? 0.0f : (float)sqrt(fmax(d2, 0.0));
                                s.D[row][col] = d;
                                s.D[col][row] = d;
                            }
                        }
                    }
                }
            }
            __syncthreads();
            // ---- adjacency (sparse_distance_matrix: i != j and d <= thr, ripser.cpp:386-395) ----
            {
                uint64_t m = 0;
                if (lane < n) {
                    for (int w2 = 0; w2 < n; ++w2)
                        if (w2 != lane && s.D[lane][w2] <= cx.thr) m |= 1ull << w2;
                }
                s.adj[lane] = lane < n ? m : 0ull;
                s.tree[lane] = 0ull;
            }
            for (int i = lane; i < (int)(sizeof(s.cleared) / 4); i += kWave) s.cleared[i] = 0u;
            __syncthreads();
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
            __syncthreads();
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
            __syncthreads();
            cx.n_p1 = 0;
            cx.n_p2 = 0;
            // ---- dim 1 ----
            if (dim_max >= 1) {
                int nna = 0;
                for (int base = 0; base < n_edges; base += kWave) {
                    const int e = base + lane;
                    bool is_col = false, apparent = false, na_col = false;
                    float birth = 0.f, death = 0.f;
                    uint64_t colkey = 0;
                    if (e < n_edges) {
                        const int i = s.edges[e] >> 8, j = s.edges[e] & 255;
                        is_col = !((s.tree[i] >> j) & 1ull);
                        if (is_col) {
                            birth = s.D[i][j];
                            colkey = make_key(birth, pack2(i, j));
                            uint64_t cand = s.adj[i] & s.adj[j];
                            if (cand) {
                                uint64_t best = kInf;
                                int kb = -1;
                                while (cand) {
                                    const int k = __ffsll((unsigned long long)cand) - 1;
                                    cand &= cand - 1;
                                    const uint64_t key = make_key(fmaxf(birth, fmaxf(s.D[i][k], s.D[j][k])), tri_with(i, j, k));
                                    if (key < best) { best = key; kb = k; }
                                }
                                death = key_diam(best);
                                // apparent iff (i,j) is the F-max facet of {i,j,kb}
                                const uint64_t f1 = cx.ekey(i, kb), f2 = cx.ekey(j, kb);
                                apparent = colkey > f1 && colkey > f2;
                                if (apparent) {
                                    const uint32_t tp = key_packed(best);
                                    cx.set_cleared((tp >> 16) & 255, (tp >> 8) & 255, tp & 255);
                                } else {
                                    na_col = true;
                                }
                            }
                        }
                    }
                    cx.append_pairs(1, apparent && death > birth, birth, death);
                    const uint64_t bal = ballot(na_col);
                    if (na_col) {
                        const int slot = nna + mask_prefix(bal);
                        if (slot < kNACap) cx.na_list()[slot] = colkey;
                    }
                    nna += __popcll(bal);
                }
                __syncthreads();
                cx.reduce_serial(1, nna);
                __syncthreads();
            }
            // ---- dim 2 ----
            if (dim_max >= 2 && cx.err == 0) {
                int nna = 0;
                // stream triangles: each lane owns an edge (a > b) and walks c < b in adj[a] & adj[b]
                int next_edge = 0;
                int ea = 0, eb = 0;
                uint64_t tmask = 0;
                while (true) {
                    // refill lanes with empty masks
                    while (true) {
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
                    uint64_t colkey = 0;
                    if (active) {
                        const int a = ea, b = eb;
                        const int c = __ffsll((unsigned long long)tmask) - 1;
                        tmask &= tmask - 1;
                        if (!cx.is_cleared(a, b, c)) {
                            birth = cx.tri_diam(a, b, c);
                            colkey = make_key(birth, pack3(a, b, c));
                            uint64_t cand = s.adj[a] & s.adj[b] & s.adj[c];
                            if (cand) {
                                uint64_t best = kInf;
                                int kb = -1;
                                while (cand) {
                                    const int k = __ffsll((unsigned long long)cand) - 1;
                                    cand &= cand - 1;
                                    const float dd = fmaxf(birth, fmaxf(fmaxf(s.D[a][k], s.D[b][k]), s.D[c][k]));
                                    const uint64_t key = make_key(dd, tet_with(a, b, c, k));
                                    if (key < best) { best = key; kb = k; }
                                }
                                death = key_diam(best);
                                // facets containing kb
                                const uint32_t tp = key_packed(best);
                                const int p = (tp >> 24) & 255, q = (tp >> 16) & 255, r = (tp >> 8) & 255, t = tp & 255;
                                uint64_t fm = cx.tkey(p, q, r);
                                uint64_t k2 = cx.tkey(p, q, t); fm = k2 > fm ? k2 : fm;
                                k2 = cx.tkey(p, r, t); fm = k2 > fm ? k2 : fm;
                                k2 = cx.tkey(q, r, t); fm = k2 > fm ? k2 : fm;
                                apparent = fm == colkey;
                                na_col = !apparent;
                            }
                        }
                    }
                    cx.append_pairs(2, apparent && death > birth, birth, death);
                    const uint64_t bal = ballot(na_col);
                    if (na_col) {
                        const int slot = nna + mask_prefix(bal);
                        if (slot < kNACap) cx.na_list()[slot] = colkey;
                    }
                    nna += __popcll(bal);
                }
                __syncthreads();
                cx.reduce_serial(2, nna);
                __syncthreads();
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
                    st[1] = sqrt(ss / (double)m);
                    st[2] = mx;
                    st[3] = mn;
                    st[4] = sum * weight;
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
            __syncthreads();
        }
    }
}

// ---------------------------------------------------------------------------------------
int betti_max_points() { return 64; }
int64_t betti_scratch_bytes_per_wave() { return ScratchLayout::total; }

static int np_for(int max_points) { return max_points <= 32 ? 32 : (max_points <= 48 ? 48 : 64); }

int betti_grid_waves(int device) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return 1024;
    // occupancy of the largest instantiation bounds the slots we allocate scratch for
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, betti_kernel<32>, kWave, 0) != hipSuccess || per_cu <= 0)
        per_cu = 8;
    return prop.multiProcessorCount * per_cu;
}

hipError_t launch_betti(hipStream_t st, const BettiLaunch& b, int max_points, int grid_waves) {
    const int np = np_for(max_points);
    int per_cu = 0;
    hipError_t e = hipSuccess;
    int dev = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    hipDeviceProp_t prop;
    if ((e = hipGetDeviceProperties(&prop, dev)) != hipSuccess) return e;
    if (np == 32) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, betti_kernel<32>, kWave, 0);
    else if (np == 48) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, betti_kernel<48>, kWave, 0);
    else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, betti_kernel<64>, kWave, 0);
    if (e != hipSuccess || per_cu <= 0) per_cu = 4;
    int grid = prop.multiProcessorCount * per_cu;
    if (grid > grid_waves) grid = grid_waves;
    const int64_t chunks = (b.num_atoms + kChunk - 1) / kChunk;
    if (grid > chunks) grid = (int)(chunks > 0 ? chunks : 1);
    if (np == 32) hipLaunchKernelGGL(betti_kernel<32>, dim3(grid), dim3(kWave), 0, st, b);
    else if (np == 48) hipLaunchKernelGGL(betti_kernel<48>, dim3(grid), dim3(kWave), 0, st, b);
    else hipLaunchKernelGGL(betti_kernel<64>, dim3(grid), dim3(kWave), 0, st, b);
    return hipGetLastError();
}

}  // namespace dgn
