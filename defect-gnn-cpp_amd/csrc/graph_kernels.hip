// graph_kernels.hip — periodic fixed-radius neighbour search, CSR compaction and Gaussian-RBF
// edge features for gfx950, plus the Betti pass's local clouds.
//
// Replaces src/graph/neighbor_list.cpp:27-94 (nanoflann KD-tree over a (2n+1)^3 image cloud),
// src/graph/edge_features.cpp:7-24, the edge loop of src/graph/crystal_graph.cpp:32-40 and the
// NeighborList(rc, SIZE_MAX) + cloud assembly of src/topology/betti_features.cpp:67-73,107.
//
// Design (MI355X-first):
//   * prep (one block per structure): geometry, the reference's image bound, the atom ->
//     structure map, the 1/count(species) Betti weight and, for structures above kStage atoms,
//     a cell list in fractional space (cells at least H wide, so a query's window spans <= 3 cells
//     per axis);
//   * one wave64 per query atom; the candidate (atom, image) set is produced by one of three
//     searches, all conservative supersets of the reference's hits:
//       - staged + one image per axis (cells wider than 2 rc): the structure's positions and
//         fractional coordinates are staged in LDS; lane j tests atom j's unique candidate image
//         with three fractional compares, survivors are ballot-compacted into a per-wave LDS ring
//         and exact-tested 64 at a time;
//       - cell list (structures above kStage atoms): lanes enumerate the <= 27 cells of the
//         window, a wave prefix sum lays their atoms out, lane t exact-tests candidate t;
//       - general (cells narrower than 2 rc): every image inside the atom's fractional slab;
//     the exact test reproduces the reference arithmetic bit for bit (offset ((na*a + nb*b) +
//     nc*c), p = pos + offset, d2 = ((dx^2 + dy^2) + dz^2), strict d2 < rc^2, self skip
//     sqrt(d2) < eps), clamped to the reference's +-nref image range; -ffp-contract=off;
//   * count: hit counts only; emit (fused): re-run the search, compact hits with ballot + mbcnt,
//     rank by (distance, j, image) — the canonical row order; the reference's nanoflann order
//     differs only among exact ties — and write the kept rows; the block's RBF region (contiguous
//     in the CSR) is then written as one flat stream of non-temporal 16-byte stores.
#include "dgn_internal.hpp"

namespace dgn {

constexpr int kW = kGraphBlock / kWave;  // waves per block

__device__ __forceinline__ int32_t uni_i32(int32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// fractional coordinates u = p . R (R = inverse lattice), one fixed operation order everywhere
__device__ __forceinline__ double frac_k(const double* R, int k, double x, double y, double z) {
    return (x * R[k] + y * R[3 + k]) + z * R[6 + k];
}

// ------------------------------------------------------------------------------------------
// Structure prep: one block per structure
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t pack_cell_atom(int j, int s0, int s1, int s2) {
    return (uint64_t)(uint32_t)j | ((uint64_t)(s0 + 512) << 32) | ((uint64_t)(s1 + 512) << 42) |
           ((uint64_t)(s2 + 512) << 52);
}

// thread per structure: geometry + the reference image bound + search strategy
__global__ __launch_bounds__(128) void prep_meta_kernel(const double* __restrict__ lattice,
                                                        const int64_t* __restrict__ atom_offset, int64_t B, double rc,
                                                        StructMeta* __restrict__ meta) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    StructMeta m;
    const double* L = lattice + 9 * b;
    for (int k = 0; k < 9; ++k) m.L[k] = L[k];
    const double a00 = L[0], a01 = L[1], a02 = L[2], a10 = L[3], a11 = L[4], a12 = L[5], a20 = L[6], a21 = L[7],
                 a22 = L[8];
    const double c00 = a11 * a22 - a12 * a21, c01 = a02 * a21 - a01 * a22, c02 = a01 * a12 - a02 * a11;
    const double c10 = a12 * a20 - a10 * a22, c11 = a00 * a22 - a02 * a20, c12 = a02 * a10 - a00 * a12;
    const double c20 = a10 * a21 - a11 * a20, c21 = a01 * a20 - a00 * a21, c22 = a00 * a11 - a01 * a10;
    const double det = a00 * c00 + a01 * c10 + a02 * c20;
    const double id = 1.0 / det;
    m.R[0] = c00 * id; m.R[1] = c01 * id; m.R[2] = c02 * id;
    m.R[3] = c10 * id; m.R[4] = c11 * id; m.R[5] = c12 * id;
    m.R[6] = c20 * id; m.R[7] = c21 * id; m.R[8] = c22 * id;
    bool one = true, few = true;
    for (int k = 0; k < 3; ++k) {
        m.H[k] = rc * sqrt(m.R[k] * m.R[k] + m.R[3 + k] * m.R[3 + k] + m.R[6 + k] * m.R[6 + k]) + 1e-9;
        one = one && m.H[k] < 0.5;
        few = few && m.H[k] < 1.0;
    }
    // Eigen Matrix3d row norm: x0 + (x1 + x2) (fixed-size unrolled redux), neighbor_list.cpp:69
    double lmin = 1e300;
    for (int r = 0; r < 3; ++r) {
        const double* v = L + 3 * r;
        lmin = fmin(lmin, sqrt(v[0] * v[0] + (v[1] * v[1] + v[2] * v[2])));
    }
    m.nref = (int32_t)ceil(rc / lmin) + 1;
    m.first = atom_offset[b];
    m.natoms = (int32_t)(atom_offset[b + 1] - atom_offset[b]);
    // one image per axis => nref == 2 (rc < half of every perpendicular width < half of every row
    // norm); the 5^3 image-offset table of the staged search relies on it
    m.one = (one && m.nref == 2) ? 1 : 0;
    m.cells = (m.one && m.natoms > kStage) ? 1 : 0;
    // every H_k < 1 (rc below every perpendicular width, so nref == 2 as well): at most two images
    // per axis can reach rc; staged structures take search_staged_few
    m.few = (!m.one && few && m.nref == 2) ? 1 : 0;
    m.diag = (L[1] == 0.0 && L[2] == 0.0 && L[3] == 0.0 && L[5] == 0.0 && L[6] == 0.0 && L[7] == 0.0) ? 1 : 0;
    // the fixed-point coordinates truncate at 2^-32: the nearest-image displacement is off by at
    // most 2^-31 (|a| + |b| + |c|) per component, d2 by 2 rc times that (for d <= rc); 64x margin
    {
        double lsum = 0.0;
        for (int r = 0; r < 3; ++r) lsum += fabs(L[3 * r]) + fabs(L[3 * r + 1]) + fabs(L[3 * r + 2]);
        m.band = 64.0 * 2.0 * rc * lsum * 0x1p-31 + 1e-12 * rc * rc;
    }
    // the count pass's f32 window (count_one_image), once per structure instead of per query:
    //   band32 bounds |approx - exact| for candidates with either value below rc^2 + band32: the
    //   fixed-point quantisation (band), f32 displacement error eps <= 5 * 2^-24 * 0.5 * sum|L| per
    //   axis (conversion of the 32-bit fraction, the rounded f32 lattice, product, two sums),
    //   2 sqrt(3) R eps + 3 eps^2 on the square (R = rc + 1e-3 bounds |d|), 3 * 2^-24 R^2 for the
    //   f32 square and sums, 2^-20 rc^2 for rounding the thresholds; the sum is doubled.
    //   `few` structures (search_staged_few) convert the fixed-point fraction (|D| <= 0.5) and add
    //   the +-1 shift in f32 (|f| < 1, one more rounding): eps <= 8 * 2^-24 * sum|L| covers it.
    {
        const double rc2 = rc * rc;
        double lsum = 0.0;
        for (int k = 0; k < 9; ++k) lsum += fabs(L[k]);
        const double eps = (m.few ? 8.0 * 0x1p-24 : 5.0 * 0x1p-24 * 0.5) * lsum, R = sqrt(rc2) + 1e-3;
        const double band32 = 2.0 * (m.band + 2.0 * 1.7320508075688772 * R * eps + 3.0 * eps * eps +
                                     3.0 * 0x1p-24 * R * R + 0x1p-20 * rc2);
        m.lo32 = (float)(rc2 - band32);
        m.hi32 = (float)(rc2 + band32);
        for (int k = 0; k < 9; ++k) m.lf[k] = (float)(L[k] * (m.few ? 1.0 : 0x1p-32));
    }
    for (int k = 0; k < 3; ++k) m.nc[k] = 1;
    if (m.cells) {
        // cells at least H wide: a query window (width 2H) spans <= 3 cells per axis
        int nc[3];
        for (int k = 0; k < 3; ++k) nc[k] = (int)fmin(floor(1.0 / m.H[k]), 64.0);
        const int cap = m.natoms < kCellMax ? m.natoms : kCellMax;
        while ((int64_t)nc[0] * nc[1] * nc[2] > cap) {
            const int k = nc[0] >= nc[1] && nc[0] >= nc[2] ? 0 : (nc[1] >= nc[2] ? 1 : 2);
            nc[k] -= 1;
        }
        for (int k = 0; k < 3; ++k) m.nc[k] = nc[k];
    }
    meta[b] = m;
}

// fractional cell coordinate of atom position p: floor s (the periodic shift of the wrapped
// coordinate) and the wrapped fraction w in [0, 1) as 32-bit fixed point W (w * 2^32)
__device__ __forceinline__ void frac_fixed(const double* R, int k, const double p[3], int& s, uint32_t& W) {
    const double u = frac_k(R, k, p[0], p[1], p[2]);
    double f = floor(u);
    uint64_t w = (uint64_t)((u - f) * 4294967296.0);
    if (w >= 4294967296ull) {  // u - f rounded to 1.0
        w -= 4294967296ull;
        f += 1.0;
    }
    s = (int)f;
    W = (uint32_t)w;
}

// block per structure: atom -> structure map, the far-position check, the per-atom
// 1/count(species) Betti weight and, for structures above kStage atoms, the cell list
__global__ __launch_bounds__(1024) void prep_atoms_kernel(const StructMeta* __restrict__ meta,
                                                         const double* __restrict__ pos,
                                                         const int32_t* __restrict__ species,
                                                         int32_t* __restrict__ atom_struct,
                                                         int32_t* __restrict__ cell_start,
                                                         double4* __restrict__ cell_pos, double* __restrict__ weight,
                                                         uint32_t* __restrict__ error_flag) {
    __shared__ int32_t hist[kCellMax + 1];
    __shared__ int32_t shist[256];
    __shared__ int32_t part[1024 / kWave];
    const int64_t b = blockIdx.x;
    const int tid = threadIdx.x;
    const StructMeta& sm = meta[b];
    const int64_t first = sm.first;
    const int natoms = sm.natoms;
    const bool one = sm.one != 0 || sm.few != 0;  // fixed-point coordinates (10-bit floors) in use
    for (int t = tid; t < natoms; t += blockDim.x) {
        atom_struct[first + t] = (int32_t)b;
        if (one) {
            const double* p = pos + 3 * (first + t);
            bool far = false;
            for (int k = 0; k < 3; ++k) {
                const double u = frac_k(sm.R, k, p[0], p[1], p[2]);
                far = far || !(fabs(u) < 500.0);
            }
            if (far) atomicOr(error_flag, kGErrFar);
        }
    }
    // 1 / count(species of i) within the structure (betti_features.cpp:62-63, 77)
    if (weight && species) {
        for (int t = tid; t < 256; t += blockDim.x) shist[t] = 0;
        __syncthreads();
        for (int t = tid; t < natoms; t += blockDim.x) {
            const int s = species[first + t];
            if (s >= 0 && s < 256) atomicAdd(&shist[s], 1);
        }
        __syncthreads();
        for (int t = tid; t < natoms; t += blockDim.x) {
            const int s = species[first + t];
            int cnt;
            if (s >= 0 && s < 256) {
                cnt = shist[s];
            } else {
                cnt = 0;
                for (int u = 0; u < natoms; ++u) cnt += species[first + u] == s;
            }
            weight[first + t] = 1.0 / (double)cnt;
        }
    }
    if (!sm.cells) return;
    // ---- cell list: counting sort of the atoms by fractional cell ----
    const int nc0 = sm.nc[0], nc1 = sm.nc[1], nc2 = sm.nc[2];
    const int ncell = nc0 * nc1 * nc2;
    for (int c = tid; c <= ncell; c += blockDim.x) hist[c] = 0;
    __syncthreads();
    auto cell_of = [&](int t, int s[3]) -> int {
        const double* p = pos + 3 * (first + t);
        int c[3];
        for (int k = 0; k < 3; ++k) {
            uint32_t W;
            frac_fixed(sm.R, k, p, s[k], W);
            const int n = sm.nc[k];
            int ck = (int)(((uint64_t)W * (uint64_t)n) >> 32);
            c[k] = ck < n ? ck : n - 1;
        }
        return (c[0] * nc1 + c[1]) * nc2 + c[2];
    };
    for (int t = tid; t < natoms; t += blockDim.x) {
        int s[3];
        atomicAdd(&hist[cell_of(t, s)], 1);
    }
    __syncthreads();
    // exclusive scan of hist[0 .. ncell) in place: per-thread chunks + wave / block scan
    const int per = (ncell + (int)blockDim.x - 1) / (int)blockDim.x;
    const int c0 = tid * per, c1 = c0 + per < ncell ? c0 + per : ncell;
    int local = 0;
    for (int c = c0; c < c1; ++c) local += hist[c];
    const int inc = wave_inclusive_sum(local);
    if (lane_id() == kWave - 1) part[tid / kWave] = inc;
    __syncthreads();
    int off = inc - local;
    for (int w = 0; w < tid / kWave; ++w) off += part[w];
    __syncthreads();
    for (int c = c0; c < c1; ++c) {
        const int v = hist[c];
        hist[c] = off;
        off += v;
    }
    __syncthreads();
    int32_t* cs = cell_start + first + b;
    for (int c = tid; c < ncell; c += blockDim.x) cs[c] = hist[c];
    if (tid == 0) cs[ncell] = natoms;
    __syncthreads();
    for (int t = tid; t < natoms; t += blockDim.x) {
        int s[3];
        const int c = cell_of(t, s);
        const int slot = atomicAdd(&hist[c], 1);
        const double* p = pos + 3 * (first + t);
        cell_pos[first + slot] = make_double4(p[0], p[1], p[2],
                                              __longlong_as_double((long long)pack_cell_atom(t, s[0], s[1], s[2])));
    }
}

// ------------------------------------------------------------------------------------------
// Block traversal shared by every search kernel: a block owns query atoms [g0, g1) of the
// range [a_begin, a_end); it walks the structures those atoms belong to, stages each structure's
// positions and fractional coordinates in LDS (SoA, when it has at most `cap` atoms; larger ones
// are read from global/L2), and hands every query atom to one wave (round-robin over the 4).
// ------------------------------------------------------------------------------------------
// LDS-typed pointers (address space 3): loads through them are ds_read, never flat loads (a flat
// load's wait also waits for every outstanding global store)
#define DGN_LDS __attribute__((address_space(3)))
template <class T>
__device__ __forceinline__ DGN_LDS T* lds(T* p) { return (DGN_LDS T*)p; }

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef double f64x4 __attribute__((ext_vector_type(4)));
struct StageView {
    DGN_LDS double *x, *y, *z;  // positions
    DGN_LDS u32x4* fx;          // fixed-point wrapped fractional coordinates W0, W1, W2 + packed floors
    DGN_LDS f64x4* offt;        // one-image structures: the 5^3 image offsets ((na*a + nb*b) + nc*c), |n| <= 2
    int cap;
};
// stage bytes per atom: 3 doubles + one uint4
constexpr int kStageBytesPerAtom = 3 * 8 + 16;
// offt == nullptr: no offset table (exact_one computes each image offset)
__device__ __forceinline__ StageView make_stage(double* base_, int cap, double4* offt) {
    DGN_LDS double* base = lds(base_);
    return {base, base + cap, base + 2 * cap, reinterpret_cast<DGN_LDS u32x4*>(base + 3 * cap),
            offt ? reinterpret_cast<DGN_LDS f64x4*>(lds(offt)) : nullptr, cap};
}
__device__ __forceinline__ uint32_t pack_floors(const int s[3]) {
    return (uint32_t)(s[0] + 512) | ((uint32_t)(s[1] + 512) << 10) | ((uint32_t)(s[2] + 512) << 20);
}
__device__ __forceinline__ int floor_of(uint32_t S, int k) { return (int)((S >> (10 * k)) & 1023u) - 512; }

struct PosSrc {
    StageView st;        // the LDS stage (valid if staged)
    bool staged;         // false -> global
    const double* gpos;  // positions of the structure's first atom
    __device__ __forceinline__ void get(int j, double p[3]) const {
        if (staged) {
            p[0] = st.x[j];
            p[1] = st.y[j];
            p[2] = st.z[j];
        } else {
            p[0] = gpos[3 * j];
            p[1] = gpos[3 * j + 1];
            p[2] = gpos[3 * j + 2];
        }
    }
};

// One structure's metadata in wave-uniform registers: lane t loads dword t (one coalesced load),
// v_readlane moves each dword to an SGPR. (Read through a global pointer the compiler must assume
// the kernel's own stores may alias it and re-loads every field with vector loads + waits.)
__device__ __forceinline__ StructMeta load_meta_uniform(const StructMeta* p) {
    constexpr int N = (int)(sizeof(StructMeta) / 4);
    static_assert(N <= 2 * kWave, "StructMeta must fit two wave loads");
    const uint32_t* src = reinterpret_cast<const uint32_t*>(p);
    const int lane = lane_id();
    const uint32_t v = lane < N ? src[lane] : 0u;
    const uint32_t v2 = N > kWave && lane + kWave < N ? src[lane + kWave] : 0u;
    StructMeta m;
    uint32_t* dst = reinterpret_cast<uint32_t*>(&m);
#pragma unroll
    for (int t = 0; t < N; ++t) dst[t] = (uint32_t)__builtin_amdgcn_readlane((int)(t < kWave ? v : v2), t & (kWave - 1));
    return m;
}

// POS = false: only the fixed-point coordinates (and offset table) are staged; positions stay in
// global memory (graph_count_one_kernel, whose tiles hold staged one-image structures only)
template <bool POS = true, class PerAtom>
__device__ __forceinline__ void for_block_atoms(const GraphLaunch& g, const StageView st, int64_t a_begin,
                                                int64_t a_end, int64_t tile, int qa, PerAtom&& per_atom) {
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
    const int64_t g0 = a_begin + tile * qa;
    const int64_t g1 = g0 + qa < a_end ? g0 + qa : a_end;
    if (g0 >= g1) return;
    const int32_t b_first = uni_i32(g.atom_struct[g0]);
    const int32_t b_last = uni_i32(g.atom_struct[g1 - 1]);
    for (int32_t b = b_first; b <= b_last; ++b) {
        const StructMeta M = load_meta_uniform(g.meta + b);
        const int64_t first = M.first;
        const int natoms = M.natoms;
        if (natoms == 0) continue;
        const bool staged = natoms <= st.cap;
        if (staged) {
            __syncthreads();  // previous segment done with the stage
            const double* src = g.pos + 3 * first;
            for (int t = threadIdx.x; t < natoms; t += kGraphBlock) {
                const double p[3] = {src[3 * t], src[3 * t + 1], src[3 * t + 2]};
                if constexpr (POS) {
                    st.x[t] = p[0];
                    st.y[t] = p[1];
                    st.z[t] = p[2];
                }
                if (M.one || M.few) {
                    int sf[3];
                    uint32_t W[3];
                    for (int k = 0; k < 3; ++k) frac_fixed(M.R, k, p, sf[k], W[k]);
                    const u32x4 v = {W[0], W[1], W[2], pack_floors(sf)};
                    st.fx[t] = v;
                }
            }
            if ((M.one || M.few) && st.offt && threadIdx.x < 125) {
                const int t = threadIdx.x;
                const double na = (double)(t / 25 - 2), nb = (double)((t / 5) % 5 - 2), nc = (double)(t % 5 - 2);
                double o[3];
                for (int k = 0; k < 3; ++k) o[k] = (na * M.L[k] + nb * M.L[3 + k]) + nc * M.L[6 + k];
                const f64x4 v = {o[0], o[1], o[2], 0.0};
                st.offt[t] = v;
            }
            __syncthreads();
        }
        const PosSrc P{st, staged, g.pos + 3 * first};
        const int64_t s0 = g0 > first ? g0 : first;
        const int64_t s1 = g1 < first + natoms ? g1 : first + natoms;
        for (int64_t gi = s0 + w; gi < s1; gi += kW) per_atom(M, P, gi, (int)(gi - g0), (int64_t)b);
    }
}

// ------------------------------------------------------------------------------------------
// Exact candidate test (the reference arithmetic) and the searches.
// visit(hit, j, na, nb, nc, d2) is invoked by every lane once per step (hit false = idle).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ double cand_d2(const StructMeta& M, const double pj[3], int na, int nb, int nc,
                                          const double q[3]) {
    const double dna = (double)na, dnb = (double)nb, dnc = (double)nc;
    double d2 = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        // offset = (na*a + nb*b) + nc*c (neighbor_list.cpp:82-84); p = pos + offset (:87)
        const double off = (dna * M.L[k] + dnb * M.L[3 + k]) + dnc * M.L[6 + k];
        const double diff = q[k] - (pj[k] + off);  // L2_Simple_Adaptor: (a - b)^2 accumulated
        d2 += diff * diff;
    }
    return d2;
}

__device__ __forceinline__ uint64_t pack_jimg(int j, int na, int nb, int nc) {
    return ((uint64_t)(uint32_t)j << 24) | ((uint64_t)((na + 128) & 255) << 16) |
           ((uint64_t)((nb + 128) & 255) << 8) | (uint64_t)((nc + 128) & 255);
}
__device__ __forceinline__ void unpack_jimg(uint64_t key, int& j, int& na, int& nb, int& nc) {
    j = (int)(key >> 24);
    na = (int)((key >> 16) & 255) - 128;
    nb = (int)((key >> 8) & 255) - 128;
    nc = (int)(key & 255) - 128;
}

// (1) staged structure, one image per axis. With W the 32-bit fixed-point wrapped fractional
// coordinates, D = W_j - W_q (mod 2^32) read as a signed fraction is the displacement to atom j's
// nearest image — its only candidate image. Its image n = (s_q - s_j) - carry (s = floors, carry =
// the wrap of W_j - W_q) and the reference arithmetic (offset from the staged 5^3 table, |n| <=
// nref = 2) give the exact d2.
// posj(j, p) yields atom j's position (LDS stage or global memory: the same doubles)
// The exact d2 of atom j's image n (|n_k| <= 2 when inr; otherwise image 0 is evaluated and the
// caller discards the value): offset from the staged 5^3 table or the table's arithmetic.
template <class PosJ>
__device__ __forceinline__ double exact_at_n(const StructMeta& M, const DGN_LDS f64x4* offt, PosJ&& posj, int j,
                                             const double q[3], const int n[3], bool inr) {
    f64x4 o;
    if (offt) {
        o = offt[inr ? (n[0] + 2) * 25 + (n[1] + 2) * 5 + (n[2] + 2) : 62];
    } else {  // the table's arithmetic: ((na*a + nb*b) + nc*c)
        const double na = inr ? (double)n[0] : 0.0, nb = inr ? (double)n[1] : 0.0, nc = inr ? (double)n[2] : 0.0;
        o.x = (na * M.L[0] + nb * M.L[3]) + nc * M.L[6];
        o.y = (na * M.L[1] + nb * M.L[4]) + nc * M.L[7];
        o.z = (na * M.L[2] + nb * M.L[5]) + nc * M.L[8];
    }
    double pj[3];
    posj(j, pj);
    const double p0 = pj[0] + o.x, p1 = pj[1] + o.y, p2 = pj[2] + o.z;  // p = pos + offset
    const double e0 = q[0] - p0, e1 = q[1] - p1, e2 = q[2] - p2;
    return ((0.0 + e0 * e0) + e1 * e1) + e2 * e2;  // L2_Simple_Adaptor accumulation
}
template <class PosJ>
__device__ __forceinline__ double exact_one_at(const StructMeta& M, const DGN_LDS f64x4* offt, const u32x4 fq,
                                               const u32x4 fj, PosJ&& posj, int j, const double q[3], int n[3],
                                               bool& inr) {
    inr = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t wj = k == 0 ? fj.x : (k == 1 ? fj.y : fj.z);
        const uint32_t wq = k == 0 ? fq.x : (k == 1 ? fq.y : fq.z);
        const int dw = (int)(wj - wq);
        const int carry = (int)(wj >= wq) - (int)(dw >= 0);
        n[k] = (floor_of(fq.w, k) - floor_of(fj.w, k)) - carry;
        inr = inr && (uint32_t)(n[k] + 2) <= 4u;  // |n| <= nref = 2
    }
    return exact_at_n(M, offt, posj, j, q, n, inr);
}
__device__ __forceinline__ double exact_one(const StructMeta& M, const StageView& st, const u32x4 fq, const u32x4 fj,
                                            int j, const double q[3], int n[3], bool& inr) {
    return exact_one_at(
        M, st.offt, fq, fj,
        [&](int jj, double p[3]) __attribute__((always_inline)) {
            p[0] = st.x[jj];
            p[1] = st.y[jj];
            p[2] = st.z[jj];
        },
        j, q, n, inr);
}
// |nearest-image displacement|^2 from the fixed-point coordinates (within M.band of the exact d2)
__device__ __forceinline__ double approx_d2(const StructMeta& M, const u32x4 fq, const u32x4 fj) {
    const double f0 = (double)(int)(fj.x - fq.x) * 0x1p-32, f1 = (double)(int)(fj.y - fq.y) * 0x1p-32,
                 f2 = (double)(int)(fj.z - fq.z) * 0x1p-32;
    double dx, dy, dz;
    if (M.diag) {
        dx = f0 * M.L[0];
        dy = f1 * M.L[4];
        dz = f2 * M.L[8];
    } else {
        dx = (f0 * M.L[0] + f1 * M.L[3]) + f2 * M.L[6];
        dy = (f0 * M.L[1] + f1 * M.L[4]) + f2 * M.L[7];
        dz = (f0 * M.L[2] + f1 * M.L[5]) + f2 * M.L[8];
    }
    return (dx * dx + dy * dy) + dz * dz;
}

// Count pass on a staged one-image structure: each lane decides atoms base + lane and base + 64 +
// lane from an approximate nearest-image distance computed for both at once in packed f32
// (v_pk_fma_f32); only candidates within `band32` of rc^2 (a few per thousand queries) take the
// exact reference test in f64. The self image (j == li, n = 0) is the only image of the query
// atom within rc. Returns m; mask[t] = the hit ballot of atom tile t (a bit per atom). The f32
// lattice and the window [lo32, hi32] = rc^2 -+ band32 come from prep_meta_kernel (derivation
// there).
typedef float f32x2 __attribute__((ext_vector_type(2)));
// skip_self: eps > 0, so the query's own image (n = 0, d2 = 0) is skipped (neighbor_list.cpp:47); its
// other images are beyond 2 rc here
template <class PosJ>
__device__ __forceinline__ int count_one_image(const StructMeta& M, const DGN_LDS u32x4* fx, const DGN_LDS f64x4* offt,
                                               PosJ&& posj, int li, double rc2, DGN_LDS uint64_t* mask_words,
                                               bool skip_self) {
    const int lane = lane_id();
    const int natoms = M.natoms;
    const u32x4 fq = fx[li];
    const float lo32 = M.lo32, hi32 = M.hi32;  // prep_meta_kernel (band32 derivation there)
    const float* Lf = M.lf;
    int m = 0;
#pragma nounroll
    for (int base = 0, t = 0; base < natoms; base += 2 * kWave, t += 2) {
        const int j0 = base + lane, j1 = base + kWave + lane;
        const u32x4 a = fx[j0 < natoms ? j0 : natoms - 1];
        const u32x4 c = fx[j1 < natoms ? j1 : natoms - 1];
        const f32x2 u0 = {(float)(int)(a.x - fq.x), (float)(int)(c.x - fq.x)};
        const f32x2 u1 = {(float)(int)(a.y - fq.y), (float)(int)(c.y - fq.y)};
        const f32x2 u2 = {(float)(int)(a.z - fq.z), (float)(int)(c.z - fq.z)};
        f32x2 dx, dy, dz;
        if (M.diag) {
            dx = u0 * Lf[0];
            dy = u1 * Lf[4];
            dz = u2 * Lf[8];
        } else {
            dx = __builtin_elementwise_fma(u2, (f32x2)Lf[6], __builtin_elementwise_fma(u1, (f32x2)Lf[3], u0 * Lf[0]));
            dy = __builtin_elementwise_fma(u2, (f32x2)Lf[7], __builtin_elementwise_fma(u1, (f32x2)Lf[4], u0 * Lf[1]));
            dz = __builtin_elementwise_fma(u2, (f32x2)Lf[8], __builtin_elementwise_fma(u1, (f32x2)Lf[5], u0 * Lf[2]));
        }
        const f32x2 d2 = __builtin_elementwise_fma(dx, dx, __builtin_elementwise_fma(dy, dy, dz * dz));
        const bool ok0 = j0 < natoms && !(skip_self && j0 == li), ok1 = j1 < natoms && !(skip_self && j1 == li);
        bool hit0 = ok0 && d2.x < lo32, hit1 = ok1 && d2.y < lo32;
        // borderline: the exact reference arithmetic decides (the query position is only read
        // here, a few times per thousand queries)
        if (ok0 && !hit0 && d2.x <= hi32) {
            int n[3];
            bool inr;
            double q[3];
            posj(li, q);
            const double e2 = exact_one_at(M, offt, fq, a, posj, j0, q, n, inr);
            hit0 = inr && e2 < rc2;
        }
        if (ok1 && !hit1 && d2.y <= hi32) {
            int n[3];
            bool inr;
            double q[3];
            posj(li, q);
            const double e2 = exact_one_at(M, offt, fq, c, posj, j1, q, n, inr);
            hit1 = inr && e2 < rc2;
        }
        const uint64_t bal0 = ballot(hit0), bal1 = ballot(hit1);
        if (mask_words && lane == 0) {
            mask_words[t] = bal0;
            if (base + kWave < natoms) mask_words[t + 1] = bal1;
        }
        m += __popcll(bal0) + __popcll(bal1);
    }
    return m;
}
__device__ __forceinline__ int count_staged_one(const StructMeta& M, const StageView st, int li, double rc2,
                                                DGN_LDS uint64_t* mask_words, bool skip_self) {
    return count_one_image(
        M, st.fx, st.offt,
        [&](int jj, double p[3]) __attribute__((always_inline)) {
            p[0] = st.x[jj];
            p[1] = st.y[jj];
            p[2] = st.z[jj];
        },
        li, rc2, mask_words, skip_self);
}

// Hit collection on a staged one-image structure (emit / Betti): `produce(base, lane, fq) -> bool`
// marks the candidates of atom tile [base, base + 64) — the count pass's exact hit mask, or the
// approximate test (hit or borderline); they queue in a per-wave LDS ring and are exact-tested 64
// at a time.
template <class Produce, class Visit>
__device__ __forceinline__ void search_staged_one(const StructMeta& M, const StageView st, const double q[3], int li,
                                                  double rc2, double eps, DGN_LDS uint32_t* ring, Produce&& produce,
                                                  Visit&& visit) {
    const int lane = lane_id();
    const int natoms = M.natoms;
    const u32x4 fq = st.fx[li];
    int head = 0, cnt = 0;
    auto flush = [&](int take) {
        wave_lds_sync();
        const bool valid = lane < take;
        const int j = valid ? (int)ring[(head + lane) & (kRing - 1)] : li;
        const u32x4 fj = st.fx[j];
        int n[3];
        bool inr;
        const double d2 = exact_one(M, st, fq, fj, j, q, n, inr);
        bool hit = valid && inr && d2 < rc2;         // RadiusResultSet: strict
        if (hit && j == li) hit = !(sqrt(d2) < eps);  // self skip (neighbor_list.cpp:47)
        visit(hit, j, n[0], n[1], n[2], d2);
        head = (head + take) & (kRing - 1);
        cnt -= take;
        wave_lds_sync();
    };
    for (int base = 0; base < natoms; base += kWave) {
        const int j = base + lane;
        const bool pass = j < natoms && produce(base, lane, fq);
        const uint64_t bal = ballot(pass);
        if (pass) ring[(head + cnt + mask_prefix(bal)) & (kRing - 1)] = (uint32_t)j;
        cnt += __popcll(bal);
        if (cnt >= kWave) flush(kWave);
    }
    while (cnt > 0) flush(cnt < kWave ? cnt : kWave);
}

// the approximate test of atom base + lane (hit or borderline; the exact test decides)
struct ApproxOne {
    StageView st;
    StructMeta M;
    int li;
    __device__ __forceinline__ bool operator()(int base, int lane, const u32x4 fq) const {
        const int j = base + lane;
        return (j != li || keep_self) && approx_d2(M, fq, st.fx[j]) <= rc2_ + M.band;
    }
    double rc2_;
    bool keep_self;  // eps <= 0: the self image (d = 0) is not skipped by the reference either
};
// the count pass's exact hits of this query (one bit per atom): lane t holds word t (one
// coalesced load per query), each tile reads its word with v_readlane
struct FromMask {
    uint32_t lo, hi;  // word lane_id() of this atom's mask
    __device__ __forceinline__ bool operator()(int base, int lane, const u32x4) const {
        const uint32_t wl = (uint32_t)__builtin_amdgcn_readlane((int)lo, base >> 6);
        const uint32_t wh = (uint32_t)__builtin_amdgcn_readlane((int)hi, base >> 6);
        return ((lane < 32 ? wl : wh) >> (lane & 31)) & 1u;
    }
};
__device__ __forceinline__ FromMask load_mask(const DGN_LDS uint64_t* m, int natoms) {
    const int lane = lane_id();
    const uint64_t w = lane < (natoms + 63) / 64 ? m[lane] : 0ull;
    return {(uint32_t)w, (uint32_t)(w >> 32)};
}

// The count pass's hits of one query as atom indices, ascending, in hit[0 .. m) (per-wave LDS):
// word t of the mask is tile t's hit ballot, so lane j's slot is the hits before it (popcounts of
// the earlier words + mbcnt). Returns m.
__device__ __forceinline__ int collect_mask_hits(const DGN_LDS uint64_t* mask, int natoms, DGN_LDS uint32_t* hit) {
    const int lane = lane_id();
    int m = 0;
    for (int t = 0; 64 * t < natoms; ++t) {
        const uint64_t wv = mask[t];  // broadcast read
        const uint64_t word = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(wv >> 32)) << 32) |
                              (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)wv);
        const int slot = m + mask_prefix(word);
        if (((word >> lane) & 1ull) && slot < kWave) hit[slot] = (uint32_t)(64 * t + lane);  // callers use <= 64
        m += __popcll(word);
    }
    wave_lds_sync();
    return m;
}
// the same for a `few` structure of <= 64 atoms: word c = combination c's hits (count_few), entries
// (c << 16 | j) in combination order
__device__ __forceinline__ int collect_few_hits(const DGN_LDS uint64_t* mask, DGN_LDS uint32_t* hit) {
    const int lane = lane_id();
    int m = 0;
#pragma unroll
    for (int c = 0; c < kFewMaskWords; ++c) {
        const uint64_t wv = mask[c];
        const uint64_t word = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(wv >> 32)) << 32) |
                              (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)wv);
        const int slot = m + mask_prefix(word);
        if (((word >> lane) & 1ull) && slot < kWave) hit[slot] = ((uint32_t)c << 16) | (uint32_t)lane;
        m += __popcll(word);
    }
    wave_lds_sync();
    return m;
}

// (1b) staged structure with every H_k < 1 (`few`: cells wider than rc but narrower than 2 rc,
// e.g. config 2's SC-64 at 5 A, H = 0.54). Per axis at most two images of atom j can reach rc:
// the nearest one (D_k of (1), image n0_k) and, when 1 - |D_k| <= H_k, the next one on the other
// side (D_k + s_k, s_k = -sign(D_k), image n0_k + s_k) — at most 2^3 (atom, image) candidates,
// each decided in f32 from the fixed-point fractions (window [lo32, hi32], prep_meta_kernel) with
// the borderline ones sent to the exact reference test. The general search (3) enumerates the same
// images through f64 slab bounds and per-lane image loops.
struct FewLane {
    float f[3][2];  // fractional displacement of option 0 / 1 per axis
    int n0[3];      // option 0's image per axis
    uint32_t up;    // bit k: axis k's option-1 shift is +1 (else -1)
    uint32_t ok;    // bit 2k + o: option o of axis k within H_k (+ f32 slack) and |n| <= nref = 2
};
__device__ __forceinline__ FewLane few_lane(const float h[3], const u32x4 fq, const u32x4 fj) {
    FewLane r;
    r.up = 0;
    r.ok = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const uint32_t wj = k == 0 ? fj.x : (k == 1 ? fj.y : fj.z);
        const uint32_t wq = k == 0 ? fq.x : (k == 1 ? fq.y : fq.z);
        const int dw = (int)(wj - wq);
        const int carry = (int)(wj >= wq) - (int)(dw >= 0);
        const int n0 = (floor_of(fq.w, k) - floor_of(fj.w, k)) - carry;
        const int s = dw >= 0 ? -1 : 1;
        const float f0 = (float)dw * 0x1p-32f;
        const float f1 = f0 + (float)s;
        r.f[k][0] = f0;
        r.f[k][1] = f1;
        r.n0[k] = n0;
        r.up |= s > 0 ? 1u << k : 0u;
        r.ok |= (__builtin_fabsf(f0) <= h[k] && (uint32_t)(n0 + 2) <= 4u) ? 1u << (2 * k) : 0u;
        r.ok |= (__builtin_fabsf(f1) <= h[k] && (uint32_t)(n0 + s + 2) <= 4u) ? 2u << (2 * k) : 0u;
    }
    return r;
}
// combination c (bit k = axis k's option) admissible for this lane
__device__ __forceinline__ bool few_combo_ok(uint32_t ok, int c) {
    return ((ok >> (c & 1)) & (ok >> (2 + ((c >> 1) & 1))) & (ok >> (4 + ((c >> 2) & 1))) & 1u) != 0;
}
__device__ __forceinline__ void few_image(const FewLane& r, int c, int n[3]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) n[k] = r.n0[k] + (((c >> k) & 1) ? (((r.up >> k) & 1) ? 1 : -1) : 0);
}
// approximate |displacement|^2 of combination c (f32 lattice rows M.lf, unscaled for `few`)
__device__ __forceinline__ float few_d2(const StructMeta& M, const FewLane& r, int c) {
    const float u0 = r.f[0][c & 1], u1 = r.f[1][(c >> 1) & 1], u2 = r.f[2][(c >> 2) & 1];
    const float* L = M.lf;
    float dx, dy, dz;
    if (M.diag) {
        dx = u0 * L[0];
        dy = u1 * L[4];
        dz = u2 * L[8];
    } else {
        dx = __builtin_fmaf(u2, L[6], __builtin_fmaf(u1, L[3], u0 * L[0]));
        dy = __builtin_fmaf(u2, L[7], __builtin_fmaf(u1, L[4], u0 * L[1]));
        dz = __builtin_fmaf(u2, L[8], __builtin_fmaf(u1, L[5], u0 * L[2]));
    }
    return __builtin_fmaf(dx, dx, __builtin_fmaf(dy, dy, dz * dz));
}
// conservative f32 half-widths: H_k plus the f32 error of the displacement (<= 2^-23)
__device__ __forceinline__ void few_halfwidths(const StructMeta& M, float h[3]) {
#pragma unroll
    for (int k = 0; k < 3; ++k) h[k] = (float)M.H[k] + 0x1p-20f;
}

// Count pass on a staged `few` structure: sure hits (below lo32) are counted from the f32 value,
// borderline ones take the exact test. The self image (j == li, n = 0, d2 = 0) is skipped exactly
// when the reference skips it (sqrt(0) < eps).
// mask_words (structures of <= 64 atoms, or null): word c = the hit ballot of combination c, which
// the emit reads instead of searching again (collect_few_hits).
template <class PosJ>
__device__ __forceinline__ int count_few(const StructMeta& M, const DGN_LDS u32x4* fx, const DGN_LDS f64x4* offt,
                                         PosJ&& posj, int li, double rc2, double eps, DGN_LDS uint64_t* mask_words) {
    const int lane = lane_id();
    const int natoms = M.natoms;
    const u32x4 fq = fx[li];
    const float lo32 = M.lo32, hi32 = M.hi32;
    float h[3];
    few_halfwidths(M, h);
    const bool skip_self = 0.0 < eps;
    int m = 0;
#pragma nounroll
    for (int base = 0; base < natoms; base += kWave) {
        const int j = base + lane;
        const bool valid = j < natoms;
        const FewLane r = few_lane(h, fq, fx[valid ? j : li]);
        const uint32_t okm = valid ? r.ok : 0u;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const bool allowed = few_combo_ok(okm, c) && !(c == 0 && skip_self && j == li);
            if (!ballot(allowed)) {  // wave-uniform: no lane has this combination
                if (mask_words && lane == 0) mask_words[c] = 0;
                continue;
            }
            const float d2 = few_d2(M, r, c);
            bool hit = allowed && d2 < lo32;
            if (allowed && !hit && d2 <= hi32) {
                int n[3];
                few_image(r, c, n);
                double q[3];
                posj(li, q);
                hit = exact_at_n(M, offt, posj, j, q, n, true) < rc2;
            }
            const uint64_t bal = ballot(hit);
            if (mask_words && lane == 0) mask_words[c] = bal;
            m += __popcll(bal);
        }
    }
    return m;
}

// Hit collection on a staged `few` structure (emit / Betti): the combinations at or below hi32
// queue in the per-wave LDS ring as (c << 16 | j) and are exact-tested 64 at a time.
template <class Visit>
__device__ __forceinline__ void search_staged_few(const StructMeta& M, const StageView st, const double q[3], int li,
                                                  double rc2, double eps, DGN_LDS uint32_t* ring, Visit&& visit) {
    const int lane = lane_id();
    const int natoms = M.natoms;
    const u32x4 fq = st.fx[li];
    const float hi32 = M.hi32;
    float h[3];
    few_halfwidths(M, h);
    auto posj = [&](int jj, double p[3]) __attribute__((always_inline)) {
        p[0] = st.x[jj];
        p[1] = st.y[jj];
        p[2] = st.z[jj];
    };
    int head = 0, cnt = 0;
    auto flush = [&](int take) {
        wave_lds_sync();
        const bool valid = lane < take;
        const uint32_t e = valid ? ring[(head + lane) & (kRing - 1)] : (uint32_t)li;
        const int j = (int)(e & 0xffffu), c = (int)(e >> 16);
        const FewLane r = few_lane(h, fq, st.fx[j]);
        int n[3];
        few_image(r, c, n);
        const double d2 = exact_at_n(M, st.offt, posj, j, q, n, valid);
        bool hit = valid && d2 < rc2;                 // RadiusResultSet: strict
        if (hit && j == li) hit = !(sqrt(d2) < eps);  // self skip (neighbor_list.cpp:47)
        visit(hit, j, n[0], n[1], n[2], d2);
        head = (head + take) & (kRing - 1);
        cnt -= take;
        wave_lds_sync();
    };
    for (int base = 0; base < natoms; base += kWave) {
        const int j = base + lane;
        const bool valid = j < natoms;
        const FewLane r = few_lane(h, fq, st.fx[valid ? j : li]);
        const uint32_t okm = valid ? r.ok : 0u;
        uint32_t bits = 0;  // the lane's combinations at or below hi32
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const bool allowed = few_combo_ok(okm, c);
            if (!ballot(allowed)) continue;
            bits |= (allowed && few_d2(M, r, c) <= hi32) ? 1u << c : 0u;
        }
        // queue them atom-major ((atom, image) order, as the general search visits them: the
        // Betti clouds keep the search order, and the 10 A wide VR kernel took 1,087 ms per
        // 32-structure batch on combination-major clouds, 1,012-1,057 ms on these), at most 64
        // entries per step so the ring never overflows
        const int nb = __builtin_popcount(bits);
        const int incl = wave_inclusive_sum(nb);
        const int total = __builtin_amdgcn_readlane(incl, kWave - 1);
        for (int w0 = 0; w0 < total; w0 += kWave) {
            int idx = incl - nb;
            for (uint32_t bb = bits; bb; bb &= bb - 1, ++idx)
                if (idx >= w0 && idx < w0 + kWave)
                    ring[(head + cnt + idx - w0) & (kRing - 1)] = ((uint32_t)__builtin_ctz(bb) << 16) | (uint32_t)j;
            cnt += total - w0 < kWave ? total - w0 : kWave;
            if (cnt >= kWave) flush(kWave);
        }
    }
    while (cnt > 0) flush(cnt < kWave ? cnt : kWave);
}

// (2) cell list (structures above kStage atoms, one image per axis)
template <class Visit>
__device__ __forceinline__ void search_cells(const GraphLaunch& g, const StructMeta& M, int64_t b, const double q[3],
                                             int li, Visit&& visit) {
    const int lane = lane_id();
    const int nc0 = M.nc[0], nc1 = M.nc[1], nc2 = M.nc[2];
    int lo[3], cw[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const double u = frac_k(M.R, k, q[0], q[1], q[2]);
        const double n = (double)M.nc[k];
        lo[k] = (int)floor((u - M.H[k]) * n);
        cw[k] = (int)floor((u + M.H[k]) * n) - lo[k] + 1;
    }
    const int ncv = cw[0] * cw[1] * cw[2];  // <= 64: each cell is at least H wide
    const int32_t* cs = g.cell_start + M.first + b;
    const double4* cp = g.cell_pos + M.first;
    int start = 0, len = 0, img0 = 0, img1 = 0, img2 = 0;
    if (lane < ncv) {
        const int plane = cw[1] * cw[2];
        const int a = lane / plane, r = lane - a * plane, bb = r / cw[2], c = r - bb * cw[2];
        const int C0 = lo[0] + a, C1 = lo[1] + bb, C2 = lo[2] + c;
        const int w0 = ((C0 % nc0) + nc0) % nc0, w1 = ((C1 % nc1) + nc1) % nc1, w2 = ((C2 % nc2) + nc2) % nc2;
        img0 = (C0 - w0) / nc0;
        img1 = (C1 - w1) / nc1;
        img2 = (C2 - w2) / nc2;
        const int cid = (w0 * nc1 + w1) * nc2 + w2;
        start = cs[cid];
        len = cs[cid + 1] - start;
    }
    const int incl = wave_inclusive_sum(len);
    const int total = __shfl(incl, kWave - 1, kWave);
    const int nref = M.nref;
    for (int t0 = 0; t0 < total; t0 += kWave) {
        const int t = t0 + lane;
        // owning cell: the first lane whose inclusive end exceeds t
        int L = 0;
#pragma unroll
        for (int step = 32; step > 0; step >>= 1) {
            const int probe = __shfl(incl, L + step - 1, kWave);
            L += probe <= t ? step : 0;
        }
        const int cst = __shfl(start, L, kWave), cin = __shfl(incl, L, kWave), cln = __shfl(len, L, kWave);
        const int i0 = __shfl(img0, L, kWave), i1 = __shfl(img1, L, kWave), i2 = __shfl(img2, L, kWave);
        bool hit = false;
        double d2 = 0.0;
        int j = 0, na = 0, nb = 0, nc = 0;
        if (t < total) {
            const double4 rec = cp[cst + (t - (cin - cln))];
            const uint64_t pk = (uint64_t)__double_as_longlong(rec.w);
            j = (int)(uint32_t)pk;
            na = i0 - ((int)((pk >> 32) & 1023) - 512);
            nb = i1 - ((int)((pk >> 42) & 1023) - 512);
            nc = i2 - ((int)((pk >> 52) & 1023) - 512);
            if (abs(na) <= nref && abs(nb) <= nref && abs(nc) <= nref) {
                const double pj[3] = {rec.x, rec.y, rec.z};
                d2 = cand_d2(M, pj, na, nb, nc, q);
                hit = d2 < g.rc2;
                if (hit && j == li) hit = !(sqrt(d2) < g.eps);
            }
        }
        visit(hit, j, na, nb, nc, d2);
    }
}

// (3) general: lane j enumerates every image whose fractional slab can reach rc, clamped to the
// reference's +-nref range, with nested counters (no integer division)
template <class Visit>
__device__ __forceinline__ void search_general(const StructMeta& M, const PosSrc& P, const double q[3], int li,
                                               double rc2, double eps, Visit&& visit) {
    const int lane = lane_id();
    const int natoms = M.natoms;
    for (int base = 0; base < natoms; base += kWave) {
        const int j = base + lane;
        double p[3] = {0.0, 0.0, 0.0};
        int lo[3] = {0, 0, 0}, hi[3] = {-1, -1, -1};
        int ni = 0;
        if (j < natoms) {
            P.get(j, p);
            const double r0 = p[0] - q[0], r1 = p[1] - q[1], r2 = p[2] - q[2];
            ni = 1;
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const double df = r0 * M.R[k] + r1 * M.R[3 + k] + r2 * M.R[6 + k];
                int l = (int)ceil(-df - M.H[k]);
                int h = (int)floor(-df + M.H[k]);
                l = l < -M.nref ? -M.nref : l;
                h = h > M.nref ? M.nref : h;
                lo[k] = l;
                hi[k] = h;
                ni = h >= l ? ni * (h - l + 1) : 0;
            }
        }
        int na = lo[0], nb = lo[1], nc = lo[2];
        for (int t = 0; ballot(t < ni); ++t) {
            bool hit = false;
            double d2 = 0.0;
            const int ca = na, cb = nb, cc = nc;
            if (t < ni) {
                d2 = cand_d2(M, p, ca, cb, cc, q);
                hit = d2 < rc2;
                if (hit && j == li) hit = !(sqrt(d2) < eps);
                if (++nc > hi[2]) {
                    nc = lo[2];
                    if (++nb > hi[1]) {
                        nb = lo[1];
                        ++na;
                    }
                }
            }
            visit(hit, j, ca, cb, cc, d2);
        }
    }
}

// mask: the count pass's exact hits of this query (staged one-image structures), or null = search
template <class Visit>
__device__ __forceinline__ void search(const GraphLaunch& g, const StructMeta& M, int64_t b, const PosSrc& P,
                                       const double q[3], int li, DGN_LDS uint32_t* ring,
                                       const DGN_LDS uint64_t* mask, Visit&& visit) {
    if (M.one && P.staged) {
        if (mask) search_staged_one(M, P.st, q, li, g.rc2, g.eps, ring, load_mask(mask, M.natoms), visit);
        else search_staged_one(M, P.st, q, li, g.rc2, g.eps, ring, ApproxOne{P.st, M, li, g.rc2, !(0.0 < g.eps)}, visit);
    } else if (M.few && P.staged) {
        search_staged_few(M, P.st, q, li, g.rc2, g.eps, ring, visit);
    } else if (M.one && M.cells) {
        search_cells(g, M, b, q, li, visit);
    } else {
        search_general(M, P, q, li, g.rc2, g.eps, visit);
    }
}

// shared memory of every staged search kernel: the stage (dynamic or static), the image-offset
// table and the per-wave candidate rings
#define DGN_SEARCH_SMEM                        \
    __shared__ double4 offt_s[125];            \
    __shared__ uint32_t ring[kW][kRing];

// Hit masks are stored per count tile of qa atoms, word-major ([tile][word][atom], kMaskWords
// words reserved per atom): the tile's stores of word w are qa consecutive u64 (whole lines; an
// atom-major layout wrote each atom's nw <= kMaskWords words as half of a 64-byte sector).
__device__ __forceinline__ int64_t mask_index(int64_t gi, int wd, int qa) {
    const int64_t t0 = gi - gi % qa;  // first atom of gi's tile
    return t0 * kMaskWords + (int64_t)wd * qa + (gi - t0);
}

// ------------------------------------------------------------------------------------------
// Kernel 1: per-atom kept counts + per-block (sum, max candidates, sum (m+1)^2, max structure
// size). No atomics on the data. For staged one-image structures it also records each query's
// exact hits as a bit per atom (word-major per tile, mask_index) so the emit and Betti passes
// skip the search. Two kernels (launch_graph_count):
//   1a graph_count_one_kernel, every tile: tiles whose structures are all staged one-image or
//      few-image ones (cells wider than rc, <= kStage atoms: config 4's FCC-256 at 5 A, config 2's
//      SC-64) are counted here; any other tile is flagged and left alone;
//   1b graph_count_kernel over the flagged tiles (every search strategy).
// 1a stages only the fixed-point coordinates (16 B per atom) and the image-offset table; the rare
// borderline exact test reads positions from global memory. Without the general / cell-list
// search code in the kernel it needs no spills and ~16 KB of LDS, where the combined kernel held
// 96 VGPRs + 12 spilled (0.45 GB of scratch writes per config-4 shard) and 29 KB of LDS.
// ------------------------------------------------------------------------------------------
#ifndef DGN_COUNT_WAVES
#define DGN_COUNT_WAVES 5
#endif
#ifndef DGN_COUNT1_WAVES
#define DGN_COUNT1_WAVES 7
#endif

// the per-wave statistics of one tile, combined and stored with the tile's counts and masks
struct CountTileOut {
    DGN_LDS int32_t* cnt;            // [qa] hits per query
    DGN_LDS int32_t* nw;             // [qa] mask words per query (0: no mask)
    DGN_LDS uint64_t (*mask)[kMaskWords];
    DGN_LDS int64_t* wsum;           // [kW] per-wave sums ...
    DGN_LDS uint64_t *wmax, *wsq, *wnat, *wm, *wwide;
};
struct CountAcc {
    int64_t sum = 0;
    uint32_t max = 0, nat = 0;
    uint64_t sq = 0, m = 0;
    // local complexes of the Betti tiers past the narrow kernels (m + 1 points): 65..kWideRegular
    // in the low word, above kWideRegular in the high word, so the host sizes those launches from
    // the count it already reads back
    uint64_t wide = 0;
    __device__ __forceinline__ void add(int m_, int natoms, uint64_t kmax) {
        wide += m_ + 1 > kWideRegular ? (uint64_t(1) << 32) : (m_ + 1 > 64 ? 1u : 0u);
        sum += (uint64_t)m_ < kmax ? (int64_t)m_ : (int64_t)kmax;
        m += (uint64_t)m_;
        max = (uint32_t)m_ > max ? (uint32_t)m_ : max;
        nat = (uint32_t)natoms > nat ? (uint32_t)natoms : nat;
        sq += (uint64_t)(m_ + 1) * (uint64_t)(m_ + 1);  // local-complex n^2
    }
};
__device__ __forceinline__ void count_tile_store(const GraphLaunch& g, int64_t tile, const CountAcc& acc,
                                                 const CountTileOut& o, int32_t* __restrict__ counts,
                                                 int64_t* __restrict__ block_sums, uint64_t* __restrict__ block_aux,
                                                 uint64_t* __restrict__ mask_out) {
    const int w = threadIdx.x / kWave;
    const int qa = g.qa;
    const int64_t g0 = tile * qa;
    if (lane_id() == 0) {
        o.wsum[w] = acc.sum;
        o.wmax[w] = acc.max;
        o.wsq[w] = acc.sq;
        o.wnat[w] = acc.nat;
        o.wm[w] = acc.m;
        o.wwide[w] = acc.wide;
    }
    __syncthreads();
    const int nq = (int)(g.num_atoms - g0 < qa ? g.num_atoms - g0 : qa);
    for (int i = threadIdx.x; i < nq; i += kGraphBlock) counts[g0 + i] = o.cnt[i];
    if (mask_out)
        for (int x = threadIdx.x; x < nq * kMaskWords; x += kGraphBlock) {
            const int wd = x / nq, a_ = x - wd * nq;  // word-major: consecutive threads, consecutive atoms
            if (wd < o.nw[a_]) mask_out[g0 * kMaskWords + (int64_t)wd * qa + a_] = o.mask[a_][wd];
        }
    if (threadIdx.x == 0) {
        int64_t s = 0;
        uint64_t mx = 0, sq = 0, nat = 0, sm = 0, wd = 0;
        for (int k = 0; k < kW; ++k) {
            s += o.wsum[k];
            wd += o.wwide[k];
            sm += o.wm[k];
            mx = o.wmax[k] > mx ? o.wmax[k] : mx;
            nat = o.wnat[k] > nat ? o.wnat[k] : nat;
            sq += o.wsq[k];
        }
        block_sums[tile] = s;
        block_aux[kAux * tile] = mx;
        block_aux[kAux * tile + 1] = sq;
        block_aux[kAux * tile + 2] = nat;
        block_aux[kAux * tile + 3] = sm;
        block_aux[kAux * tile + 4] = wd;
    }
}

#define DGN_COUNT_SMEM                                                                   \
    __shared__ int32_t cnt_s[kQA], nw_s[kQA]; /* block outputs, written at the end */    \
    __shared__ uint64_t mask_s[kQA][kMaskWords];                                         \
    __shared__ int64_t wsum[kW];                                                         \
    __shared__ uint64_t wmax[kW], wsq[kW], wnat[kW], wm[kW], wwide[kW];                  \
    const CountTileOut out{lds(cnt_s), lds(nw_s), reinterpret_cast<DGN_LDS uint64_t(*)[kMaskWords]>(lds(&mask_s[0][0])), \
                           lds(wsum), lds(wmax), lds(wsq), lds(wnat), lds(wm), lds(wwide)};

__global__ __launch_bounds__(kGraphBlock) __attribute__((amdgpu_waves_per_eu(DGN_COUNT1_WAVES))) void graph_count_one_kernel(
    GraphLaunch g, int32_t* __restrict__ counts, int64_t* __restrict__ block_sums, uint64_t* __restrict__ block_aux,
    uint64_t* __restrict__ mask_out, uint8_t* __restrict__ defer) {
    __shared__ u32x4 fx_s[kStage];
    __shared__ double4 offt_s[125];
    DGN_COUNT_SMEM
    const int lane = lane_id();
    const int64_t tile = blockIdx.x;
    const int64_t g0 = tile * g.qa;
    const int64_t g1 = g0 + g.qa < g.num_atoms ? g0 + g.qa : g.num_atoms;
    // every structure of the tile staged and one-image or few-image? (wave-uniform: metadata in
    // SGPRs)
    bool one = true, all_one = true;
    for (int32_t b = uni_i32(g.atom_struct[g0]), bl = uni_i32(g.atom_struct[g1 - 1]); b <= bl && one; ++b) {
        const StructMeta M = load_meta_uniform(g.meta + b);
        one = M.natoms == 0 || ((M.one || M.few) && M.natoms <= kStage);
        all_one = all_one && (M.natoms == 0 || M.one);
    }
    if (threadIdx.x == 0) defer[tile] = one ? 0 : 1;  // every tile's flag is written: no memset
    if (!one) return;
    // stage view without positions (for_block_atoms<false> stores fx and the offset table only)
    const StageView st{nullptr, nullptr, nullptr, lds(fx_s), reinterpret_cast<DGN_LDS f64x4*>(lds(offt_s)), kStage};
    CountAcc acc;
    // per query atom: M.one -> the one-image count, else the few-image count; the all-one-image
    // tiles (config 4) take a loop of their own, so their code is laid out as without the few path
    auto per_atom = [&](const StructMeta& M, const PosSrc& P, int64_t gi, int t, bool only_one) __attribute__((always_inline)) {
        const int li = (int)(gi - M.first);
        const double* gp = P.gpos;
        auto posj = [&](int jj, double p[3]) __attribute__((always_inline)) {
            p[0] = gp[3 * jj];
            p[1] = gp[3 * jj + 1];
            p[2] = gp[3 * jj + 2];
        };
        int m, nw;
        if (only_one || M.one) {
            m = count_one_image(M, st.fx, st.offt, posj, li, g.rc2, lds(mask_s[t]), 0.0 < g.eps);
            nw = (M.natoms + 63) / 64;
        } else {
            const bool words = M.natoms <= kWave;  // a hit word per image combination (collect_few_hits)
            m = count_few(M, st.fx, st.offt, posj, li, g.rc2, g.eps, words ? lds(mask_s[t]) : nullptr);
            nw = words ? kFewMaskWords : 0;
        }
        if (lane == 0) {
            cnt_s[t] = (int32_t)m;
            nw_s[t] = nw;
        }
        acc.add(m, M.natoms, g.kmax);
    };
    if (all_one)
        for_block_atoms<false>(g, st, 0, g.num_atoms, tile, g.qa, [&](const StructMeta& M, const PosSrc& P, int64_t gi, int t, int64_t)
                                   __attribute__((always_inline)) { per_atom(M, P, gi, t, true); });
    else
        for_block_atoms<false>(g, st, 0, g.num_atoms, tile, g.qa, [&](const StructMeta& M, const PosSrc& P, int64_t gi, int t, int64_t)
                                   __attribute__((always_inline)) { per_atom(M, P, gi, t, false); });
    count_tile_store(g, tile, acc, out, counts, block_sums, block_aux, mask_out);
}

// defer: graph_count_one_kernel's per-tile flags (the grid strides over the tiles: lane k of every
// wave loads the flag of tile blockIdx.x + k * gridDim.x of the current round, the ballot lists the
// block's deferred tiles), or null: tile = blockIdx.x (no 1a pass, e.g. without hit masks)
__global__ __launch_bounds__(kGraphBlock) __attribute__((amdgpu_waves_per_eu(DGN_COUNT_WAVES))) void graph_count_kernel(GraphLaunch g, int32_t* __restrict__ counts,
                                                                   int64_t* __restrict__ block_sums,
                                                                   uint64_t* __restrict__ block_aux,
                                                                   uint64_t* __restrict__ mask_out,
                                                                   const uint8_t* __restrict__ defer) {
    __shared__ double stage_mem[kStage * kStageBytesPerAtom / 8];
    DGN_SEARCH_SMEM
    DGN_COUNT_SMEM
    const StageView st = make_stage(stage_mem, kStage, offt_s);
    const int w = threadIdx.x / kWave;
    const int lane = lane_id();
    auto run_tile = [&](int64_t tile) __attribute__((always_inline)) {
        CountAcc acc;
        for_block_atoms(g, st, 0, g.num_atoms, tile, g.qa, [&](const StructMeta& M, const PosSrc& P, int64_t gi, int t, int64_t b) __attribute__((always_inline)) {
            const int li = (int)(gi - M.first);
            int m = 0, nw = 0;
            if (M.one && P.staged) {
                m = count_staged_one(M, P.st, li, g.rc2, mask_out ? lds(mask_s[t]) : nullptr, 0.0 < g.eps);
                nw = mask_out ? (M.natoms + 63) / 64 : 0;
            } else if (M.few && P.staged) {
                m = count_few(
                    M, P.st.fx, P.st.offt,
                    [&](int jj, double p[3]) __attribute__((always_inline)) {
                        p[0] = P.st.x[jj];
                        p[1] = P.st.y[jj];
                        p[2] = P.st.z[jj];
                    },
                    li, g.rc2, g.eps, (mask_out && M.natoms <= kWave) ? lds(mask_s[t]) : nullptr);
                nw = (mask_out && M.natoms <= kWave) ? kFewMaskWords : 0;
            } else {
                double q[3];
                P.get(li, q);
                search(g, M, b, P, q, li, lds(ring[w]), nullptr,
                       [&](bool hit, int, int, int, int, double) { m += __popcll(ballot(hit)); });
            }
            if (lane == 0) {
                cnt_s[t] = (int32_t)m;  // every hit: the emit keeps min(m, kmax), a Betti pass at this rc reuses m
                nw_s[t] = nw;
            }
            acc.add(m, M.natoms, g.kmax);
        });
        count_tile_store(g, tile, acc, out, counts, block_sums, block_aux, mask_out);
        __syncthreads();  // the next tile reuses the block's LDS outputs
    };
    if (!defer) {
        run_tile(blockIdx.x);
        return;
    }
    const int64_t nt = (g.num_atoms + g.qa - 1) / g.qa, G = gridDim.x;
    for (int64_t base = blockIdx.x; base < nt; base += (int64_t)kWave * G) {
        const int64_t mine = base + (int64_t)lane * G;
        uint64_t bal = ballot(mine < nt && defer[mine] != 0);  // the same in every wave of the block
        while (bal) {
            const int k = __builtin_ctzll(bal);
            bal &= bal - 1;
            run_tile(base + (int64_t)k * G);
        }
    }
}

// ------------------------------------------------------------------------------------------
// Kernel 2: exclusive scan of the per-block sums (one workgroup) -> *total, and the max /
// sum reductions of block_aux -> *max_candidates, *sum_sq.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kScanThreads) void block_scan_kernel(int64_t* __restrict__ v,
                                                                  const uint64_t* __restrict__ aux, int64_t n,
                                                                  int64_t* __restrict__ total,
                                                                  uint32_t* __restrict__ max_candidates,
                                                                  unsigned long long* __restrict__ sum_sq,
                                                                  uint32_t* __restrict__ max_natoms,
                                                                  unsigned long long* __restrict__ sum_m,
                                                                  unsigned long long* __restrict__ wide_atoms) {
    __shared__ int64_t wtot[kScanThreads / kWave];
    __shared__ uint64_t wmx[kScanThreads / kWave], wsq[kScanThreads / kWave], wna[kScanThreads / kWave],
        wsm[kScanThreads / kWave], wwd[kScanThreads / kWave];
    const int tid = threadIdx.x, lane = lane_id(), w = tid / kWave;
    __shared__ int64_t carry_s;
    if (tid == 0) carry_s = 0;
    // reductions of the block aux words: coalesced, independent loads
    uint64_t mx = 0, sq = 0, na = 0, sm = 0, wd = 0;
    for (int64_t i = tid; i < n; i += kScanThreads) {
        mx = aux[kAux * i] > mx ? aux[kAux * i] : mx;
        sq += aux[kAux * i + 1];
        na = aux[kAux * i + 2] > na ? aux[kAux * i + 2] : na;
        sm += aux[kAux * i + 3];
        wd += aux[kAux * i + 4];
    }
    __syncthreads();
    // exclusive scan, 8 consecutive sums per thread (two 32-byte loads per lane: coalesced), 8192
    // per step
    constexpr int kPer = 8;
    typedef int64_t i64x4 __attribute__((ext_vector_type(4)));
    for (int64_t base = 0; base < n; base += (int64_t)kScanThreads * kPer) {
        const int64_t i0 = base + (int64_t)tid * kPer;
        int64_t x[kPer];
        if (i0 + kPer <= n && (((uintptr_t)(v + i0)) & 31) == 0) {
            const i64x4 a = *reinterpret_cast<const i64x4*>(v + i0), b = *reinterpret_cast<const i64x4*>(v + i0 + 4);
            x[0] = a.x, x[1] = a.y, x[2] = a.z, x[3] = a.w, x[4] = b.x, x[5] = b.y, x[6] = b.z, x[7] = b.w;
        } else {
#pragma unroll
            for (int k = 0; k < kPer; ++k) x[k] = i0 + k < n ? v[i0 + k] : 0;
        }
        int64_t tot = 0;
#pragma unroll
        for (int k = 0; k < kPer; ++k) tot += x[k];
        const int64_t inc = wave_inclusive_sum(tot);
        if (lane == kWave - 1) wtot[w] = inc;
        __syncthreads();
        int64_t woff = 0;
        for (int k = 0; k < w; ++k) woff += wtot[k];
        const int64_t carry = carry_s;
        int64_t acc = carry + woff + inc - tot;
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            if (i0 + k < n) v[i0 + k] = acc;
            acc += x[k];
        }
        __syncthreads();
        if (tid == kScanThreads - 1) carry_s = acc;
        __syncthreads();
    }
    if (tid == 0) *total = carry_s;
    mx = wave_max(mx);
    sq = wave_sum(sq);
    na = wave_max(na);
    sm = wave_sum(sm);
    wd = wave_sum(wd);
    if (lane == 0) {
        wmx[w] = mx;
        wsq[w] = sq;
        wna[w] = na;
        wsm[w] = sm;
        wwd[w] = wd;
    }
    __syncthreads();
    if (tid == 0) {
        uint64_t m = 0, s = 0, a = 0, t = 0, x = 0;
        for (int k = 0; k < kScanThreads / kWave; ++k) {
            x += wwd[k];
            m = wmx[k] > m ? wmx[k] : m;
            s += wsq[k];
            a = wna[k] > a ? wna[k] : a;
            t += wsm[k];
        }
        *max_candidates = (uint32_t)m;
        *sum_sq = s;
        *max_natoms = (uint32_t)a;
        *sum_m = t;
        *wide_atoms = x;
    }
}

// ------------------------------------------------------------------------------------------
// Ranking of one atom's compacted hits by (distance, j, image), the canonical row order.
// ------------------------------------------------------------------------------------------
// m <= 64: lane s ranks entry s by counting strictly smaller distances (broadcast LDS reads, one
// f64 compare each; 8 entries per step with the next step's reads in flight; kd[m, round8(m)) must
// hold +inf); exact distance ties collide on a rank, which a claim byte detects, and only then is
// the (j, image) tie-break counted.
typedef double f64x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int rank_small(const DGN_LDS double* kd, const DGN_LDS uint64_t* kj, int m,
                                          DGN_LDS uint8_t* claim) {
    m = uni_i32(m);
    const int lane = lane_id();
    const bool act = lane < m;
    const double me = act ? kd[lane] : 0.0;
    const DGN_LDS f64x2* kv = reinterpret_cast<const DGN_LDS f64x2*>(kd);
    const int m8 = (m + 7) >> 3;
    int r = 0;
    f64x2 c0 = kv[0], c1 = kv[1], c2 = kv[2], c3 = kv[3];
    for (int s = 0; s < m8; ++s) {
        const int nx = s + 1 < m8 ? 4 * (s + 1) : 4 * s;
        const f64x2 n0 = kv[nx], n1 = kv[nx + 1], n2 = kv[nx + 2], n3 = kv[nx + 3];
        r += ((int)(c0.x < me) + (int)(c0.y < me)) + ((int)(c1.x < me) + (int)(c1.y < me)) +
             ((int)(c2.x < me) + (int)(c2.y < me)) + ((int)(c3.x < me) + (int)(c3.y < me));
        c0 = n0;
        c1 = n1;
        c2 = n2;
        c3 = n3;
    }
    if (act) claim[r] = (uint8_t)lane;
    wave_lds_sync();
    const bool lost = act && claim[r] != (uint8_t)lane;
    if (ballot(lost)) {
        const uint64_t mj = act ? kj[lane] : 0ull;
        int extra = 0;
        for (int u = 0; u < m; ++u) extra += (int)((kd[u] == me) & (kj[u] < mj));
        r += extra;
    }
    return r;
}
// m > 64: lane s ranks entries s, s + 64, ... with the full key (broadcast reads; LDS, or the
// global key rows of the large-row emit)
template <class PD, class PJ, class Visit>
__device__ __forceinline__ void rank_large(PD kd, PJ kj, int m, Visit&& visit) {
    for (int s = lane_id(); s < m; s += kWave) {
        const double d = kd[s];
        const uint64_t j = kj[s];
        int rank = 0;
        for (int u = 0; u < m; ++u) {
            const double ud = kd[u];
            const uint64_t uj = kj[u];
            rank += (int)((ud < d) | ((ud == d) & (uj < j)));
        }
        visit(rank, d, j);
    }
}

// ------------------------------------------------------------------------------------------
// RBF values (edge_features.cpp:7-24): g_k(d) = norm * exp(-0.5 (k dr - d)^2 / sigma^2)
// ------------------------------------------------------------------------------------------
// f32 output: t = k dr - d in f64; the exponent x = t^2 * c2 (c2 = -0.5 log2(e) / sigma^2, |x| <=
// 6.5 because |t| <= rc = 3 sigma) in f64, rounded to f32 once (abs error <= 2.4e-7), v_exp_f32
// (1 ulp), times the f32 normaliser: |rel err| < 4.1e-7 against the f64 value.
__device__ __forceinline__ float rbf_f32(double t, const RbfSpec& r) {
    const float x = (float)((t * t) * r.c2);
    return __builtin_amdgcn_exp2f(x) * r.norm_f;
}
__device__ __forceinline__ double rbf_value_f64(double d, int k, const RbfSpec& r) {
    const double center = k * r.dr;  // edge_features.cpp:20
    const double t = center - d;
    return r.norm * exp(-0.5 * (t * t) * r.inv_sigma2);
}

// flat element f of an edge block -> (edge, bin); exact for f < 2^24
__device__ __forceinline__ void rbf_split(int f, const RbfSpec& r, int& e, int& k) {
    e = (int)((float)f * r.inv_nbins);
    if (e * r.nbins > f) --e;
    else if ((e + 1) * r.nbins <= f) ++e;
    k = f - e * r.nbins;
}

// Write the RBF of `total` = edges x nbins flat values starting at `out` from the edge distances
// sd[] with `threads` cooperating threads (thread index tix): scalar head to a 16-byte boundary,
// non-temporal 16-byte body (written once, never re-read here), scalar tail.
template <typename T, class PS>
__device__ __forceinline__ void write_rbf_flat(T* __restrict__ out, int total, PS sd, const RbfSpec& rs, int tix,
                                               int threads) {
    constexpr int V = 16 / sizeof(T);
    const int nb = rs.nbins;
    const int mis = (int)(((uintptr_t)out / sizeof(T)) & (V - 1));
    int head = mis ? V - mis : 0;
    head = head < total ? head : total;
    auto one = [&](int f) -> T {
        int e, k;
        rbf_split(f, rs, e, k);
        if constexpr (sizeof(T) == 4) return rbf_f32((double)k * rs.dr - sd[e], rs);
        else return rbf_value_f64(sd[e], k, rs);
    };
    if (tix < head) out[tix] = one(tix);
    const int nvec = (total - head) / V;
    for (int v = tix; v < nvec; v += threads) {
        const int f = head + V * v;
        int e, k;
        rbf_split(f, rs, e, k);
        if constexpr (sizeof(T) == 4) {
            double d = sd[e];
            double t = (double)k * rs.dr - d;
            float o[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                o[u] = rbf_f32(t, rs);
                if (++k == nb) {
                    k = 0;
                    d = sd[++e];  // sd has one slack entry past the last edge
                    t = -d;
                } else {
                    t += rs.dr;
                }
            }
            typedef float float4_t __attribute__((ext_vector_type(4)));
            const float4_t ov = {o[0], o[1], o[2], o[3]};
            __builtin_nontemporal_store(ov, reinterpret_cast<float4_t*>(out + f));
        } else {
            double o[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                o[u] = rbf_value_f64(sd[e], k, rs);
                if (++k == nb) {
                    k = 0;
                    ++e;
                }
            }
            typedef double double2_t __attribute__((ext_vector_type(2)));
            const double2_t ov = {o[0], o[1]};
            __builtin_nontemporal_store(ov, reinterpret_cast<double2_t*>(out + f));
        }
    }
    const int t0 = head + V * nvec;
    if (t0 + tix < total) out[t0 + tix] = one(t0 + tix);
}

// ------------------------------------------------------------------------------------------
// Block RBF stream (STREAM emit): the block's edges (distances re-read from the just written
// `dist` rows, L2-resident) are processed EP at a time per wave; lane =
// (edge, segment of h bins). With t0 = k0 dr - d the segment start's offset from the centre,
//   g_{k0+i} = norm exp(-0.5 (t0 + i dr)^2 / s^2) = G_i C_i,   G_i = g_{k0} B^i,
//   B = exp(-t0 dr / s^2),   C_i = exp(-0.5 i^2 dr^2 / s^2)  (table),
// G_i runs as an f64 product chain (<= 1e-14 relative for i <= 100). f64 output: G_i C_i in f64.
// f32 output: per pair of bins, g = f32(G_i), (g, g f32(B)) x (C_i, C_{i+1}) as one packed f32
// multiply, G_{i+2} = G_i B^2 in f64: at most 5 f32 roundings, < 3.5e-7 relative, inside the f32
// path's 1e-6. Values go to a per-wave LDS buffer laid out like the output (shifted to the
// output's 16-byte phase) and leave as non-temporal 16-byte stores.
// ------------------------------------------------------------------------------------------
#ifndef DGN_RBF_BUF_BYTES
#define DGN_RBF_BUF_BYTES 4352  // per wave: 21 edges x 50 f32 bins (3 lanes per edge)
#endif
struct RbfStreamGeom {
    int ep, seg, h;  // edges per pass, lanes per edge, bins per lane
};
__host__ __device__ inline RbfStreamGeom rbf_stream_geom(int nb, int elem) {
    // fewest lanes per edge (most edges per exp pair) whose pass fits the buffer
    int sg = 1;
    while (sg < kWave && (kWave / sg) * nb * elem + 16 > DGN_RBF_BUF_BYTES) ++sg;
    int ep = kWave / sg;
    if (ep < 1) ep = 1;
    sg = sg > nb ? nb : sg;
    return {ep, sg, (nb + sg - 1) / sg};
}
__host__ __device__ inline int rbf_stream_buf_bytes(const RbfStreamGeom& gm, int nb, int elem) {
    return ((gm.ep * nb + 16 / elem) * elem + 16 + 15) / 16 * 16;
}
// exp(x) for |x| < 700 (no range checks): x = n ln2 + r, |r| <= ln2 / 2, Taylor polynomial of
// degree DEG in r by Horner with the coefficients 1/k! (DEG 12: < 2e-16 truncation; DEG 8:
// < 6e-9), times 2^n
template <int DEG>
__device__ __forceinline__ double exp_bounded(double x) {
    constexpr double kInvFact[13] = {1.0, 1.0, 1.0 / 2, 1.0 / 6, 1.0 / 24, 1.0 / 120, 1.0 / 720, 1.0 / 5040,
                                     1.0 / 40320, 1.0 / 362880, 1.0 / 3628800, 1.0 / 39916800, 1.0 / 479001600};
    const double n = __builtin_rint(x * 1.4426950408889634);
    double r = __builtin_fma(-n, 6.93147180369123816490e-01, x);
    r = __builtin_fma(-n, 1.90821492927058770002e-10, r);
    double p = kInvFact[DEG];
#pragma unroll
    for (int k = DEG - 1; k >= 0; --k) p = __builtin_fma(p, r, kInvFact[k]);
    return __builtin_ldexp(p, (int)n);
}
template <typename T>
__device__ __forceinline__ void rbf_stream_wave(T* __restrict__ out, int ne, const DGN_LDS double* dl,
                                                const DGN_LDS double* ctab, DGN_LDS T* buf, const RbfSpec& rs,
                                                const RbfStreamGeom gm, int w) {
    constexpr int V = 16 / sizeof(T);
    const int lane = lane_id();
    const int nb = rs.nbins;
    const int le = lane / gm.seg, sgi = lane - le * gm.seg;
    const int k0 = sgi * gm.h;
    const int cnt0 = nb - k0 < gm.h ? nb - k0 : gm.h;
    const DGN_LDS f32x2* ctf = reinterpret_cast<const DGN_LDS f32x2*>(ctab + gm.h + 1);  // f32 (C_i, C_i+1)
    for (int e = w * gm.ep; e < ne; e += kW * gm.ep) {
        const int nedge = ne - e < gm.ep ? ne - e : gm.ep;
        T* o = out + (int64_t)e * nb;
        const int phase = (int)(((uintptr_t)o / sizeof(T)) & (V - 1));  // o - phase is 16-byte aligned
        const double d = le < nedge ? dl[e + le] : 0.0;
        if (le < nedge && cnt0 > 0) {
            const double t0 = (double)k0 * rs.dr - d;
            const double s = rs.inv_sigma2;
            DGN_LDS T* dst = buf + phase + le * nb + k0;
            if constexpr (sizeof(T) == 8) {
                double G = rs.norm * exp_bounded<12>(-0.5 * (t0 * t0) * s);
                const double B = exp_bounded<12>(-(t0 * rs.dr) * s);
                for (int i = 0; i < cnt0; ++i) {
                    dst[i] = G * ctab[i];
                    G *= B;
                }
            } else {
                double G = rs.norm * exp_bounded<8>(-0.5 * (t0 * t0) * s);
                const double B = exp_bounded<8>(-(t0 * rs.dr) * s);
                const double B2 = B * B;
                const float bf = (float)B;
                int i = 0;
                auto pair = [&](int at, const f32x2 c) __attribute__((always_inline)) {
                    const float g = (float)G;
                    const f32x2 gg = {g, g * bf};
                    const f32x2 v = gg * c;
                    dst[at] = v.x;
                    dst[at + 1] = v.y;
                    G *= B2;
                };
                for (; i + 8 <= cnt0; i += 8) {  // the table reads of 4 pairs in flight together
                    const f32x2 c0 = ctf[(i >> 1)], c1 = ctf[(i >> 1) + 1], c2 = ctf[(i >> 1) + 2],
                                c3 = ctf[(i >> 1) + 3];
                    pair(i, c0);
                    pair(i + 2, c1);
                    pair(i + 4, c2);
                    pair(i + 6, c3);
                }
                for (; i + 2 <= cnt0; i += 2) {
                    const float g = (float)G;
                    const f32x2 gg = {g, g * bf};
                    const f32x2 v = gg * ctf[i >> 1];
                    dst[i] = v.x;
                    dst[i + 1] = v.y;
                    G *= B2;
                }
                if (i < cnt0) dst[i] = (float)G * ctf[i >> 1].x;
            }
        }
        wave_lds_sync();
        // stream buf[phase, phase + nedge * nb) -> o[0, nedge * nb): lanes cover 16-byte units;
        // whole units [1 or 0, nfull) without checks, the partial head / tail unit element-wise
        const int total = nedge * nb + phase;  // in units of T from the aligned base o - phase
        const int v0 = phase ? 1 : 0, nfull = total / V;
        typedef T vec_t __attribute__((ext_vector_type(V)));
        T* ob = o - phase;
        for (int v = v0 + lane; v < nfull; v += kWave) {
            const vec_t val = *reinterpret_cast<const DGN_LDS vec_t*>(buf + V * v);
            // f32: non-temporal 16-byte stores; f64 (the reference's edge_attr dtype, twice the
            // bytes): plain stores, which the L2 merges into full lines -- measured on the fused
            // emit, config-4 shard: f64 4.01 -> 3.46 ms with plain stores, f32 2.23 -> 2.37 ms
            // (worse) with them (tools/r03_graph_exp.sh)
            constexpr bool plain = sizeof(T) == 8;
            if constexpr (plain) *reinterpret_cast<vec_t*>(ob + V * v) = val;
            else __builtin_nontemporal_store(val, reinterpret_cast<vec_t*>(ob + V * v));
        }
        if (lane < V) {
            const int fh = lane, ft = V * nfull + lane;  // head unit 0 (phase > 0), tail unit nfull
            if (phase && fh >= phase && fh < total) ob[fh] = buf[fh];
            if (ft < total && ft >= phase) ob[ft] = buf[ft];
        }
        wave_lds_sync();
    }
}

// The tile's RBF block as flat 16-byte units, one per thread per step (all kGraphBlock threads,
// consecutive threads -> consecutive units): element f of the block is (edge f / nb, bin f % nb);
// d[] (LDS) holds the block's distances with one slack entry past the last edge.
template <typename T>
__device__ __forceinline__ void rbf_direct(T* __restrict__ out, int total, const DGN_LDS double* d, const RbfSpec& rs) {
    constexpr int V = 16 / sizeof(T);
    const int nb = rs.nbins;
    const int mis = (int)(((uintptr_t)out / sizeof(T)) & (V - 1));
    int head = mis ? V - mis : 0;
    head = head < total ? head : total;
    auto one = [&](int f) -> T {
        int e, k;
        rbf_split(f, rs, e, k);
        const double t = (double)k * rs.dr - d[e];
        if constexpr (sizeof(T) == 4) return rbf_f32(t, rs);
        else return rs.norm * exp_bounded<12>(-0.5 * (t * t) * rs.inv_sigma2);
    };
    const int tix = threadIdx.x;
    if (tix < head) out[tix] = one(tix);
    const int nvec = (total - head) / V;
    typedef T vec_t __attribute__((ext_vector_type(V)));
    for (int v = tix; v < nvec; v += kGraphBlock) {
        const int f = head + V * v;
        int e, k;
        rbf_split(f, rs, e, k);
        double de = d[e];
        double t = (double)k * rs.dr - de;
        vec_t o;
#pragma unroll
        for (int u = 0; u < V; ++u) {
            // f64: t = k dr - d afresh per value (edge_features.cpp:20-21); f32: t steps by dr
            if constexpr (sizeof(T) == 4) o[u] = rbf_f32(t, rs);
            else o[u] = rs.norm * exp_bounded<12>(-0.5 * (t * t) * rs.inv_sigma2);
            if (++k == nb) {
                k = 0;
                de = d[++e];  // d has one slack entry past the last edge
            }
            if constexpr (sizeof(T) == 4) t = k ? t + rs.dr : -de;
            else t = (double)k * rs.dr - de;
        }
        __builtin_nontemporal_store(o, reinterpret_cast<vec_t*>(out + f));
    }
    const int t0 = head + V * nvec;
    if (t0 + tix < total) out[t0 + tix] = one(t0 + tix);
}

// ------------------------------------------------------------------------------------------
// Kernel 3: fused emit. Per atom (one wave): compact the hits (the count pass's mask, or a search)
// into LDS, rank, write the kept rows (col, distance, displacement). STREAM (max_neighbors <=
// kStreamMaxK): after the block's atoms, its whole RBF region (contiguous in the CSR) is written
// by the 4 waves from the block's distance rows, through per-wave LDS buffers as 16-byte
// non-temporal stores; otherwise each wave writes its atom's RBF rows (write_rbf_flat).
// `dist` must be non-null when STREAM writes an RBF (the host passes a scratch row buffer).
// ------------------------------------------------------------------------------------------
// Dynamic LDS of the emit (bytes): region A (search phase: stage, hit lists, hit masks, sorted
// distances) is dead once the block's atoms are placed and is reused as region B (the per-wave
// RBF buffers); then the tile's kept distances and the RBF C table, which live to the end.
struct EmitLayout {
    int stage, keyd, keyj, mask, sorted, dl, rbf, ctab, total;
    RbfStreamGeom gm;
    int wbytes;
};
__host__ __device__ inline EmitLayout emit_layout(int stage_cap, int cap, bool stream, int K, int nb, int elem,
                                                  int nwm) {
    EmitLayout l{};
    int o = 0;
    auto take = [&](int bytes) {
        const int at = o;
        o += (bytes + 15) / 16 * 16;
        return at;
    };
    l.stage = take(stage_cap * kStageBytesPerAtom);
    l.keyd = take(kW * cap * 8);
    l.keyj = take(kW * cap * 8);
    l.mask = take(kQA * nwm * 8);
    l.sorted = take(stream || cap == 0 ? 0 : kW * (cap + 1) * 8);
    const int a_end = o;
    l.gm = rbf_stream_geom(nb > 0 ? nb : 1, elem > 0 ? elem : 4);
    l.wbytes = (stream && nb > 0) ? rbf_stream_buf_bytes(l.gm, nb, elem > 0 ? elem : 4) : 0;
    // region B: the per-wave RBF buffers; then (live throughout) the tile's kept distances, which
    // the rows phase leaves in LDS so the RBF phase issues no global load (a load issued after a
    // wave's stores waits for them)
    l.rbf = 0;
    const int b_end = kW * l.wbytes;
    o = a_end > b_end ? a_end : (b_end + 15) / 16 * 16;
    l.dl = take((stream && nb > 0) ? (kQA * K + 1) * 8 : 0);
    l.ctab = take(stream ? (l.gm.h + 1) * 8 + (l.gm.h + 2) * 4 : 0);  // f64 C_i, then f32 C_i
    l.total = o;
    return l;
}

// the tiles (kQA atoms) of one emit launch: row tiles [row0, row0 + nrow) and RBF tiles
// [rbf0, rbf0 + nrbf) whose rows an earlier launch wrote; fused: each row block streams its own
// RBF after its rows (one launch, nrbf = 0)
struct EmitTiles {
    int64_t row0, nrow, rbf0, nrbf;
    int fused;
};

// CAP = 0 (kEmitGlobalKeys, rows of more candidates than the LDS instantiations hold): each wave's
// hit list, keys and sorted distances live in its own global row, [3 cap + 1] doubles at
// base + (block of the launch * kW + wave) * (3 cap + 1); the host launches the tiles in chunks so
// the rows stay bounded
struct EmitKeys {
    double* base;
    int32_t cap;
    int32_t chunk;  // tiles per launch (host side; 0 = emit_key_chunk_tiles)
};

template <int CAP, bool STREAM>
__global__ __launch_bounds__(kGraphBlock) void graph_emit_kernel(GraphLaunch g, int stage_cap, int nwm,
                                                                  const int32_t* __restrict__ counts,
                                                                  const int64_t* __restrict__ block_offsets,
                                                                  int64_t* __restrict__ row_ptr,
                                                                  int32_t* __restrict__ col, double* __restrict__ dist,
                                                                  double* __restrict__ disp, void* __restrict__ rbf,
                                                                  RbfSpec rs, uint32_t* __restrict__ error_flag,
                                                                  EmitTiles tl, EmitKeys gk) {
    constexpr bool GK = CAP == 0;
    extern __shared__ double dyn[];
    __shared__ uint32_t ring[kW][kRing];
    __shared__ uint8_t claim[kW][kWave];
    __shared__ int64_t row_start[kQA + 1];
    const int K = g.kmax < (uint64_t)0x7fffffff ? (int)g.kmax : 0x7fffffff;
    const int elem = rs.dtype == 2 ? 8 : 4;
    const EmitLayout ly = emit_layout(stage_cap, CAP, STREAM, K, rs.dtype ? rs.nbins : 0, elem, nwm);
    DGN_LDS uint8_t* base = reinterpret_cast<DGN_LDS uint8_t*>(lds(dyn));
    const StageView st = make_stage(reinterpret_cast<double*>(dyn) + ly.stage / 8, stage_cap, nullptr);
    DGN_LDS double* dl = reinterpret_cast<DGN_LDS double*>(base + ly.dl);
    DGN_LDS uint64_t* mask_s = reinterpret_cast<DGN_LDS uint64_t*>(base + ly.mask);
    DGN_LDS double* ctab = reinterpret_cast<DGN_LDS double*>(base + ly.ctab);
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / kWave));
    const int lane = lane_id();
    const int cap = GK ? gk.cap : CAP;
    using PD = std::conditional_t<GK, double*, DGN_LDS double*>;
    using PJ = std::conditional_t<GK, uint64_t*, DGN_LDS uint64_t*>;
    PD kd, sd;
    PJ kj;
    // lane-to-lane hand-off through the key rows: LDS (wave order), or global (the agent-scope
    // fence waits for the wave's stores and invalidates the CU's L1 before the reads)
    auto key_rows_sync = [&]() __attribute__((always_inline)) {
        if constexpr (GK) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
        else wave_lds_sync();
    };
    if constexpr (GK) {
        double* r = gk.base + ((int64_t)blockIdx.x * kW + w) * (3 * (int64_t)gk.cap + 1);
        kd = r;
        kj = reinterpret_cast<uint64_t*>(r + gk.cap);
        sd = r + 2 * (int64_t)gk.cap;
    } else {
        kd = reinterpret_cast<DGN_LDS double*>(base + ly.keyd) + w * CAP;
        kj = reinterpret_cast<DGN_LDS uint64_t*>(base + ly.keyj) + w * CAP;
        sd = reinterpret_cast<DGN_LDS double*>(base + ly.sorted) + w * (CAP + 1);
    }
    // this block's job: row tiles and RBF tiles alternate in the grid (every CU gets both)
    const int64_t both = tl.nrow < tl.nrbf ? tl.nrow : tl.nrbf;
    const int64_t x = blockIdx.x;
    const bool is_rbf = x < 2 * both ? (x & 1) != 0 : tl.nrbf > tl.nrow;
    const int64_t tile = (is_rbf ? tl.rbf0 : tl.row0) + (x < 2 * both ? x >> 1 : x - both);
    const int qa = g.qa;
    const int64_t g0 = tile * qa;
    const int nq = (int)(g.num_atoms - g0 < qa ? g.num_atoms - g0 : qa);
    // the RBF of this tile from its rows (row_ptr, dist), by the block's 4 waves; region A must be dead
    auto rbf_tile = [&](bool rows_in_lds) __attribute__((always_inline)) {
        for (int i = threadIdx.x; i <= ly.gm.h + 1; i += kGraphBlock) {
            const double xx = (double)i * rs.dr;
            const double c = exp(-0.5 * (xx * xx) * rs.inv_sigma2);  // C_i
            if (i <= ly.gm.h) ctab[i] = c;
            reinterpret_cast<DGN_LDS float*>(ctab + ly.gm.h + 1)[i] = (float)c;
        }
        __syncthreads();
        // the tile's own rows only: row_ptr[g0 + nq] belongs to the next tile, whose rows may be
        // written by this same launch
        const int64_t e0 = row_ptr[g0], e1 = row_ptr[g0 + nq - 1] + min(counts[g0 + nq - 1], K);
        const int ne = (int)(e1 - e0);
        if (!rows_in_lds) {  // RBF tile of an earlier launch's rows
            for (int i = threadIdx.x; i < ne; i += kGraphBlock) dl[i] = dist[e0 + i];
            __syncthreads();
        }
        if (rs.dtype == 1)
            rbf_stream_wave(reinterpret_cast<float*>(rbf) + e0 * rs.nbins, ne, dl, ctab,
                            reinterpret_cast<DGN_LDS float*>(base + ly.rbf + w * ly.wbytes), rs, ly.gm, w);
        else
            rbf_stream_wave(reinterpret_cast<double*>(rbf) + e0 * rs.nbins, ne, dl, ctab,
                            reinterpret_cast<DGN_LDS double*>(base + ly.rbf + w * ly.wbytes), rs, ly.gm, w);
    };
    if constexpr (STREAM) {
        if (is_rbf) {
            rbf_tile(false);
            return;
        }
    }

    // local scan of this block's counts -> row starts (and row_ptr); qa <= kQA == one wave
    if (w == 0) {
        const int64_t gi = g0 + lane;
        const bool mine = lane < qa && gi < g.num_atoms;
        const int64_t c = mine ? min(counts[gi], K) : 0;  // kept rows: min(m, max_neighbors)
        const int64_t inc = wave_inclusive_sum(c);
        const int64_t start = block_offsets[tile] + inc - c;
        row_start[lane] = start;
        if (lane == kWave - 1) row_start[kQA] = start + c;
        if (mine) {
            row_ptr[gi] = start;
            if (gi == g.num_atoms - 1) row_ptr[g.num_atoms] = start + c;
        }
    }
    // the count pass's hit masks of the block's atoms (staged one-image structures)
    if (g.mask)
        for (int x = threadIdx.x; x < nq * nwm; x += kGraphBlock) {
            const int wd = x / nq, a_ = x - wd * nq;  // coalesced: consecutive threads, consecutive atoms
            mask_s[a_ * nwm + wd] = g.mask[mask_index(g0 + a_, wd, qa)];
        }
    __syncthreads();
    for_block_atoms(g, st, 0, g.num_atoms, tile, qa, [&](const StructMeta& M, const PosSrc& P, int64_t gi, int t, int64_t b)
                                               __attribute__((always_inline)) {
        const int li = (int)(gi - M.first);
        double q[3];
        P.get(li, q);
        // 1. compact the hits into the wave's LDS list (staged one-image structures: only the
        // count pass's hits are evaluated)
        int m = 0;
        bool fast = false;
        // (`few` structures of <= 64 atoms: a hit word per image combination, collect_few_hits)
        const bool few_mask = M.few && M.natoms <= kWave && nwm >= kFewMaskWords;
        const DGN_LDS uint64_t* mk = (g.mask && (M.one || few_mask) && P.staged) ? mask_s + t * nwm : nullptr;
        if (mk) {
            // fast path: at most 64 hits, one lane each, straight from the count pass's mask
            const int mh = M.one ? collect_mask_hits(mk, M.natoms, lds(ring[w])) : collect_few_hits(mk, lds(ring[w]));
            if (mh <= kWave) {
                fast = true;
                m = mh;
                bool ok = true;
                if (lane < m) {
                    const uint32_t e = ring[w][lane];
                    const int j = (int)(e & 0xffffu);
                    int n[3];
                    bool inr = true;
                    double d2;
                    if (M.one) {
                        d2 = exact_one(M, P.st, P.st.fx[li], P.st.fx[j], j, q, n, inr);
                    } else {
                        float h[3];
                        few_halfwidths(M, h);
                        few_image(few_lane(h, P.st.fx[li], P.st.fx[j]), (int)(e >> 16), n);
                        d2 = exact_at_n(
                            M, P.st.offt,
                            [&](int jj, double p[3]) __attribute__((always_inline)) { P.get(jj, p); }, j, q, n, true);
                    }
                    ok = inr && d2 < g.rc2;
                    kd[lane] = sqrt(d2);  // neighbor_list.cpp:53
                    kj[lane] = pack_jimg(j, n[0], n[1], n[2]);
                }
                if (ballot(!ok)) {
                    if (lane == 0) atomicOr(error_flag, kGErrMissedHit);
                    return;
                }
            }
        }
        if (!fast)
            search(g, M, b, P, q, li, lds(ring[w]), mk, [&](bool hit, int j, int na, int nb, int nc, double d2) {
                const uint64_t bal = ballot(hit);
                if (hit) {
                    const int slot = m + mask_prefix(bal);
                    if (slot < cap) {
                        kd[slot] = sqrt(d2);  // neighbor_list.cpp:53
                        kj[slot] = pack_jimg(j, na, nb, nc);
                    }
                }
                m += __popcll(bal);
            });
        const int64_t rs0 = row_start[t];
        const int kept = (int)(row_start[t + 1] - rs0);
        if (m > cap || kept != (m < K ? m : K)) {
            if (lane == 0) atomicOr(error_flag, m > cap ? kGErrCap : kGErrMismatch);
            return;
        }
        key_rows_sync();
        // 2. rank by (distance, j, image) and place the kept rows
        auto put = [&](int rank, double d, uint64_t key) __attribute__((always_inline)) {
            if (rank >= kept) return;
            const int64_t e = rs0 + rank;
            int j, na, nb, nc;
            unpack_jimg(key, j, na, nb, nc);
            if constexpr (STREAM) dl[e - row_start[0]] = d;
            else sd[rank] = d;
            col[e] = j;
            if (dist) dist[e] = d;
            if (disp) {
                double pj[3];
                P.get(j, pj);
                for (int k = 0; k < 3; ++k) {
                    const double off = ((double)na * M.L[k] + (double)nb * M.L[3 + k]) + (double)nc * M.L[6 + k];
                    disp[3 * e + k] = (pj[k] + off) - q[k];  // delta_r = p - q (neighbor_list.cpp:51)
                }
            }
        };
        if (!GK && m <= kWave) {
            if constexpr (!GK) {
                if (lane >= m && lane < ((m + 7) & ~7)) kd[lane] = __builtin_inf();  // rank_small reads groups of 8
                wave_lds_sync();
                const int r = rank_small(kd, kj, m, lds(claim[w]));
                if (lane < m) put(r, kd[lane], kj[lane]);
            }
        } else {
            rank_large(kd, kj, m, put);
        }
        key_rows_sync();
        if constexpr (!STREAM) {
            // 3. this atom's RBF rows: kept x nbins contiguous values from rs0 * nbins
            if (rs.dtype != 0 && rbf) {
                const int total = kept * rs.nbins;
                if (rs.dtype == 1)
                    write_rbf_flat(reinterpret_cast<float*>(rbf) + rs0 * rs.nbins, total, sd, rs, lane, kWave);
                else
                    write_rbf_flat(reinterpret_cast<double*>(rbf) + rs0 * rs.nbins, total, sd, rs, lane, kWave);
            }
            key_rows_sync();
        }
    });
    if constexpr (STREAM) {
        if (tl.fused) {
            __syncthreads();  // the block's rows are in dl; region A is dead
            rbf_tile(true);
        }
    }
}

// ------------------------------------------------------------------------------------------
// Betti distance pass with its own neighbour search: complex c = atom `first + c`, cloud row 0 =
// pos_i, row k = pos_i + disp_k over every neighbour within rc (betti_features.cpp:67-73 with
// NeighborList(rc, SIZE_MAX), :107). The persistence diagram and the 35 statistics do not depend
// on the order of the cloud's rows (every distance depends only on its two points; the pairing
// values of a filtration do not depend on its tie-breaking order), so the rows keep the search's
// order instead of the sorted one. Writes the f32 lower triangle (the reference's Gram arithmetic,
// gram_triangle_*) + npoints.
// ------------------------------------------------------------------------------------------
// The Betti search + distance kernel (f64 VALU pairs for n <= 64, matrix-core tiles above) writes ~1 KB of triangle per complex with little reuse:
// compiled for 4 waves per SIMD (128 VGPRs, a few spills) it keeps more stores in flight than at
// its natural 161 VGPRs (3 waves): 7.6 -> 5.9 ms per config-4 shard (tools/ab_dist.sh)
// (the 64-point instantiation; the wide ones are LDS-bound anyway). A 256-thread block is one wave
// per SIMD, so DGN_DIST_WPE blocks per CU = DGN_DIST_WPE waves per SIMD.
#ifndef DGN_DIST_WPE
#define DGN_DIST_WPE 4
#endif
template <int CAP>
__global__ __launch_bounds__(kGraphBlock, CAP <= kWave ? DGN_DIST_WPE : 1) void betti_dist_search_kernel(GraphLaunch g, int64_t first, int64_t count,
                                                                         int64_t tri_stride,
                                                                         const int32_t* __restrict__ counts,
                                                                         float* __restrict__ lower,
                                                                         int32_t* __restrict__ npoints,
                                                                         uint32_t* __restrict__ error_flag,
                                                                         uint64_t* __restrict__ keys_out,
                                                                         int key_stride) {
    __shared__ double stage_mem[kStage * kStageBytesPerAtom / 8];
    DGN_SEARCH_SMEM
    // per wave: the neighbour keys (CAP u64), then the wide triangle's squared norms (CAP + 1);
    // the narrow triangle's point records (4 x 64 doubles) overlay both once the cloud is built
    constexpr int kWaveDoubles = 2 * CAP + 1 > 4 * kWave ? 2 * CAP + 1 : 4 * kWave;
    __shared__ double cloud_s[kW][kWaveDoubles];
    __shared__ uint64_t mask_s[kQA][kMaskWords];
    const StageView st = make_stage(stage_mem, kStage, offt_s);
    const int w = threadIdx.x / kWave;
    const int lane = lane_id();
    uint64_t* key_j = reinterpret_cast<uint64_t*>(cloud_s[w]);
    const int64_t g0 = first + (int64_t)blockIdx.x * kQA;
    const int nq = (int)(first + count - g0 < kQA ? first + count - g0 : kQA);
    if (g.mask) {
        for (int x = threadIdx.x; x < nq * kMaskWords; x += kGraphBlock) {
            const int wd = x / nq, a_ = x - wd * nq;
            mask_s[a_][wd] = g.mask[mask_index(g0 + a_, wd, g.qa)];
        }
        __syncthreads();
    }
    for_block_atoms(g, st, first, first + count, blockIdx.x, kQA, [&](const StructMeta& M, const PosSrc& P, int64_t gi, int, int64_t b) __attribute__((always_inline)) {
        const int li = (int)(gi - M.first);
        const int64_t c = gi - first;
        double q[3];
        P.get(li, q);
        int m = 0;
        bool fast = false;
        const DGN_LDS uint64_t* mk = (g.mask && M.one && P.staged) ? lds(mask_s[gi - g0]) : nullptr;
        if (mk) {
            // at most 63 hits: the count pass's mask, the images from the fixed-point coordinates
            const int mh = collect_mask_hits(mk, M.natoms, lds(ring[w]));
            if (mh < kWave) {
                fast = true;
                m = mh;
                bool ok = true;
                if (lane < m) {
                    const int j = (int)ring[w][lane];
                    int n[3];
                    bool inr;
                    const double d2 = exact_one(M, P.st, P.st.fx[li], P.st.fx[j], j, q, n, inr);
                    ok = inr && d2 < g.rc2;
                    key_j[lane] = pack_jimg(j, n[0], n[1], n[2]);
                }
                if (ballot(!ok)) {
                    if (lane == 0) atomicOr(error_flag, kGErrMismatch);
                    return;
                }
            }
        }
        if (!fast)
            search(g, M, b, P, q, li, lds(ring[w]), mk, [&](bool hit, int j, int na, int nb, int nc, double) {
                const uint64_t bal = ballot(hit);
                if (hit) {
                    const int slot = m + mask_prefix(bal);
                    if (slot < CAP) key_j[slot] = pack_jimg(j, na, nb, nc);
                }
                m += __popcll(bal);
            });
        const int n = m + 1;
        if (lane == 0) npoints[c] = n;
        if (m > CAP || m != counts[gi]) {
            if (lane == 0) atomicOr(error_flag, m > CAP ? kGErrCap : kGErrMismatch);
            return;
        }
        wave_lds_sync();
        if (keys_out)  // diagnostics (dgn_debug_betti_clouds): cloud row p >= 1 is (j, image) key p - 1
            for (int p = lane; p < m && p < key_stride; p += kWave) keys_out[c * key_stride + p] = key_j[p];
        // cloud row p: p = 0 the centre, else centre + ((p_j + offset) - centre)
        auto point = [&](int p, double x[3]) __attribute__((always_inline)) {
            if (p == 0) {
                x[0] = q[0];
                x[1] = q[1];
                x[2] = q[2];
                return;
            }
            int j, na, nb, nc;
            unpack_jimg(key_j[p - 1], j, na, nb, nc);
            double pj[3];
            P.get(j, pj);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const double off = ((double)na * M.L[k] + (double)nb * M.L[3 + k]) + (double)nc * M.L[6 + k];
                x[k] = q[k] + ((pj[k] + off) - q[k]);  // betti_features.cpp:71: pos_i + disp_k
            }
        };
        float* L = lower + c * tri_stride;
        if (n <= kWave) {
            double px[3];
            point(lane < n ? lane : n - 1, px);
            gram_triangle_narrow(px, n, cloud_s[w], L, tri_stride);
        } else {
            gram_triangle_wide(n, cloud_s[w] + CAP, L, point, tri_stride);
        }
    });
}

hipError_t launch_betti_dist_search(hipStream_t s, const GraphLaunch& g, int64_t first, int64_t count, int max_points,
                                    int64_t tri_stride, const int32_t* counts, float* lower, int32_t* npoints,
                                    uint32_t* error_flag, uint64_t* keys_out, int key_stride) {
    if (count <= 0) return hipSuccess;
    const int64_t nb = graph_blocks(count);
    if (max_points <= kWave)
        hipLaunchKernelGGL(betti_dist_search_kernel<kWave>, dim3((unsigned)nb), dim3(kGraphBlock), 0, s, g, first,
                           count, tri_stride, counts, lower, npoints, error_flag, keys_out, key_stride);
    else if (max_points <= kWideRegular)
        hipLaunchKernelGGL(betti_dist_search_kernel<kWideRegular>, dim3((unsigned)nb), dim3(kGraphBlock), 0, s, g,
                           first, count, tri_stride, counts, lower, npoints, error_flag, keys_out, key_stride);
    else
        hipLaunchKernelGGL(betti_dist_search_kernel<kWideMaxPoints>, dim3((unsigned)nb), dim3(kGraphBlock), 0, s, g,
                           first, count, tri_stride, counts, lower, npoints, error_flag, keys_out, key_stride);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// RBF of caller-given distances (CrystalGraph edge_attr), flat over the output so stores are
// coalesced in either layout: layout 0 row-major [E][nb], layout 1 column-major (k*E + e).
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void rbf_kernel(const double* __restrict__ d, int64_t E, RbfSpec rs, int layout,
                                                  void* __restrict__ out) {
    const int64_t total = E * rs.nbins;
    for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < total; f += (int64_t)gridDim.x * blockDim.x) {
        int64_t e;
        int k;
        if (layout == 0) {
            e = f / rs.nbins;
            k = (int)(f - e * rs.nbins);
        } else {
            k = (int)(f / E);
            e = f - (int64_t)k * E;
        }
        if (rs.dtype == 1) reinterpret_cast<float*>(out)[f] = rbf_f32((double)k * rs.dr - d[e], rs);
        else reinterpret_cast<double*>(out)[f] = rbf_value_f64(d[e], k, rs);
    }
}

hipError_t launch_rbf(hipStream_t s, const double* d, int64_t E, const RbfSpec& rs, int layout, void* out) {
    const int64_t total = E * rs.nbins;
    if (total <= 0) return hipSuccess;
    int64_t blocks = (total + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(rbf_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d, E, rs, layout, out);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------
hipError_t launch_prep_structures(hipStream_t s, const double* lattice, const int64_t* atom_offset, const double* pos,
                                  const int32_t* species, int64_t B, double rc, StructMeta* meta, int32_t* atom_struct,
                                  int32_t* cell_start, double4* cell_pos, double* weight, uint32_t* error_flag) {
    if (B <= 0) return hipSuccess;
    hipLaunchKernelGGL(prep_meta_kernel, dim3((unsigned)((B + 127) / 128)), dim3(128), 0, s, lattice, atom_offset, B,
                       rc, meta);
    // block per structure; small batches (a few large cells, e.g. BASELINE config 5's supercell)
    // get 1024 threads per block for the cell-list sort
    const unsigned threads = B < 512 ? 1024u : 256u;
    hipLaunchKernelGGL(prep_atoms_kernel, dim3((unsigned)B), dim3(threads), 0, s, meta, pos, species, atom_struct,
                       cell_start, cell_pos, weight, error_flag);
    return hipGetLastError();
}

hipError_t launch_graph_count(hipStream_t s, const GraphLaunch& g, int32_t* counts, int64_t* block_sums,
                              uint64_t* block_aux, uint64_t* mask_out, uint8_t* defer) {
    const int64_t nb = graph_blocks(g.num_atoms, g.qa);
    if (nb <= 0) return hipSuccess;
    if (!mask_out || !defer) {
        hipLaunchKernelGGL(graph_count_kernel, dim3((unsigned)nb), dim3(kGraphBlock), 0, s, g, counts, block_sums,
                           block_aux, mask_out, (const uint8_t*)nullptr);
        return hipGetLastError();
    }
    // 1a over every tile, then 1b over the tiles 1a flagged (a fixed grid strides over the flags,
    // so a launch with nothing deferred costs one short launch and no host read)
    hipLaunchKernelGGL(graph_count_one_kernel, dim3((unsigned)nb), dim3(kGraphBlock), 0, s, g, counts, block_sums,
                       block_aux, mask_out, defer);
    const unsigned grid = (unsigned)(nb < kCountListGrid ? nb : kCountListGrid);
    hipLaunchKernelGGL(graph_count_kernel, dim3(grid), dim3(kGraphBlock), 0, s, g, counts, block_sums, block_aux,
                       mask_out, (const uint8_t*)defer);
    return hipGetLastError();
}

hipError_t launch_block_scan(hipStream_t s, int64_t* v, const uint64_t* aux, int64_t n, int64_t* total,
                             uint32_t* max_candidates, unsigned long long* sum_sq, uint32_t* max_natoms,
                             unsigned long long* sum_m, unsigned long long* wide_atoms) {
    hipLaunchKernelGGL(block_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, v, aux, n, total, max_candidates,
                       sum_sq, max_natoms, sum_m, wide_atoms);
    return hipGetLastError();
}

int graph_emit_cap(uint32_t m, uint64_t kmax) {
    if (m <= 64) return 64;
    if (m <= 128) return 128;
    if (m <= 256) return 256;
    if (m <= 512) return 512;
    if (m <= 1024) return 1024;
    // 1,025..2,048 candidates (cutoffs up to ~20 A at FCC density) with max_neighbors <=
    // kStreamMaxK: the streamed emit (no per-wave sorted-distance buffer) still fits the LDS
    if (m <= 2048 && kmax <= (uint64_t)kStreamMaxK) return 2048;
    return kEmitGlobalKeys;  // larger rows: key rows in global memory (emit_key_row_doubles)
}

int64_t emit_key_row_doubles(uint32_t m) { return 3 * (int64_t)((m + 63) / 64 * 64) + 1; }
// a chunk's key rows take at most kEmitGkChunkBytes whatever max_candidates is (at least one tile)
int64_t emit_key_chunk_tiles(uint32_t m) {
    const int64_t tile_bytes = emit_key_row_doubles(m) * (int64_t)sizeof(double) * kW;
    return std::max<int64_t>(1, std::min<int64_t>(kEmitGkChunkBlocks, kEmitGkChunkBytes / tile_bytes));
}
int64_t emit_key_rows_per_chunk(uint32_t m) { return emit_key_chunk_tiles(m) * kW; }

template <int CAP, bool STREAM>
static void launch_emit_t(hipStream_t s, const GraphLaunch& g, int stage, const int32_t* counts,
                          const int64_t* block_offsets, int64_t* row_ptr, int32_t* col, double* dist, double* disp,
                          void* rbf, const RbfSpec& rs, uint32_t* error_flag, EmitKeys gk) {
    const int64_t nt = graph_blocks(g.num_atoms, g.qa);
    // mask words per atom staged by the emit: the atom tiles of the largest structure, and at least
    // kFewMaskWords when every structure has <= 64 atoms (a `few` structure's combination words)
    const int nwm = stage <= kWave ? kFewMaskWords : (stage + 63) / 64;
    const int K = g.kmax < (uint64_t)0x7fffffff ? (int)g.kmax : 0x7fffffff;
    const EmitLayout ly = emit_layout(stage, CAP, STREAM, K, rs.dtype ? rs.nbins : 0, rs.dtype == 2 ? 8 : 4, nwm);
    const int fused = STREAM && rs.dtype != 0 && rbf ? 1 : 0;
    auto go = [&](EmitTiles tl) {
        const int64_t blocks = tl.nrow + tl.nrbf;
        if (blocks > 0)
            hipLaunchKernelGGL((graph_emit_kernel<CAP, STREAM>), dim3((unsigned)blocks), dim3(kGraphBlock),
                               (size_t)ly.total, s, g, stage, nwm, counts, block_offsets, row_ptr, col, dist, disp, rbf,
                               rs, error_flag, tl, gk);
    };
    if (CAP == 0) {
        // global key rows: one row per wave of a chunk of emit_key_chunk_tiles tiles, launched in turn
        const int64_t chunk = gk.chunk > 0 ? std::min<int64_t>(gk.chunk, emit_key_chunk_tiles((uint32_t)gk.cap))
                                           : emit_key_chunk_tiles((uint32_t)gk.cap);
        for (int64_t t0 = 0; t0 < nt; t0 += chunk) go({t0, std::min<int64_t>(chunk, nt - t0), 0, 0, fused});
        return;
    }
    // one launch, each block writes its rows, then its tile's RBF (round 3 A/B: all rows then all
    // RBF in two launches, and a chunk pipeline overlapping rows of chunk i with the RBF of chunk
    // i - 1, were both slower: RBF-only blocks stream at ~4 TB/s and take slots from row blocks)
    go({0, nt, 0, 0, fused});
}

hipError_t launch_graph_emit(hipStream_t s, const GraphLaunch& g, int cap, int stage, const int32_t* counts,
                             const int64_t* block_offsets, int64_t* row_ptr, int32_t* col, double* dist,
                             double* disp, void* rbf, const RbfSpec& rs, uint32_t* error_flag, double* key_rows,
                             uint32_t max_candidates, int chunk_tiles) {
    const int64_t nb = graph_blocks(g.num_atoms, g.qa);
    if (nb <= 0) return hipSuccess;
    const bool stream = g.kmax <= (uint64_t)kStreamMaxK;
    EmitKeys gk{nullptr, 0, 0};
#define DGN_EMIT(C)                                                                                              \
    case C:                                                                                                      \
        if (stream) launch_emit_t<C, true>(s, g, stage, counts, block_offsets, row_ptr, col, dist, disp, rbf, rs, \
                                           error_flag, gk);                                                      \
        else launch_emit_t<C, false>(s, g, stage, counts, block_offsets, row_ptr, col, dist, disp, rbf, rs,      \
                                     error_flag, gk);                                                            \
        break;
    switch (cap) {
        DGN_EMIT(64)
        DGN_EMIT(128)
        DGN_EMIT(256)
        DGN_EMIT(512)
        DGN_EMIT(1024)
        case 2048:  // streamed emit only (graph_emit_cap)
            if (!stream) return hipErrorInvalidValue;
            launch_emit_t<2048, true>(s, g, stage, counts, block_offsets, row_ptr, col, dist, disp, rbf, rs, error_flag,
                                      gk);
            break;
        case kEmitGlobalKeys:
            if (!key_rows) return hipErrorInvalidValue;
            gk = {key_rows, (int32_t)((emit_key_row_doubles(max_candidates) - 1) / 3), chunk_tiles};
            if (stream) launch_emit_t<0, true>(s, g, stage, counts, block_offsets, row_ptr, col, dist, disp, rbf, rs,
                                               error_flag, gk);
            else launch_emit_t<0, false>(s, g, stage, counts, block_offsets, row_ptr, col, dist, disp, rbf, rs,
                                         error_flag, gk);
            break;
        default:
            return hipErrorInvalidValue;
    }
#undef DGN_EMIT
    return hipGetLastError();
}

}  // namespace dgn

