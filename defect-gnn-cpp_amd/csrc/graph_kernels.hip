// graph_kernels.hip — periodic fixed-radius neighbour search, CSR compaction and Gaussian-RBF
// edge features for gfx950.
//
// Replaces src/graph/neighbor_list.cpp:27-94 (nanoflann KD-tree over a (2n+1)^3 image cloud),
// src/graph/edge_features.cpp:7-24 and the edge loop of src/graph/crystal_graph.cpp:32-40.
//
// Design (MI355X-first):
//   * one wave64 per query atom; lane j owns structure atom j of the current 64-atom tile and
//     enumerates ONLY the periodic images whose fractional slab can reach rc (<= 27 for cells
//     wider than rc, vs the reference's fixed 125), clamped to the reference's own image range
//     so the candidate set is exactly the reference's;
//   * the membership test reproduces the reference arithmetic bit for bit (offset
//     ((na*a + nb*b) + nc*c), p = pos + offset, d2 = ((dx^2 + dy^2) + dz^2), strict d2 < rc^2,
//     self-skip sqrt(d2) < eps) — compiled with -ffp-contract=off;
//   * hits are compacted with ballot + mbcnt into an LDS candidate list, ranked by
//     (distance, j, image) with broadcast LDS reads, truncated to max_neighbors, and written
//     to the CSR slot row_ptr[i] + rank;
//   * the RBF block of an atom (cnt x n_rbf values) is contiguous in HBM and written by the
//     whole wave in flat, coalesced order; exp is range-reduced in f64 and finished with
//     v_exp_f32 for the f32 output (|rel err| < 3e-7), or computed in f64 for the f64 output.
//   * three launches: count (+ per-block sums), block-sum scan, emit (recomputes its rows and
//     scans its 16 atoms locally). No spin waits.
#include "dgn_internal.hpp"

namespace dgn {

// ------------------------------------------------------------------------------------------
// Structure metadata + atom -> structure map
// ------------------------------------------------------------------------------------------
__global__ void prep_structures_kernel(const double* __restrict__ lattice, const int64_t* __restrict__ atom_offset,
                                       int64_t B, double rc, StructMeta* __restrict__ meta) {
    const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    StructMeta m;
    const double* L = lattice + 9 * b;
    for (int k = 0; k < 9; ++k) m.L[k] = L[k];
    const double a00 = L[0], a01 = L[1], a02 = L[2], a10 = L[3], a11 = L[4], a12 = L[5], a20 = L[6],
                 a21 = L[7], a22 = L[8];
    const double c00 = a11 * a22 - a12 * a21, c01 = a02 * a21 - a01 * a22, c02 = a01 * a12 - a02 * a11;
    const double c10 = a12 * a20 - a10 * a22, c11 = a00 * a22 - a02 * a20, c12 = a02 * a10 - a00 * a12;
    const double c20 = a10 * a21 - a11 * a20, c21 = a01 * a20 - a00 * a21, c22 = a00 * a11 - a01 * a10;
    const double det = a00 * c00 + a01 * c10 + a02 * c20;
    const double id = 1.0 / det;
    m.R[0] = c00 * id; m.R[1] = c01 * id; m.R[2] = c02 * id;
    m.R[3] = c10 * id; m.R[4] = c11 * id; m.R[5] = c12 * id;
    m.R[6] = c20 * id; m.R[7] = c21 * id; m.R[8] = c22 * id;
    for (int k = 0; k < 3; ++k)
        m.h[k] = rc * sqrt(m.R[k] * m.R[k] + m.R[3 + k] * m.R[3 + k] + m.R[6 + k] * m.R[6 + k]);
    // Eigen Matrix3d row norm: x0 + (x1 + x2) (fixed-size unrolled redux), neighbor_list.cpp:69
    double lmin = 1e300;
    for (int r = 0; r < 3; ++r) {
        const double* v = L + 3 * r;
        lmin = fmin(lmin, sqrt(v[0] * v[0] + (v[1] * v[1] + v[2] * v[2])));
    }
    m.nref = (int32_t)ceil(rc / lmin) + 1;
    m.first = atom_offset[b];
    m.natoms = (int32_t)(atom_offset[b + 1] - atom_offset[b]);
    meta[b] = m;
}

// one block per structure: atom_struct[first .. first + natoms) = b
__global__ __launch_bounds__(256) void map_atoms_kernel(const int64_t* __restrict__ atom_offset,
                                                        int32_t* __restrict__ atom_struct) {
    const int64_t b = blockIdx.x;
    const int64_t a0 = atom_offset[b], a1 = atom_offset[b + 1];
    for (int64_t a = a0 + threadIdx.x; a < a1; a += blockDim.x) atom_struct[a] = (int32_t)b;
}

// ------------------------------------------------------------------------------------------
// Block traversal shared by count and emit: a block owns query atoms [g0, g0 + kQA); it walks
// the structures those atoms belong to, stages each structure's positions in LDS (SoA, when it
// has at most kStage atoms; larger ones are read from global/L2), and hands every query atom
// to one wave (atoms round-robin over the 4 waves).
// ------------------------------------------------------------------------------------------
struct StagedPos {
    double x[kStage], y[kStage], z[kStage];
};

struct PosSrc {
    const StagedPos* lds;     // null -> global
    const double* gpos;       // positions of the structure's first atom
    __device__ __forceinline__ void get(int j, double p[3]) const {
        if (lds) {
            p[0] = lds->x[j];
            p[1] = lds->y[j];
            p[2] = lds->z[j];
        } else {
            p[0] = gpos[3 * j];
            p[1] = gpos[3 * j + 1];
            p[2] = gpos[3 * j + 2];
        }
    }
};

__device__ __forceinline__ int32_t uni_i32(int32_t x) { return __builtin_amdgcn_readfirstlane(x); }

template <class PerAtom>
__device__ __forceinline__ void for_block_atoms(const GraphLaunch& g, StagedPos& st, PerAtom&& per_atom) {
    const int w = threadIdx.x / kWave;
    const int64_t g0 = (int64_t)blockIdx.x * kQA;
    const int64_t g1 = g0 + kQA < g.num_atoms ? g0 + kQA : g.num_atoms;
    const int32_t b_first = uni_i32(g.atom_struct[g0]);
    const int32_t b_last = uni_i32(g.atom_struct[g1 - 1]);
    for (int32_t b = b_first; b <= b_last; ++b) {
        const StructMeta& M = g.meta[b];
        const int64_t first = M.first;
        const int natoms = M.natoms;
        if (natoms == 0) continue;
        const bool staged = natoms <= kStage;
        if (staged) {
            __syncthreads();  // previous segment done with the stage
            const double* src = g.pos + 3 * first;
            for (int t = threadIdx.x; t < natoms; t += kGraphBlock) {
                st.x[t] = src[3 * t];
                st.y[t] = src[3 * t + 1];
                st.z[t] = src[3 * t + 2];
            }
            __syncthreads();
        }
        const PosSrc P{staged ? &st : nullptr, g.pos + 3 * first};
        const int64_t s0 = g0 > first ? g0 : first;
        const int64_t s1 = g1 < first + natoms ? g1 : first + natoms;
        for (int64_t gi = s0 + w; gi < s1; gi += kGraphBlock / kWave) per_atom(M, P, gi, (int)(gi - g0));
    }
}

// ------------------------------------------------------------------------------------------
// Candidate enumeration: all (j, image) with d2 < rc^2 around query atom q (wave-uniform call).
// Lane j enumerates only the images whose fractional slab can reach rc, clamped to the
// reference's +-nref range, with nested counters (no integer division).
// visit(hit, j, na, nb, nc, d) is invoked by every lane once per step (hit false = idle).
// ------------------------------------------------------------------------------------------
template <class Visit>
__device__ __forceinline__ void for_each_candidate(const StructMeta& M, const PosSrc& P, const double q[3], int li,
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
                int l = (int)ceil(-df - M.h[k] - 1e-9);
                int h = (int)floor(-df + M.h[k] + 1e-9);
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
            double d = 0.0;
            const int ca = na, cb = nb, cc = nc;
            if (t < ni) {
                const double dna = (double)ca, dnb = (double)cb, dnc = (double)cc;
                double d2 = 0.0;
#pragma unroll
                for (int k = 0; k < 3; ++k) {
                    // offset = (na*a + nb*b) + nc*c (neighbor_list.cpp:82-84); p = pos + offset (:87)
                    const double off = (dna * M.L[k] + dnb * M.L[3 + k]) + dnc * M.L[6 + k];
                    const double diff = q[k] - (p[k] + off);  // L2_Simple_Adaptor: (a - b)^2 accumulated
                    d2 += diff * diff;
                }
                if (d2 < rc2) {  // RadiusResultSet: strict
                    d = sqrt(d2);
                    hit = !(j == li && d < eps);  // self skip (neighbor_list.cpp:47)
                }
                if (++nc > hi[2]) {
                    nc = lo[2];
                    if (++nb > hi[1]) {
                        nb = lo[1];
                        ++na;
                    }
                }
            }
            visit(hit, j, ca, cb, cc, d);
        }
    }
}

__device__ __forceinline__ uint64_t pack_jimg(int j, int na, int nb, int nc) {
    return ((uint64_t)(uint32_t)j << 24) | ((uint64_t)((na + 128) & 255) << 16) |
           ((uint64_t)((nb + 128) & 255) << 8) | (uint64_t)((nc + 128) & 255);
}

// ------------------------------------------------------------------------------------------
// Ranking of one atom's compacted candidates by (distance, j, image) — the canonical row order
// (the reference's nanoflann order differs only among exact ties). Lane s ranks entry s by
// counting smaller keys (broadcast LDS reads); visit(rank, kd, kj) for every entry.
// ------------------------------------------------------------------------------------------
template <class Visit>
__device__ __forceinline__ void rank_candidates(const uint64_t* kd_, const uint64_t* kj_, int m, Visit&& visit) {
    for (int s = lane_id(); s < m; s += kWave) {
        const uint64_t kd = kd_[s], kj = kj_[s];
        int rank = 0;
        for (int u = 0; u < m; ++u) {
            const uint64_t ud = kd_[u], uj = kj_[u];
            rank += (ud < kd) | ((ud == kd) & (uj < kj));
        }
        visit(rank, kd, kj);
    }
}

// ------------------------------------------------------------------------------------------
// Kernel 1: per-atom kept counts + per-block (sum, max candidates, sum (m+1)^2). No atomics.
// ROWS: also rank each atom's candidates and store its kept rows (distance bits, packed
// j/image) at rows[gi * K + rank], K = max_neighbors <= kRowsMaxK, so the emit pass only
// streams; atoms with more than kRowsCap candidates set the block's overflow bit instead.
// ------------------------------------------------------------------------------------------
template <bool ROWS>
__global__ __launch_bounds__(kGraphBlock) void graph_count_kernel(GraphLaunch g, int32_t* __restrict__ counts,
                                                                   int64_t* __restrict__ block_sums,
                                                                   uint64_t* __restrict__ block_aux,
                                                                   uint64_t* __restrict__ rows_d,
                                                                   uint64_t* __restrict__ rows_j) {
    constexpr int W = kGraphBlock / kWave;
    constexpr int CAP = ROWS ? kRowsCap : 1;
    __shared__ StagedPos st;
    __shared__ int64_t wsum[W];
    __shared__ uint64_t wmax[W], wsq[W];
    __shared__ uint64_t key_d[W][CAP];
    __shared__ uint64_t key_j[W][CAP];
    const int w = threadIdx.x / kWave;
    const int lane = lane_id();
    int64_t my_sum = 0;
    uint32_t my_max = 0;
    uint64_t my_sq = 0;
    for_block_atoms(g, st, [&](const StructMeta& M, const PosSrc& P, int64_t gi, int) {
        const int li = (int)(gi - M.first);
        double q[3];
        P.get(li, q);
        int m = 0;
        if constexpr (ROWS) {
            for_each_candidate(M, P, q, li, g.rc2, g.eps, [&](bool hit, int j, int na, int nb, int nc, double d) {
                const uint64_t bal = ballot(hit);
                if (hit) {
                    const int slot = m + mask_prefix(bal);
                    if (slot < CAP) {
                        key_d[w][slot] = f64_bits(d);
                        key_j[w][slot] = pack_jimg(j, na, nb, nc);
                    }
                }
                m += __popcll(bal);
            });
        } else {
            for_each_candidate(M, P, q, li, g.rc2, g.eps,
                               [&](bool hit, int, int, int, int, double) { m += __popcll(ballot(hit)); });
        }
        const int64_t c = (uint64_t)m < g.kmax ? (int64_t)m : (int64_t)g.kmax;
        if (lane == 0) counts[gi] = (int32_t)c;
        if constexpr (ROWS) {
            if (m <= CAP) {
                __builtin_amdgcn_wave_barrier();
                const int64_t base = gi * (int64_t)g.kmax;
                rank_candidates(key_d[w], key_j[w], m, [&](int rank, uint64_t kd, uint64_t kj) {
                    if (rank < c) {
                        rows_d[base + rank] = kd;
                        rows_j[base + rank] = kj;
                    }
                });
                __builtin_amdgcn_wave_barrier();
            }
        }
        my_sum += c;
        my_max = (uint32_t)m > my_max ? (uint32_t)m : my_max;
        my_sq += (uint64_t)(m + 1) * (uint64_t)(m + 1);  // local-complex n^2
    });
    if (lane == 0) {
        wsum[w] = my_sum;
        wmax[w] = my_max;
        wsq[w] = my_sq;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int64_t s = 0;
        uint64_t mx = 0, sq = 0;
        for (int k = 0; k < W; ++k) {
            s += wsum[k];
            mx = wmax[k] > mx ? wmax[k] : mx;
            sq += wsq[k];
        }
        block_sums[blockIdx.x] = s;
        block_aux[2 * blockIdx.x] = mx;
        block_aux[2 * blockIdx.x + 1] = sq;
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
                                                                  unsigned long long* __restrict__ sum_sq) {
    __shared__ int64_t wtot[kScanThreads / kWave];
    __shared__ uint64_t wmx[kScanThreads / kWave], wsq[kScanThreads / kWave];
    __shared__ int64_t carry_s;
    const int tid = threadIdx.x, lane = lane_id(), w = tid / kWave;
    if (tid == 0) carry_s = 0;
    uint64_t mx = 0, sq = 0;
    __syncthreads();
    for (int64_t base = 0; base < n; base += kScanThreads) {
        const int64_t i = base + tid;
        const int64_t x = i < n ? v[i] : 0;
        if (i < n) {
            mx = aux[2 * i] > mx ? aux[2 * i] : mx;
            sq += aux[2 * i + 1];
        }
        const int64_t inc = wave_inclusive_sum(x);
        if (lane == kWave - 1) wtot[w] = inc;
        __syncthreads();
        int64_t woff = 0;
        for (int k = 0; k < w; ++k) woff += wtot[k];
        const int64_t carry = carry_s;
        if (i < n) v[i] = carry + woff + inc - x;
        __syncthreads();
        if (tid == kScanThreads - 1) carry_s = carry + woff + inc;
        __syncthreads();
    }
    mx = wave_max(mx);
    sq = wave_sum(sq);
    if (lane == 0) {
        wmx[w] = mx;
        wsq[w] = sq;
    }
    __syncthreads();
    if (tid == 0) {
        *total = carry_s;
        uint64_t m = 0, s = 0;
        for (int k = 0; k < kScanThreads / kWave; ++k) {
            m = wmx[k] > m ? wmx[k] : m;
            s += wsq[k];
        }
        *max_candidates = (uint32_t)m;
        *sum_sq = s;
    }
}

// ------------------------------------------------------------------------------------------
// Kernel 3: emit CSR rows + edge features.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float rbf_value_f32(double d, int k, const RbfSpec& r) {
    const double center = k * r.dr;  // edge_features.cpp:20
    const double t = center - d;
    const double arg = -0.5 * (t * t) * r.inv_sigma2;  // -0.5 * pow(c - d, 2) * inv_sigma_squared
    const double x = arg * 1.4426950408889634074;      // log2(e)
    const double n = rint(x);
    const float e = __builtin_amdgcn_exp2f((float)(x - n));  // |x - n| <= 0.5
    return (float)(r.norm * ldexp((double)e, (int)n));
}
__device__ __forceinline__ double rbf_value_f64(double d, int k, const RbfSpec& r) {
    const double center = k * r.dr;
    const double t = center - d;
    return r.norm * exp(-0.5 * (t * t) * r.inv_sigma2);
}

// flat element f of an atom's RBF block -> (edge, bin); exact for f < 2^24
__device__ __forceinline__ void rbf_split(int f, const RbfSpec& r, int& e, int& k) {
    e = (int)((float)f * r.inv_nbins);
    if (e * r.nbins > f) --e;
    else if ((e + 1) * r.nbins <= f) ++e;
    k = f - e * r.nbins;
}

// write the kept x nbins RBF block of one atom: scalar head to a 16-byte boundary, 16-byte
// vector body, scalar tail (all lanes of the wave, coalesced)
template <typename T>
__device__ __forceinline__ void write_rbf_block(T* __restrict__ out, int total, const double* sd, const RbfSpec& rs) {
    constexpr int V = 16 / sizeof(T);
    const int lane = lane_id();
    const int mis = (int)(((uintptr_t)out / sizeof(T)) & (V - 1));
    int head = mis ? V - mis : 0;
    head = head < total ? head : total;
    auto val = [&](int f) -> T {
        int e, k;
        rbf_split(f, rs, e, k);
        if constexpr (sizeof(T) == 4) return rbf_value_f32(sd[e], k, rs);
        else return rbf_value_f64(sd[e], k, rs);
    };
    if (lane < head) out[lane] = val(lane);
    const int nvec = (total - head) / V;
    for (int v = lane; v < nvec; v += kWave) {
        const int f = head + V * v;
        if constexpr (sizeof(T) == 4) {
            float4 o;
            o.x = val(f);
            o.y = val(f + 1);
            o.z = val(f + 2);
            o.w = val(f + 3);
            *reinterpret_cast<float4*>(out + f) = o;
        } else {
            double2 o;
            o.x = val(f);
            o.y = val(f + 1);
            *reinterpret_cast<double2*>(out + f) = o;
        }
    }
    const int tail0 = head + V * nvec;
    if (tail0 + lane < total) out[tail0 + lane] = val(tail0 + lane);
}

template <int CAP>
__global__ __launch_bounds__(kGraphBlock) void graph_emit_kernel(GraphLaunch g, const int32_t* __restrict__ counts,
                                                                  const int64_t* __restrict__ block_offsets,
                                                                  int64_t* __restrict__ row_ptr,
                                                                  int32_t* __restrict__ col, double* __restrict__ dist,
                                                                  double* __restrict__ disp, void* __restrict__ rbf,
                                                                  RbfSpec rs, uint32_t* __restrict__ error_flag) {
    constexpr int W = kGraphBlock / kWave;
    __shared__ StagedPos st;
    __shared__ uint64_t key_d[W][CAP];
    __shared__ uint64_t key_j[W][CAP];
    __shared__ double sorted_d[W][CAP];
    __shared__ int64_t row_start[kQA];
    const int w = threadIdx.x / kWave;
    const int lane = lane_id();
    const int64_t g0 = (int64_t)blockIdx.x * kQA;

    // local scan of this block's counts -> row starts (and row_ptr); kQA == one wave
    if (w == 0) {
        const int64_t gi = g0 + lane;
        const int64_t c = gi < g.num_atoms ? counts[gi] : 0;
        const int64_t inc = wave_inclusive_sum(c);
        const int64_t start = block_offsets[blockIdx.x] + inc - c;
        row_start[lane] = start;
        if (gi < g.num_atoms) {
            row_ptr[gi] = start;
            if (gi == g.num_atoms - 1) row_ptr[g.num_atoms] = start + c;
        }
    }
    __syncthreads();
    for_block_atoms(g, st, [&](const StructMeta& M, const PosSrc& P, int64_t gi, int t) {
        const int li = (int)(gi - M.first);
        double q[3];
        P.get(li, q);
        // 1. compact hits into the wave's LDS candidate list
        int m = 0;
        for_each_candidate(M, P, q, li, g.rc2, g.eps, [&](bool hit, int j, int na, int nb, int nc, double d) {
            const uint64_t bal = ballot(hit);
            if (hit) {
                const int slot = m + mask_prefix(bal);
                if (slot < CAP) {
                    key_d[w][slot] = f64_bits(d);
                    key_j[w][slot] = pack_jimg(j, na, nb, nc);
                }
            }
            m += __popcll(bal);
        });
        const int cnt = counts[gi];
        const int64_t rs0 = row_start[t];
        const int kept = (uint64_t)m < g.kmax ? m : (int)g.kmax;
        if (m > CAP || kept != cnt) {
            if (lane == 0) atomicOr(error_flag, m > CAP ? 1u : 2u);
            return;
        }
        __builtin_amdgcn_wave_barrier();
        // 2. rank by (distance, j, image) and write the kept rows
        rank_candidates(key_d[w], key_j[w], m, [&](int rank, uint64_t kd, uint64_t kj) {
            if (rank < kept) {
                const int64_t e = rs0 + rank;
                const int j = (int)(kj >> 24);
                const double d = __longlong_as_double((long long)kd);
                col[e] = j;
                if (dist) dist[e] = d;
                sorted_d[w][rank] = d;
                if (disp) {
                    const int na = (int)((kj >> 16) & 255) - 128, nb = (int)((kj >> 8) & 255) - 128,
                              nc = (int)(kj & 255) - 128;
                    double pj[3];
                    P.get(j, pj);
                    for (int k = 0; k < 3; ++k) {
                        const double off = ((double)na * M.L[k] + (double)nb * M.L[3 + k]) + (double)nc * M.L[6 + k];
                        disp[3 * e + k] = (pj[k] + off) - q[k];  // delta_r = p - q (neighbor_list.cpp:51)
                    }
                }
            }
        });
        __builtin_amdgcn_wave_barrier();
        // 3. RBF block: kept x nbins contiguous values starting at rs0 * nbins
        if (rs.dtype != 0 && rbf) {
            const int total = kept * rs.nbins;
            if (rs.dtype == 1) write_rbf_block(reinterpret_cast<float*>(rbf) + rs0 * rs.nbins, total, sorted_d[w], rs);
            else write_rbf_block(reinterpret_cast<double*>(rbf) + rs0 * rs.nbins, total, sorted_d[w], rs);
        }
        __builtin_amdgcn_wave_barrier();
    });
}

// ------------------------------------------------------------------------------------------
// Kernel 3b: streaming emit from the rows the count pass stored (ROWS mode). A block covers
// kQA atoms, whose edges and RBF rows are contiguous in the CSR: phase 1 places the kept rows
// (col, dist, displacement) edge-parallel and keeps the distances in LDS; phase 2 writes the
// block's whole RBF region as one flat stream of 16-byte stores.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ float rbf_value_f32_fast(double d, int k, const RbfSpec& r) {
    const double t = (double)k * r.dr - d;  // center - distance (edge_features.cpp:20-21)
    const double x = ((-0.5 * (t * t)) * r.inv_sigma2) * 1.4426950408889634074;
    const double n = rint(x);
    const float e = __builtin_amdgcn_exp2f((float)(x - n));  // |x - n| <= 0.5
    return __builtin_ldexpf(e, (int)n) * r.norm_f;
}

__global__ __launch_bounds__(kGraphBlock) void graph_emit_rows_kernel(
    GraphLaunch g, const int32_t* __restrict__ counts, const int64_t* __restrict__ block_offsets,
    const uint64_t* __restrict__ rows_d, const uint64_t* __restrict__ rows_j, int64_t* __restrict__ row_ptr,
    int32_t* __restrict__ col, double* __restrict__ dist, double* __restrict__ disp, void* __restrict__ rbf,
    RbfSpec rs) {
    extern __shared__ double dl[];  // [kQA * K] distances of the block's edges, CSR order
    __shared__ int64_t row_start[kQA + 1];
    __shared__ int32_t cnt[kQA];
    const int tid = threadIdx.x, lane = lane_id();
    const int64_t g0 = (int64_t)blockIdx.x * kQA;
    const int K = (int)g.kmax;
    if (tid < kWave) {
        const int64_t gi = g0 + lane;
        const int64_t c = gi < g.num_atoms ? counts[gi] : 0;
        const int64_t inc = wave_inclusive_sum(c);
        const int64_t start = block_offsets[blockIdx.x] + inc - c;
        row_start[lane] = start;
        cnt[lane] = (int32_t)c;
        if (lane == kWave - 1) row_start[kQA] = start + c;
        if (gi < g.num_atoms) {
            row_ptr[gi] = start;
            if (gi == g.num_atoms - 1) row_ptr[g.num_atoms] = start + c;
        }
    }
    __syncthreads();
    const int64_t e0 = row_start[0];
    // phase 1: slot p = (atom a, rank r), r < K; stored rows are read in order (coalesced)
    const float invK = 1.0f / (float)K;
    for (int p = tid; p < kQA * K; p += kGraphBlock) {
        int a = (int)((float)p * invK);
        if (a * K > p) --a;
        else if ((a + 1) * K <= p) ++a;
        const int r = p - a * K;
        const int64_t gi = g0 + a;
        if (gi >= g.num_atoms || r >= cnt[a]) continue;
        const uint64_t kd = rows_d[gi * K + r], kj = rows_j[gi * K + r];
        const int64_t e = row_start[a] + r;
        const double d = __longlong_as_double((long long)kd);
        const int j = (int)(kj >> 24);
        col[e] = j;
        if (dist) dist[e] = d;
        dl[e - e0] = d;
        if (disp) {
            const StructMeta& M = g.meta[g.atom_struct[gi]];
            const int na = (int)((kj >> 16) & 255) - 128, nb = (int)((kj >> 8) & 255) - 128, nc = (int)(kj & 255) - 128;
            const double* pj = g.pos + 3 * (M.first + j);
            const double* q = g.pos + 3 * gi;
            for (int k = 0; k < 3; ++k) {
                const double off = ((double)na * M.L[k] + (double)nb * M.L[3 + k]) + (double)nc * M.L[6 + k];
                disp[3 * e + k] = (pj[k] + off) - q[k];  // delta_r = p - q (neighbor_list.cpp:51)
            }
        }
    }
    if (rs.dtype == 0 || !rbf) return;
    __syncthreads();
    // phase 2: the block's RBF region [e0 * nb, e1 * nb) as one flat stream
    const int nb = rs.nbins;
    const int total = (int)(row_start[kQA] - e0) * nb;
    auto split = [&](int f, int& le, int& k) {
        le = (int)((float)f * rs.inv_nbins);
        if (le * nb > f) --le;
        else if ((le + 1) * nb <= f) ++le;
        k = f - le * nb;
    };
    if (rs.dtype == 1) {
        float* out = reinterpret_cast<float*>(rbf) + e0 * nb;
        const int mis = (int)(((uintptr_t)out >> 2) & 3);
        int head = mis ? 4 - mis : 0;
        head = head < total ? head : total;
        if (tid < head) {
            int le, k;
            split(tid, le, k);
            out[tid] = rbf_value_f32_fast(dl[le], k, rs);
        }
        const int nvec = (total - head) >> 2;
        for (int v = tid; v < nvec; v += kGraphBlock) {
            const int f = head + 4 * v;
            int le, k;
            split(f, le, k);
            float o[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                o[u] = rbf_value_f32_fast(dl[le], k, rs);
                if (++k == nb) {
                    k = 0;
                    ++le;
                }
            }
            // streaming (non-temporal) 16-byte store: the RBF block is written once, never re-read here
            typedef float float4_t __attribute__((ext_vector_type(4)));
            const float4_t ov = {o[0], o[1], o[2], o[3]};
            __builtin_nontemporal_store(ov, reinterpret_cast<float4_t*>(out + f));
        }
        const int t0 = head + 4 * nvec;
        if (t0 + tid < total) {
            int le, k;
            split(t0 + tid, le, k);
            out[t0 + tid] = rbf_value_f32_fast(dl[le], k, rs);
        }
    } else {
        double* out = reinterpret_cast<double*>(rbf) + e0 * nb;
        const int head = ((((uintptr_t)out >> 3) & 1) && total > 0) ? 1 : 0;
        if (tid < head) out[0] = rbf_value_f64(dl[0], 0, rs);
        const int nvec = (total - head) >> 1;
        for (int v = tid; v < nvec; v += kGraphBlock) {
            const int f = head + 2 * v;
            int le, k;
            split(f, le, k);
            double o[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                o[u] = rbf_value_f64(dl[le], k, rs);
                if (++k == nb) {
                    k = 0;
                    ++le;
                }
            }
            typedef double double2_t __attribute__((ext_vector_type(2)));
            const double2_t ov = {o[0], o[1]};
            __builtin_nontemporal_store(ov, reinterpret_cast<double2_t*>(out + f));
        }
        const int t0 = head + 2 * nvec;
        if (t0 + tid < total) {
            int le, k;
            split(t0 + tid, le, k);
            out[t0 + tid] = rbf_value_f64(dl[le], k, rs);
        }
    }
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
        if (rs.dtype == 1) reinterpret_cast<float*>(out)[f] = rbf_value_f32(d[e], k, rs);
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
hipError_t launch_prep_structures(hipStream_t s, const double* lattice, const int64_t* atom_offset, int64_t B,
                                  double rc, StructMeta* meta, int32_t* atom_struct) {
    if (B <= 0) return hipSuccess;
    const int t = 128;
    hipLaunchKernelGGL(prep_structures_kernel, dim3((unsigned)((B + t - 1) / t)), dim3(t), 0, s, lattice, atom_offset,
                       B, rc, meta);
    hipLaunchKernelGGL(map_atoms_kernel, dim3((unsigned)B), dim3(256), 0, s, atom_offset, atom_struct);
    return hipGetLastError();
}

hipError_t launch_graph_count(hipStream_t s, const GraphLaunch& g, int32_t* counts, int64_t* block_sums,
                              uint64_t* block_aux, uint64_t* rows_d, uint64_t* rows_j) {
    const int64_t nb = graph_blocks(g.num_atoms);
    if (nb <= 0) return hipSuccess;
    if (rows_d)
        hipLaunchKernelGGL(graph_count_kernel<true>, dim3((unsigned)nb), dim3(kGraphBlock), 0, s, g, counts,
                           block_sums, block_aux, rows_d, rows_j);
    else
        hipLaunchKernelGGL(graph_count_kernel<false>, dim3((unsigned)nb), dim3(kGraphBlock), 0, s, g, counts,
                           block_sums, block_aux, rows_d, rows_j);
    return hipGetLastError();
}

hipError_t launch_graph_emit_rows(hipStream_t s, const GraphLaunch& g, const int32_t* counts,
                                  const int64_t* block_offsets, const uint64_t* rows_d, const uint64_t* rows_j,
                                  int64_t* row_ptr, int32_t* col, double* dist, double* disp, void* rbf,
                                  const RbfSpec& rs) {
    const int64_t nb = graph_blocks(g.num_atoms);
    if (nb <= 0) return hipSuccess;
    const size_t shmem = sizeof(double) * (size_t)kQA * (size_t)g.kmax;
    hipLaunchKernelGGL(graph_emit_rows_kernel, dim3((unsigned)nb), dim3(kGraphBlock), shmem, s, g, counts,
                       block_offsets, rows_d, rows_j, row_ptr, col, dist, disp, rbf, rs);
    return hipGetLastError();
}

hipError_t launch_block_scan(hipStream_t s, int64_t* v, const uint64_t* aux, int64_t n, int64_t* total,
                             uint32_t* max_candidates, unsigned long long* sum_sq) {
    hipLaunchKernelGGL(block_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, v, aux, n, total, max_candidates,
                       sum_sq);
    return hipGetLastError();
}

int graph_emit_cap(uint32_t m) {
    if (m <= 64) return 64;
    if (m <= 128) return 128;
    if (m <= 256) return 256;
    if (m <= 512) return 512;
    return 0;
}

hipError_t launch_graph_emit(hipStream_t s, const GraphLaunch& g, int cap, const int32_t* counts,
                             const int64_t* block_offsets, int64_t* row_ptr, int32_t* col, double* dist,
                             double* disp, void* rbf, const RbfSpec& rs, uint32_t* error_flag) {
    const int64_t nb = graph_blocks(g.num_atoms);
    if (nb <= 0) return hipSuccess;
    const dim3 grid((unsigned)nb), block(kGraphBlock);
    switch (cap) {
        case 64:
            hipLaunchKernelGGL(graph_emit_kernel<64>, grid, block, 0, s, g, counts, block_offsets, row_ptr, col,
                               dist, disp, rbf, rs, error_flag);
            break;
        case 128:
            hipLaunchKernelGGL(graph_emit_kernel<128>, grid, block, 0, s, g, counts, block_offsets, row_ptr, col,
                               dist, disp, rbf, rs, error_flag);
            break;
        case 256:
            hipLaunchKernelGGL(graph_emit_kernel<256>, grid, block, 0, s, g, counts, block_offsets, row_ptr, col,
                               dist, disp, rbf, rs, error_flag);
            break;
        case 512:
            hipLaunchKernelGGL(graph_emit_kernel<512>, grid, block, 0, s, g, counts, block_offsets, row_ptr, col,
                               dist, disp, rbf, rs, error_flag);
            break;
        default:
            return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace dgn
