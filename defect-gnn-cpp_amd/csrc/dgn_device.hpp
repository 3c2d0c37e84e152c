// dgn_device.hpp — shared device-side types and wave64 primitives for gfx950 (CDNA4).
//
// Every kernel in this library is compiled with -ffp-contract=off: the reference's double
// arithmetic (x86-64 SSE2, no -march) is never contracted to FMA, and bit-exact CSR
// membership / distances depend on reproducing its exact operation order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace dgn {

constexpr int kWave = 64;  // CDNA wavefront; never 32

// Per-structure geometry, prepared once per call by prep_structures_kernel.
struct StructMeta {
    double L[9];     // lattice rows a, b, c (row-major)
    double R[9];     // inverse lattice; column k = reciprocal vector of fractional axis k
    double H[3];     // rc * |column k of R| + 1e-9: the conservative fractional half-widths every
                     // search uses (|frac_k| bound of any vector shorter than rc, plus a margin)
    int64_t first;   // first atom (global index)
    int32_t natoms;  // atoms in the structure
    int32_t nref;    // reference image range: ceil(rc / min row norm) + 1 (neighbor_list.cpp:68-72)
    int32_t one;     // every H_k < 0.5: at most one periodic image of an atom per axis can reach rc
    int32_t cells;   // a cell list was built (natoms > kStage and one)
    int32_t nc[3];   // cells per fractional axis (cell list), each cell at least H_k wide
    int32_t diag;    // lattice rows are axis-aligned (a = (a0,0,0), b = (0,b1,0), c = (0,0,c2))
    double band;     // |d2_approx - d2| bound of the fixed-point nearest-image distance (x64 margin)
    // the one-image count pass's packed-f32 prefilter (count_one_image): lattice * 2^-32 in f32 and
    // the d2 window (rc^2 -+ its rigorous band) outside which the f32 value decides
    // (unscaled for `few` structures, whose f32 displacements are fractions, not fixed point)
    float lf[9];
    float lo32, hi32;
    int32_t few;     // not one, every H_k < 1 and nref == 2: at most two images per axis (search_staged_few)
};

__device__ __forceinline__ int lane_id() {
    int l = (int)(threadIdx.x & (kWave - 1));
    asm volatile("" : "+v"(l));
    return l;
}

// element i of a per-wave scratch array as (scalar base) + (32-bit byte offset): the load/store
// takes the base in SGPRs and one vector offset register (global_* vN, s[base]) instead of a
// 64-bit vector address built per access (every scratch array here is far below 4 GB)
template <class T>
__device__ __forceinline__ T& at(T* base, uint32_t i) {
    return *reinterpret_cast<T*>(reinterpret_cast<uint8_t*>(const_cast<std::remove_const_t<T>*>(base)) +
                                 i * (uint32_t)sizeof(T));
}
template <class T>
__device__ __forceinline__ const T& at(const T* base, uint32_t i) {
    return *reinterpret_cast<const T*>(reinterpret_cast<const uint8_t*>(base) + i * (uint32_t)sizeof(T));
}


__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// number of set bits of m strictly below this lane
__device__ __forceinline__ int mask_prefix(uint64_t m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, kWave);
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        T w = __shfl_xor(v, o, kWave);
        v = w > v ? w : v;
    }
    return v;
}
template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        T w = __shfl_xor(v, o, kWave);
        v = w < v ? w : v;
    }
    return v;
}
// inclusive prefix sum over the wave
template <typename T>
__device__ __forceinline__ T wave_inclusive_sum(T v) {
    const int l = lane_id();
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        T w = __shfl_up(v, o, kWave);
        if (l >= o) v += w;
    }
    return v;
}

// Wave reductions to a SCALAR: DPP row rotations (every lane of a 16-lane row gets the row's
// result), row_bcast:15 / row_bcast:31 carry rows 0..2 into row 3, and one v_readlane of lane 63.
// The result is uniform to the compiler; a __shfl-based reduction is a vector value to it, and a
// branch on one turns every later branch on data derived from it into exec-masked code.
// Precondition: the whole wave is active (EXEC = all 64 lanes), i.e. the call sits in wave-uniform
// control flow. An inactive lane would be read by the DPP steps as the bound value (the identity,
// harmless), but an inactive lane 63 would hand back a stale register. Builds with
// -DDGN_DEVICE_CHECKS=1 trap on a call that breaks the precondition.
__device__ __forceinline__ void dgn_check_full_exec() {
#if defined(DGN_DEVICE_CHECKS) && DGN_DEVICE_CHECKS
    if (__builtin_amdgcn_read_exec() != ~0ull) __builtin_trap();
#endif
}
// Bounds checks of stores whose index a kernel derives (DGN_DEVICE_CHECKS builds only: a trap
// names the faulting kernel in the HIP error instead of a write past the buffer)
__device__ __forceinline__ void dgn_check(bool ok) {
#if defined(DGN_DEVICE_CHECKS) && DGN_DEVICE_CHECKS
    if (!ok) __builtin_trap();
#else
    (void)ok;
#endif
}
__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
    dgn_check_full_exec();
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x121, 0xf, 0xf, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x122, 0xf, 0xf, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x124, 0xf, 0xf, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x128, 0xf, 0xf, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x142, 0xa, 0xf, false));
    x = min(x, (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)x, 0x143, 0xc, 0xf, false));
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}
// 64-bit minimum in two 32-bit stages: the high words, then the low words of the lanes holding
// the minimal high word
__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
    const uint32_t hi = (uint32_t)(v >> 32);
    const uint32_t mh = wave_min_u32(hi);
    const uint32_t ml = wave_min_u32(hi == mh ? (uint32_t)v : 0xFFFFFFFFu);
    return ((uint64_t)mh << 32) | ml;
}
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t x) {
    dgn_check_full_exec();
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x121, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x122, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x124, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x128, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
}

__device__ __forceinline__ uint64_t f64_bits(double d) { return (uint64_t)__double_as_longlong(d); }

// One-wave LDS hand-off: a wave's LDS instructions execute in order, so lane-to-lane exchange
// through LDS only needs the compiler not to move memory operations across this point.
__device__ __forceinline__ void wave_lds_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront"); }

__device__ __forceinline__ int tri_c2(int x) { return x * (x - 1) / 2; }

// ---- local distance matrices (ripser_wrapper.cpp:60-70 + 17-24) ----
// The reference's Gram arithmetic: dot = (x_i0 x_j0 + x_i1 x_j1) + x_i2 x_j2 (Eigen's GEBP k
// order, each product rounded, no FMA), sq_i = the same sum of squares, then
// sqrt(max(0, (sq_i + sq_j) - 2 dot)) -> f32; the strict lower triangle in the reference's packing
// (row i, j < i at i(i-1)/2 + j).
//
// sqrt_lean: the f64 square root the compiler emits for sqrt() (v_rsq_f64 seed, one Newton step
// on the pair (y ~ sqrt x, h ~ 1/(2 sqrt x)), two residual corrections), without its rescaling of
// x < 2^-767 and its +-0 / inf pass-through: the same operations in the same order, so for
// 2^-767 <= x < inf it returns the same bits. The callers take the full sqrt() for a wave with
// any lane outside that range.
__device__ __forceinline__ double sqrt_lean(double x) {
    const double r = __builtin_amdgcn_rsq(x);
    double y = x * r;
    double h = r * 0.5;
    const double e = __builtin_fma(-h, y, 0.5);
    y = __builtin_fma(y, e, y);
    h = __builtin_fma(h, e, h);
    double d = __builtin_fma(-y, y, x);
    y = __builtin_fma(d, h, y);
    d = __builtin_fma(-y, y, x);
    return __builtin_fma(d, h, y);
}
constexpr double kLeanSqrtMin = 0x1p-767;  // the compiler's rescaling threshold

// Narrow form: n <= 64, lane p holds cloud row p in px (lanes >= n: any value); rec = per-wave
// LDS [4 * 64] doubles (x, y, z, squared norm per row; it may overlay the storage px came from).
// One pair per lane and round over the packed triangle, so every lane of a round but the last
// computes a wanted distance and the stores are contiguous (a 16 x 16 Gram tile on the matrix
// cores leaves 37 % of the lanes idle at n = 43 and its products need the same VALU tail: the
// MFMA form measured 4.55 ms of the 5.94 ms config-4 distance kernel, the search 1.39 ms).
// cap: floats the caller reserved for this complex's triangle (bounds check of DGN_DEVICE_CHECKS builds)
__device__ __forceinline__ void gram_triangle_narrow(const double px[3], int n, double* rec, float* __restrict__ L,
                                                     int64_t cap) {
    typedef double double2_t __attribute__((ext_vector_type(2)));
    const int lane = lane_id();
    dgn_check(n >= 1 && n <= kWave && tri_c2(n) <= cap);
    const double sq = (px[0] * px[0] + px[1] * px[1]) + px[2] * px[2];  // rowwise().squaredNorm()
    wave_lds_sync();
    if (lane < n) {
        double2_t* R = reinterpret_cast<double2_t*>(rec + 4 * lane);
        R[0] = double2_t{px[0], px[1]};
        R[1] = double2_t{px[2], sq};
    }
    wave_lds_sync();
    const int tot = __builtin_amdgcn_readfirstlane(tri_c2(n));  // n is wave-uniform
    for (int base = 0; base < tot; base += kWave) {  // wave-uniform rounds; the last one partial
        const uint32_t t = (uint32_t)min(base + lane, tot - 1);
        // row i of packed index t < 2016: (1 + sqrt(8t + 1)) / 2 is i exactly at the row's first
        // index and at most i + 1 - 2 / 127 at its last, so a 0.004 bias absorbs the f32 root's
        // error (one ulp) without the two integer corrections
        const uint32_t i = (uint32_t)__builtin_fmaf(__builtin_amdgcn_sqrtf((float)(8 * t + 1)), 0.5f, 0.504f);
        const uint32_t j = t - ((i * (i - 1)) >> 1);
        const double2_t* Ri = reinterpret_cast<const double2_t*>(rec + 4 * i);
        const double2_t* Rj = reinterpret_cast<const double2_t*>(rec + 4 * j);
        const double2_t a0 = Ri[0], a1 = Ri[1], b0 = Rj[0], b1 = Rj[1];
        const double dot = (a0.x * b0.x + a0.y * b0.y) + a1.x * b1.x;  // GEBP k order, no FMA
        const double d2 = fmax((a1.y + b1.y) - 2.0 * dot, 0.0);
        double dd;
        if (ballot(!(d2 >= kLeanSqrtMin && d2 < __builtin_inf()))) dd = sqrt(d2);
        else dd = sqrt_lean(d2);
        if (base + lane < tot) {
            dgn_check(t < (uint32_t)tot && j < i);
            L[t] = (float)dd;
        }
    }
    wave_lds_sync();
}

// Wide form (n > 64): row p comes from point(p, x) (x[0..2] = the row's coordinates, static
// indices only); sq = LDS [n].
__device__ __forceinline__ double sel3(int k, double a, double b, double c) { return k == 0 ? a : (k == 1 ? b : c); }
template <class Point>
__device__ __forceinline__ void gram_triangle_wide(int n, double* sq, float* __restrict__ L, Point&& point, int64_t cap) {
    typedef double double4_t __attribute__((ext_vector_type(4)));
    const int lane = lane_id();
    dgn_check((int64_t)n * (n - 1) / 2 <= cap);
    const int kq = lane >> 4;
    for (int p = lane; p < n; p += kWave) {
        double x[3];
        point(p, x);
        sq[p] = (x[0] * x[0] + x[1] * x[1]) + x[2] * x[2];
    }
    wave_lds_sync();
    const int T = (n + 15) / 16;
    for (int I = 0; I < T; ++I) {
        const int ra = 16 * I + (lane & 15);
        double xa = 0.0;
        if (ra < n && kq < 3) {
            double x[3];
            point(ra, x);
            xa = sel3(kq, x[0], x[1], x[2]);
        }
        for (int J = 0; J <= I; ++J) {
            const int cb = 16 * J + (lane & 15);
            double xb = 0.0;
            if (cb < n && kq < 3) {
                double x[3];
                point(cb, x);
                xb = sel3(kq, x[0], x[1], x[2]);
            }
            const double4_t z = {0.0, 0.0, 0.0, 0.0};
            const double4_t p0 = __builtin_amdgcn_mfma_f64_16x16x4f64(kq == 0 ? xa : 0.0, kq == 0 ? xb : 0.0, z, 0, 0, 0);
            const double4_t p1 = __builtin_amdgcn_mfma_f64_16x16x4f64(kq == 1 ? xa : 0.0, kq == 1 ? xb : 0.0, z, 0, 0, 0);
            const double4_t p2 = __builtin_amdgcn_mfma_f64_16x16x4f64(kq == 2 ? xa : 0.0, kq == 2 ? xb : 0.0, z, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 16 * I + (lane >> 4) + 4 * r;
                if (row < n && cb < row) {
                    dgn_check(tri_c2(row) + cb < tri_c2(n));
                    const double dot = (p0[r] + p1[r]) + p2[r];
                    const double d2 = (sq[row] + sq[cb]) - 2.0 * dot;
                    L[tri_c2(row) + cb] = (float)sqrt(fmax(d2, 0.0));
                }
            }
        }
    }
    wave_lds_sync();
}

// ---- DPP wave reductions of doubles: row_ror 1/2/4/8 inside each 16-lane row (VALU latency,
// no LDS round trips), then the four row results by v_readlane ----
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)b, CTRL, 0xf, 0xf, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(b >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
struct OpAdd { __device__ static double f(double a, double b) { return a + b; } };
struct OpMax { __device__ static double f(double a, double b) { return fmax(a, b); } };
struct OpMin { __device__ static double f(double a, double b) { return fmin(a, b); } };
template <class Op>
__device__ __forceinline__ double wave_reduce_f64(double v) {
    v = Op::f(v, dpp_f64<0x121>(v));
    v = Op::f(v, dpp_f64<0x122>(v));
    v = Op::f(v, dpp_f64<0x124>(v));
    v = Op::f(v, dpp_f64<0x128>(v));
    return Op::f(Op::f(readlane_f64(v, 0), readlane_f64(v, 16)), Op::f(readlane_f64(v, 32), readlane_f64(v, 48)));
}

// The 35 Betti statistics of one atom (betti_features.cpp:24-55, 87-98; utils/math.hpp:9-28):
// groups 0 dim-0 death | 1..3 dim-1 persistence, birth, death | 4..6 dim-2 persistence, birth,
// death; each mean, population std (two-pass), max, min, sum * weight; zeros for an empty
// diagram. One group at a time (few live uniform values), DPP reductions (no LDS round trips).
// Returns feature `lane` for lanes < 35.
__device__ __forceinline__ double betti_stats35(const float* d0, int n0, const float2* P1, int n1, const float2* P2,
                                                int n2, double weight) {
    const int lane = lane_id();
    double out = 0.0;
#pragma unroll 1
    for (int g = 0; g < 7; ++g) {
        const int m = g == 0 ? n0 : (g <= 3 ? n1 : n2);
        if (m == 0) continue;
        const float2* P = g <= 3 ? P1 : P2;
        const int which = g == 0 ? 1 : (g - 1) % 3;  // 0 persistence, 1 birth, 2 death (dims 1, 2)
        auto val = [&](int i) -> double {
            if (g == 0) return (double)at(d0, i);
            const float2 pr = at(P, i);
            return which == 0 ? (double)pr.y - (double)pr.x : (which == 1 ? (double)pr.x : (double)pr.y);
        };
        double sm = 0.0, mx = -INFINITY, mn = INFINITY;
        for (int i = lane; i < m; i += kWave) {
            const double v = val(i);
            sm += v;
            mx = fmax(mx, v);
            mn = fmin(mn, v);
        }
        sm = wave_reduce_f64<OpAdd>(sm);
        mx = wave_reduce_f64<OpMax>(mx);
        mn = wave_reduce_f64<OpMin>(mn);
        const double mean = sm / (double)m;
        double ss = 0.0;
        for (int i = lane; i < m; i += kWave) {
            const double v = val(i);
            ss += (v - mean) * (v - mean);
        }
        ss = wave_reduce_f64<OpAdd>(ss);
        const int r = lane - 5 * g;
        if (r == 0) out = mean;
        if (r == 1) out = sqrt(ss / (double)m);  // population std (math.hpp:13-16)
        if (r == 2) out = mx;
        if (r == 3) out = mn;
        if (r == 4) out = sm * weight;  // weighted_sum = sum * weight (math.hpp:26-28)
    }
    return out;
}

}  // namespace dgn
