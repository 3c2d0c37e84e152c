// dgn_device.hpp — shared device-side types and wave64 primitives for gfx950 (CDNA4).
//
// Every kernel in this library is compiled with -ffp-contract=off: the reference's double
// arithmetic (x86-64 SSE2, no -march) is never contracted to FMA, and bit-exact CSR
// membership / distances depend on reproducing its exact operation order.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dgn {

constexpr int kWave = 64;  // CDNA wavefront; never 32

// Per-structure geometry, prepared once per call by prep_structures_kernel.
struct StructMeta {
    double L[9];     // lattice rows a, b, c (row-major)
    double R[9];     // inverse lattice; column k = reciprocal vector of fractional axis k
    double h[3];     // rc * |column k of R|: |frac_k| bound of any vector shorter than rc
    int64_t first;   // first atom (global index)
    int32_t natoms;  // atoms in the structure
    int32_t nref;    // reference image range: ceil(rc / min row norm) + 1 (neighbor_list.cpp:68-72)
};

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & (kWave - 1)); }

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

__device__ __forceinline__ uint64_t f64_bits(double d) { return (uint64_t)__double_as_longlong(d); }

}  // namespace dgn
