// betti_rank.hip — rank codes of local distance matrices for complexes above 512 points.
//
// The wide reduction keys a simplex by (diameter, combinatorial index) in 64 bits. With f32
// diameter bits that leaves 32 bits of index, and C(n, 4) passes 2^32 at n ~ 570. Above 512 points
// the retry launch therefore runs on rank codes: code(d) = the index of d's first occurrence in the
// complex's sorted packed triangle, < C(1024, 2) < 2^20, order- and equality-preserving (so every
// comparison the reduction makes on distances, ripser.cpp:318-324, gives the same answer), and the
// sorted triangle itself maps a code back to its f32 value for the emitted (birth, death) pairs.
//   gather : keys = f32 bits of each retry complex's packed lower triangle, values = positions
//   sort   : rocprim segmented radix sort, one segment per complex
//   codes  : lower_bound of each sorted key in its segment, scattered back to the position
#include <rocprim/device/device_segmented_radix_sort.hpp>

#include "dgn_internal.hpp"

namespace dgn {
namespace {

constexpr int kRankBlock = 256;

__global__ __launch_bounds__(kRankBlock) void rank_gather_kernel(const float* __restrict__ lower, int64_t tri_stride,
                                                                 const int32_t* __restrict__ npoints,
                                                                 const int32_t* __restrict__ list, int64_t count,
                                                                 int64_t stride, uint32_t* __restrict__ keys,
                                                                 uint32_t* __restrict__ vals, int32_t* __restrict__ beg,
                                                                 int32_t* __restrict__ end,
                                                                 const uint32_t* __restrict__ dev_len) {
    const int64_t r = blockIdx.y;
    // slots past the list's length on the device (launches sized by an upper bound): empty segments
    if (dev_len && r >= (int64_t)*dev_len) {
        if (blockIdx.x == 0 && threadIdx.x == 0) beg[r] = end[r] = (int32_t)(r * stride);
        return;
    }
    const int64_t gi = list[r];
    const int64_t n = npoints[gi];
    const int64_t m = n * (n - 1) / 2;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        beg[r] = (int32_t)(r * stride);
        end[r] = (int32_t)(r * stride + m);
    }
    const float* L = lower + gi * tri_stride;
    for (int64_t t = (int64_t)blockIdx.x * kRankBlock + threadIdx.x; t < m; t += (int64_t)gridDim.x * kRankBlock) {
        keys[r * stride + t] = __float_as_uint(L[t]);  // distances >= 0: bit order = value order
        vals[r * stride + t] = (uint32_t)t;
    }
}

__global__ __launch_bounds__(kRankBlock) void rank_codes_kernel(const int32_t* __restrict__ npoints,
                                                                const int32_t* __restrict__ list, int64_t stride,
                                                                const uint32_t* __restrict__ sorted,
                                                                const uint32_t* __restrict__ pos,
                                                                uint32_t* __restrict__ codes,
                                                                const uint32_t* __restrict__ dev_len) {
    const int64_t r = blockIdx.y;
    if (dev_len && r >= (int64_t)*dev_len) return;
    const int64_t n = npoints[list[r]];
    const int64_t m = n * (n - 1) / 2;
    const uint32_t* S = sorted + r * stride;
    for (int64_t t = (int64_t)blockIdx.x * kRankBlock + threadIdx.x; t < m; t += (int64_t)gridDim.x * kRankBlock) {
        const uint32_t key = S[t];
        int64_t lo = 0, hi = t;  // first index with S[idx] == key (S sorted ascending)
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (S[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        codes[r * stride + pos[r * stride + t]] = (uint32_t)lo;
    }
}

struct RankTemp {
    uint32_t *keys, *vals, *pos;
    int32_t *beg, *end;
    void* sort_tmp;
    size_t sort_bytes, total;
};

RankTemp rank_temp_layout(void* base, int64_t count, int64_t stride, size_t sort_bytes) {
    auto al = [](size_t x) { return (x + 255) / 256 * 256; };
    RankTemp t{};
    uint8_t* p = reinterpret_cast<uint8_t*>(base);
    size_t o = 0;
    const size_t arr = al(sizeof(uint32_t) * (size_t)count * (size_t)stride);
    t.keys = reinterpret_cast<uint32_t*>(p + o), o += arr;
    t.vals = reinterpret_cast<uint32_t*>(p + o), o += arr;
    t.pos = reinterpret_cast<uint32_t*>(p + o), o += arr;
    t.beg = reinterpret_cast<int32_t*>(p + o), o += al(sizeof(int32_t) * (size_t)count);
    t.end = reinterpret_cast<int32_t*>(p + o), o += al(sizeof(int32_t) * (size_t)count);
    t.sort_tmp = p + o;
    t.sort_bytes = sort_bytes;
    t.total = o + al(sort_bytes);
    return t;
}

size_t sort_temp_bytes(int64_t count, int64_t stride) {
    size_t bytes = 0;
    (void)rocprim::segmented_radix_sort_pairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                              (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                              (unsigned int)(count * stride), (unsigned int)count,
                                              (const int32_t*)nullptr, (const int32_t*)nullptr);
    return bytes;
}

}  // namespace

size_t betti_rank_temp_bytes(int64_t count, int64_t stride) {
    return rank_temp_layout(nullptr, count, stride, sort_temp_bytes(count, stride)).total;
}

hipError_t betti_rank_codes(hipStream_t s, const float* lower, int64_t tri_stride, const int32_t* npoints,
                            const int32_t* list, int64_t count, int64_t stride, uint32_t* codes, uint32_t* sorted,
                            void* temp, size_t temp_bytes, const uint32_t* dev_len) {
    if (count <= 0) return hipSuccess;
    if (count * stride > INT32_MAX) return hipErrorInvalidValue;  // rocprim item counts are 32-bit
    size_t sb = sort_temp_bytes(count, stride);
    RankTemp t = rank_temp_layout(temp, count, stride, sb);
    if (t.total > temp_bytes) return hipErrorInvalidValue;
    const int64_t per = (stride + kRankBlock - 1) / kRankBlock;
    const dim3 grid((unsigned)(per < 64 ? per : 64), (unsigned)count);
    hipLaunchKernelGGL(rank_gather_kernel, grid, dim3(kRankBlock), 0, s, lower, tri_stride, npoints, list, count,
                       stride, t.keys, t.vals, t.beg, t.end, dev_len);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    e = rocprim::segmented_radix_sort_pairs(t.sort_tmp, sb, (const uint32_t*)t.keys, sorted, (const uint32_t*)t.vals,
                                            t.pos, (unsigned int)(count * stride), (unsigned int)count,
                                            (const int32_t*)t.beg, (const int32_t*)t.end, 0, 32, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(rank_codes_kernel, grid, dim3(kRankBlock), 0, s, npoints, list, stride, sorted, t.pos, codes,
                       dev_len);
    return hipGetLastError();
}

// slice q of a list of *total entries: sl[2q] = its length, clamp(*total - q slice, 0, slice), and
// sl[2q + 1] = 0 (its launch's work queue), for q < nsl -- so the slices of a list whose length
// only the device knows are launched without a host read (grids sized by the host's upper bound)
__global__ void slice_lengths_kernel(const uint32_t* __restrict__ total, int64_t slice, int64_t nsl,
                                     uint32_t* __restrict__ sl) {
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < nsl; q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t left = (int64_t)*total - q * slice;
        sl[2 * q] = (uint32_t)(left < 0 ? 0 : (left < slice ? left : slice));
        sl[2 * q + 1] = 0u;
    }
}

hipError_t launch_slice_lengths(hipStream_t s, const uint32_t* total, int64_t slice, int64_t nsl, uint32_t* sl) {
    if (nsl <= 0) return hipSuccess;
    const int64_t blocks = (nsl + 255) / 256;
    hipLaunchKernelGGL(slice_lengths_kernel, dim3((unsigned)(blocks < 1024 ? blocks : 1024)), dim3(256), 0, s, total,
                       slice, nsl, sl);
    return hipGetLastError();
}

}  // namespace dgn
