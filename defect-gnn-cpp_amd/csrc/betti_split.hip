// betti_split.hip — local complexes above kWideMaxPoints (2,048) points, split into the connected
// components of their threshold graph.
//
// The Vietoris-Rips complex at threshold thr (ripser.cpp:386-395: sparse_distance_matrix keeps
// d <= thr) has no simplex across two components of the graph {d <= thr}: its coboundary matrix is
// block-diagonal by component, a column is only ever added to a column of its own block (they share
// the pivot, a cofacet inside the block), and Kruskal's forest is the union of the components'
// forests. So the persistence pairs of the complex are the union of its components' pairs
// (ripser.cpp:514-1269 applied to each component gives the same multiset), and a component of one
// point contributes one essential dim-0 class. Complexes of any size whose components each have
// at most kWideGiantPoints (4,096) points are therefore reduced by the ordinary tiers, one
// sub-complex per component (components of 2,049..4,096 points on the GIANT instantiation, round 6);
// a single larger component stays outside the envelope (DGN_ERR_UNSUPPORTED).
//
//   big_gram_kernel        distances of clouds above 2,048 points (the reference's Gram arithmetic,
//                          ripser_wrapper.cpp:64-67, on the VALU: the same rounded products and sums
//                          as the ordinary distance kernels), f32 packed lower triangle
//   components_kernel      union-find over the pairs d <= thr (one workgroup per complex; roots
//                          link larger -> smaller with a compare-and-swap, so parents only decrease)
//   gather_sub_kernel      a component's packed sub-triangle (vertices in ascending order)
#include "dgn_internal.hpp"

namespace dgn {
namespace {

constexpr int kSplitBlock = 1024;

__device__ __forceinline__ int64_t c2l(int64_t x) { return x * (x - 1) / 2; }

// row i of the packing holds (i, j) for j < i at c2(i) + j (ripser_wrapper.cpp:20-24)
__global__ __launch_bounds__(256) void big_gram_kernel(const double* __restrict__ clouds, int64_t cloud_stride,
                                                       const int32_t* __restrict__ npoints, int64_t first,
                                                       float* __restrict__ lower, int64_t tri_stride) {
    const int64_t c = blockIdx.y;
    const int64_t n = npoints[first + c];
    const double* X = clouds + (first + c) * cloud_stride * 3;
    float* L = lower + c * tri_stride;
    const int64_t tot = c2l(n);
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < tot; t += (int64_t)gridDim.x * blockDim.x) {
        int64_t i = (int64_t)((1.0 + sqrt(1.0 + 8.0 * (double)t)) * 0.5);
        i -= c2l(i) > t;
        i += c2l(i + 1) <= t;
        const int64_t j = t - c2l(i);
        const double xi0 = X[3 * i], xi1 = X[3 * i + 1], xi2 = X[3 * i + 2];
        const double xj0 = X[3 * j], xj1 = X[3 * j + 1], xj2 = X[3 * j + 2];
        const double si = (xi0 * xi0 + xi1 * xi1) + xi2 * xi2;  // rowwise().squaredNorm()
        const double sj = (xj0 * xj0 + xj1 * xj1) + xj2 * xj2;
        const double dot = (xi0 * xj0 + xi1 * xj1) + xi2 * xj2;  // GEBP k order, no FMA
        const double d2 = (si + sj) - 2.0 * dot;
        L[t] = (float)sqrt(fmax(d2, 0.0));
    }
}

__device__ __forceinline__ int32_t uf_find(int32_t* P, int32_t x) {
    // path halving; every store writes a smaller index of the same set (parents only decrease)
    int32_t p = __atomic_load_n(&P[x], __ATOMIC_RELAXED);
    while (p != x) {
        const int32_t g = __atomic_load_n(&P[p], __ATOMIC_RELAXED);
        if (g != p) __atomic_store_n(&P[x], g, __ATOMIC_RELAXED);
        x = p;
        p = g;
    }
    return x;
}

// the parent array lives in LDS (dynamic, n int32), so every find and link of the workgroup is
// coherent; the roots go to labels[c][v] at the end
__global__ __launch_bounds__(kSplitBlock) void components_kernel(const float* __restrict__ lower, int64_t tri_stride,
                                                                 const int32_t* __restrict__ npoints, int64_t first,
                                                                 float thr, int32_t* __restrict__ labels,
                                                                 int64_t label_stride) {
    extern __shared__ int32_t P[];
    const int64_t c = blockIdx.x;
    const int32_t n = npoints[first + c];
    const float* L = lower + c * tri_stride;
    for (int32_t v = threadIdx.x; v < n; v += kSplitBlock) P[v] = v;
    __syncthreads();
    const int64_t tot = c2l(n);
    int64_t i = (int64_t)((1.0 + sqrt(1.0 + 8.0 * (double)threadIdx.x)) * 0.5);
    i -= c2l(i) > (int64_t)threadIdx.x;
    i += c2l(i + 1) <= (int64_t)threadIdx.x;
    int64_t j = (int64_t)threadIdx.x - c2l(i);
    for (int64_t t = threadIdx.x; t < tot; t += kSplitBlock) {
        if (L[t] <= thr) {
            int32_t a = (int32_t)i, b = (int32_t)j;
            for (;;) {
                a = uf_find(P, a);
                b = uf_find(P, b);
                if (a == b) break;
                if (a < b) {
                    const int32_t x = a;
                    a = b;
                    b = x;
                }
                // link the larger root under the smaller one; a lost race re-reads both roots
                if (atomicCAS(&P[a], a, b) == a) break;
            }
        }
        j += kSplitBlock;
        while (j >= i) {
            j -= i;
            ++i;
        }
    }
    __syncthreads();  // every union done: the forest no longer changes, finds return the roots
    int32_t* out = labels + c * label_stride;
    for (int32_t v = threadIdx.x; v < n; v += kSplitBlock) out[v] = uf_find(P, v);
}

// sub-complex q: vertices map[off[q] .. off[q] + size[q]) (ascending) of complex src[q]
__global__ __launch_bounds__(256) void gather_sub_kernel(const float* __restrict__ lower, int64_t tri_stride,
                                                         const int32_t* __restrict__ src, const int64_t* __restrict__ off,
                                                         const int32_t* __restrict__ size, const int32_t* __restrict__ map,
                                                         float* __restrict__ sub, int64_t sub_stride) {
    const int64_t q = blockIdx.y;
    const int64_t s = size[q];
    const int32_t* M = map + off[q];
    const float* L = lower + (int64_t)src[q] * tri_stride;
    float* O = sub + q * sub_stride;
    const int64_t tot = c2l(s);
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < tot; t += (int64_t)gridDim.x * blockDim.x) {
        int64_t i = (int64_t)((1.0 + sqrt(1.0 + 8.0 * (double)t)) * 0.5);
        i -= c2l(i) > t;
        i += c2l(i + 1) <= t;
        const int64_t j = t - c2l(i);
        const int64_t a = M[i], b = M[j];  // a > b (ascending map)
        O[t] = L[c2l(a) + b];
    }
}

}  // namespace

hipError_t launch_big_gram(hipStream_t s, const double* clouds, int64_t cloud_stride, const int32_t* npoints,
                           int64_t first, int64_t count, float* lower, int64_t tri_stride) {
    if (count <= 0) return hipSuccess;
    const int64_t per = (tri_stride + 255) / 256;
    hipLaunchKernelGGL(big_gram_kernel, dim3((unsigned)(per < 4096 ? per : 4096), (unsigned)count), dim3(256), 0, s,
                       clouds, cloud_stride, npoints, first, lower, tri_stride);
    return hipGetLastError();
}

hipError_t launch_components(hipStream_t s, const float* lower, int64_t tri_stride, const int32_t* npoints,
                             int64_t first, int64_t count, float thr, int32_t* labels, int64_t label_stride) {
    if (count <= 0) return hipSuccess;
    if (label_stride * 4 > 160 * 1024) return hipErrorInvalidValue;  // kSplitMaxPoints
    hipLaunchKernelGGL(components_kernel, dim3((unsigned)count), dim3(kSplitBlock), (size_t)(4 * label_stride), s,
                       lower, tri_stride, npoints, first, thr, labels, label_stride);
    return hipGetLastError();
}

hipError_t launch_gather_sub(hipStream_t s, const float* lower, int64_t tri_stride, const int32_t* src,
                             const int64_t* off, const int32_t* size, const int32_t* map, int64_t count,
                             float* sub, int64_t sub_stride) {
    if (count <= 0) return hipSuccess;
    const int64_t per = (sub_stride + 255) / 256;
    hipLaunchKernelGGL(gather_sub_kernel, dim3((unsigned)(per < 4096 ? per : 4096), (unsigned)count), dim3(256), 0, s,
                       lower, tri_stride, src, off, size, map, sub, sub_stride);
    return hipGetLastError();
}

}  // namespace dgn
