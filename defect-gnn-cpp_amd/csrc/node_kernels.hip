// node_kernels.hip — per-atom node features of CrystalGraph with the topological block appended
// (SURVEY 8(f) row 3): the species-keyed embedding gather (reference crystal_graph.cpp:19-21,
// node_features_.row(i) = atom_embeddings.at(element)), PCA::transform of the 35 Betti statistics
// (pca.cpp:36-44: (x - mean) * components, an A x 35 by 35 x k f64 product) and their N x (D + k)
// concatenation, the layout add_topo_features (crystal_graph.cpp:65-67) names.
// HBM-bound: per atom 4 B species + 280 B Betti row in, 8 (D + k) B out; the embedding table,
// mean and components are tiny and stay in L2 / LDS.
#include "dgn_internal.hpp"

namespace dgn {

constexpr int kNodeBlock = 256;
constexpr int kNodeAtoms = 32;  // atoms per block
constexpr int kBettiDims = 35;
constexpr int kMaxPcaK = 35;

__global__ __launch_bounds__(kNodeBlock) void node_features_kernel(const int32_t* __restrict__ species, int64_t A,
                                                                    const double* __restrict__ embed, int32_t nkeys,
                                                                    int32_t D, const double* __restrict__ betti,
                                                                    const double* __restrict__ mean,
                                                                    const double* __restrict__ comp, int32_t k,
                                                                    double* __restrict__ out,
                                                                    uint32_t* __restrict__ error_flag) {
    __shared__ double mean_s[kBettiDims];
    __shared__ double comp_s[kBettiDims * kMaxPcaK];       // [t][j], row-major 35 x k
    __shared__ double cent_s[kNodeAtoms][kBettiDims + 1];  // centred Betti rows of the block's atoms
    __shared__ int32_t sp_s[kNodeAtoms];
    const int64_t a0 = (int64_t)blockIdx.x * kNodeAtoms;
    const int na = (int)(A - a0 < kNodeAtoms ? A - a0 : kNodeAtoms);
    const int W = D + k;
    if (betti && k > 0) {
        for (int t = threadIdx.x; t < kBettiDims; t += kNodeBlock) mean_s[t] = mean[t];
        for (int t = threadIdx.x; t < kBettiDims * k; t += kNodeBlock) comp_s[t] = comp[t];
    }
    for (int i = threadIdx.x; i < na; i += kNodeBlock) {
        const int32_t s = species[a0 + i];
        if (s < 0 || s >= nkeys) atomicOr(error_flag, 1u);  // atom_embeddings.at(): unknown key
        sp_s[i] = s < 0 || s >= nkeys ? 0 : s;
    }
    __syncthreads();
    if (betti && k > 0) {
        for (int x = threadIdx.x; x < na * kBettiDims; x += kNodeBlock) {  // coalesced rows
            const int i = x / kBettiDims, t = x - i * kBettiDims;
            cent_s[i][t] = betti[a0 * kBettiDims + x] - mean_s[t];  // x.rowwise() - mean
        }
    }
    __syncthreads();
    // the block's output rows are contiguous: [a0, a0 + na) x W, written coalesced
    const int64_t total = (int64_t)na * W;
    double* o = out + a0 * W;
    for (int64_t x = threadIdx.x; x < total; x += kNodeBlock) {
        const int i = (int)(x / W), c = (int)(x - (int64_t)i * W);
        double v;
        if (c < D) {
            v = embed[(int64_t)sp_s[i] * D + c];
        } else {
            const int j = c - D;
            double acc = 0.0;
#pragma unroll 5
            for (int t = 0; t < kBettiDims; ++t) acc = __builtin_fma(cent_s[i][t], comp_s[t * k + j], acc);
            v = acc;
        }
        o[x] = v;
    }
}

hipError_t launch_node_features(hipStream_t s, const int32_t* species, int64_t A, const double* embed, int32_t nkeys,
                                int32_t D, const double* betti, const double* mean, const double* comp, int32_t k,
                                double* out, uint32_t* error_flag) {
    if (A <= 0) return hipSuccess;
    if (k > kMaxPcaK) return hipErrorInvalidValue;
    const int64_t nb = (A + kNodeAtoms - 1) / kNodeAtoms;
    hipLaunchKernelGGL(node_features_kernel, dim3((unsigned)nb), dim3(kNodeBlock), 0, s, species, A, embed, nkeys, D,
                       betti, mean, comp, k, out, error_flag);
    return hipGetLastError();
}

}  // namespace dgn

namespace dgn {

// Flat per-edge arrays of a CSR, the WasmAPI graph accessors (reference src/viz/wasm_bindings.cpp:
// 206-294: get_edge_sources / get_edge_targets / get_edge_distances / get_edge_displacements,
// float32 casts of Neighbor::distance / displacement, sources = the row atom's index within its
// structure). One block per 256 atom rows: the rows' CSR offsets and in-structure indices are
// staged in LDS, then the block's contiguous edge range is written edge-parallel (coalesced).
// HBM-bound: per edge 4 (col) + 8 (dist) + 24 (disp) B in, 4 + 4 + 4 + 12 B out.
constexpr int kEdgeRows = 256;

__global__ __launch_bounds__(kEdgeRows) void edge_arrays_kernel(const int64_t* __restrict__ row_ptr,
                                                                 const int64_t* __restrict__ atom_offset, int64_t B,
                                                                 int64_t A, const int32_t* __restrict__ col,
                                                                 const double* __restrict__ dist,
                                                                 const double* __restrict__ disp,
                                                                 int32_t* __restrict__ src, int32_t* __restrict__ tgt,
                                                                 float* __restrict__ dist32,
                                                                 float* __restrict__ disp32) {
    __shared__ int64_t rp_s[kEdgeRows + 1];
    __shared__ int32_t local_s[kEdgeRows];
    const int64_t a0 = (int64_t)blockIdx.x * kEdgeRows;
    const int na = (int)(A - a0 < kEdgeRows ? A - a0 : kEdgeRows);
    const int t = threadIdx.x;
    if (t < na) rp_s[t] = row_ptr[a0 + t];
    if (t == 0) rp_s[na] = row_ptr[a0 + na];  // na <= kEdgeRows: one past the block's last row
    if (t < na && src) {
        // structure of atom a0 + t: the last s with atom_offset[s] <= a (binary search)
        const int64_t a = a0 + t;
        int64_t lo = 0, hi = B - 1;
        while (lo < hi) {
            const int64_t mid = (lo + hi + 1) >> 1;
            if (atom_offset[mid] <= a) lo = mid;
            else hi = mid - 1;
        }
        local_s[t] = (int32_t)(a - atom_offset[lo]);
    }
    __syncthreads();
    const int64_t e0 = rp_s[0], e1 = rp_s[na];
    for (int64_t e = e0 + t; e < e1; e += kEdgeRows) {
        if (src) {
            int lo = 0, hi = na - 1;  // row r: rp_s[r] <= e < rp_s[r + 1]
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (rp_s[mid] <= e) lo = mid;
                else hi = mid - 1;
            }
            src[e] = local_s[lo];
        }
        if (tgt) tgt[e] = col[e];
        if (dist32) dist32[e] = (float)dist[e];
    }
    if (disp32)
        for (int64_t x = 3 * e0 + t; x < 3 * e1; x += kEdgeRows) disp32[x] = (float)disp[x];
}

hipError_t launch_edge_arrays(hipStream_t s, const int64_t* row_ptr, const int64_t* atom_offset, int64_t B, int64_t A,
                              const int32_t* col, const double* dist, const double* disp, int32_t* src, int32_t* tgt,
                              float* dist32, float* disp32) {
    if (A <= 0) return hipSuccess;
    const int64_t nb = (A + kEdgeRows - 1) / kEdgeRows;
    hipLaunchKernelGGL(edge_arrays_kernel, dim3((unsigned)nb), dim3(kEdgeRows), 0, s, row_ptr, atom_offset, B, A, col,
                       dist, disp, src, tgt, dist32, disp32);
    return hipGetLastError();
}

}  // namespace dgn
