// Persistence front end over the GPU VR reduction (dgn_host_persistence[_lower]); reference
// src/topology/ripser_wrapper.cpp:11-70. Pairs are returned per dimension sorted by
// (birth, death) — the multiset Ripser emits; dim0 ends with one (0, inf) per component
// (ripser.cpp:759-761). Complexes up to 512 points (64-point wave kernel + wide kernel); above that
// the library returns DGN_ERR_UNSUPPORTED.
#include <algorithm>
#include <cmath>
#include <limits>
#include <stdexcept>

#include "dgn/runtime.hpp"
#include "topology/ripser_wrapper.hpp"

namespace defect_gnn::topology {

namespace {

int32_t pair_capacity(int64_t n) {
    const int64_t e = n * (n - 1) / 2, t = e * (n - 2) / 3;
    return static_cast<int32_t>(std::max<int64_t>({n, e, t, 1}));
}

PersistenceResult unpack(const std::vector<float>& pairs, const int32_t counts[4], int32_t cap) {
    PersistenceResult r;
    auto take = [&](int dim, int cnt, PersistenceDiagram& d) {
        const float* p = pairs.data() + static_cast<size_t>(dim) * cap * 2;
        d.reserve(static_cast<size_t>(cnt));
        for (int i = 0; i < cnt; ++i) d.push_back({static_cast<double>(p[2 * i]), static_cast<double>(p[2 * i + 1])});
    };
    take(0, counts[0], r.dim0);
    for (int i = 0; i < counts[1]; ++i) r.dim0.push_back({0.0, static_cast<double>(std::numeric_limits<float>::infinity())});
    take(1, counts[2], r.dim1);
    take(2, counts[3], r.dim2);
    return r;
}

}  // namespace

PersistenceResult compute_persistence_from_distances(const dgn::MatrixXd& distance_matrix, double threshold,
                                                     unsigned /*num_threads*/) {
    const auto n = distance_matrix.rows();
    if (n != distance_matrix.cols()) throw std::invalid_argument("distance matrix must be square");
    if (n == 0) return {};
    std::vector<float> lower;
    lower.reserve(static_cast<size_t>(n * (n - 1) / 2));
    for (std::ptrdiff_t i = 1; i < n; ++i)
        for (std::ptrdiff_t j = 0; j < i; ++j) lower.push_back(static_cast<float>(distance_matrix(i, j)));
    if (lower.empty()) lower.push_back(0.0F);
    const int32_t cap = pair_capacity(n), np = static_cast<int32_t>(n);
    std::vector<float> pairs(static_cast<size_t>(3) * cap * 2);
    int32_t counts[4] = {0, 0, 0, 0};
    auto& rt = dgn::runtime();
    {
        std::lock_guard<std::mutex> lk(rt.mu);
        dgn::check(dgn_host_persistence_lower(rt.ctx, lower.data(), &np, 1, np, threshold, pairs.data(), cap, counts),
                   "compute_persistence_from_distances");
    }
    return unpack(pairs, counts, cap);
}

PersistenceResult compute_persistence(const dgn::MatrixXd& point_cloud, double threshold, unsigned /*num_threads*/) {
    const auto n = point_cloud.rows();
    if (point_cloud.cols() != 3) throw std::invalid_argument("point cloud must be N x 3");
    if (n == 0) return {};
    std::vector<double> cloud(static_cast<size_t>(3 * n));
    for (std::ptrdiff_t i = 0; i < n; ++i)
        for (int k = 0; k < 3; ++k) cloud[static_cast<size_t>(3 * i + k)] = point_cloud(i, k);
    const int32_t cap = pair_capacity(n), np = static_cast<int32_t>(n);
    std::vector<float> pairs(static_cast<size_t>(3) * cap * 2);
    int32_t counts[4] = {0, 0, 0, 0};
    auto& rt = dgn::runtime();
    {
        std::lock_guard<std::mutex> lk(rt.mu);
        dgn::check(dgn_host_persistence(rt.ctx, cloud.data(), &np, 1, np, threshold, pairs.data(), cap, counts),
                   "compute_persistence");
    }
    return unpack(pairs, counts, cap);
}

}  // namespace defect_gnn::topology
