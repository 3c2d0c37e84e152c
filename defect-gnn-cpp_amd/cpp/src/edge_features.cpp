// Gaussian RBF expansion on the GPU (dgn_host_rbf), reference src/graph/edge_features.cpp:7-24.
#include <cmath>

#include "dgn/runtime.hpp"
#include "graph/edge_features.hpp"

namespace defect_gnn::graph {

dgn::MatrixXd gaussian_rbf_batch(const std::vector<double>& distances, double r_cutoff, double dr) {
    const int n = dgn_rbf_bins(r_cutoff, dr);
    dgn::MatrixXd out(static_cast<std::ptrdiff_t>(distances.size()), n > 0 ? n : 0);
    if (distances.empty() || n <= 0) return out;
    auto& rt = dgn::runtime();
    std::lock_guard<std::mutex> lk(rt.mu);
    dgn::check(dgn_host_rbf(rt.ctx, distances.data(), static_cast<int64_t>(distances.size()), r_cutoff, dr, DGN_F64,
                            /*layout=*/1, out.data()),
               "gaussian_rbf");
    return out;
}

dgn::VectorXd gaussian_rbf(double distance, double r_cutoff, double dr) {
    const dgn::MatrixXd m = gaussian_rbf_batch({distance}, r_cutoff, dr);
    dgn::VectorXd g(m.cols());
    for (std::ptrdiff_t k = 0; k < m.cols(); ++k) g[k] = m(0, k);
    return g;
}

}  // namespace defect_gnn::graph
