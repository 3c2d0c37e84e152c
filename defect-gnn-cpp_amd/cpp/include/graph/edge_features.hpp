// Gaussian RBF expansion (replaces reference include/graph/edge_features.hpp:14):
// n = floor(r_cutoff / dr) bins, sigma = r_cutoff / 3, g[k] = exp(-0.5 (k dr - d)^2 / sigma^2)
// / (sigma sqrt(2 pi)). Evaluated on the GPU; for many edges use gaussian_rbf_batch.
#pragma once
#include <vector>

#include "dgn/matrix.hpp"

namespace defect_gnn::graph {

dgn::VectorXd gaussian_rbf(double distance, double r_cutoff, double dr);
// E x n_rbf, column-major like Eigen's MatrixXd (CrystalGraph::edge_attr layout)
dgn::MatrixXd gaussian_rbf_batch(const std::vector<double>& distances, double r_cutoff, double dr);

}  // namespace defect_gnn::graph
