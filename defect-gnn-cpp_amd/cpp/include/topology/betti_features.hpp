// Per-atom 35-d topological descriptor (replaces reference include/topology/betti_features.hpp).
#pragma once
#include <string>
#include <vector>

#include "crystal/structure.hpp"
#include "dgn/matrix.hpp"
#include "graph/neighbor_list.hpp"
#include "topology/ripser_wrapper.hpp"

namespace defect_gnn::topology {

static constexpr int BETTI_FEATURE_DIM = 35;

struct BettiStatistics {
    double mean = 0.0;
    double std = 0.0;
    double max = 0.0;
    double min = 0.0;
    double weighted_sum = 0.0;
};

inline void append_to(BettiStatistics stats, std::vector<double>& vec) {
    vec.insert(vec.end(), {stats.mean, stats.std, stats.max, stats.min, stats.weighted_sum});
}

// values_type: "birth", "death" or "persistence"; infinite deaths are skipped
BettiStatistics compute_statistics(const PersistenceDiagram& diagram, const std::string& values_type,
                                   double weight = 1.0);

dgn::VectorXd compute_atom_betti_features(const crystal::Structure& structure, size_t atom_idx,
                                          const graph::NeighborList& neighbor_list, double r_cutoff,
                                          unsigned num_threads);

// N x 35, column-major (reference MatrixXd layout); batched on the GPU
dgn::MatrixXd compute_structure_betti_features(const crystal::Structure& structure, double r_cutoff = 10,
                                               unsigned num_threads = 8);

// many structures in one GPU batch (the preprocess driver's path)
std::vector<dgn::MatrixXd> compute_batch_betti_features(const std::vector<const crystal::Structure*>& structures,
                                                        double r_cutoff = 10);

// binary: int32 rows, int32 cols, rows*cols f64 column-major (betti_features.cpp:121-153)
void save_betti_features(const std::string& filepath, const dgn::MatrixXd& features);
dgn::MatrixXd load_betti_features(const std::string& filepath);

}  // namespace defect_gnn::topology
