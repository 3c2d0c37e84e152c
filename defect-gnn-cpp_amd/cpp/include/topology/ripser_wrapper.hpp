// Persistence front end (replaces reference include/topology/ripser_wrapper.hpp:9-31):
// VR persistence up to dim 2 over Z/2 at `threshold`, computed by the wave64 reduction kernel.
// num_threads is accepted and ignored.
#pragma once
#include <vector>

#include "dgn/matrix.hpp"

namespace defect_gnn::topology {

struct PersistencePair {
    double birth;
    double death;
};

[[nodiscard]] inline double persistence(const PersistencePair& p) { return p.death - p.birth; }

using PersistenceDiagram = std::vector<PersistencePair>;

struct PersistenceResult {
    PersistenceDiagram dim0;  // includes (0, inf) per connected component, like Ripser
    PersistenceDiagram dim1;
    PersistenceDiagram dim2;
};

PersistenceResult compute_persistence_from_distances(const dgn::MatrixXd& distance_matrix, double threshold,
                                                     unsigned num_threads);

PersistenceResult compute_persistence(const dgn::MatrixXd& point_cloud, double threshold, unsigned num_threads);

}  // namespace defect_gnn::topology
