// graph::NeighborList (replaces reference include/graph/neighbor_list.hpp:11-71). Rows are
// computed on the GPU (dgn_host_graph); same defaults, same row contents and order (by
// distance; ties in canonical (idx, image) order).
#pragma once
#include <cstddef>
#include <vector>

#include "crystal/structure.hpp"
#include "dgn/matrix.hpp"

namespace defect_gnn::graph {

struct Neighbor {
    size_t idx;
    double distance;
    dgn::Vector3d displacement;
};

class NeighborList {
public:
    explicit NeighborList(const crystal::Structure& structure, double r_cutoff = 10.0,
                          size_t max_neighbors = 20, double epsilon = 1e-10);

    [[nodiscard]] const std::vector<Neighbor>& neighbors(size_t atom_idx) const;

private:
    double r_cutoff_;
    size_t max_neighbors_;
    double epsilon_;
    std::vector<std::vector<Neighbor>> neighbor_lists_;
};

}  // namespace defect_gnn::graph
