// graph::CrystalGraph (replaces reference include/graph/crystal_graph.hpp:12-40).
#pragma once
#include <map>

#include "crystal/structure.hpp"
#include "dgn/matrix.hpp"
#include "graph/neighbor_list.hpp"

namespace defect_gnn::graph {

class CrystalGraph {
public:
    CrystalGraph(const crystal::Structure& structure, const NeighborList& neighbors,
                 const std::map<int, dgn::VectorXd>& atom_embeddings, int atom_embedding_dims = 92,
                 double r_cutoff = 10, double dr = 0.1);

    [[nodiscard]] const dgn::MatrixXd& node_features() const;
    [[nodiscard]] const dgn::MatrixXi& edge_index() const;
    [[nodiscard]] const dgn::MatrixXd& edge_attr() const;

    [[nodiscard]] double target() const;
    void set_target(double y);

    // reference: unimplemented TODO (crystal_graph.cpp:65-67); kept as a no-op
    void add_topo_features(const dgn::MatrixXd& topo);

    [[nodiscard]] size_t num_nodes() const;
    [[nodiscard]] size_t num_edges() const;

private:
    dgn::MatrixXd node_features_;
    dgn::MatrixXi edge_index_;
    dgn::MatrixXd edge_attr_;
    double target_ = 0.0;
};

}  // namespace defect_gnn::graph
