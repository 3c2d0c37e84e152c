// graph::CrystalGraph (reference src/graph/crystal_graph.cpp:9-44): node features by species
// embedding lookup, edge_index 2 x E in row order, edge_attr E x n_rbf computed for all edges
// in one GPU call.
#include <stdexcept>

#include "dgn.h"
#include "graph/crystal_graph.hpp"
#include "graph/edge_features.hpp"

namespace defect_gnn::graph {

CrystalGraph::CrystalGraph(const crystal::Structure& structure, const NeighborList& neighbors,
                           const std::map<int, dgn::VectorXd>& atom_embeddings, int atom_embedding_dims,
                           double r_cutoff, double dr) {
    const auto n = static_cast<std::ptrdiff_t>(structure.num_atoms());
    node_features_.resize(n, atom_embedding_dims);
    for (std::ptrdiff_t i = 0; i < n; ++i) {
        const dgn::VectorXd& emb = atom_embeddings.at(structure.atoms()[static_cast<size_t>(i)].element);
        if (emb.size() != atom_embedding_dims) throw std::invalid_argument("CrystalGraph: embedding size mismatch");
        for (std::ptrdiff_t k = 0; k < atom_embedding_dims; ++k) node_features_(i, k) = emb[k];
    }
    std::vector<double> dist;
    std::ptrdiff_t edges = 0;
    for (std::ptrdiff_t i = 0; i < n; ++i) edges += static_cast<std::ptrdiff_t>(neighbors.neighbors(static_cast<size_t>(i)).size());
    edge_index_.resize(2, edges);
    dist.reserve(static_cast<size_t>(edges));
    std::ptrdiff_t e = 0;
    for (std::ptrdiff_t i = 0; i < n; ++i)
        for (const Neighbor& nb : neighbors.neighbors(static_cast<size_t>(i))) {
            edge_index_(0, e) = static_cast<int>(i);
            edge_index_(1, e) = static_cast<int>(nb.idx);
            dist.push_back(nb.distance);
            ++e;
        }
    edge_attr_ = gaussian_rbf_batch(dist, r_cutoff, dr);
    if (edges == 0) edge_attr_.resize(0, dgn_rbf_bins(r_cutoff, dr));
    target_ = 0;
}

const dgn::MatrixXd& CrystalGraph::node_features() const { return node_features_; }
const dgn::MatrixXi& CrystalGraph::edge_index() const { return edge_index_; }
const dgn::MatrixXd& CrystalGraph::edge_attr() const { return edge_attr_; }
double CrystalGraph::target() const { return target_; }
void CrystalGraph::set_target(double y) { target_ = y; }
void CrystalGraph::add_topo_features(const dgn::MatrixXd&) {}
size_t CrystalGraph::num_nodes() const { return static_cast<size_t>(node_features_.rows()); }
size_t CrystalGraph::num_edges() const { return static_cast<size_t>(edge_index_.cols()); }

}  // namespace defect_gnn::graph
