// graph::NeighborList over the GPU neighbour kernels (dgn_host_graph). Row contents and order
// match reference src/graph/neighbor_list.cpp:14-94 (see DESIGN.md for the tie order).
#include <cstdint>
#include <limits>
#include <memory>
#include <stdexcept>

#include "dgn/runtime.hpp"
#include "graph/neighbor_list.hpp"

namespace defect_gnn::graph {

NeighborList::NeighborList(const crystal::Structure& structure, double r_cutoff, size_t max_neighbors,
                           double epsilon)
    : r_cutoff_(r_cutoff), max_neighbors_(max_neighbors), epsilon_(epsilon) {
    const auto n = static_cast<int64_t>(structure.num_atoms());
    neighbor_lists_.resize(static_cast<size_t>(n));
    if (n == 0) return;
    std::vector<double> lattice(9), pos(static_cast<size_t>(3 * n));
    std::vector<int32_t> species(static_cast<size_t>(n));
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) lattice[static_cast<size_t>(3 * r + c)] = structure.lattice()(r, c);
    for (int64_t i = 0; i < n; ++i) {
        const auto& a = structure.atoms()[static_cast<size_t>(i)];
        for (int k = 0; k < 3; ++k) pos[static_cast<size_t>(3 * i + k)] = a.position[k];
        species[static_cast<size_t>(i)] = a.element;
    }
    const int64_t offs[2] = {0, n};
    const dgn_batch batch{1, n, lattice.data(), pos.data(), species.data(), offs};
    dgn_graph_params p;
    dgn_graph_params_default(&p);
    p.r_cutoff = r_cutoff;
    p.max_neighbors = max_neighbors == std::numeric_limits<size_t>::max() ? UINT64_MAX : max_neighbors;
    p.epsilon = epsilon;
    p.rbf_dtype = DGN_NONE;
    p.write_displacement = 1;
    auto& rt = dgn::runtime();
    dgn_graph_result* res = nullptr;
    {
        std::lock_guard<std::mutex> lk(rt.mu);
        dgn::check(dgn_host_graph(rt.ctx, &batch, &p, &res), "NeighborList");
    }
    std::unique_ptr<dgn_graph_result, void (*)(dgn_graph_result*)> guard(res, dgn_graph_result_free);
    for (int64_t i = 0; i < n; ++i) {
        auto& row = neighbor_lists_[static_cast<size_t>(i)];
        row.reserve(static_cast<size_t>(res->row_ptr[i + 1] - res->row_ptr[i]));
        for (int64_t e = res->row_ptr[i]; e < res->row_ptr[i + 1]; ++e)
            row.push_back(Neighbor{static_cast<size_t>(res->col_idx[e]), res->distance[e],
                                   dgn::Vector3d(res->displacement[3 * e], res->displacement[3 * e + 1],
                                                 res->displacement[3 * e + 2])});
    }
}

const std::vector<Neighbor>& NeighborList::neighbors(size_t atom_idx) const {
    return neighbor_lists_.at(atom_idx);
}

}  // namespace defect_gnn::graph
