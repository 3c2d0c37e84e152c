// viz::WasmAPI over the C ABI: the graph is NeighborList(r_cutoff, max_neighbors) computed on the
// GPU and flattened there (dgn_host_edge_arrays, edge_arrays_kernel), so the accessors are copies of
// the arrays the device wrote. Same behaviour as reference src/viz/wasm_bindings.cpp:120-294:
// load_structure returns false on any parse error, build_graph without a structure is a no-op,
// accessors without a structure / graph return empty arrays.
#include <cstdint>
#include <limits>
#include <sstream>
#include <stdexcept>

#include "dgn/runtime.hpp"
#include "viz/wasm_api.hpp"

namespace defect_gnn::viz {

io::VASPStructure parse_vasp_string(const std::string& content) {
    io::VASPStructure r;
    std::istringstream in(content);
    std::string line;
    std::getline(in, line);  // comment
    std::getline(in, line);
    const double scale = std::stod(line);  // throws on a malformed scale line
    for (int i = 0; i < 3; ++i) {
        std::getline(in, line);
        std::istringstream ls(line);
        ls >> r.lattice(i, 0) >> r.lattice(i, 1) >> r.lattice(i, 2);
    }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r.lattice(i, j) *= scale;
    std::getline(in, line);
    {
        std::istringstream es(line);
        std::string e;
        while (es >> e) r.elements.push_back(e);
    }
    std::getline(in, line);
    int total = 0;
    {
        std::istringstream cs(line);
        int c = 0;
        while (cs >> c) {
            r.counts.push_back(c);
            total += c;
        }
    }
    std::getline(in, line);  // Direct / Cartesian: the WASM reader takes fractional coordinates
    r.frac_coords.resize(total, 3);
    r.atom_types.resize(static_cast<size_t>(total));
    int idx = 0;
    for (size_t t = 0; t < r.counts.size(); ++t)
        for (int i = 0; i < r.counts[t]; ++i, ++idx) {
            std::getline(in, line);
            std::istringstream ps(line);
            ps >> r.frac_coords(idx, 0) >> r.frac_coords(idx, 1) >> r.frac_coords(idx, 2);
            r.atom_types[static_cast<size_t>(idx)] = static_cast<int>(t);
        }
    return r;
}

bool WasmAPI::load_structure(const std::string& vasp_content) {
    try {
        vasp_ = std::make_unique<io::VASPStructure>(parse_vasp_string(vasp_content));
        structure_ = std::make_unique<crystal::Structure>(*vasp_);
        edges_.reset();
        return true;
    } catch (const std::exception&) {
        return false;
    }
}

void WasmAPI::build_graph(double r_cutoff, size_t max_neighbors) {
    if (!structure_) return;
    const auto n = static_cast<int64_t>(structure_->num_atoms());
    std::vector<double> lattice(9), pos(static_cast<size_t>(3 * n));
    std::vector<int32_t> species(static_cast<size_t>(n));
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) lattice[static_cast<size_t>(3 * r + c)] = structure_->lattice()(r, c);
    for (int64_t i = 0; i < n; ++i) {
        const auto& a = structure_->atoms()[static_cast<size_t>(i)];
        for (int k = 0; k < 3; ++k) pos[static_cast<size_t>(3 * i + k)] = a.position[k];
        species[static_cast<size_t>(i)] = a.element;
    }
    const int64_t offs[2] = {0, n};
    const dgn_batch batch{1, n, lattice.data(), pos.data(), species.data(), offs};
    const uint64_t k = max_neighbors == std::numeric_limits<size_t>::max() ? UINT64_MAX : max_neighbors;
    auto& rt = dgn::runtime();
    dgn_edge_arrays* ea = nullptr;
    {
        std::lock_guard<std::mutex> lk(rt.mu);
        dgn::check(dgn_host_edge_arrays(rt.ctx, &batch, r_cutoff, k, 1e-10, &ea), "WasmAPI::build_graph");
    }
    std::unique_ptr<dgn_edge_arrays, void (*)(dgn_edge_arrays*)> guard(ea, dgn_edge_arrays_free);
    auto e = std::make_unique<Edges>();
    const auto E = static_cast<size_t>(ea->num_edges);
    e->sources.assign(ea->sources, ea->sources + E);
    e->targets.assign(ea->targets, ea->targets + E);
    e->distances.assign(ea->distances, ea->distances + E);
    e->displacements.assign(ea->displacements, ea->displacements + 3 * E);
    edges_ = std::move(e);
}

size_t WasmAPI::num_atoms() const { return structure_ ? structure_->num_atoms() : 0; }

std::vector<float> WasmAPI::get_positions() const {
    std::vector<float> out;
    if (!structure_) return out;
    out.reserve(3 * structure_->num_atoms());
    for (const auto& a : structure_->atoms())
        for (int k = 0; k < 3; ++k) out.push_back(static_cast<float>(a.position[k]));
    return out;
}

std::vector<int> WasmAPI::get_atom_types() const { return vasp_ ? vasp_->atom_types : std::vector<int>{}; }
std::vector<std::string> WasmAPI::get_elements() const {
    return vasp_ ? vasp_->elements : std::vector<std::string>{};
}
std::vector<int> WasmAPI::get_element_counts() const { return vasp_ ? vasp_->counts : std::vector<int>{}; }

std::vector<float> WasmAPI::get_lattice_vectors() const {
    std::vector<float> out;
    if (!structure_) return out;
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) out.push_back(static_cast<float>(structure_->lattice()(i, j)));
    return out;
}

size_t WasmAPI::num_edges() const { return edges_ && structure_ ? edges_->sources.size() : 0; }
std::vector<int> WasmAPI::get_edge_sources() const {
    return edges_ && structure_ ? edges_->sources : std::vector<int>{};
}
std::vector<int> WasmAPI::get_edge_targets() const {
    return edges_ && structure_ ? edges_->targets : std::vector<int>{};
}
std::vector<float> WasmAPI::get_edge_distances() const {
    return edges_ && structure_ ? edges_->distances : std::vector<float>{};
}
std::vector<float> WasmAPI::get_edge_displacements() const {
    return edges_ && structure_ ? edges_->displacements : std::vector<float>{};
}

}  // namespace defect_gnn::viz
