// viz::WasmAPI (replaces reference include/viz/wasm_api.hpp + src/viz/wasm_bindings.cpp:120-294,
// without the emscripten bindings): load a POSCAR string, build the neighbour graph on the GPU and
// read the structure / edges back as flat float32 / int arrays. build_graph runs NeighborList +
// the flat-array pass on the device (dgn_host_edge_arrays) and keeps the arrays; the accessors
// return copies, like the reference's.
#pragma once
#include <cstddef>
#include <memory>
#include <string>
#include <vector>

#include "crystal/structure.hpp"
#include "io/vasp_parser.hpp"

namespace defect_gnn::viz {

// The WASM path's own POSCAR reader (wasm_bindings.cpp:14-118): coordinates always fractional.
io::VASPStructure parse_vasp_string(const std::string& content);

class WasmAPI {
public:
    WasmAPI() = default;

    bool load_structure(const std::string& vasp_content);
    void build_graph(double r_cutoff, size_t max_neighbors);

    // === Structure accessors (unit cell) ===
    [[nodiscard]] size_t num_atoms() const;
    [[nodiscard]] std::vector<float> get_positions() const;
    [[nodiscard]] std::vector<int> get_atom_types() const;
    [[nodiscard]] std::vector<std::string> get_elements() const;
    [[nodiscard]] std::vector<int> get_element_counts() const;
    [[nodiscard]] std::vector<float> get_lattice_vectors() const;

    // === Graph accessors (edges) ===
    [[nodiscard]] size_t num_edges() const;
    [[nodiscard]] std::vector<int> get_edge_sources() const;
    [[nodiscard]] std::vector<int> get_edge_targets() const;
    [[nodiscard]] std::vector<float> get_edge_distances() const;
    [[nodiscard]] std::vector<float> get_edge_displacements() const;

private:
    struct Edges {
        std::vector<int> sources, targets;
        std::vector<float> distances, displacements;
    };
    std::unique_ptr<io::VASPStructure> vasp_;
    std::unique_ptr<crystal::Structure> structure_;
    std::unique_ptr<Edges> edges_;
};

}  // namespace defect_gnn::viz
