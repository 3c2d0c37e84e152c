// Per-atom 35-d topological descriptor; reference src/topology/betti_features.cpp:24-153.
// compute_structure_betti_features and the batched variant run the whole chain (neighbour
// search, local VR persistence, statistics) in the fused GPU kernels (dgn_host_betti);
// compute_statistics / compute_atom_betti_features keep the reference's single-atom API.
#include <cmath>
#include <fstream>
#include <limits>
#include <stdexcept>

#include "dgn/runtime.hpp"
#include "topology/betti_features.hpp"

namespace defect_gnn::topology {

BettiStatistics compute_statistics(const PersistenceDiagram& diagram, const std::string& values_type,
                                   double weight) {
    std::vector<double> v;
    for (const PersistencePair& p : diagram) {
        if (p.death == INFINITY) continue;  // betti_features.cpp:30-32
        if (values_type == "birth")
            v.push_back(p.birth);
        else if (values_type == "death")
            v.push_back(p.death);
        else if (values_type == "persistence")
            v.push_back(persistence(p));
    }
    if (v.empty()) return {};
    double sum = 0.0, mx = v[0], mn = v[0];
    for (double x : v) {
        sum += x;
        mx = x > mx ? x : mx;
        mn = x < mn ? x : mn;
    }
    const double mean = sum / static_cast<double>(v.size());
    double ss = 0.0;
    for (double x : v) ss += (x - mean) * (x - mean);
    return {mean, std::sqrt(ss / static_cast<double>(v.size())), mx, mn, sum * weight};  // utils/math.hpp:9-27
}

dgn::VectorXd compute_atom_betti_features(const crystal::Structure& structure, size_t atom_idx,
                                          const graph::NeighborList& neighbor_list, double r_cutoff,
                                          unsigned num_threads) {
    const crystal::Atom& centre = structure.atoms().at(atom_idx);
    const int element_count = structure.count(centre.element);
    const auto& nb = neighbor_list.neighbors(atom_idx);
    dgn::MatrixXd cloud(static_cast<std::ptrdiff_t>(nb.size() + 1), 3);
    for (int k = 0; k < 3; ++k) cloud(0, k) = centre.position[k];
    for (size_t i = 0; i < nb.size(); ++i)
        for (int k = 0; k < 3; ++k)
            cloud(static_cast<std::ptrdiff_t>(i + 1), k) = centre.position[k] + nb[i].displacement[k];
    const PersistenceResult r = compute_persistence(cloud, r_cutoff, num_threads);
    const double weight = 1.0 / element_count;
    std::vector<double> f;
    f.reserve(BETTI_FEATURE_DIM);
    append_to(compute_statistics(r.dim0, "death", weight), f);
    for (const char* t : {"persistence", "birth", "death"}) append_to(compute_statistics(r.dim1, t, weight), f);
    for (const char* t : {"persistence", "birth", "death"}) append_to(compute_statistics(r.dim2, t, weight), f);
    dgn::VectorXd out(BETTI_FEATURE_DIM);
    for (int k = 0; k < BETTI_FEATURE_DIM; ++k) out[k] = f[static_cast<size_t>(k)];
    return out;
}

std::vector<dgn::MatrixXd> compute_batch_betti_features(const std::vector<const crystal::Structure*>& structures,
                                                        double r_cutoff) {
    const auto B = static_cast<int64_t>(structures.size());
    std::vector<int64_t> offs(static_cast<size_t>(B + 1), 0);
    for (int64_t s = 0; s < B; ++s) offs[static_cast<size_t>(s + 1)] = offs[static_cast<size_t>(s)] +
                                                                      static_cast<int64_t>(structures[static_cast<size_t>(s)]->num_atoms());
    const int64_t A = offs.back();
    std::vector<dgn::MatrixXd> out;
    out.reserve(static_cast<size_t>(B));
    if (A == 0) {
        for (int64_t s = 0; s < B; ++s) out.emplace_back(0, BETTI_FEATURE_DIM);
        return out;
    }
    std::vector<double> lattice(static_cast<size_t>(9 * B)), pos(static_cast<size_t>(3 * A));
    std::vector<int32_t> species(static_cast<size_t>(A));
    for (int64_t s = 0; s < B; ++s) {
        const crystal::Structure& st = *structures[static_cast<size_t>(s)];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) lattice[static_cast<size_t>(9 * s + 3 * r + c)] = st.lattice()(r, c);
        for (size_t i = 0; i < st.num_atoms(); ++i) {
            const auto a = static_cast<size_t>(offs[static_cast<size_t>(s)]) + i;
            for (int k = 0; k < 3; ++k) pos[3 * a + static_cast<size_t>(k)] = st.atoms()[i].position[k];
            species[a] = st.atoms()[i].element;
        }
    }
    const dgn_batch batch{B, A, lattice.data(), pos.data(), species.data(), offs.data()};
    const dgn_betti_params p{r_cutoff};
    std::vector<double> feat(static_cast<size_t>(A) * BETTI_FEATURE_DIM);
    auto& rt = dgn::runtime();
    {
        std::lock_guard<std::mutex> lk(rt.mu);
        dgn::check(dgn_host_betti(rt.ctx, &batch, &p, feat.data(), nullptr), "compute_structure_betti_features");
    }
    for (int64_t s = 0; s < B; ++s) {
        const int64_t n = offs[static_cast<size_t>(s + 1)] - offs[static_cast<size_t>(s)];
        dgn::MatrixXd m(n, BETTI_FEATURE_DIM);
        for (int64_t i = 0; i < n; ++i)
            for (int k = 0; k < BETTI_FEATURE_DIM; ++k)
                m(i, k) = feat[static_cast<size_t>((offs[static_cast<size_t>(s)] + i) * BETTI_FEATURE_DIM + k)];
        out.push_back(std::move(m));
    }
    return out;
}

dgn::MatrixXd compute_structure_betti_features(const crystal::Structure& structure, double r_cutoff,
                                               unsigned /*num_threads*/) {
    return std::move(compute_batch_betti_features({&structure}, r_cutoff)[0]);
}

void save_betti_features(const std::string& filepath, const dgn::MatrixXd& features) {
    std::ofstream file(filepath, std::ios::binary);
    if (!file) throw std::runtime_error("Cannot open file for writing: " + filepath);
    const auto rows = static_cast<int32_t>(features.rows()), cols = static_cast<int32_t>(features.cols());
    file.write(reinterpret_cast<const char*>(&rows), sizeof rows);
    file.write(reinterpret_cast<const char*>(&cols), sizeof cols);
    file.write(reinterpret_cast<const char*>(features.data()),
               static_cast<std::streamsize>(static_cast<size_t>(rows) * static_cast<size_t>(cols) * sizeof(double)));
}

dgn::MatrixXd load_betti_features(const std::string& filepath) {
    std::ifstream file(filepath, std::ios::binary);
    if (!file) throw std::runtime_error("Cannot open file for reading: " + filepath);
    int32_t rows = 0, cols = 0;
    file.read(reinterpret_cast<char*>(&rows), sizeof rows);
    file.read(reinterpret_cast<char*>(&cols), sizeof cols);
    if (!file || rows < 0 || cols < 0) throw std::runtime_error("Corrupt Betti feature file: " + filepath);
    dgn::MatrixXd m(rows, cols);
    file.read(reinterpret_cast<char*>(m.data()),
              static_cast<std::streamsize>(static_cast<size_t>(rows) * static_cast<size_t>(cols) * sizeof(double)));
    if (!file) throw std::runtime_error("Truncated Betti feature file: " + filepath);
    return m;
}

}  // namespace defect_gnn::topology
