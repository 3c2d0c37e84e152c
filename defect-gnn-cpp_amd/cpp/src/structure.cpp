// crystal::Structure — behaviour of reference src/crystal/structure.cpp:7-66. Input-model
// construction on the host (positions = L^T * frac); the hot path consumes positions on the GPU.
#include <cmath>
#include <stdexcept>

#include "crystal/structure.hpp"

namespace defect_gnn::crystal {

namespace {
// L^T * f with the fixed-size redux order x0 + (x1 + x2) (Eigen 3.4; unpinned)
dgn::Vector3d lt_times(const dgn::Matrix3d& L, const double f[3]) {
    dgn::Vector3d p;
    for (int k = 0; k < 3; ++k) p[k] = L(0, k) * f[0] + (L(1, k) * f[1] + L(2, k) * f[2]);
    return p;
}
dgn::Matrix3d inverse3(const dgn::Matrix3d& a) {
    dgn::Matrix3d r;
    const double det = a(0, 0) * (a(1, 1) * a(2, 2) - a(1, 2) * a(2, 1)) -
                       a(0, 1) * (a(1, 0) * a(2, 2) - a(1, 2) * a(2, 0)) +
                       a(0, 2) * (a(1, 0) * a(2, 1) - a(1, 1) * a(2, 0));
    r(0, 0) = (a(1, 1) * a(2, 2) - a(1, 2) * a(2, 1)) / det;
    r(0, 1) = (a(0, 2) * a(2, 1) - a(0, 1) * a(2, 2)) / det;
    r(0, 2) = (a(0, 1) * a(1, 2) - a(0, 2) * a(1, 1)) / det;
    r(1, 0) = (a(1, 2) * a(2, 0) - a(1, 0) * a(2, 2)) / det;
    r(1, 1) = (a(0, 0) * a(2, 2) - a(0, 2) * a(2, 0)) / det;
    r(1, 2) = (a(0, 2) * a(1, 0) - a(0, 0) * a(1, 2)) / det;
    r(2, 0) = (a(1, 0) * a(2, 1) - a(1, 1) * a(2, 0)) / det;
    r(2, 1) = (a(0, 1) * a(2, 0) - a(0, 0) * a(2, 1)) / det;
    r(2, 2) = (a(0, 0) * a(1, 1) - a(0, 1) * a(1, 0)) / det;
    return r;
}
}  // namespace

Structure::Structure(const io::VASPStructure& vasp) : lattice_(vasp.lattice), inv_lattice_(inverse3(vasp.lattice)) {
    for (size_t e = 0; e < vasp.counts.size(); ++e) counts_[static_cast<int>(e)] = vasp.counts[e];
    for (std::ptrdiff_t i = 0; i < vasp.frac_coords.rows(); ++i) {
        Atom a;
        a.element = vasp.atom_types[static_cast<size_t>(i)];
        const double f[3] = {vasp.frac_coords(i, 0), vasp.frac_coords(i, 1), vasp.frac_coords(i, 2)};
        a.frac_position = dgn::Vector3d(f[0], f[1], f[2]);
        a.position = lt_times(lattice_, f);
        atoms_.push_back(a);
    }
}

Structure::Structure(const dgn::Matrix3d& lattice, const std::vector<dgn::Vector3d>& positions,
                     const std::vector<int>& species)
    : lattice_(lattice), inv_lattice_(inverse3(lattice)) {
    if (positions.size() != species.size()) throw std::invalid_argument("Structure: positions/species size mismatch");
    for (size_t i = 0; i < positions.size(); ++i) {
        Atom a;
        a.element = species[i];
        a.position = positions[i];
        // frac = pos * L^-1 (row vector)
        for (int k = 0; k < 3; ++k)
            a.frac_position[k] = positions[i][0] * inv_lattice_(0, k) + positions[i][1] * inv_lattice_(1, k) +
                                 positions[i][2] * inv_lattice_(2, k);
        counts_[species[i]] += 1;
        atoms_.push_back(a);
    }
}

const dgn::Matrix3d& Structure::lattice() const { return lattice_; }
const std::vector<Atom>& Structure::atoms() const { return atoms_; }
size_t Structure::num_atoms() const { return atoms_.size(); }

dgn::Vector3d Structure::displacement(size_t i, size_t j) const {  // minimum image (structure.cpp:38-46)
    double df[3];
    for (int k = 0; k < 3; ++k) {
        df[k] = atoms_.at(j).frac_position[k] - atoms_.at(i).frac_position[k];
        df[k] -= std::round(df[k]);
    }
    return lt_times(lattice_, df);
}

double Structure::distance(size_t i, size_t j) const {
    const dgn::Vector3d d = displacement(i, j);
    return std::sqrt(d[0] * d[0] + (d[1] * d[1] + d[2] * d[2]));
}

int Structure::count(int element) const { return counts_.at(element); }

dgn::MatrixXd Structure::compute_distance_matrix() const {
    const auto n = static_cast<std::ptrdiff_t>(atoms_.size());
    dgn::MatrixXd d(n, n);
    for (std::ptrdiff_t i = 0; i < n; ++i)
        for (std::ptrdiff_t j = i + 1; j < n; ++j) d(i, j) = d(j, i) = distance(static_cast<size_t>(i), static_cast<size_t>(j));
    return d;
}

}  // namespace defect_gnn::crystal
