// crystal::Structure (replaces reference include/crystal/structure.hpp:19-38).
#pragma once
#include <map>
#include <vector>

#include "dgn/matrix.hpp"
#include "io/vasp_parser.hpp"

namespace defect_gnn::crystal {

class Atom {
public:
    int element;
    dgn::Vector3d position;
    dgn::Vector3d frac_position;
};

class Structure {
public:
    explicit Structure(const io::VASPStructure& vasp);
    // direct construction from Cartesian positions (synthetic batches)
    Structure(const dgn::Matrix3d& lattice, const std::vector<dgn::Vector3d>& positions,
              const std::vector<int>& species);

    [[nodiscard]] const dgn::Matrix3d& lattice() const;
    [[nodiscard]] const std::vector<Atom>& atoms() const;
    [[nodiscard]] size_t num_atoms() const;

    [[nodiscard]] double distance(size_t i, size_t j) const;
    [[nodiscard]] dgn::Vector3d displacement(size_t i, size_t j) const;
    [[nodiscard]] dgn::MatrixXd compute_distance_matrix() const;

    [[nodiscard]] int count(int element) const;  // throws std::out_of_range (structure.cpp:49)

private:
    dgn::Matrix3d lattice_;
    dgn::Matrix3d inv_lattice_;
    std::vector<Atom> atoms_;
    std::map<int, int> counts_;
};

}  // namespace defect_gnn::crystal
