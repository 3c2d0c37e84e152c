// POSCAR reader (replaces io::parse_vasp, reference src/io/vasp_parser.cpp:13-78).
#pragma once
#include <string>
#include <vector>

#include "dgn/matrix.hpp"

namespace defect_gnn::io {

struct VASPStructure {
    dgn::Matrix3d lattice;  // rows a, b, c (scaled by the POSCAR scale factor)
    std::vector<std::string> elements;
    std::vector<int> counts;
    dgn::MatrixXd frac_coords;  // N x 3
    std::vector<int> atom_types;  // species index per atom
};

// Throws std::runtime_error if the file cannot be opened (vasp_parser.cpp:15-17).
VASPStructure parse_vasp(const std::string& filepath);

}  // namespace defect_gnn::io
