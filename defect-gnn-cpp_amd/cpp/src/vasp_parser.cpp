// POSCAR reader — behaviour of reference src/io/vasp_parser.cpp:13-78: scale factor on line 2
// applies to the lattice only; "Direct"/"direct" coordinates are fractional; Cartesian
// coordinates are converted with the inverse lattice (and are not scaled, as in the reference).
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "io/vasp_parser.hpp"

namespace defect_gnn::io {

namespace {
dgn::Matrix3d inverse(const dgn::Matrix3d& a) {
    dgn::Matrix3d r;
    const double c00 = a(1, 1) * a(2, 2) - a(1, 2) * a(2, 1), c01 = a(0, 2) * a(2, 1) - a(0, 1) * a(2, 2),
                 c02 = a(0, 1) * a(1, 2) - a(0, 2) * a(1, 1), c10 = a(1, 2) * a(2, 0) - a(1, 0) * a(2, 2),
                 c11 = a(0, 0) * a(2, 2) - a(0, 2) * a(2, 0), c12 = a(0, 2) * a(1, 0) - a(0, 0) * a(1, 2),
                 c20 = a(1, 0) * a(2, 1) - a(1, 1) * a(2, 0), c21 = a(0, 1) * a(2, 0) - a(0, 0) * a(2, 1),
                 c22 = a(0, 0) * a(1, 1) - a(0, 1) * a(1, 0);
    const double det = a(0, 0) * c00 + a(0, 1) * c10 + a(0, 2) * c20;
    const double c[3][3] = {{c00, c01, c02}, {c10, c11, c12}, {c20, c21, c22}};
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) r(i, j) = c[i][j] / det;
    return r;
}
}  // namespace

VASPStructure parse_vasp(const std::string& filepath) {
    std::ifstream file(filepath);
    if (!file.is_open()) throw std::runtime_error("Could not open file: " + filepath);
    std::vector<std::string> lines;
    std::string line;
    while (std::getline(file, line)) lines.push_back(line);
    if (lines.size() < 8) throw std::runtime_error("Truncated POSCAR: " + filepath);
    VASPStructure v;
    double scale = 1.0;
    std::stringstream(lines[1]) >> scale;
    for (int i = 0; i < 3; ++i) {
        std::stringstream ss(lines[2 + i]);
        ss >> v.lattice(i, 0) >> v.lattice(i, 1) >> v.lattice(i, 2);
    }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) v.lattice(i, j) *= scale;
    {
        std::stringstream ss(lines[5]);
        std::string e;
        while (ss >> e) v.elements.push_back(e);
    }
    {
        std::stringstream ss(lines[6]);
        int c;
        while (ss >> c) v.counts.push_back(c);
    }
    const bool direct = !lines[7].empty() && (lines[7][0] == 'd' || lines[7][0] == 'D');
    int total = 0;
    for (int c : v.counts) total += c;
    if (static_cast<int>(lines.size()) < 8 + total) throw std::runtime_error("Truncated POSCAR: " + filepath);
    v.frac_coords.resize(total, 3);
    v.atom_types.resize(total);
    int idx = 0;
    for (size_t e = 0; e < v.counts.size(); ++e)
        for (int j = 0; j < v.counts[e]; ++j, ++idx) {
            std::stringstream ss(lines[8 + idx]);
            ss >> v.frac_coords(idx, 0) >> v.frac_coords(idx, 1) >> v.frac_coords(idx, 2);
            v.atom_types[idx] = static_cast<int>(e);
        }
    if (!direct) {  // frac = cart * L^-1 (row vector times inverse)
        const dgn::Matrix3d inv = inverse(v.lattice);
        for (int i = 0; i < total; ++i) {
            const double x = v.frac_coords(i, 0), y = v.frac_coords(i, 1), z = v.frac_coords(i, 2);
            for (int k = 0; k < 3; ++k) v.frac_coords(i, k) = x * inv(0, k) + y * inv(1, k) + z * inv(2, k);
        }
    }
    return v;
}

}  // namespace defect_gnn::io
