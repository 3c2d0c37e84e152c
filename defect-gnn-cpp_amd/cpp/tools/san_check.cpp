// san_check: host-code sanitizer driver (`make sanitize`, ASan + UBSan). Exercises the CPU
// oracle (test infrastructure) and the facade's host-only code paths (POSCAR parser, Structure,
// PCA fit/transform/save/load) on the committed fixtures and synthetic inputs; GPU entry points
// are not called (no device in the build container). Exit status 0 = clean run.
//   san_check <poscar_dir> <tmp_dir>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>
#include <string>
#include <vector>

#include "crystal/structure.hpp"
#include "io/vasp_parser.hpp"
#include "oracle.h"
#include "topology/pca.hpp"

using namespace defect_gnn;

static int check_structure_oracle(const crystal::Structure& s, double rc) {
    const int64_t n = (int64_t)s.num_atoms();
    std::vector<double> lat(9), pos(3 * n);
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) lat[3 * r + c] = s.lattice()(r, c);
    std::vector<int32_t> sp(n);
    for (int64_t i = 0; i < n; ++i) {
        for (int k = 0; k < 3; ++k) pos[3 * i + k] = s.atoms()[i].position[k];
        sp[i] = s.atoms()[i].element;
    }
    std::vector<int64_t> rp(n + 1);
    const int64_t E = oracle_neighbor_list(lat.data(), pos.data(), n, rc, 20, 1e-10, rp.data(), nullptr, nullptr,
                                           nullptr, nullptr);
    std::vector<int32_t> col(E), img(3 * E);
    std::vector<double> dist(E), disp(3 * E);
    oracle_neighbor_list(lat.data(), pos.data(), n, rc, 20, 1e-10, rp.data(), col.data(), dist.data(), disp.data(),
                         img.data());
    const int nb = oracle_rbf_bins(rc, 0.1);
    std::vector<double> rbf(nb);
    for (int64_t e = 0; e < E; e += 7) oracle_gaussian_rbf(dist[e], rc, 0.1, rbf.data());
    std::vector<double> feat(35 * n);
    std::vector<int32_t> cnt(4 * n);
    if (oracle_structure_betti(lat.data(), pos.data(), sp.data(), n, rc, feat.data(), cnt.data()) != 0) return 1;
    for (double f : feat)
        if (!std::isfinite(f)) return 2;
    return 0;
}

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: san_check <poscar_dir> <tmp_dir>\n");
        return 2;
    }
    const std::string dir = argv[1], tmp = argv[2];
    int bad = 0;
    for (const char* name : {"1", "741", "1046"}) {
        const io::VASPStructure v = io::parse_vasp(dir + "/" + name + ".vasp");
        const crystal::Structure s(v);
        (void)s.compute_distance_matrix();
        bad |= check_structure_oracle(s, 5.0);
    }
    // KAT clouds + random clouds with ties through the restated reduction
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> U(0.0, 3.0);
    for (int c = 0; c < 40; ++c) {
        const int n = 2 + c % 40;
        std::vector<double> cloud(3 * n);
        for (double& x : cloud) x = c % 3 == 0 ? std::floor(U(rng)) : U(rng);
        std::vector<float> lower((size_t)n * (n - 1) / 2);
        oracle_local_distances(cloud.data(), n, lower.data());
        const int cap = n * n * 4 + 16;
        std::vector<float> d0(2 * cap), d1(2 * cap), d2(2 * cap);
        oracle_counts k{};
        int64_t st[8];
        if (oracle_persistence(lower.data(), n, 2.5f, d0.data(), d1.data(), d2.data(), cap, &k, st) != 0) bad |= 4;
        double out[5];
        oracle_statistics(d1.data(), k.n_dim1, 2, 0.5, out);
    }
    // PCA fit / transform / save / load round trip
    dgn::MatrixXd x(300, 35);
    for (int i = 0; i < 300; ++i)
        for (int j = 0; j < 35; ++j) x(i, j) = U(rng) * (1 + j % 5);
    topology::PCA p;
    const dgn::MatrixXd y = p.fit_transform(x, 6);
    p.save(tmp + "/san_pca.bin");
    topology::PCA q;
    q.load(tmp + "/san_pca.bin");
    const dgn::MatrixXd z = q.transform(x);
    for (int i = 0; i < y.rows(); ++i)
        for (int j = 0; j < y.cols(); ++j)
            if (std::fabs(y(i, j) - z(i, j)) > 1e-9) bad |= 8;
    std::printf("san_check %s\n", bad ? "FAILED" : "ok");
    return bad;
}
