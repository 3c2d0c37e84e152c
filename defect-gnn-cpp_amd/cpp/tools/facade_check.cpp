// facade_check — exercises the C++ facade end to end on one POSCAR and dumps every result as
// text ("<key> <count> v0 v1 ...", %.17g) for tests/test_gpu_facade.py to compare with the oracle.
//   facade_check <poscar> <r_cutoff> <max_neighbors> <out.txt>   (GPU: graph, Betti, persistence)
//   facade_check parse <poscar> <out.txt>                           (host: POSCAR -> Structure)
//   facade_check pca <features.bin> <n_components> <out.txt>        (host: load_betti_features + PCA)
#include <cmath>
#include <cstdio>
#include <fstream>
#include <sstream>
#include <limits>
#include <map>
#include <string>
#include <vector>

#include "crystal/structure.hpp"
#include "graph/crystal_graph.hpp"
#include "graph/edge_features.hpp"
#include "graph/neighbor_list.hpp"
#include "io/vasp_parser.hpp"
#include "topology/betti_features.hpp"
#include "topology/pca.hpp"
#include "topology/ripser_wrapper.hpp"
#include "viz/wasm_api.hpp"

using namespace defect_gnn;

static void dump(FILE* f, const char* key, const std::vector<double>& v) {
    std::fprintf(f, "%s %zu", key, v.size());
    for (double x : v) std::fprintf(f, " %.17g", x);
    std::fprintf(f, "\n");
}

static int host_modes(int argc, char** argv) {
    const std::string mode = argv[1];
    if (mode == "parse" && argc == 4) {
        const io::VASPStructure v = io::parse_vasp(argv[2]);
        const crystal::Structure s(v);
        FILE* f = std::fopen(argv[3], "w");
        if (!f) return 3;
        std::vector<double> lat, pos, frac, sp, cnt;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) lat.push_back(s.lattice()(r, c));
        for (const auto& a : s.atoms()) {
            for (int k = 0; k < 3; ++k) pos.push_back(a.position[k]);
            for (int k = 0; k < 3; ++k) frac.push_back(a.frac_position[k]);
            sp.push_back(a.element);
        }
        for (size_t e = 0; e < v.elements.size(); ++e) cnt.push_back(s.count(static_cast<int>(e)));
        dump(f, "lattice", lat);
        dump(f, "positions", pos);
        dump(f, "frac", frac);
        dump(f, "species", sp);
        dump(f, "counts", cnt);
        const dgn::MatrixXd dm = s.compute_distance_matrix();
        dump(f, "distance_matrix", std::vector<double>(dm.data(), dm.data() + dm.size()));
        std::fclose(f);
        return 0;
    }
    if (mode == "pca" && argc == 5) {
        const dgn::MatrixXd x = topology::load_betti_features(argv[2]);
        topology::PCA pca;
        const dgn::MatrixXd t = pca.fit_transform(x, std::stoi(argv[3]));
        const std::string model = std::string(argv[4]) + ".pca_model.bin";
        pca.save(model);
        topology::PCA back;
        back.load(model);
        FILE* f = std::fopen(argv[4], "w");
        if (!f) return 3;
        dump(f, "mean", std::vector<double>(pca.mean().data(), pca.mean().data() + pca.mean().size()));
        dump(f, "components", std::vector<double>(back.components().data(), back.components().data() + back.components().size()));
        dump(f, "ratio", std::vector<double>(back.explained_variance_ratio().data(),
                                              back.explained_variance_ratio().data() + back.explained_variance_ratio().size()));
        dump(f, "transform", std::vector<double>(t.data(), t.data() + t.size()));
        std::fclose(f);
        return 0;
    }
    return -1;
}

// facade_check wasm <poscar> <r_cutoff> <max_neighbors> <out.txt>: viz::WasmAPI end to end (GPU)
static int wasm_mode(char** argv) {
    std::ifstream in(argv[2]);
    if (!in) return 3;
    std::stringstream ss;
    ss << in.rdbuf();
    viz::WasmAPI api;
    if (!api.load_structure(ss.str())) return 4;
    viz::WasmAPI empty;
    empty.build_graph(5.0, 20);  // no structure: no-op, empty accessors
    if (empty.num_edges() != 0 || !empty.get_positions().empty() || empty.load_structure("garbage\nx\n")) return 5;
    api.build_graph(std::stod(argv[3]), static_cast<size_t>(std::stoul(argv[4])));
    FILE* f = std::fopen(argv[5], "w");
    if (!f) return 3;
    auto fl = [](const std::vector<float>& v) { return std::vector<double>(v.begin(), v.end()); };
    auto in_ = [](const std::vector<int>& v) { return std::vector<double>(v.begin(), v.end()); };
    dump(f, "num_atoms", {static_cast<double>(api.num_atoms())});
    dump(f, "num_edges", {static_cast<double>(api.num_edges())});
    dump(f, "positions", fl(api.get_positions()));
    dump(f, "lattice", fl(api.get_lattice_vectors()));
    dump(f, "atom_types", in_(api.get_atom_types()));
    dump(f, "element_counts", in_(api.get_element_counts()));
    dump(f, "sources", in_(api.get_edge_sources()));
    dump(f, "targets", in_(api.get_edge_targets()));
    dump(f, "distances", fl(api.get_edge_distances()));
    dump(f, "displacements", fl(api.get_edge_displacements()));
    std::fclose(f);
    return 0;
}

int main(int argc, char** argv) {
    if (argc == 6 && std::string(argv[1]) == "wasm") {
        try {
            return wasm_mode(argv);
        } catch (const std::exception& e) {
            std::fprintf(stderr, "facade_check: %s\n", e.what());
            return 1;
        }
    }
    if (argc >= 2 && (std::string(argv[1]) == "parse" || std::string(argv[1]) == "pca")) {
        try {
            const int rc = host_modes(argc, argv);
            if (rc >= 0) return rc;
        } catch (const std::exception& e) {
            std::fprintf(stderr, "facade_check: %s\n", e.what());
            return 1;
        }
    }
    if (argc != 5) {
        std::fprintf(stderr, "usage: facade_check <poscar> <r_cutoff> <max_neighbors> <out.txt>\n");
        return 2;
    }
    try {
        const double rc = std::stod(argv[2]);
        const size_t K = static_cast<size_t>(std::stoul(argv[3]));
        const io::VASPStructure v = io::parse_vasp(argv[1]);
        const crystal::Structure s(v);
        FILE* f = std::fopen(argv[4], "w");
        if (!f) return 3;
        std::vector<double> lat, pos, sp;
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) lat.push_back(s.lattice()(r, c));
        for (const auto& a : s.atoms()) {
            for (int k = 0; k < 3; ++k) pos.push_back(a.position[k]);
            sp.push_back(a.element);
        }
        dump(f, "lattice", lat);
        dump(f, "positions", pos);
        dump(f, "species", sp);

        const graph::NeighborList nl(s, rc, K);
        std::vector<double> rp{0}, col, dist, disp;
        for (size_t i = 0; i < s.num_atoms(); ++i) {
            for (const auto& nb : nl.neighbors(i)) {
                col.push_back(static_cast<double>(nb.idx));
                dist.push_back(nb.distance);
                for (int k = 0; k < 3; ++k) disp.push_back(nb.displacement[k]);
            }
            rp.push_back(static_cast<double>(col.size()));
        }
        dump(f, "row_ptr", rp);
        dump(f, "col", col);
        dump(f, "dist", dist);
        dump(f, "disp", disp);

        std::map<int, dgn::VectorXd> emb;
        for (size_t e = 0; e < v.elements.size(); ++e) {
            dgn::VectorXd x(4);
            for (int k = 0; k < 4; ++k) x[k] = 10.0 * static_cast<double>(e) + k;
            emb[static_cast<int>(e)] = x;
        }
        const graph::CrystalGraph g(s, nl, emb, 4, rc, 0.1);
        dump(f, "node_features", std::vector<double>(g.node_features().data(), g.node_features().data() + g.node_features().size()));
        std::vector<double> ei;
        for (std::ptrdiff_t k = 0; k < g.edge_index().size(); ++k) ei.push_back(g.edge_index().data()[k]);
        dump(f, "edge_index", ei);
        dump(f, "edge_attr", std::vector<double>(g.edge_attr().data(), g.edge_attr().data() + g.edge_attr().size()));
        const dgn::VectorXd one = graph::gaussian_rbf(1.2345, rc, 0.1);
        dump(f, "rbf_one", std::vector<double>(one.data(), one.data() + one.size()));

        const dgn::MatrixXd feat = topology::compute_structure_betti_features(s, rc, 8);
        dump(f, "betti", std::vector<double>(feat.data(), feat.data() + feat.size()));

        // single-atom path (reference call sequence) for atom 0
        const graph::NeighborList nl_all(s, rc, std::numeric_limits<size_t>::max());
        const dgn::VectorXd a0 = topology::compute_atom_betti_features(s, 0, nl_all, rc, 1);
        dump(f, "atom0", std::vector<double>(a0.data(), a0.data() + a0.size()));
        // persistence from an explicit distance matrix (atom 0's local cloud)
        const auto& nb0 = nl_all.neighbors(0);
        dgn::MatrixXd cloud(static_cast<std::ptrdiff_t>(nb0.size() + 1), 3);
        for (int k = 0; k < 3; ++k) cloud(0, k) = s.atoms()[0].position[k];
        for (size_t i = 0; i < nb0.size(); ++i)
            for (int k = 0; k < 3; ++k) cloud(static_cast<std::ptrdiff_t>(i + 1), k) = s.atoms()[0].position[k] + nb0[i].displacement[k];
        dgn::MatrixXd dm(cloud.rows(), cloud.rows());
        for (std::ptrdiff_t i = 0; i < cloud.rows(); ++i)
            for (std::ptrdiff_t j = 0; j < cloud.rows(); ++j) {
                double d2 = 0;
                for (int k = 0; k < 3; ++k) d2 += (cloud(i, k) - cloud(j, k)) * (cloud(i, k) - cloud(j, k));
                dm(i, j) = std::sqrt(d2);
            }
        const topology::PersistenceResult pr = topology::compute_persistence_from_distances(dm, rc, 1);
        for (const auto& [key, d] : {std::pair<const char*, const topology::PersistenceDiagram*>{"pd0", &pr.dim0},
                                     {"pd1", &pr.dim1}, {"pd2", &pr.dim2}}) {
            std::vector<double> flat;
            for (const auto& p : *d) {
                flat.push_back(p.birth);
                flat.push_back(p.death);
            }
            dump(f, key, flat);
        }
        dump(f, "cloud0", std::vector<double>(cloud.data(), cloud.data() + cloud.size()));

        // PCA round trip + betti .bin round trip
        topology::PCA pca;
        pca.fit(feat, 6);
        dump(f, "pca_components", std::vector<double>(pca.components().data(), pca.components().data() + pca.components().size()));
        dump(f, "pca_ratio", std::vector<double>(pca.explained_variance_ratio().data(),
                                                  pca.explained_variance_ratio().data() + pca.explained_variance_ratio().size()));
        const std::string bin = std::string(argv[4]) + ".betti.bin";
        topology::save_betti_features(bin, feat);
        const dgn::MatrixXd back = topology::load_betti_features(bin);
        bool same = back.rows() == feat.rows() && back.cols() == feat.cols();
        for (std::ptrdiff_t k = 0; same && k < feat.size(); ++k) same = back.data()[k] == feat.data()[k];
        dump(f, "bin_roundtrip", {same ? 1.0 : 0.0});
        std::fclose(f);
    } catch (const std::exception& e) {
        std::fprintf(stderr, "facade_check: %s\n", e.what());
        return 1;
    }
    return 0;
}
