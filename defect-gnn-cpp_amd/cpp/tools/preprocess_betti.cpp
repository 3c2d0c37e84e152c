// preprocess_betti — batch driver equivalent to reference src/preprocess/preprocess_betti.cpp:30-143.
//   preprocess_betti [--resume] [raw_path processed_path [r_cutoff [n_pca_components [batch_structures]]]]
// Scans raw_path/*.vasp, orders ids "X_Y" by (X, Y) (:21-28,43-46), computes the N x 35 Betti
// features of every structure, writes processed_path/betti/<id>.bin (save_betti_features format),
// fits the PCA over all atoms and writes processed_path/pca_model.bin. Structures are sent to the
// GPU in batches (one dgn_host_betti call per batch) instead of one OpenMP loop per structure.
// --resume: a structure whose betti/<id>.bin already exists (and matches its POSCAR's atom count) is
// loaded (load_betti_features) instead of parsed and recomputed, and its file is left untouched, as the Python upstream skips existing outputs
// (.reference_code/Defect_GNN/Betti_number.py:208-209); the PCA is still fitted over every atom.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <filesystem>
#include <fstream>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "crystal/structure.hpp"
#include "io/vasp_parser.hpp"
#include "topology/betti_features.hpp"
#include "topology/pca.hpp"

namespace fs = std::filesystem;
using namespace defect_gnn;

static std::pair<int, int> parse_structure_id(const std::string& id) {
    const size_t u = id.find('_');
    if (u == std::string::npos) return {std::stoi(id), 0};
    return {std::stoi(id.substr(0, u)), std::stoi(id.substr(u + 1))};
}

// atom count of a POSCAR from its header alone (line 7: the per-species counts, as io::parse_vasp
// reads them): the --resume shape check of a saved betti/<id>.bin without parsing the coordinates
static size_t vasp_atom_count(const std::string& path) {
    std::ifstream f(path);
    if (!f.is_open()) throw std::runtime_error("Could not open file: " + path);
    std::string line;
    for (int i = 0; i < 7; ++i)
        if (!std::getline(f, line)) throw std::runtime_error("Truncated POSCAR: " + path);
    std::stringstream ss(line);
    size_t total = 0;
    int c;
    while (ss >> c) total += static_cast<size_t>(c);
    if (total == 0) throw std::runtime_error("No atom counts in POSCAR: " + path);
    return total;
}

static void log(const std::string& msg) { std::fprintf(stderr, "[preprocess_betti] %s\n", msg.c_str()); }

int main(int argc_in, char** argv_in) {
    std::string raw_path = "data/raw/defective_structures", processed_path = "data/processed";
    double r_cutoff = 10;
    int n_pca = 6;
    size_t batch = 1024;
    bool resume = false;
    std::vector<char*> args;
    for (int i = 0; i < argc_in; ++i) {
        if (i > 0 && std::string(argv_in[i]) == "--resume") resume = true;
        else args.push_back(argv_in[i]);
    }
    const int argc = static_cast<int>(args.size());
    char** argv = args.data();
    if (argc >= 3) {
        raw_path = argv[1];
        processed_path = argv[2];
    }
    if (argc >= 4) r_cutoff = std::stod(argv[3]);
    if (argc >= 5) n_pca = std::stoi(argv[4]);
    if (argc >= 6) batch = static_cast<size_t>(std::max(1, std::stoi(argv[5])));
    try {
        fs::create_directories(processed_path + "/betti");
        std::vector<std::string> ids;
        for (const auto& e : fs::directory_iterator(raw_path))
            if (e.path().extension() == ".vasp") ids.push_back(e.path().stem().string());
        std::sort(ids.begin(), ids.end(),
                  [](const std::string& a, const std::string& b) { return parse_structure_id(a) < parse_structure_id(b); });
        std::map<int, int> defects;
        for (const auto& id : ids) defects[parse_structure_id(id).first]++;
        log("found " + std::to_string(ids.size()) + " defective structures from " + std::to_string(defects.size()) +
            " base structures; r_cutoff=" + std::to_string(r_cutoff) + " batch=" + std::to_string(batch));

        const auto t0 = std::chrono::steady_clock::now();
        std::vector<dgn::MatrixXd> all;
        size_t total_atoms = 0;
        size_t skipped = 0;
        for (size_t lo = 0; lo < ids.size(); lo += batch) {
            const size_t hi = std::min(ids.size(), lo + batch);
            std::vector<crystal::Structure> st;
            std::vector<size_t> todo;  // ids[i] to compute in this batch
            std::vector<dgn::MatrixXd> feats(hi - lo);
            // --resume reads only the header of a structure whose betti/<id>.bin exists (shape check)
            // and parses in full only the structures it computes: a raw file that no longer parses
            // does not abort a batch whose features were saved
            for (size_t i = lo; i < hi; ++i) {
                const std::string out = processed_path + "/betti/" + ids[i] + ".bin";
                bool have = false;
                if (resume && fs::exists(out)) {
                    // an unreadable file (a run killed mid-write before round 5 wrote them in place) or
                    // one of another shape (other structure) is recomputed, not trusted
                    try {
                        dgn::MatrixXd m = topology::load_betti_features(out);
                        std::ptrdiff_t want = m.rows();
                        try {
                            want = static_cast<std::ptrdiff_t>(vasp_atom_count(raw_path + "/" + ids[i] + ".vasp"));
                        } catch (const std::exception& e) {
                            log(std::string("resume: ") + e.what() + "; keeping the saved " + out);
                        }
                        if (m.rows() == want && m.cols() == topology::BETTI_FEATURE_DIM) {
                            feats[i - lo] = std::move(m);
                            have = true;
                            ++skipped;
                        } else {
                            log("resume: " + out + " has the wrong shape; recomputed");
                        }
                    } catch (const std::exception& e) {
                        log(std::string("resume: ") + e.what() + "; recomputed");
                    }
                }
                if (!have) todo.push_back(i);
            }
            st.reserve(todo.size());
            for (size_t i : todo) st.emplace_back(io::parse_vasp(raw_path + "/" + ids[i] + ".vasp"));
            std::vector<const crystal::Structure*> ptrs;
            for (const auto& s : st) ptrs.push_back(&s);
            if (!ptrs.empty()) {
                std::vector<dgn::MatrixXd> got = topology::compute_batch_betti_features(ptrs, r_cutoff);
                for (size_t t = 0; t < todo.size(); ++t) {
                    // written under a temporary name and renamed into place: a killed run never
                    // leaves a truncated betti/<id>.bin behind for --resume
                    const std::string out = processed_path + "/betti/" + ids[todo[t]] + ".bin";
                    topology::save_betti_features(out + ".tmp", got[t]);
                    fs::rename(out + ".tmp", out);
                    feats[todo[t] - lo] = std::move(got[t]);
                }
            }
            for (size_t i = lo; i < hi; ++i) {
                total_atoms += static_cast<size_t>(feats[i - lo].rows());
                all.push_back(std::move(feats[i - lo]));
            }
            log("[" + std::to_string(hi) + "/" + std::to_string(ids.size()) + "] structures done");
        }
        if (resume) log("resume: " + std::to_string(skipped) + " existing betti/<id>.bin loaded, not recomputed");
        const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        log("Betti features: " + std::to_string(ids.size()) + " structures, " + std::to_string(total_atoms) +
            " atoms in " + std::to_string(secs) + " s");

        dgn::MatrixXd stacked(static_cast<std::ptrdiff_t>(total_atoms), topology::BETTI_FEATURE_DIM);
        std::ptrdiff_t row = 0;
        for (const auto& f : all)
            for (std::ptrdiff_t i = 0; i < f.rows(); ++i, ++row)
                for (std::ptrdiff_t k = 0; k < f.cols(); ++k) stacked(row, k) = f(i, k);
        if (total_atoms > 1) {
            topology::PCA pca;
            pca.fit(stacked, n_pca);
            pca.save(processed_path + "/pca_model.bin");
            double ratio = 0;
            for (std::ptrdiff_t k = 0; k < pca.explained_variance_ratio().size(); ++k) ratio += pca.explained_variance_ratio()[k];
            log("PCA explained variance ratio: " + std::to_string(ratio));
        }
        log("done");
    } catch (const std::exception& e) {
        std::fprintf(stderr, "[preprocess_betti] error: %s\n", e.what());
        return 1;
    }
    return 0;
}
