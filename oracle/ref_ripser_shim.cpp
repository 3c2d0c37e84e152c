/*
 * ref_ripser_shim.cpp — C entry points over the VERBATIM vendored Ripser of the reference
 * (TEST INFRASTRUCTURE ONLY; built by oracle/Makefile into oracle/_ref/, never committed).
 *
 * The Ripser sources are compiled where they lie, through include paths into
 * /root/reference/third_party (exactly as src/topology/ripser_wrapper.cpp:5-6 includes them);
 * nothing of the reference is copied into this repository. The Eigen front end of
 * ripser_wrapper.cpp cannot be built offline (Eigen 3.4.0 absent), so the f32 packing and
 * threshold of ripser_wrapper.cpp:11-34 are restated here around the verbatim engine.
 */
#define RIPSER_AS_LIBRARY
#include <ripser/ripser.cpp>  // /root/reference/third_party/ripser/ripser.cpp

#include <omp.h>

#include <algorithm>
#include <cstdint>
#include <limits>
#include <vector>

#include "oracle.h"

namespace {
void collect(const std::vector<std::pair<value_t, value_t>>& v, std::vector<std::pair<float, float>>& out) {
    out.assign(v.begin(), v.end());
    std::sort(out.begin(), out.end());
}
struct RefPairs {
    std::vector<std::pair<float, float>> d0, d1, d2;
    int n_inf0 = 0;
};
void run_ripser(const float* lower, int n, float thr, unsigned threads, RefPairs& P) {
    std::vector<value_t> distances(lower, lower + (size_t)n * (n - 1) / 2);
    compressed_lower_distance_matrix dist(std::move(distances));
    // ripser_wrapper.cpp:32-34: sparse matrix at thresh, dim 2, ratio 1, modulus 2
    ripser<sparse_distance_matrix> r(sparse_distance_matrix(dist, thr), 2, thr, 1.0f, 2, threads);
    r.compute_barcodes();
    std::vector<std::pair<float, float>> d0all;
    if (r.persistence_pairs.size() > 0) collect(r.persistence_pairs[0], d0all);
    if (r.persistence_pairs.size() > 1) collect(r.persistence_pairs[1], P.d1);
    if (r.persistence_pairs.size() > 2) collect(r.persistence_pairs[2], P.d2);
    P.d0.clear();
    P.n_inf0 = 0;
    for (auto& p : d0all) {
        if (p.second == std::numeric_limits<float>::infinity()) ++P.n_inf0;
        else P.d0.push_back(p);
    }
}
}  // namespace

extern "C" {

/* Same contract as oracle_persistence (sorted finite pairs, counts). n must be >= 2:
 * an isolated point segfaults the reference (ripser.cpp:761). */
int ref_ripser_persistence(const float* lower, int n, float thr, unsigned threads, float* dim0, float* dim1,
                           float* dim2, int cap, oracle_counts* counts) {
    if (n < 2) return -2;
    RefPairs P;
    run_ripser(lower, n, thr, threads, P);
    if (counts) {
        counts->n_dim0_finite = (int32_t)P.d0.size();
        counts->n_dim0_inf = P.n_inf0;
        counts->n_dim1 = (int32_t)P.d1.size();
        counts->n_dim2 = (int32_t)P.d2.size();
    }
    auto put = [&](const std::vector<std::pair<float, float>>& v, float* o) -> bool {
        if (!o) return true;
        if ((int)v.size() > cap) return false;
        for (size_t k = 0; k < v.size(); ++k) {
            o[2 * k] = v[k].first;
            o[2 * k + 1] = v[k].second;
        }
        return true;
    };
    return (put(P.d0, dim0) && put(P.d1, dim1) && put(P.d2, dim2)) ? 0 : -1;
}

/* Whole-structure Betti features the reference way (betti_features.cpp:103-119): restated
 * neighbour list + Gram distances, VERBATIM Ripser, restated statistics; OpenMP over atoms
 * with omp_threads threads and ripser_threads per Ripser call (reference default 8 x 8). */
int ref_structure_betti(const double* L, const double* pos, const int32_t* species, int64_t n, double rc,
                        int omp_threads, unsigned ripser_threads, double* features, int32_t* counts) {
    std::vector<int64_t> row_ptr(n + 1);
    int64_t E = oracle_neighbor_list(L, pos, n, rc, UINT64_MAX, 1e-10, row_ptr.data(), nullptr, nullptr, nullptr,
                                     nullptr);
    std::vector<int32_t> col(E);
    std::vector<double> dist(E), disp(3 * E);
    oracle_neighbor_list(L, pos, n, rc, UINT64_MAX, 1e-10, row_ptr.data(), col.data(), dist.data(), disp.data(),
                         nullptr);
    const float thr = (float)rc;
    int bad = 0;
#pragma omp parallel for schedule(dynamic) num_threads(omp_threads) reduction(+ : bad)
    for (int64_t i = 0; i < n; ++i) {
        int cnt = 0;
        for (int64_t j = 0; j < n; ++j) cnt += (species[j] == species[i]);
        const double w = 1.0 / cnt;
        const int m = (int)(row_ptr[i + 1] - row_ptr[i]) + 1;
        double* f = features + 35 * i;
        if (m < 2) {  // reference UB; defined as zeros
            for (int k = 0; k < 35; ++k) f[k] = 0;
            if (counts) {
                counts[4 * i] = 0;
                counts[4 * i + 1] = 1;
                counts[4 * i + 2] = counts[4 * i + 3] = 0;
            }
            continue;
        }
        std::vector<double> cloud(3 * (size_t)m);
        for (int k = 0; k < 3; ++k) cloud[k] = pos[3 * i + k];
        for (int r = 0; r < m - 1; ++r)
            for (int k = 0; k < 3; ++k) cloud[3 * (r + 1) + k] = pos[3 * i + k] + disp[3 * (row_ptr[i] + r) + k];
        std::vector<float> lower((size_t)m * (m - 1) / 2);
        oracle_local_distances(cloud.data(), m, lower.data());
        RefPairs P;
        run_ripser(lower.data(), m, thr, ripser_threads, P);
        auto flat = [](const std::vector<std::pair<float, float>>& v) {
            std::vector<float> o(2 * v.size());
            for (size_t k = 0; k < v.size(); ++k) {
                o[2 * k] = v[k].first;
                o[2 * k + 1] = v[k].second;
            }
            return o;
        };
        std::vector<float> a = flat(P.d0), b = flat(P.d1), c = flat(P.d2);
        oracle_statistics(a.data(), (int)P.d0.size(), 1, w, f + 0);
        oracle_statistics(b.data(), (int)P.d1.size(), 2, w, f + 5);
        oracle_statistics(b.data(), (int)P.d1.size(), 0, w, f + 10);
        oracle_statistics(b.data(), (int)P.d1.size(), 1, w, f + 15);
        oracle_statistics(c.data(), (int)P.d2.size(), 2, w, f + 20);
        oracle_statistics(c.data(), (int)P.d2.size(), 0, w, f + 25);
        oracle_statistics(c.data(), (int)P.d2.size(), 1, w, f + 30);
        if (counts) {
            counts[4 * i] = (int32_t)P.d0.size();
            counts[4 * i + 1] = P.n_inf0;
            counts[4 * i + 2] = (int32_t)P.d1.size();
            counts[4 * i + 3] = (int32_t)P.d2.size();
        }
    }
    return bad;
}

}  // extern "C"
