/*
 * oracle.cpp — CPU restatement of the reference hot path. TEST INFRASTRUCTURE ONLY:
 * loaded by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, never by
 * the product library. See oracle.h for the parity-pinning statement.
 *
 * Build: g++ -O2 -ffp-contract=off (x86-64 SSE2 baseline, no FMA) — the reference is built
 * without -march, so its double arithmetic is never contracted.
 */
#include "oracle.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

namespace {

// ---------------------------------------------------------------------------------------
// Neighbour list — restates src/graph/neighbor_list.cpp:27-94.
// ---------------------------------------------------------------------------------------

// Eigen Matrix3d::row(k).norm(): fixed-size 3 redux unrolls as x0 + (x1 + x2)
// (Eigen 3.4 redux_novec_unroller halves the range). neighbor_list.cpp:69.
double lattice_row_norm(const double* r) {
    return std::sqrt(r[0] * r[0] + (r[1] * r[1] + r[2] * r[2]));
}

struct Candidate {
    double distance;
    int32_t j;
    int32_t img[3];
    double disp[3];
};

// Canonical order: (distance, j, n_a, n_b, n_c). The reference's order among exact ties is
// implementation-defined (nanoflann sort, then an unstable std::sort at :56-58).
bool candidate_less(const Candidate& a, const Candidate& b) {
    if (a.distance != b.distance) return a.distance < b.distance;
    if (a.j != b.j) return a.j < b.j;
    if (a.img[0] != b.img[0]) return a.img[0] < b.img[0];
    if (a.img[1] != b.img[1]) return a.img[1] < b.img[1];
    return a.img[2] < b.img[2];
}

void neighbor_rows(const double* L, const double* pos, int64_t n, double rc, uint64_t kmax,
                   double eps, std::vector<std::vector<Candidate>>& rows) {
    const int N = oracle_num_images(L, rc);
    const double rc2 = rc * rc;  // nanoflann radiusSearch(q, r_cutoff * r_cutoff) :40
    rows.assign(n, {});
    // bounding box of the atoms, used only to skip images that cannot hold a point within rc
    double lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    for (int64_t j = 0; j < n; ++j)
        for (int k = 0; k < 3; ++k) {
            lo[k] = std::min(lo[k], pos[3 * j + k]);
            hi[k] = std::max(hi[k], pos[3 * j + k]);
        }
    for (int64_t i = 0; i < n; ++i) {
        const double* q = pos + 3 * i;
        std::vector<Candidate>& out = rows[i];
        // create_image_cloud order: n_a outer, n_b, n_c inner, then atoms (:79-91)
        for (int na = -N; na <= N; ++na)
            for (int nb = -N; nb <= N; ++nb)
                for (int nc = -N; nc <= N; ++nc) {
                    // offset = n_a*a + n_b*b + n_c*c, Eigen evaluates ((na*a + nb*b) + nc*c) :82-84
                    double off[3];
                    for (int k = 0; k < 3; ++k)
                        off[k] = (double(na) * L[k] + double(nb) * L[3 + k]) + double(nc) * L[6 + k];
                    // conservative skip: squared distance from q to the shifted bounding box
                    double gap2 = 0;
                    for (int k = 0; k < 3; ++k) {
                        double g = std::max({lo[k] + off[k] - q[k], q[k] - (hi[k] + off[k]), 0.0});
                        gap2 += g * g;
                    }
                    if (gap2 > rc2 * (1.0 + 1e-9) + 1e-9) continue;
                    for (int64_t j = 0; j < n; ++j) {
                        double p[3];
                        for (int k = 0; k < 3; ++k) p[k] = pos[3 * j + k] + off[k];
                        // nanoflann L2_Simple_Adaptor::evalMetric: result += (a-b)^2, k = 0,1,2
                        double d2 = 0.0;
                        for (int k = 0; k < 3; ++k) {
                            double diff = q[k] - p[k];
                            d2 += diff * diff;
                        }
                        if (!(d2 < rc2)) continue;  // RadiusResultSet::addPoint: dist < radius
                        double dist = std::sqrt(d2);
                        if (j == i && dist < eps) continue;  // self skip :47
                        Candidate c;
                        c.distance = dist;  // :53
                        c.j = (int32_t)j;
                        c.img[0] = na;
                        c.img[1] = nb;
                        c.img[2] = nc;
                        for (int k = 0; k < 3; ++k) c.disp[k] = p[k] - q[k];  // delta_r :51
                        out.push_back(c);
                    }
                }
        std::sort(out.begin(), out.end(), candidate_less);  // :56-58
        if (out.size() > kmax) out.resize(kmax);             // :60-62
    }
}

// ---------------------------------------------------------------------------------------
// VR persistence — Ripser semantics (third_party/ripser/ripser.cpp), own reduction code.
//   * sparse_distance_matrix keeps i != j with d <= threshold (:386-395)
//   * dim_max = min(2, n - 2) (:560)
//   * filtration order F: diameter ascending, then combinatorial index DESCENDING
//     (greater_diameter_or_smaller_index, :318-324); pivots are F-minimal cofacets
//   * dim 0: Kruskal in F order, emit (0,d) for d != 0 and (0,inf) per component (:725-762)
//   * dim >= 1: cohomology with clearing; emit (birth, death) only if death > birth (:1240);
//     essential classes are NOT emitted in the parallel build (:1209-1225)
// Any correct reduction yields the same (birth, death) multiset because the persistence
// pairing of a total order is unique; this one is the plain standard algorithm.
// ---------------------------------------------------------------------------------------

struct Key {
    float d;
    int64_t idx;
};
// F order: a before b
inline bool f_less(const Key& a, const Key& b) {
    return a.d < b.d || (a.d == b.d && a.idx > b.idx);
}
inline bool key_eq(const Key& a, const Key& b) { return a.idx == b.idx; }

struct Binom {
    std::vector<int64_t> t;
    int n, k;
    Binom(int n_, int k_) : t((size_t)(n_ + 1) * (k_ + 1), 0), n(n_), k(k_) {
        for (int i = 0; i <= n; ++i) {
            t[(size_t)i * (k + 1)] = 1;
            for (int j = 1; j <= std::min(i, k); ++j)
                t[(size_t)i * (k + 1) + j] =
                    t[(size_t)(i - 1) * (k + 1) + j - 1] + (j <= i - 1 ? t[(size_t)(i - 1) * (k + 1) + j] : 0);
        }
    }
    int64_t operator()(int v, int kk) const { return (kk > v) ? 0 : t[(size_t)v * (k + 1) + kk]; }
};

struct Simplex {
    Key key;
    int v[4];  // vertices, strictly descending
    int dim;
};

struct VR {
    int n;
    float thr;
    std::vector<float> D;  // dense n*n (diagonal 0)
    Binom B;
    int64_t* stats;
    VR(const float* lower, int n_, float thr_, int64_t* stats_)
        : n(n_), thr(thr_), D((size_t)n_ * n_, 0.0f), B(n_ + 1, 5), stats(stats_) {
        // compute_persistence_from_distances packs row i = 1..n-1, j < i (ripser_wrapper.cpp:20-24)
        size_t p = 0;
        for (int i = 1; i < n; ++i)
            for (int j = 0; j < i; ++j) {
                D[(size_t)i * n + j] = lower[p];
                D[(size_t)j * n + i] = lower[p];
                ++p;
            }
    }
    float dist(int a, int b) const { return D[(size_t)a * n + b]; }
    bool adjacent(int a, int b) const { return a != b && dist(a, b) <= thr; }

    int64_t index_of(const int* v, int dim) const {  // v strictly descending, dim+1 vertices
        int64_t idx = 0;
        for (int t = 0; t <= dim; ++t) idx += B(v[t], dim + 1 - t);
        return idx;
    }

    // all cofacets of s (dimension s.dim+1), with diameter <= thr, sorted by F order
    void coboundary(const Simplex& s, std::vector<Simplex>& out) const {
        out.clear();
        for (int w = 0; w < n; ++w) {
            bool ok = true;
            float diam = s.key.d;
            for (int t = 0; t <= s.dim && ok; ++t) {
                if (w == s.v[t] || !adjacent(w, s.v[t])) ok = false;
                else diam = std::max(diam, dist(w, s.v[t]));
            }
            if (!ok || !(diam <= thr)) continue;
            Simplex c;
            c.dim = s.dim + 1;
            int t = 0, o = 0;
            bool placed = false;
            for (; t <= s.dim; ++t) {
                if (!placed && w > s.v[t]) {
                    c.v[o++] = w;
                    placed = true;
                }
                c.v[o++] = s.v[t];
            }
            if (!placed) c.v[o++] = w;
            c.key.d = diam;
            c.key.idx = index_of(c.v, c.dim);
            out.push_back(c);
        }
        std::sort(out.begin(), out.end(), [](const Simplex& a, const Simplex& b) { return f_less(a.key, b.key); });
    }
};

// symmetric difference of two F-sorted columns (Z/2 addition)
void column_add(std::vector<Key>& a, const std::vector<Key>& b, std::vector<Key>& tmp) {
    tmp.clear();
    size_t i = 0, j = 0;
    while (i < a.size() && j < b.size()) {
        if (key_eq(a[i], b[j])) {
            ++i;
            ++j;
        } else if (f_less(a[i], b[j])) {
            tmp.push_back(a[i++]);
        } else {
            tmp.push_back(b[j++]);
        }
    }
    while (i < a.size()) tmp.push_back(a[i++]);
    while (j < b.size()) tmp.push_back(b[j++]);
    a.swap(tmp);
}

struct Pairs {
    std::vector<std::pair<float, float>> d0, d1, d2;
    int n_inf0 = 0;
};

// union-find (any correct one: the dim-0 pairing in F order is unique)
int uf_find(std::vector<int>& p, int x) {
    while (p[x] != x) {
        p[x] = p[p[x]];
        x = p[x];
    }
    return x;
}

void persistence(const float* lower, int n, float thr, Pairs& out, int64_t* stats) {
    out = Pairs();
    if (n <= 0) return;
    if (n == 1) {  // reference segfaults (ripser.cpp:761); defined here as one essential class
        out.n_inf0 = 1;
        return;
    }
    VR vr(lower, n, thr, stats);
    const int dim_max = std::min(2, n - 2);

    // ---- dim 0: Kruskal in F order (ripser.cpp:725-762) ----
    std::vector<Simplex> edges;
    for (int i = 1; i < n; ++i)
        for (int j = 0; j < i; ++j)
            if (vr.dist(i, j) <= thr) {
                Simplex e;
                e.dim = 1;
                e.v[0] = i;
                e.v[1] = j;
                e.key.d = vr.dist(i, j);
                e.key.idx = vr.index_of(e.v, 1);
                edges.push_back(e);
            }
    std::sort(edges.begin(), edges.end(), [](const Simplex& a, const Simplex& b) { return f_less(a.key, b.key); });
    std::vector<int> parent(n);
    for (int i = 0; i < n; ++i) parent[i] = i;
    std::vector<Simplex> columns;  // non-tree edges
    for (const Simplex& e : edges) {
        int u = uf_find(parent, e.v[0]), v = uf_find(parent, e.v[1]);
        if (u != v) {
            if (e.key.d != 0) out.d0.push_back({0.0f, e.key.d});
            parent[u] = v;
        } else {
            columns.push_back(e);
        }
    }
    for (int i = 0; i < n; ++i)
        if (uf_find(parent, i) == i) ++out.n_inf0;
    if (dim_max < 1) return;

    std::vector<Simplex> cob;
    std::vector<Key> tmp;
    std::vector<int64_t> cleared;  // dim-1 pivots (triangle indices), for clearing in dim 2
    for (int dim = 1; dim <= dim_max; ++dim) {
        if (dim == 2) {
            // assemble_columns_to_reduce (ripser.cpp:596-723): all triangles <= thr that are not
            // dim-1 pivots. Enumerate triangles a > b > c.
            std::sort(cleared.begin(), cleared.end());
            columns.clear();
            for (int a = 2; a < n; ++a)
                for (int b = 1; b < a; ++b) {
                    if (!vr.adjacent(a, b)) continue;
                    for (int c = 0; c < b; ++c) {
                        if (!vr.adjacent(a, c) || !vr.adjacent(b, c)) continue;
                        Simplex t;
                        t.dim = 2;
                        t.v[0] = a;
                        t.v[1] = b;
                        t.v[2] = c;
                        t.key.d = std::max(vr.dist(a, b), std::max(vr.dist(a, c), vr.dist(b, c)));
                        t.key.idx = vr.index_of(t.v, 2);
                        if (stats) stats[6]++;
                        if (std::binary_search(cleared.begin(), cleared.end(), t.key.idx)) continue;
                        columns.push_back(t);
                    }
                }
        }
        // reduce in F-descending order (columns_to_reduce sorted by greater_diameter_or_smaller_index)
        std::sort(columns.begin(), columns.end(), [](const Simplex& a, const Simplex& b) { return f_less(b.key, a.key); });
        std::vector<std::vector<Key>> R(columns.size());
        std::vector<std::pair<Key, int>> owner;  // pivot -> column (kept sorted by idx)
        auto find_owner = [&](int64_t idx) -> int {
            auto it = std::lower_bound(owner.begin(), owner.end(), idx,
                                       [](const std::pair<Key, int>& a, int64_t v) { return a.first.idx < v; });
            return (it != owner.end() && it->first.idx == idx) ? it->second : -1;
        };
        std::vector<Key> col;
        for (size_t c = 0; c < columns.size(); ++c) {
            vr.coboundary(columns[c], cob);
            if (stats) stats[dim == 1 ? 0 : 3]++;
            if (stats) stats[7] += (int64_t)cob.size();
            col.clear();
            for (const Simplex& s : cob) col.push_back(s.key);
            bool first = true;
            while (!col.empty()) {
                int o = find_owner(col.front().idx);
                if (o < 0) break;
                column_add(col, R[o], tmp);
                if (stats) stats[dim == 1 ? 2 : 5]++;
                first = false;
            }
            if (first && stats && !col.empty()) stats[dim == 1 ? 1 : 4]++;
            if (col.empty()) continue;  // essential class: not emitted (ripser.cpp:1209-1225)
            Key piv = col.front();
            float birth = columns[c].key.d, death = piv.d;
            if (death > birth) (dim == 1 ? out.d1 : out.d2).push_back({birth, death});
            if (dim == 1) cleared.push_back(piv.idx);
            R[c] = col;
            auto it = std::lower_bound(owner.begin(), owner.end(), piv.idx,
                                       [](const std::pair<Key, int>& a, int64_t v) { return a.first.idx < v; });
            owner.insert(it, {piv, (int)c});
        }
    }
}

void sort_pairs(std::vector<std::pair<float, float>>& v) { std::sort(v.begin(), v.end()); }

// ---------------------------------------------------------------------------------------
// Statistics — betti_features.cpp:24-55 and utils/math.hpp:9-28.
// Summation is sequential in the given (sorted) order; the reference's pair order is the
// hash-map slot order of a lock-free map (nondeterministic), so only ~1e-15 agreement exists.
// ---------------------------------------------------------------------------------------
void stats5(const std::vector<double>& v, double weight, double* out) {
    for (int k = 0; k < 5; ++k) out[k] = 0.0;
    if (v.empty()) return;  // BettiStatistics{} (betti_features.cpp:43-45)
    double s = 0;
    for (double x : v) s += x;
    double m = s / (double)v.size();  // Eigen mean = sum / size
    double ss = 0;
    for (double x : v) ss += (x - m) * (x - m);
    double mx = v[0], mn = v[0];
    for (double x : v) {
        mx = std::max(mx, x);
        mn = std::min(mn, x);
    }
    out[0] = m;
    out[1] = std::sqrt(ss / (double)v.size());  // population std (math.hpp:13-16)
    out[2] = mx;
    out[3] = mn;
    out[4] = s * weight;  // weighted_sum = sum * weight (math.hpp:26-28)
}

void diagram_stats(const std::vector<std::pair<float, float>>& pd, int which, double w, double* out) {
    std::vector<double> v;
    for (const auto& p : pd) {
        double b = p.first, d = p.second;  // PersistencePair holds doubles (ripser_wrapper.cpp:36-45)
        if (d == INFINITY) continue;       // betti_features.cpp:30-32
        v.push_back(which == 0 ? b : which == 1 ? d : d - b);
    }
    stats5(v, w, out);
}

}  // namespace

// ======================================= C ABI ==========================================
extern "C" {

int oracle_num_images(const double* L, double rc) {
    double lmin = std::min({lattice_row_norm(L), lattice_row_norm(L + 3), lattice_row_norm(L + 6)});
    return static_cast<int>(std::ceil(rc / lmin)) + 1;
}

int64_t oracle_neighbor_list(const double* L, const double* pos, int64_t n, double rc, uint64_t kmax,
                             double eps, int64_t* row_ptr, int32_t* col, double* dist, double* disp,
                             int32_t* image) {
    std::vector<std::vector<Candidate>> rows;
    neighbor_rows(L, pos, n, rc, kmax, eps, rows);
    int64_t e = 0;
    if (row_ptr) row_ptr[0] = 0;
    for (int64_t i = 0; i < n; ++i) {
        for (const Candidate& c : rows[i]) {
            if (col) col[e] = c.j;
            if (dist) dist[e] = c.distance;
            if (disp)
                for (int k = 0; k < 3; ++k) disp[3 * e + k] = c.disp[k];
            if (image)
                for (int k = 0; k < 3; ++k) image[3 * e + k] = c.img[k];
            ++e;
        }
        if (row_ptr) row_ptr[i + 1] = e;
    }
    return e;
}

int oracle_rbf_bins(double rc, double dr) { return (int)std::floor(rc / dr); }

int64_t oracle_structure_graph(const double* L, const double* pos, int64_t n, double rc, uint64_t kmax, double eps,
                               double rbf_rc, double dr, double* rbf_out) {
    // CrystalGraph edge part (crystal_graph.cpp:23-40): NeighborList rows, one gaussian_rbf per edge
    std::vector<std::vector<Candidate>> rows;
    neighbor_rows(L, pos, n, rc, kmax, eps, rows);
    const int nb = oracle_rbf_bins(rbf_rc, dr);
    std::vector<double> g(nb);
    int64_t e = 0;
    double sink = 0;
    for (int64_t i = 0; i < n; ++i)
        for (const Candidate& c : rows[i]) {
            oracle_gaussian_rbf(c.distance, rbf_rc, dr, rbf_out ? rbf_out + e * nb : g.data());
            sink += g[0];
            ++e;
        }
    if (sink == -1.0) e = -1;  // keep the work observable
    return e;
}

void oracle_gaussian_rbf(double distance, double rc, double dr, double* g) {
    // edge_features.cpp:7-24, same operation sequence
    int n = std::floor(rc / dr);
    double sigma = rc / 3;
    double inv_sigma_squared = 1 / std::pow(sigma, 2);
    double norm = 1 / (sigma * std::sqrt(2 * M_PI));
    for (int k = 0; k < n; k++) {
        double center = k * dr;
        g[k] = (norm * std::exp(-0.5 * std::pow(center - distance, 2) * inv_sigma_squared));
    }
}

void oracle_local_distances(const double* X, int n, float* lower) {
    // ripser_wrapper.cpp:64-67: sq = rowwise squaredNorm, D = sqrt(max(0, sq_i + sq_j - 2 X X^T))
    std::vector<double> sq(n);
    for (int i = 0; i < n; ++i) {
        const double* a = X + 3 * i;
        sq[i] = (a[0] * a[0] + a[1] * a[1]) + a[2] * a[2];  // Eigen dynamic redux: sequential
    }
    size_t p = 0;
    for (int i = 1; i < n; ++i)
        for (int j = 0; j < i; ++j) {
            const double* a = X + 3 * i;
            const double* b = X + 3 * j;
            double dot = (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];  // GEBP k-order, no FMA
            double d2 = (sq[i] + sq[j]) - 2.0 * dot;
            double d = std::sqrt(std::max(d2, 0.0));
            lower[p++] = static_cast<float>(d);  // value_t = float (ripser_wrapper.cpp:22)
        }
}

int oracle_persistence(const float* lower, int n, float thr, float* dim0, float* dim1, float* dim2,
                       int cap, oracle_counts* counts, int64_t* stats) {
    Pairs P;
    persistence(lower, n, thr, P, stats);
    sort_pairs(P.d0);
    sort_pairs(P.d1);
    sort_pairs(P.d2);
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
    bool ok = put(P.d0, dim0) && put(P.d1, dim1) && put(P.d2, dim2);
    return ok ? 0 : -1;
}

void oracle_statistics(const float* pairs, int m, int which, double weight, double* out) {
    std::vector<std::pair<float, float>> pd(m);
    for (int k = 0; k < m; ++k) pd[k] = {pairs[2 * k], pairs[2 * k + 1]};
    diagram_stats(pd, which, weight, out);
}

int oracle_structure_betti(const double* L, const double* pos, const int32_t* species, int64_t n,
                           double rc, double* features, int32_t* counts) {
    std::vector<std::vector<Candidate>> rows;
    // compute_structure_betti_features: NeighborList(structure, rc, SIZE_MAX) (betti_features.cpp:107)
    neighbor_rows(L, pos, n, rc, std::numeric_limits<uint64_t>::max(), 1e-10, rows);
    const float thr = static_cast<float>(rc);  // ripser_wrapper.cpp:28
    for (int64_t i = 0; i < n; ++i) {
        int cnt = 0;
        for (int64_t j = 0; j < n; ++j) cnt += (species[j] == species[i]);
        const double weight = 1.0 / cnt;  // betti_features.cpp:77
        const std::vector<Candidate>& nb = rows[i];
        const int m = (int)nb.size() + 1;
        std::vector<double> cloud(3 * (size_t)m);
        for (int k = 0; k < 3; ++k) cloud[k] = pos[3 * i + k];  // row 0 = centre (:68)
        for (int r = 0; r < (int)nb.size(); ++r)
            for (int k = 0; k < 3; ++k) cloud[3 * (r + 1) + k] = pos[3 * i + k] + nb[r].disp[k];  // :70-73
        std::vector<float> lower((size_t)m * (m - 1) / 2);
        oracle_local_distances(cloud.data(), m, lower.data());
        Pairs P;
        persistence(lower.data(), m, thr, P, nullptr);
        sort_pairs(P.d0);
        sort_pairs(P.d1);
        sort_pairs(P.d2);
        double* f = features + 35 * i;
        diagram_stats(P.d0, 1, weight, f + 0);  // dim0 death (:87-88)
        diagram_stats(P.d1, 2, weight, f + 5);  // dim1 persistence, birth, death (:90-93)
        diagram_stats(P.d1, 0, weight, f + 10);
        diagram_stats(P.d1, 1, weight, f + 15);
        diagram_stats(P.d2, 2, weight, f + 20);  // dim2 persistence, birth, death (:95-98)
        diagram_stats(P.d2, 0, weight, f + 25);
        diagram_stats(P.d2, 1, weight, f + 30);
        if (counts) {
            counts[4 * i + 0] = (int32_t)P.d0.size();
            counts[4 * i + 1] = P.n_inf0;
            counts[4 * i + 2] = (int32_t)P.d1.size();
            counts[4 * i + 3] = (int32_t)P.d2.size();
        }
    }
    return 0;
}

}  // extern "C"
