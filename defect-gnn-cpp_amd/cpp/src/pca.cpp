// PCA: the reference takes a thin SVD of the centred N x 35 matrix (pca.cpp:15-34); the right
// singular vectors and s^2/(N-1) are the eigenpairs of the 35 x 35 covariance, which is what
// this computes (cyclic Jacobi, converged to machine precision).
#include <algorithm>
#include <cmath>
#include <fstream>
#include <numeric>
#include <stdexcept>
#include <vector>

#include "topology/betti_features.hpp"
#include "topology/pca.hpp"

namespace defect_gnn::topology {

namespace {

// symmetric eigen-decomposition A = V diag(w) V^T, A (d x d, row-major, destroyed)
void jacobi_eigen(std::vector<double>& a, int d, std::vector<double>& w, std::vector<double>& v) {
    v.assign(static_cast<size_t>(d * d), 0.0);
    for (int i = 0; i < d; ++i) v[static_cast<size_t>(i * d + i)] = 1.0;
    auto A = [&](int i, int j) -> double& { return a[static_cast<size_t>(i * d + j)]; };
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0.0, diag = 0.0;
        for (int i = 0; i < d; ++i) {
            diag += A(i, i) * A(i, i);
            for (int j = i + 1; j < d; ++j) off += A(i, j) * A(i, j);
        }
        if (off <= 1e-30 * diag || off == 0.0) break;
        for (int p = 0; p < d; ++p)
            for (int q = p + 1; q < d; ++q) {
                const double apq = A(p, q);
                if (apq == 0.0) continue;
                const double theta = (A(q, q) - A(p, p)) / (2.0 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < d; ++k) {  // A <- A J (columns p, q)
                    const double akp = A(k, p), akq = A(k, q);
                    A(k, p) = c * akp - s * akq;
                    A(k, q) = s * akp + c * akq;
                }
                for (int k = 0; k < d; ++k) {  // A <- J^T A (rows p, q)
                    const double apk = A(p, k), aqk = A(q, k);
                    A(p, k) = c * apk - s * aqk;
                    A(q, k) = s * apk + c * aqk;
                }
                for (int k = 0; k < d; ++k) {
                    double& vkp = v[static_cast<size_t>(k * d + p)];
                    double& vkq = v[static_cast<size_t>(k * d + q)];
                    const double x = vkp, y = vkq;
                    vkp = c * x - s * y;
                    vkq = s * x + c * y;
                }
            }
    }
    w.resize(static_cast<size_t>(d));
    for (int i = 0; i < d; ++i) w[static_cast<size_t>(i)] = A(i, i);
}

}  // namespace

void PCA::fit(const dgn::MatrixXd& x, int n_components) {
    if (x.cols() != BETTI_FEATURE_DIM)
        throw std::runtime_error("Inputted Matrix does not have the correct number of columns");  // pca.cpp:16-18
    const auto n = x.rows();
    const int d = BETTI_FEATURE_DIM;
    if (n_components < 0 || n_components > d) throw std::invalid_argument("PCA: bad n_components");
    mean_.resize(d);
    for (int k = 0; k < d; ++k) {
        double s = 0.0;
        for (std::ptrdiff_t i = 0; i < n; ++i) s += x(i, k);
        mean_[k] = n ? s / static_cast<double>(n) : 0.0;
    }
    std::vector<double> cov(static_cast<size_t>(d * d), 0.0);
    for (int a = 0; a < d; ++a)
        for (int b = a; b < d; ++b) {
            double s = 0.0;
            for (std::ptrdiff_t i = 0; i < n; ++i) s += (x(i, a) - mean_[a]) * (x(i, b) - mean_[b]);
            cov[static_cast<size_t>(a * d + b)] = cov[static_cast<size_t>(b * d + a)] = s;
        }
    std::vector<double> w, v;
    jacobi_eigen(cov, d, w, v);
    std::vector<int> order(static_cast<size_t>(d));
    std::iota(order.begin(), order.end(), 0);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return w[static_cast<size_t>(a)] > w[static_cast<size_t>(b)]; });
    const double denom = n > 1 ? static_cast<double>(n - 1) : 1.0;
    double total = 0.0;
    for (double e : w) total += std::max(e, 0.0) / denom;
    components_.resize(d, n_components);
    explained_var_.resize(n_components);
    for (int c = 0; c < n_components; ++c) {
        const int src = order[static_cast<size_t>(c)];
        int big = 0;
        for (int k = 1; k < d; ++k)
            if (std::fabs(v[static_cast<size_t>(k * d + src)]) > std::fabs(v[static_cast<size_t>(big * d + src)])) big = k;
        const double sign = v[static_cast<size_t>(big * d + src)] < 0 ? -1.0 : 1.0;
        for (int k = 0; k < d; ++k) components_(k, c) = sign * v[static_cast<size_t>(k * d + src)];
        explained_var_[c] = total > 0 ? std::max(w[static_cast<size_t>(src)], 0.0) / denom / total : 0.0;
    }
    n_components_ = n_components;
    fitted_ = true;
}

dgn::MatrixXd PCA::transform(const dgn::MatrixXd& x) const {
    if (!fitted_) throw std::runtime_error("PCA::transform called before fit() or load()");
    if (x.cols() != mean_.size()) throw std::runtime_error("PCA::transform: column count mismatch");
    dgn::MatrixXd out(x.rows(), components_.cols());
    for (std::ptrdiff_t i = 0; i < x.rows(); ++i)
        for (std::ptrdiff_t c = 0; c < components_.cols(); ++c) {
            double s = 0.0;
            for (std::ptrdiff_t k = 0; k < x.cols(); ++k) s += (x(i, k) - mean_[k]) * components_(k, c);
            out(i, c) = s;
        }
    return out;
}

dgn::MatrixXd PCA::fit_transform(const dgn::MatrixXd& x, int n_components) {
    fit(x, n_components);
    return transform(x);
}

// pca_model.bin: int32 k, int32 D, D f64 mean, int32 rows, int32 cols, rows*cols f64
// (column-major), int32 k, k f64 explained ratio (pca.cpp:52-78)
void PCA::save(const std::string& filepath) const {
    if (!fitted_) throw std::runtime_error("PCA::save called before fit() or load()");
    std::ofstream f(filepath, std::ios::binary);
    if (!f) throw std::runtime_error("Cannot open file for writing: " + filepath);
    auto put_i = [&](int32_t v) { f.write(reinterpret_cast<const char*>(&v), sizeof v); };
    auto put_d = [&](const double* p, size_t cnt) {
        f.write(reinterpret_cast<const char*>(p), static_cast<std::streamsize>(cnt * sizeof(double)));
    };
    put_i(n_components_);
    put_i(static_cast<int32_t>(mean_.size()));
    put_d(mean_.data(), static_cast<size_t>(mean_.size()));
    put_i(static_cast<int32_t>(components_.rows()));
    put_i(static_cast<int32_t>(components_.cols()));
    put_d(components_.data(), static_cast<size_t>(components_.size()));
    put_i(static_cast<int32_t>(explained_var_.size()));
    put_d(explained_var_.data(), static_cast<size_t>(explained_var_.size()));
}

void PCA::load(const std::string& filepath) {
    std::ifstream f(filepath, std::ios::binary);
    if (!f) throw std::runtime_error("Cannot open file for reading: " + filepath);
    auto get_i = [&]() {
        int32_t v = 0;
        f.read(reinterpret_cast<char*>(&v), sizeof v);
        if (!f || v < 0) throw std::runtime_error("Corrupt PCA model: " + filepath);
        return v;
    };
    auto get_d = [&](double* p, size_t cnt) {
        f.read(reinterpret_cast<char*>(p), static_cast<std::streamsize>(cnt * sizeof(double)));
        if (!f) throw std::runtime_error("Truncated PCA model: " + filepath);
    };
    n_components_ = get_i();
    mean_.resize(get_i());
    get_d(mean_.data(), static_cast<size_t>(mean_.size()));
    const int32_t r = get_i(), c = get_i();
    components_.resize(r, c);
    get_d(components_.data(), static_cast<size_t>(components_.size()));
    explained_var_.resize(get_i());
    get_d(explained_var_.data(), static_cast<size_t>(explained_var_.size()));
    fitted_ = true;
}

}  // namespace defect_gnn::topology
