// matrix.hpp — minimal dense, column-major matrix/vector types with the subset of the Eigen
// API the reference's public headers expose (Eigen 3.4 is not available on this platform).
// MatrixXd / MatrixXi / VectorXd / Matrix3d / Vector3d keep Eigen's storage order
// (column-major), so element (i, j) of an R x C matrix is data()[j * R + i].
#pragma once
#include <cstddef>
#include <initializer_list>
#include <stdexcept>
#include <vector>

namespace dgn {

template <typename T>
class Matrix {
public:
    using Index = std::ptrdiff_t;
    Matrix() = default;
    Matrix(Index rows, Index cols) : r_(rows), c_(cols), v_(static_cast<size_t>(rows * cols), T()) {}
    void resize(Index rows, Index cols) {
        r_ = rows;
        c_ = cols;
        v_.assign(static_cast<size_t>(rows * cols), T());
    }
    Index rows() const { return r_; }
    Index cols() const { return c_; }
    Index size() const { return r_ * c_; }
    T* data() { return v_.data(); }
    const T* data() const { return v_.data(); }
    T& operator()(Index i, Index j) { return v_[static_cast<size_t>(j * r_ + i)]; }
    const T& operator()(Index i, Index j) const { return v_[static_cast<size_t>(j * r_ + i)]; }
    // vector-style access (column vectors)
    T& operator[](Index i) { return v_[static_cast<size_t>(i)]; }
    const T& operator[](Index i) const { return v_[static_cast<size_t>(i)]; }
    T& operator()(Index i) { return v_[static_cast<size_t>(i)]; }
    const T& operator()(Index i) const { return v_[static_cast<size_t>(i)]; }
    std::vector<T> row(Index i) const {
        std::vector<T> out(static_cast<size_t>(c_));
        for (Index j = 0; j < c_; ++j) out[static_cast<size_t>(j)] = (*this)(i, j);
        return out;
    }
    void set_row(Index i, const std::vector<T>& x) {
        if (static_cast<Index>(x.size()) != c_) throw std::invalid_argument("set_row: size mismatch");
        for (Index j = 0; j < c_; ++j) (*this)(i, j) = x[static_cast<size_t>(j)];
    }

private:
    Index r_ = 0, c_ = 0;
    std::vector<T> v_;
};

using MatrixXd = Matrix<double>;
using MatrixXi = Matrix<int>;

// fixed 3-vectors / 3x3 matrices as value types
struct Vector3d {
    double v[3] = {0.0, 0.0, 0.0};
    Vector3d() = default;
    Vector3d(double x, double y, double z) : v{x, y, z} {}
    double& operator[](int i) { return v[i]; }
    double operator[](int i) const { return v[i]; }
    double& operator()(int i) { return v[i]; }
    double operator()(int i) const { return v[i]; }
    const double* data() const { return v; }
};

struct Matrix3d {
    double m[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};  // m[row][col]
    double& operator()(int i, int j) { return m[i][j]; }
    double operator()(int i, int j) const { return m[i][j]; }
};

class VectorXd {
public:
    VectorXd() = default;
    explicit VectorXd(std::ptrdiff_t n) : v_(static_cast<size_t>(n), 0.0) {}
    void resize(std::ptrdiff_t n) { v_.assign(static_cast<size_t>(n), 0.0); }
    std::ptrdiff_t size() const { return static_cast<std::ptrdiff_t>(v_.size()); }
    double& operator[](std::ptrdiff_t i) { return v_[static_cast<size_t>(i)]; }
    double operator[](std::ptrdiff_t i) const { return v_[static_cast<size_t>(i)]; }
    double& operator()(std::ptrdiff_t i) { return v_[static_cast<size_t>(i)]; }
    double operator()(std::ptrdiff_t i) const { return v_[static_cast<size_t>(i)]; }
    double* data() { return v_.data(); }
    const double* data() const { return v_.data(); }

private:
    std::vector<double> v_;
};

}  // namespace dgn
