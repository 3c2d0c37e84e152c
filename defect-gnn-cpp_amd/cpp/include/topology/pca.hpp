// topology::PCA over the 35-d Betti features (replaces reference include/topology/pca.hpp,
// src/topology/pca.cpp:15-121). Same fit/transform/save/load API and pca_model.bin layout.
// Components are unique up to sign; this build fixes the sign so that each component's
// largest-magnitude coefficient is positive (the reference's JacobiSVD sign is arbitrary).
#pragma once
#include <string>

#include "dgn/matrix.hpp"

namespace defect_gnn::topology {

class PCA {
public:
    void fit(const dgn::MatrixXd& x, int n_components = 6);
    [[nodiscard]] dgn::MatrixXd transform(const dgn::MatrixXd& x) const;
    dgn::MatrixXd fit_transform(const dgn::MatrixXd& x, int n_components = 6);

    void save(const std::string& path) const;
    void load(const std::string& path);

    [[nodiscard]] const int& n_components() const { return n_components_; }
    [[nodiscard]] const dgn::VectorXd& mean() const { return mean_; }
    [[nodiscard]] const dgn::MatrixXd& components() const { return components_; }
    [[nodiscard]] const dgn::VectorXd& explained_variance_ratio() const { return explained_var_; }

private:
    bool fitted_ = false;
    int n_components_ = 0;
    dgn::VectorXd mean_;
    dgn::MatrixXd components_;  // D x k
    dgn::VectorXd explained_var_;
};

}  // namespace defect_gnn::topology
