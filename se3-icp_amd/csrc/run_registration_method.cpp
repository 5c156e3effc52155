// run_registration_method — drop-in for examples/run_registration_method.cpp (CLI:8-63).
//
//   run_registration_method <AlgorithmName> <SourcePointCloudFilePath> <TargetPointCloudFilePath>
//
// Same argv, method whitelist, parameter overrides, stdout lines and exit codes as the
// reference; the registration runs on the GPU through libse3icp.so's object surface
// (the C-ABI mirror of IterativeSE3Registration).
#include <iomanip>
#include <iostream>
#include <sstream>
#include <string>
#include <vector>

#include "ply.hpp"
#include "se3icp.h"

namespace {

// Eigen's default IOFormat for `std::cout << Matrix4d`: stream precision (6 significant
// digits), columns right-aligned to the widest coefficient, " " between columns.
void print_matrix(const double* T) {
    std::string cells[16];
    size_t width = 0;
    for (int i = 0; i < 16; ++i) {
        std::ostringstream ss;
        ss.copyfmt(std::cout);
        ss << T[i];
        cells[i] = ss.str();
        width = std::max(width, cells[i].size());
    }
    for (int r = 0; r < 4; ++r) {
        if (r) std::cout << "\n";
        for (int c = 0; c < 4; ++c) {
            if (c) std::cout << " ";
            std::cout << std::setw((int)width) << cells[r * 4 + c];
        }
    }
}

}  // namespace

int main(int argc, char* argv[]) {
    if (argc != 4) {
        std::cerr << "Usage: " << argv[0] << " <AlgorithmName> <SourcePointCloudFilePath> <TargetPointCloudFilePath>"
                  << std::endl;
        return 1;
    }
    const std::string algorithmName = argv[1];
    const std::string sourceCloudPath = argv[2];
    const std::string targetCloudPath = argv[3];
    if (algorithmName != "pt2pt" && algorithmName != "pt2pl" && algorithmName != "gicp" &&
        algorithmName != "se3_pt2pt" && algorithmName != "se3_pt2pl" && algorithmName != "se3_gicp") {
        std::cerr << "Not a valid algorithm name\n"
                  << "Available names are: pt2pt, pt2pl, gicp, se3_pt2pt, se3_pt2pl, and se3_gicp\n";
        return 1;
    }
    std::vector<double> src, tgt;
    std::string err;
    if (!se3icp::read_ply_xyz(sourceCloudPath, src, err)) {
        std::cerr << "Failed to read " << sourceCloudPath << ": " << err << std::endl;
        return 1;
    }
    std::cout << "source point cloud size = " << src.size() / 3 << std::endl;
    if (!se3icp::read_ply_xyz(targetCloudPath, tgt, err)) {
        std::cerr << "Failed to read " << targetCloudPath << ": " << err << std::endl;
        return 1;
    }
    std::cout << "target point cloud size = " << tgt.size() / 3 << std::endl;

    se3icp_registration* reg = se3icp_registration_new();
    se3icp_set_source_cloud(reg, src.data(), (int64_t)(src.size() / 3));
    se3icp_set_target_cloud(reg, tgt.data(), (int64_t)(tgt.size() / 3));
    se3icp_params* p = se3icp_params_of(reg);  // CLI:38-42
    p->estimated_overlap = 1.0;
    p->max_num_se3_iterations = 10;
    p->mse = 0.00001;
    p->mse_switch_error = 5 * p->mse;
    p->number_of_nn_for_LRF = 90;

    int rc;
    if (algorithmName == "pt2pt" || algorithmName == "pt2pl" || algorithmName == "gicp") {
        std::cout << "Running standard ICP variant: " << algorithmName << std::endl;
        rc = se3icp_run_icp(reg, algorithmName.c_str());
    } else {
        std::cout << "Running SE(3)-ICP variant: " << algorithmName.substr(4) << std::endl;
        rc = se3icp_run_se3_icp(reg, algorithmName.substr(4).c_str());
    }
    if (rc != SE3ICP_OK && rc != SE3ICP_ERR_NONFINITE) {
        std::cerr << "se3icp: " << se3icp_status_string(rc) << std::endl;
        se3icp_registration_free(reg);
        return 2;
    }
    se3icp_result res;
    se3icp_get_result(reg, &res);
    std::cout << "Estimated transformation = \n";
    print_matrix(res.T);
    std::cout << std::endl;
    se3icp_registration_free(reg);
    return 0;
}
