// gen_ref.cpp — the reference's synthetic registration problems, number for number
// (examples/benchmark_synthetic.cpp:91-160, host).  See refrand.hpp for what pins each step.
//
// The driver's streams, in its order of use:
//   Open3D's engine: utility::random::Seed(1), then RandomDownSample(0.02) of the x50 bunny
//     (the source, shared by every case, B_SYN:94-99) and, per case, of the transformed
//     full cloud (B_SYN:147-148);
//   std::mt19937 gen(1) with uniform_real_distribution<double>: per case t = (U, U, U)
//     (braced list: left to right) then rot_3d(U, U, U) (B_SYN:113-116; function arguments:
//     right to left as GCC evaluates them, or left to right with SE3ICP_GEN_ARGS_LTR);
//   add_noise_to_point_cloud (B_SYN:13-56): ONE static std::mt19937{1} and
//     normal_distribution<double> for the whole run; each point += sqrt(noise) * (z0, z1, z2)
//     (the eigen-decomposition of noise * I is sqrt(noise) * I), source copy first, then
//     the target, case after case.
// The standard-library algorithms are libstdc++'s (the reference's Linux toolchain); this
// library is built against the same libstdc++.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <random>
#include <vector>

#include "refrand.hpp"
#include "se3icp.h"

using namespace se3icp::refrand;

extern "C" {

int64_t se3icp_random_downsample(const double* xyz, int64_t n, double ratio, uint32_t seed, double* out) {
    if (!xyz || n < 0 || !(ratio >= 0.0 && ratio <= 1.0)) return SE3ICP_ERR_INVALID_ARG;
    std::mt19937 engine(seed);
    const std::vector<int64_t> keep = random_downsample(n, ratio, engine);
    if (out)
        for (size_t k = 0; k < keep.size(); ++k) std::memcpy(out + 3 * k, xyz + 3 * keep[k], 3 * sizeof(double));
    return (int64_t)keep.size();
}

int64_t se3icp_synthetic_reference(const double* cloud, int64_t n, int32_t n_cases, double ratio, double noise_var,
                                   double t_range, double r_range, int32_t flags, double* src_out, double* tgt_out,
                                   double* T_out) {
    if (!cloud || n <= 0 || n_cases < 0 || !(ratio >= 0.0 && ratio <= 1.0) || !(noise_var >= 0.0))
        return SE3ICP_ERR_INVALID_ARG;
    std::mt19937 o3d_engine(1);                      // open3d::utility::random::Seed(1)
    const std::vector<int64_t> src_idx = random_downsample(n, ratio, o3d_engine);
    const int64_t k = (int64_t)src_idx.size();
    std::mt19937 gen(1);                             // B_SYN:103
    std::uniform_real_distribution<double> dist_T(-t_range, t_range), dist_R(-r_range, r_range);
    std::mt19937 noise_gen{1};                       // B_SYN:34-35 (static)
    std::normal_distribution<> noise_dist;
    const double sd = std::sqrt(noise_var);
    auto add_noise = [&](double* p, int64_t m) {
        for (int64_t i = 0; i < m; ++i) {
            const double z0 = noise_dist(noise_gen), z1 = noise_dist(noise_gen), z2 = noise_dist(noise_gen);
            p[3 * i] += sd * z0;
            p[3 * i + 1] += sd * z1;
            p[3 * i + 2] += sd * z2;
        }
    };
    std::vector<double> moved((size_t)n * 3);
    for (int32_t c = 0; c < n_cases; ++c) {
        double t[3];
        for (double& v : t) v = dist_T(gen);
        double roll, pitch, yaw;
        if (flags & SE3ICP_GEN_ARGS_LTR) {
            roll = dist_R(gen); pitch = dist_R(gen); yaw = dist_R(gen);
        } else {
            yaw = dist_R(gen); pitch = dist_R(gen); roll = dist_R(gen);
        }
        double R[9], T[16];
        rot_3d(roll, pitch, yaw, R);
        for (int r = 0; r < 3; ++r) {
            for (int cc = 0; cc < 3; ++cc) T[4 * r + cc] = R[3 * r + cc];
            T[4 * r + 3] = t[r];
        }
        T[12] = T[13] = T[14] = 0.0;
        T[15] = 1.0;
        if (T_out) std::memcpy(T_out + 16 * (size_t)c, T, sizeof(T));
        for (int64_t i = 0; i < n; ++i) transform_point(T, cloud + 3 * i, moved.data() + 3 * i);
        const std::vector<int64_t> tgt_idx = random_downsample(n, ratio, o3d_engine);
        double* so = src_out ? src_out + (size_t)c * k * 3 : nullptr;
        double* to = tgt_out ? tgt_out + (size_t)c * k * 3 : nullptr;
        std::vector<double> tmp_s, tmp_t;
        if (!so) { tmp_s.resize((size_t)k * 3); so = tmp_s.data(); }
        if (!to) { tmp_t.resize((size_t)k * 3); to = tmp_t.data(); }
        for (int64_t i = 0; i < k; ++i) std::memcpy(so + 3 * i, cloud + 3 * src_idx[(size_t)i], 3 * sizeof(double));
        for (int64_t i = 0; i < k; ++i) std::memcpy(to + 3 * i, moved.data() + 3 * tgt_idx[(size_t)i], 3 * sizeof(double));
        add_noise(so, k);  // B_SYN:154-155: source copy first, then the target
        add_noise(to, k);
    }
    return k;
}

}  // extern "C"
