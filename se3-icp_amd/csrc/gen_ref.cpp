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
#include <algorithm>
#include <random>
#include <vector>

#include "refrand.hpp"
#include "se3icp.h"

using namespace se3icp::refrand;

namespace se3icp {
namespace refrand {

ReferenceDraws draw_reference(int64_t n, int32_t n_cases, double ratio, double t_range, double r_range,
                              bool args_left_to_right, bool want_noise) {
    ReferenceDraws D;
    std::mt19937 o3d_engine(1);                      // open3d::utility::random::Seed(1)
    const std::vector<int64_t> src_idx = random_downsample(n, ratio, o3d_engine);
    const int64_t k = (int64_t)src_idx.size();
    D.k = k;
    D.src_idx.assign(src_idx.begin(), src_idx.end());
    D.tgt_idx.resize((size_t)n_cases * k);
    D.T.resize((size_t)n_cases * 16);
    if (want_noise) D.z.resize((size_t)n_cases * 6 * k);
    std::mt19937 gen(1);                             // B_SYN:103
    std::uniform_real_distribution<double> dist_T(-t_range, t_range), dist_R(-r_range, r_range);
    std::mt19937 noise_gen{1};                       // B_SYN:34-35 (static)
    std::normal_distribution<> noise_dist;
    for (int32_t c = 0; c < n_cases; ++c) {
        double t[3];
        for (double& v : t) v = dist_T(gen);
        double roll, pitch, yaw;
        if (args_left_to_right) {
            roll = dist_R(gen); pitch = dist_R(gen); yaw = dist_R(gen);
        } else {
            yaw = dist_R(gen); pitch = dist_R(gen); roll = dist_R(gen);
        }
        double R[9];
        double* T = D.T.data() + 16 * (size_t)c;
        rot_3d(roll, pitch, yaw, R);
        for (int r = 0; r < 3; ++r) {
            for (int cc = 0; cc < 3; ++cc) T[4 * r + cc] = R[3 * r + cc];
            T[4 * r + 3] = t[r];
        }
        T[12] = T[13] = T[14] = 0.0;
        T[15] = 1.0;
        const std::vector<int64_t> tgt_idx = random_downsample(n, ratio, o3d_engine);  // B_SYN:147-148
        std::copy(tgt_idx.begin(), tgt_idx.end(), D.tgt_idx.begin() + (size_t)c * k);
        // B_SYN:154-155: the source copy's noise first, then the target's
        if (want_noise)
            for (int64_t i = 0; i < 6 * k; ++i) D.z[(size_t)c * 6 * k + i] = noise_dist(noise_gen);
    }
    return D;
}

}  // namespace refrand
}  // namespace se3icp

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
    const ReferenceDraws D = draw_reference(n, n_cases, ratio, t_range, r_range, (flags & SE3ICP_GEN_ARGS_LTR) != 0,
                                            src_out || tgt_out);
    const int64_t k = D.k;
    const double sd = std::sqrt(noise_var);
    for (int32_t c = 0; c < n_cases; ++c) {
        const double* T = D.T.data() + 16 * (size_t)c;
        if (T_out) std::memcpy(T_out + 16 * (size_t)c, T, 16 * sizeof(double));
        const double* zs = D.z.data() + (size_t)c * 6 * k;
        const double* zt = zs + 3 * k;
        for (int64_t i = 0; i < k && src_out; ++i) {  // add_noise_to_point_cloud: p += sd * z
            double* o = src_out + ((size_t)c * k + i) * 3;
            const double* p = cloud + 3 * (size_t)D.src_idx[(size_t)i];
            for (int a = 0; a < 3; ++a) o[a] = p[a] + sd * zs[3 * i + a];
        }
        for (int64_t i = 0; i < k && tgt_out; ++i) {  // Transform(T) of the full cloud, then the subset
            double* o = tgt_out + ((size_t)c * k + i) * 3;
            double q[3];
            transform_point(T, cloud + 3 * (size_t)D.tgt_idx[(size_t)c * k + i], q);
            for (int a = 0; a < 3; ++a) o[a] = q[a] + sd * zt[3 * i + a];
        }
    }
    return k;
}

}  // extern "C"
