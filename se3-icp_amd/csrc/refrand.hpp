// refrand.hpp — the arithmetic the reference's synthetic drivers use to make problems,
// restated on raw doubles so that it reproduces their numbers bit for bit (host only).
//   * cc::rot_3d (src/cc.cpp:22-30): Eigen AngleAxisd -> Quaterniond product
//     yaw * pitch * roll -> toRotationMatrix (Eigen's scalar formulas);
//   * PointCloud::Transform (ISR.cpp:706 and the drivers): each coordinate
//     ((R0 x + R1 y) + R2 z) + t, no FMA (the 4x4 * (x, y, z, 1) product, / w = 1);
//   * PointCloud::RandomDownSample (Open3D 0.19) under utility::random::Seed(s): std::shuffle
//     of 0..n-1 with the std::mt19937 engine, the first (int)(ratio * n) kept, selected in
//     index order.
// Pinned by the reference's own fixture: created_example_reg_problem/source.ply is the
// RandomDownSample(0.02) of stanford_bunny.ply x 50 under Seed(1), and target.ply its
// Transform by rot_3d(pi/9, pi/8, -pi/7), t = (1, 2, 3) -- both reproduced exactly
// (tests/test_reference_streams.py).
#pragma once
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <numeric>
#include <random>
#include <vector>

namespace se3icp {
namespace refrand {

#pragma clang fp contract(off)

struct Quat { double w, x, y, z; };
inline Quat angle_axis(double angle, int axis) {  // Eigen: Quaternion(AngleAxis)
    const double s = std::sin(0.5 * angle), c = std::cos(0.5 * angle);
    Quat q{c, 0.0, 0.0, 0.0};
    (axis == 0 ? q.x : axis == 1 ? q.y : q.z) = s;
    return q;
}
inline Quat qmul(const Quat& a, const Quat& b) {  // Eigen quat_product (generic)
    return Quat{a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
                a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z, a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x};
}
// cc::rot_3d(roll, pitch, yaw), row-major R[9]
inline void rot_3d(double roll, double pitch, double yaw, double R[9]) {
    const Quat q = qmul(qmul(angle_axis(yaw, 2), angle_axis(pitch, 1)), angle_axis(roll, 0));
    const double tx = 2.0 * q.x, ty = 2.0 * q.y, tz = 2.0 * q.z;
    const double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    const double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    const double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz;         R[2] = txz + twy;
    R[3] = txy + twz;         R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
    R[6] = txz - twy;         R[7] = tyz + twx;         R[8] = 1.0 - (txx + tyy);
}
// PointCloud::Transform of one point by the row-major 4x4 T
inline void transform_point(const double* T, const double* p, double* q) {
    for (int r = 0; r < 3; ++r) q[r] = ((T[4 * r] * p[0] + T[4 * r + 1] * p[1]) + T[4 * r + 2] * p[2]) + T[4 * r + 3] * 1.0;
}
// PointCloud::RandomDownSample with the (continuing) engine: kept indices, ascending
inline std::vector<int64_t> random_downsample(int64_t n, double ratio, std::mt19937& engine) {
    std::vector<size_t> idx((size_t)n);
    std::iota(idx.begin(), idx.end(), (size_t)0);
    std::shuffle(idx.begin(), idx.end(), engine);
    idx.resize((size_t)(int)(ratio * (double)n));
    std::vector<char> mask((size_t)n, 0);
    for (size_t i : idx) mask[i] = 1;
    std::vector<int64_t> out;
    out.reserve(idx.size());
    for (int64_t i = 0; i < n; ++i)
        if (mask[(size_t)i]) out.push_back(i);
    return out;
}

// Every random draw of examples/benchmark_synthetic.cpp:91-160 for n_cases cases, in the
// driver's order of use (gen_ref.cpp): the shared source subset, per case T and the target
// subset, and the N(0, 1) noise words (source copy then target, case after case).  Applied
// by se3icp_synthetic_reference on the host and by k_gen.hip k_apply_reference on the GPU
// with the same arithmetic (no FMA), so both give the same bits.
struct ReferenceDraws {
    int64_t k = 0;                  // (int)(ratio * n) points per cloud
    std::vector<int32_t> src_idx;   // [k] kept indices of the shared source subset, ascending
    std::vector<int32_t> tgt_idx;   // [n_cases * k] per case, ascending
    std::vector<double> T;          // [n_cases * 16] row-major
    std::vector<double> z;          // [n_cases * 2 * k * 3]: case c: source (k x 3) then target (k x 3)
};
ReferenceDraws draw_reference(int64_t n, int32_t n_cases, double ratio, double t_range, double r_range,
                              bool args_left_to_right, bool want_noise);

}  // namespace refrand
}  // namespace se3icp
