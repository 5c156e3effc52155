// cc.cpp — metrics and pose-file formats of the reference's benchmark drivers
// (include/se3icp_cc.h).  Host code; restated from src/cc.cpp and examples/*.cpp.
#include "se3icp_cc.h"

#include "refrand.hpp"

#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

namespace {

constexpr double kRadToDeg = 180.0 / M_PI;

// C = A^T B (3x3 row-major)
void mul_at_b(const double* A, const double* B, double* C) {
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
            C[r * 3 + c] = A[0 * 3 + r] * B[0 * 3 + c] + A[1 * 3 + r] * B[1 * 3 + c] + A[2 * 3 + r] * B[2 * 3 + c];
}

void apply(const double* T, const double* p, double* q) {
    for (int r = 0; r < 3; ++r) q[r] = T[r * 4] * p[0] + T[r * 4 + 1] * p[1] + T[r * 4 + 2] * p[2] + T[r * 4 + 3];
}

double safe_acos(double x) {  // cc.cpp:39-47
    if (x <= -1.0) return M_PI;
    if (x >= 1.0) return 0.0;
    return std::acos(x);
}

// [R|t] rows from 12 whitespace-separated values
bool parse12(const std::string& line, double* M) {
    std::istringstream s(line);
    double v[12];
    for (int j = 0; j < 12; ++j)
        if (!(s >> v[j])) return false;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 4; ++c) M[r * 4 + c] = v[r * 4 + c];
    M[12] = M[13] = M[14] = 0.0;
    M[15] = 1.0;
    return true;
}

int64_t read12(const char* path, double* out, int64_t cap, int stride) {
    std::ifstream f(path);
    if (!f.is_open()) return -1;
    std::string line;
    int64_t n = 0, k = 0;
    while (std::getline(f, line)) {
        const bool use = (k++ % stride) == 0;  // benchmark_kitti.cpp:80-97 reads every other line
        if (!use) continue;
        double M[16];
        if (!parse12(line, M)) continue;
        if (out && n < cap) std::memcpy(out + 16 * n, M, sizeof(M));
        ++n;
    }
    return n;
}

}  // namespace

extern "C" {

// cc::rot_3d (cc.cpp:22-30): Rz(yaw) Ry(pitch) Rx(roll) through Eigen's quaternion
// arithmetic, bit for bit (refrand.hpp; pinned by the reference's fixture)
void se3icp_cc_rot_3d(double roll, double pitch, double yaw, double R[9]) { se3icp::refrand::rot_3d(roll, pitch, yaw, R); }

double se3icp_cc_angular_error_so3(const double R1[9], const double R2[9]) {
    // |vee(log M)| = theta; sin(theta) from the skew part, cos(theta) from the trace
    double M[9];
    mul_at_b(R1, R2, M);
    const double wx = M[7] - M[5], wy = M[2] - M[6], wz = M[3] - M[1];
    const double s = 0.5 * std::sqrt(wx * wx + wy * wy + wz * wz);
    const double c = 0.5 * (M[0] + M[4] + M[8] - 1.0);
    return std::atan2(s, c) * kRadToDeg;
}

double se3icp_cc_angular_error_so3_alt(const double R1[9], const double R2[9]) {
    double M[9];
    mul_at_b(R1, R2, M);
    return std::abs(safe_acos((M[0] + M[4] + M[8] - 1.0) / 2.0)) * kRadToDeg;
}

double se3icp_cc_error_filterreg(const double* xyz, int64_t n, const double T_gt[16], const double T_est[16]) {
    if (n <= 0) return 0.0;
    double acc = 0.0;
    for (int64_t i = 0; i < n; ++i) {
        double a[3], b[3];
        apply(T_gt, xyz + 3 * i, a);
        apply(T_est, xyz + 3 * i, b);
        const double dx = a[0] - b[0], dy = a[1] - b[1], dz = a[2] - b[2];
        acc += std::sqrt(dx * dx + dy * dy + dz * dz);
    }
    return acc / (double)n;
}

void se3icp_cc_rot2euler(const double R[9], double euler[3]) {
    const double m00 = R[0], m02 = R[2], m10 = R[3], m11 = R[4], m12 = R[5], m20 = R[6], m22 = R[8];
    double bank, attitude, heading;
    if (m10 > 0.998) {  // singularity at north pole
        bank = 0;
        attitude = M_PI / 2;
        heading = std::atan2(m02, m22);
    } else if (m10 < -0.998) {
        bank = 0;
        attitude = -M_PI / 2;
        heading = std::atan2(m02, m22);
    } else {
        bank = std::atan2(-m12, m11);
        attitude = std::asin(m10);
        heading = std::atan2(-m20, m00);
    }
    euler[0] = bank;
    euler[1] = attitude;
    euler[2] = heading;
}

static double angle_difference(double a, double b) {  // benchmark_lounge.cpp:52-56
    double diff = std::fmod(a - b, 360.0);
    if (diff > 180.0) diff = 360.0 - diff;
    return std::abs(diff);
}

double se3icp_cc_avg_eul_error(const double R1[9], const double R2[9]) {
    double E[3], K[3];
    se3icp_cc_rot2euler(R1, E);
    se3icp_cc_rot2euler(R2, K);
    double s = 0.0;
    for (int i = 0; i < 3; ++i)
        s += angle_difference(std::fmod(E[i] * kRadToDeg, 360.0), std::fmod(K[i] * kRadToDeg, 360.0));
    return s / 3.0;
}

double se3icp_cc_evaluate_lrf_quality(const double* src_frames, const double* tgt_frames, const double map_gt[16],
                                      const int32_t* pairs, int64_t n_pairs) {
    if (n_pairs <= 0) return 0.0;
    double acc = 0.0;
    for (int64_t k = 0; k < n_pairs; ++k) {
        const double* S = src_frames + 16 * (int64_t)pairs[2 * k];
        const double* T = tgt_frames + 16 * (int64_t)pairs[2 * k + 1];
        double A[9], B[9];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) {
                A[r * 3 + c] = map_gt[r * 4] * S[c] + map_gt[r * 4 + 1] * S[4 + c] + map_gt[r * 4 + 2] * S[8 + c];
                B[r * 3 + c] = T[r * 4 + c];
            }
        acc += se3icp_cc_angular_error_so3_alt(A, B);
    }
    return acc / (double)n_pairs;
}

int se3icp_cc_evaluate_trajectory(const double* gt, const double* est, int64_t n, double out[3]) {
    if (!gt || !est || !out || n <= 0) return -1;
    double rot = 0.0, tra = 0.0;
    int64_t fails = 0;
    for (int64_t i = 0; i < n; ++i) {
        const double* G = gt + 16 * i;
        const double* E = est + 16 * i;
        double RG[9], RE[9];
        for (int r = 0; r < 3; ++r)
            for (int c = 0; c < 3; ++c) { RG[r * 3 + c] = G[r * 4 + c]; RE[r * 3 + c] = E[r * 4 + c]; }
        const double ri = se3icp_cc_angular_error_so3(RG, RE);
        const double dx = G[3] - E[3], dy = G[7] - E[7], dz = G[11] - E[11];
        const double ti = std::sqrt(dx * dx + dy * dy + dz * dz);
        rot += ri;
        tra += ti;
        if (ri > 2.0 || ti > 0.25) ++fails;
    }
    out[0] = tra / (double)n;
    out[1] = rot / (double)n;
    out[2] = (double)(n - fails) / (double)n;
    return 0;
}

int64_t se3icp_cc_read_trajectory(const char* path, double* out, int64_t cap) { return read12(path, out, cap, 1); }
int64_t se3icp_cc_read_kitti_poses(const char* path, double* out, int64_t cap) { return read12(path, out, cap, 2); }

int64_t se3icp_cc_read_redwood_log(const char* path, double* out, int32_t* ids, int64_t cap) {
    FILE* f = std::fopen(path, "r");
    if (!f) return -1;
    char buf[1024];
    int64_t n = 0;
    while (std::fgets(buf, sizeof(buf), f)) {
        if (std::strlen(buf) == 0 || buf[0] == '#') continue;
        int id1 = 0, id2 = 0, frame = 0;
        if (std::sscanf(buf, "%d %d %d", &id1, &id2, &frame) != 3) continue;
        double M[16];
        bool ok = true;
        for (int r = 0; r < 4 && ok; ++r) {
            ok = std::fgets(buf, sizeof(buf), f) &&
                 std::sscanf(buf, "%lf %lf %lf %lf", &M[r * 4], &M[r * 4 + 1], &M[r * 4 + 2], &M[r * 4 + 3]) == 4;
        }
        if (!ok) break;
        if (n < cap) {
            if (out) std::memcpy(out + 16 * n, M, sizeof(M));
            if (ids) { ids[3 * n] = id1; ids[3 * n + 1] = id2; ids[3 * n + 2] = frame; }
        }
        ++n;
    }
    std::fclose(f);
    return n;
}

int se3icp_cc_write_trajectory(const char* path, const double* poses, int64_t n) {
    FILE* f = std::fopen(path, "w");
    if (!f) return -1;
    for (int64_t i = 0; i < n; ++i) {
        const double* M = poses + 16 * i;
        for (int k = 0; k < 12; ++k) std::fprintf(f, k ? " %.17g" : "%.17g", M[k]);
        std::fprintf(f, "\n");
    }
    return std::fclose(f) == 0 ? 0 : -1;
}

int se3icp_cc_write_redwood_log(const char* path, const double* poses, const int32_t* ids, int64_t n) {
    FILE* f = std::fopen(path, "w");  // RGBDTrajectory::SaveToFile, benchmark_lounge.cpp:127-139
    if (!f) return -1;
    for (int64_t i = 0; i < n; ++i) {
        const double* M = poses + 16 * i;
        std::fprintf(f, "%d\t%d\t%d\n", ids[3 * i], ids[3 * i + 1], ids[3 * i + 2]);
        for (int r = 0; r < 4; ++r)
            std::fprintf(f, "%.8f %.8f %.8f %.8f\n", M[r * 4], M[r * 4 + 1], M[r * 4 + 2], M[r * 4 + 3]);
    }
    return std::fclose(f) == 0 ? 0 : -1;
}

}  // extern "C"
