// loopdev.hpp — device helpers shared by the per-iteration kernels (k_nn.hip, k_loop.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>
#include <cmath>

#include "view.hpp"

namespace se3icp {
namespace loopdev {

// query = T * M0 for the 12-vector packing [R(:,0) R(:,1) R(:,2) t]; equal to the
// reference's per-iteration update source_se3_cloud_[k] = T_i * source_se3_cloud_[k]
// (ISR.cpp:713-716) composed over the iterations, T = T_n ... T_1 (ISR.cpp:710).
__device__ __forceinline__ void pose_frame(const double* T, const double* m, double* q) {
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r)
            q[c * 3 + r] = T[r * 4 + 0] * m[c * 3 + 0] + T[r * 4 + 1] * m[c * 3 + 1] + T[r * 4 + 2] * m[c * 3 + 2];
#pragma unroll
    for (int r = 0; r < 3; ++r) q[9 + r] = T[r * 4 + 0] * m[9] + T[r * 4 + 1] * m[10] + T[r * 4 + 2] * m[11] + T[r * 4 + 3];
}
// source_moving_ point = T * p0 (PointCloud::Transform composed, ISR.cpp:706)
__device__ __forceinline__ void pose_point(const double* T, double x, double y, double z, double* q) {
#pragma unroll
    for (int r = 0; r < 3; ++r) q[r] = T[r * 4 + 0] * x + T[r * 4 + 1] * y + T[r * 4 + 2] * z + T[r * 4 + 3];
}

__device__ __forceinline__ void load_T(const PairDev* P, double* T) {
#pragma unroll
    for (int i = 0; i < 12; ++i) T[i] = P->T[i];
}

// f64 query vector of source point g (global slot) in the phase's search space
template <int D>
__device__ __forceinline__ void query_f64(const View& v, const double* T, int g, double* q) {
    if constexpr (D == 12) {
        double m[12];
#pragma unroll
        for (int r = 0; r < 12; ++r) m[r] = v.fr64[(size_t)g * 12 + r];
        pose_frame(T, m, q);
    } else {
        pose_point(T, v.xyz64[g], v.xyz64[v.ld + g], v.xyz64[2 * (size_t)v.ld + g], q);
    }
}

// Rigorous bound on |f32 squared distance - exact squared distance of the f64 vectors|
// (DESIGN.md "Certified f32 arg-min"): both vectors rounded to f32 (u = 2^-24), D
// differences and a D-term FMA chain; na, nb bound the two vector norms.
__device__ __forceinline__ float f32_err(float d, float na, float nb, int D) {
    const float u = 5.9604645e-08f;
    const float s = na + nb;
    return 1.25f * (2.f * u * s * sqrtf(fmaxf(d, 0.f)) + (float)(D + 3) * u * d + 4.f * u * u * s * s) + 1e-30f;
}

// nanoflann L2_Adaptor::evalMetric order (groups of 4), no FMA contraction
__device__ __forceinline__ double l2_nanoflann12(const double* a, const double* b) {
#pragma clang fp contract(off)
    double result = 0.0;
#pragma unroll
    for (int d = 0; d < 12; d += 4) {
        const double d0 = a[d] - b[d], d1 = a[d + 1] - b[d + 1], d2 = a[d + 2] - b[d + 2], d3 = a[d + 3] - b[d + 3];
        result += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
    }
    return result;
}
__device__ __forceinline__ double l2_nanoflann3(const double* a, const double* b) {
#pragma clang fp contract(off)
    const double d0 = a[0] - b[0], d1 = a[1] - b[1], d2 = a[2] - b[2];
    return (d0 * d0 + d1 * d1) + d2 * d2;
}

// target 12-D search vector j (alpha-weighted rotation rows + translation rows; for
// run_se3_icp_with_cf the translation rows are the points, ISR.cpp:834-836)
__device__ __forceinline__ void target12(const View& v, const CloudDev& ct, bool cf, int j, double* b) {
    const int gt = ct.off + j;
#pragma unroll
    for (int r = 0; r < 9; ++r) b[r] = v.fr64[(size_t)gt * 12 + r];
    if (cf) {
        b[9] = v.xyz64[gt]; b[10] = v.xyz64[v.ld + gt]; b[11] = v.xyz64[2 * (size_t)v.ld + gt];
    } else {
        b[9] = v.fr64[(size_t)gt * 12 + 9]; b[10] = v.fr64[(size_t)gt * 12 + 10]; b[11] = v.fr64[(size_t)gt * 12 + 11];
    }
}

// distance stored with the correspondence: the R3 distance between translation parts
// in the SE(3) phase (ISR.cpp:465-468, beta-weighted target_se3_cloud_ translation even
// in the cf variant) and the 3-D NN distance in the R3 phase (ISR.cpp:411-413), f64 -> float
__device__ __forceinline__ float stored_dist(const View& v, int phase, const CloudDev& ct, const double* Q, int j) {
    const int gt = ct.off + j;
    if (phase == PHASE_SE3) {
        const double dx = Q[9] - v.fr64[(size_t)gt * 12 + 9];
        const double dy = Q[10] - v.fr64[(size_t)gt * 12 + 10];
        const double dz = Q[11] - v.fr64[(size_t)gt * 12 + 11];
        return (float)sqrt((dx * dx + dy * dy) + dz * dz);
    }
    const double b[3] = {v.xyz64[gt], v.xyz64[v.ld + gt], v.xyz64[2 * (size_t)v.ld + gt]};
    return (float)sqrt(l2_nanoflann3(Q, b));
}

__device__ __forceinline__ bool key_less(double da, int ia, double db, int ib) {
    return da < db || (da == db && ia < ib);
}

}  // namespace loopdev
}  // namespace se3icp
