// devmath.hpp — f64 small-matrix math used by the setup kernels (device only).
//
// Restates, for the GPU, the third-party arithmetic the reference calls per point:
//   * Eigen::SelfAdjointEigenSolver<Matrix3d> (TOLDI normal, ISR.cpp:275-281)
//     -> cyclic Jacobi, eigenvalues ascending;
//   * Open3D FastEigen3x3 (EstimateNormals fast path, ISR.cpp:643 / :43);
//   * GetRotationFromE1ToX (ISR.cpp:4-14).
#pragma once
#include <hip/hip_runtime.h>

namespace se3icp {

struct d3 { double x, y, z; };
__device__ __forceinline__ d3 mk3(double a, double b, double c) { return d3{a, b, c}; }
__device__ __forceinline__ d3 operator-(d3 a, d3 b) { return d3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ d3 operator+(d3 a, d3 b) { return d3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ d3 operator*(double s, d3 a) { return d3{s * a.x, s * a.y, s * a.z}; }
__device__ __forceinline__ double dot3(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ d3 cross3(d3 a, d3 b) {
    return d3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// Symmetric 3x3 eigen-decomposition by cyclic Jacobi rotations.  a is symmetric
// (row-major, only a[0..8] used); returns eigenvector of the smallest eigenvalue.
__device__ inline d3 jacobi_smallest_evec(double a00, double a01, double a02, double a11, double a12, double a22) {
    double a[3][3] = {{a00, a01, a02}, {a01, a11, a12}, {a02, a12, a22}};
    double v[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int sweep = 0; sweep < 32; ++sweep) {
        const double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
        const double dg = a[0][0] * a[0][0] + a[1][1] * a[1][1] + a[2][2] * a[2][2];
        if (off == 0.0 || off <= 1e-36 * dg) break;
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            const int p = (r == 2) ? 1 : 0;
            const int q = (r == 0) ? 1 : 2;
            const double apq = a[p][q];
            if (apq != 0.0) {
                const double theta = (a[q][q] - a[p][p]) / (2.0 * apq);
                const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
                const double c = 1.0 / sqrt(t * t + 1.0);
                const double s = t * c;
    #pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double akp = a[k][p], akq = a[k][q];
                    a[k][p] = c * akp - s * akq;
                    a[k][q] = s * akp + c * akq;
                }
    #pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double apk = a[p][k], aqk = a[q][k];
                    a[p][k] = c * apk - s * aqk;
                    a[q][k] = s * apk + c * aqk;
                }
    #pragma unroll
                for (int k = 0; k < 3; ++k) {
                    const double vkp = v[k][p], vkq = v[k][q];
                    v[k][p] = c * vkp - s * vkq;
                    v[k][q] = s * vkp + c * vkq;
                }
            }
        }
    }
    // column of the smallest diagonal entry, as a 0/1-weighted sum: a select between
    // array elements would be turned back into a runtime-indexed (scratch) load
    const bool m1 = a[1][1] < a[0][0];
    const bool m2 = a[2][2] < (m1 ? a[1][1] : a[0][0]);
    const double w2 = m2 ? 1.0 : 0.0, w1 = (!m2 && m1) ? 1.0 : 0.0, w0 = 1.0 - w1 - w2;
    return d3{w0 * v[0][0] + w1 * v[0][1] + w2 * v[0][2], w0 * v[1][0] + w1 * v[1][1] + w2 * v[1][2],
              w0 * v[2][0] + w1 * v[2][1] + w2 * v[2][2]};
}

// Open3D FastEigen3x3 helpers (Geometric Tools "RobustEigenSymmetric3x3").
__device__ inline d3 fe_evec0(const double A[3][3], double eval0) {
    const d3 row0{A[0][0] - eval0, A[0][1], A[0][2]};
    const d3 row1{A[0][1], A[1][1] - eval0, A[1][2]};
    const d3 row2{A[0][2], A[1][2], A[2][2] - eval0};
    const d3 r0xr1 = cross3(row0, row1), r0xr2 = cross3(row0, row2), r1xr2 = cross3(row1, row2);
    const double d0 = dot3(r0xr1, r0xr1), d1 = dot3(r0xr2, r0xr2), d2 = dot3(r1xr2, r1xr2);
    double dmax = d0;
    int imax = 0;
    if (d1 > dmax) { dmax = d1; imax = 1; }
    if (d2 > dmax) { imax = 2; }
    if (imax == 0) return (1.0 / sqrt(d0)) * r0xr1;
    if (imax == 1) return (1.0 / sqrt(d1)) * r0xr2;
    return (1.0 / sqrt(d2)) * r1xr2;
}
__device__ inline d3 fe_evec1(const double A[3][3], d3 e0, double eval1) {
    d3 U;
    if (fabs(e0.x) > fabs(e0.y)) {
        const double il = 1 / sqrt(e0.x * e0.x + e0.z * e0.z);
        U = d3{-e0.z * il, 0, e0.x * il};
    } else {
        const double il = 1 / sqrt(e0.y * e0.y + e0.z * e0.z);
        U = d3{0, e0.z * il, -e0.y * il};
    }
    const d3 V = cross3(e0, U);
    const d3 AU{A[0][0] * U.x + A[0][1] * U.y + A[0][2] * U.z, A[0][1] * U.x + A[1][1] * U.y + A[1][2] * U.z,
                A[0][2] * U.x + A[1][2] * U.y + A[2][2] * U.z};
    const d3 AV{A[0][0] * V.x + A[0][1] * V.y + A[0][2] * V.z, A[0][1] * V.x + A[1][1] * V.y + A[1][2] * V.z,
                A[0][2] * V.x + A[1][2] * V.y + A[2][2] * V.z};
    double m00 = U.x * AU.x + U.y * AU.y + U.z * AU.z - eval1;
    double m01 = U.x * AV.x + U.y * AV.y + U.z * AV.z;
    double m11 = V.x * AV.x + V.y * AV.y + V.z * AV.z - eval1;
    const double a00 = fabs(m00), a01 = fabs(m01), a11 = fabs(m11);
    if (a00 >= a11) {
        if (fmax(a00, a01) > 0) {
            if (a00 >= a01) { m01 /= m00; m00 = 1 / sqrt(1 + m01 * m01); m01 *= m00; }
            else { m00 /= m01; m01 = 1 / sqrt(1 + m00 * m00); m00 *= m01; }
            return m01 * U - m00 * V;
        }
        return U;
    }
    if (fmax(a11, a01) > 0) {
        if (a11 >= a01) { m01 /= m11; m11 = 1 / sqrt(1 + m01 * m01); m01 *= m11; }
        else { m11 /= m01; m01 = 1 / sqrt(1 + m11 * m11); m11 *= m01; }
        return m11 * U - m01 * V;
    }
    return U;
}
// Open3D FastEigen3x3: eigenvector of the smallest eigenvalue of a covariance.
__device__ inline d3 fast_eigen3x3(double c00, double c01, double c02, double c11, double c12, double c22) {
    double A[3][3] = {{c00, c01, c02}, {c01, c11, c12}, {c02, c12, c22}};
    double mc = A[0][0];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) mc = fmax(mc, A[i][j]);
    if (mc == 0) return d3{0, 0, 0};
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) A[i][j] /= mc;
    const double nrm = A[0][1] * A[0][1] + A[0][2] * A[0][2] + A[1][2] * A[1][2];
    if (nrm > 0) {
        const double q = (A[0][0] + A[1][1] + A[2][2]) / 3;
        const double b00 = A[0][0] - q, b11 = A[1][1] - q, b22 = A[2][2] - q;
        const double p = sqrt((b00 * b00 + b11 * b11 + b22 * b22 + nrm * 2) / 6);
        const double c00_ = b11 * b22 - A[1][2] * A[1][2];
        const double c01_ = A[0][1] * b22 - A[1][2] * A[0][2];
        const double c02_ = A[0][1] * A[1][2] - b11 * A[0][2];
        const double det = (b00 * c00_ - A[0][1] * c01_ + A[0][2] * c02_) / (p * p * p);
        double half_det = fmin(fmax(det * 0.5, -1.0), 1.0);
        const double angle = acos(half_det) / 3.0;
        const double two_thirds_pi = 2.09439510239319549;
        const double beta2 = cos(angle) * 2;
        const double beta0 = cos(angle + two_thirds_pi) * 2;
        const double beta1 = -(beta0 + beta2);
        const double e0 = q + p * beta0, e1 = q + p * beta1, e2 = q + p * beta2;
        if (half_det >= 0) {
            const d3 v2 = fe_evec0(A, e2);
            if (e2 < e0 && e2 < e1) return v2;
            const d3 v1 = fe_evec1(A, v2, e1);
            if (e1 < e0 && e1 < e2) return v1;
            return cross3(v1, v2);
        }
        const d3 v0 = fe_evec0(A, e0);
        if (e0 < e1 && e0 < e2) return v0;
        const d3 v1 = fe_evec1(A, v0, e1);
        if (e1 < e0 && e1 < e2) return v1;
        return cross3(v0, v1);
    }
    if (A[0][0] < A[1][1] && A[0][0] < A[2][2]) return d3{1, 0, 0};
    if (A[1][1] < A[0][0] && A[1][1] < A[2][2]) return d3{0, 1, 0};
    return d3{0, 0, 1};
}

// The SE(3) 12-vector of point gp as its rows of the frame buffers (fr64 [ld][12] f64,
// fr32 [ld][12] f32; 16-byte stores).  f32 translation rows: the point itself for a cf
// target (ISR.cpp:834-836), else the beta-weighted translation.
__device__ __forceinline__ void store_frame_rows(double* fr64, float* fr32, int gp, const double* f12, bool cf_target,
                                                 double qx, double qy, double qz) {
    double2* r64 = reinterpret_cast<double2*>(fr64 + (size_t)gp * 12);
#pragma unroll
    for (int k = 0; k < 6; ++k) r64[k] = make_double2(f12[2 * k], f12[2 * k + 1]);
    float4* r32 = reinterpret_cast<float4*>(fr32 + (size_t)gp * 12);
    r32[0] = make_float4((float)f12[0], (float)f12[1], (float)f12[2], (float)f12[3]);
    r32[1] = make_float4((float)f12[4], (float)f12[5], (float)f12[6], (float)f12[7]);
    r32[2] = cf_target ? make_float4((float)f12[8], (float)qx, (float)qy, (float)qz)
                       : make_float4((float)f12[8], (float)f12[9], (float)f12[10], (float)f12[11]);
}

// GetRotationFromE1ToX (ISR.cpp:4-14) and Cov = Rx diag(eps,1,1) Rx^T (ISR.cpp:46-51),
// returned as the 6 unique entries (xx xy xz yy yz zz).  k_reduce recomputes it from the
// stored normal for every correspondence (no covariance array); no FMA contraction, so
// every call site rounds the same way.
__device__ inline void gicp_cov_from_normal(d3 n, double eps, double out[6]) {
#pragma clang fp contract(off)
    double R[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    const double c = n.x;  // e1 . n
    if (!(c < -0.99)) {
        const d3 v{0.0, -n.z, n.y};  // e1 x n
        const double S[3][3] = {{0, -v.z, v.y}, {v.z, 0, -v.x}, {-v.y, v.x, 0}};
        const double f = 1 / (1 + c);
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const double s2 = S[i][0] * S[0][j] + S[i][1] * S[1][j] + S[i][2] * S[2][j];
                R[i][j] = (i == j ? 1.0 : 0.0) + S[i][j] + s2 * f;
            }
    }
    // C = R diag(eps,1,1) R^T
    double C[3][3];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) C[i][j] = R[i][0] * eps * R[j][0] + R[i][1] * R[j][1] + R[i][2] * R[j][2];
    out[0] = C[0][0]; out[1] = C[0][1]; out[2] = C[0][2];
    out[3] = C[1][1]; out[4] = C[1][2]; out[5] = C[2][2];
}

}  // namespace se3icp
