// refcpu.cpp — CPU restatement of kenahm/se3-icp's IterativeSE3Registration.
//
// TEST INFRASTRUCTURE ONLY (the oracle / CPU baseline).  The product never links it.
//
// Every function cites the reference line(s) it restates (ISR.cpp =
// src/iterative_SE3_registration.cpp, ISR.hpp = include/iterative_SE3_registration.hpp).
// Third-party arithmetic the reference calls but does not vendor (Open3D v0.19,
// PCL 1.14, Eigen 3.x) is restated from their published algorithms; those
// restatements are marked [3P] and are pinned only end-to-end through the
// reference fixture created_example_reg_problem/ (see DESIGN.md "Oracle").
//
// Build: g++ -O3 -fopenmp -ffp-contract=off (no FMA contraction, like the
// reference's default x86-64 GCC build, so the nanoflann distance arithmetic
// below is reproduced operation for operation).

#include "refcpu.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <limits>
#include <numeric>
#include <vector>
#ifdef _OPENMP
#include <omp.h>
#endif

namespace {

// ---------------------------------------------------------------- small linear algebra
struct Vec3 {
    double x = 0, y = 0, z = 0;
    Vec3() = default;
    Vec3(double a, double b, double c) : x(a), y(b), z(c) {}
    double& operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
    double operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
inline Vec3 operator+(const Vec3& a, const Vec3& b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline Vec3 operator-(const Vec3& a, const Vec3& b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline Vec3 operator*(double s, const Vec3& a) { return {s * a.x, s * a.y, s * a.z}; }
inline Vec3 operator-(const Vec3& a) { return {-a.x, -a.y, -a.z}; }
inline Vec3& operator+=(Vec3& a, const Vec3& b) { a.x += b.x; a.y += b.y; a.z += b.z; return a; }
inline double dot(const Vec3& a, const Vec3& b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline Vec3 cross(const Vec3& a, const Vec3& b) {
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
inline double norm(const Vec3& a) { return std::sqrt(dot(a, a)); }

struct Mat3 {
    double m[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    static Mat3 I() { Mat3 r; r.m[0][0] = r.m[1][1] = r.m[2][2] = 1; return r; }
};
inline Mat3 mul(const Mat3& a, const Mat3& b) {
    Mat3 r;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) r.m[i][j] = a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j];
    return r;
}
inline Mat3 transpose(const Mat3& a) {
    Mat3 r;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) r.m[i][j] = a.m[j][i];
    return r;
}
inline Vec3 mul(const Mat3& a, const Vec3& v) {
    return {a.m[0][0] * v.x + a.m[0][1] * v.y + a.m[0][2] * v.z, a.m[1][0] * v.x + a.m[1][1] * v.y + a.m[1][2] * v.z,
            a.m[2][0] * v.x + a.m[2][1] * v.y + a.m[2][2] * v.z};
}
inline Mat3 add(const Mat3& a, const Mat3& b) {
    Mat3 r;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) r.m[i][j] = a.m[i][j] + b.m[i][j];
    return r;
}
inline Mat3 skew(const Vec3& v) {  // open3d::utility::SkewMatrix
    Mat3 r;
    r.m[0][1] = -v.z; r.m[0][2] = v.y;
    r.m[1][0] = v.z;  r.m[1][2] = -v.x;
    r.m[2][0] = -v.y; r.m[2][1] = v.x;
    return r;
}

struct Mat4 {
    double m[4][4];
    static Mat4 I() {
        Mat4 r;
        for (int i = 0; i < 4; i++)
            for (int j = 0; j < 4; j++) r.m[i][j] = (i == j) ? 1.0 : 0.0;
        return r;
    }
};
inline Mat4 mul(const Mat4& a, const Mat4& b) {
    Mat4 r;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            r.m[i][j] = ((a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j]) + a.m[i][2] * b.m[2][j]) + a.m[i][3] * b.m[3][j];
    return r;
}
inline double frob_diff(const Mat4& a, const Mat4& b) {
    double s = 0;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) { double d = a.m[i][j] - b.m[i][j]; s += d * d; }
    return std::sqrt(s);
}

// ------------------------------------------------ [3P] Eigen::SelfAdjointEigenSolver<Matrix3d>
// Restated as cyclic Jacobi (accurate to working precision; eigenvalues sorted
// ascending, eigenvectors as columns, like Eigen).  Used at ISR.cpp:275-281.
void sym_eig3(const Mat3& A, double w[3], Mat3& V) {
    double a[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) a[i][j] = 0.5 * (A.m[i][j] + A.m[j][i]);
    double v[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int sweep = 0; sweep < 64; sweep++) {
        double off = a[0][1] * a[0][1] + a[0][2] * a[0][2] + a[1][2] * a[1][2];
        double diag = a[0][0] * a[0][0] + a[1][1] * a[1][1] + a[2][2] * a[2][2];
        if (off == 0.0 || off <= 1e-36 * diag) break;
        static const int P[3] = {0, 0, 1}, Q[3] = {1, 2, 2};
        for (int r = 0; r < 3; r++) {
            int p = P[r], q = Q[r];
            double apq = a[p][q];
            if (apq == 0.0) continue;
            double theta = (a[q][q] - a[p][p]) / (2.0 * apq);
            double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
            double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
            for (int k = 0; k < 3; k++) {  // A <- A J  (columns p,q)
                double akp = a[k][p], akq = a[k][q];
                a[k][p] = c * akp - s * akq;
                a[k][q] = s * akp + c * akq;
            }
            for (int k = 0; k < 3; k++) {  // A <- J^T A (rows p,q)
                double apk = a[p][k], aqk = a[q][k];
                a[p][k] = c * apk - s * aqk;
                a[q][k] = s * apk + c * aqk;
            }
            for (int k = 0; k < 3; k++) {
                double vkp = v[k][p], vkq = v[k][q];
                v[k][p] = c * vkp - s * vkq;
                v[k][q] = s * vkp + c * vkq;
            }
        }
    }
    int ord[3] = {0, 1, 2};
    std::sort(ord, ord + 3, [&](int i, int j) { return a[i][i] < a[j][j]; });
    for (int c = 0; c < 3; c++) {
        w[c] = a[ord[c]][ord[c]];
        for (int k = 0; k < 3; k++) V.m[k][c] = v[k][ord[c]];
    }
}

// ------------------------------------------------ [3P] Open3D FastEigen3x3 (geometry/EstimateNormals.cpp)
// Robust closed-form eigenvector of the smallest eigenvalue (Geometric Tools).
Vec3 ComputeEigenvector0(const Mat3& A, double eval0) {
    Vec3 row0(A.m[0][0] - eval0, A.m[0][1], A.m[0][2]);
    Vec3 row1(A.m[0][1], A.m[1][1] - eval0, A.m[1][2]);
    Vec3 row2(A.m[0][2], A.m[1][2], A.m[2][2] - eval0);
    Vec3 r0xr1 = cross(row0, row1), r0xr2 = cross(row0, row2), r1xr2 = cross(row1, row2);
    double d0 = dot(r0xr1, r0xr1), d1 = dot(r0xr2, r0xr2), d2 = dot(r1xr2, r1xr2);
    double dmax = d0;
    int imax = 0;
    if (d1 > dmax) { dmax = d1; imax = 1; }
    if (d2 > dmax) { imax = 2; }
    if (imax == 0) return (1.0 / std::sqrt(d0)) * r0xr1;
    if (imax == 1) return (1.0 / std::sqrt(d1)) * r0xr2;
    return (1.0 / std::sqrt(d2)) * r1xr2;
}
Vec3 ComputeEigenvector1(const Mat3& A, const Vec3& evec0, double eval1) {
    Vec3 U, V;
    if (std::fabs(evec0.x) > std::fabs(evec0.y)) {
        double inv_length = 1 / std::sqrt(evec0.x * evec0.x + evec0.z * evec0.z);
        U = Vec3(-evec0.z * inv_length, 0, evec0.x * inv_length);
    } else {
        double inv_length = 1 / std::sqrt(evec0.y * evec0.y + evec0.z * evec0.z);
        U = Vec3(0, evec0.z * inv_length, -evec0.y * inv_length);
    }
    V = cross(evec0, U);
    Vec3 AU(A.m[0][0] * U.x + A.m[0][1] * U.y + A.m[0][2] * U.z, A.m[0][1] * U.x + A.m[1][1] * U.y + A.m[1][2] * U.z,
            A.m[0][2] * U.x + A.m[1][2] * U.y + A.m[2][2] * U.z);
    Vec3 AV(A.m[0][0] * V.x + A.m[0][1] * V.y + A.m[0][2] * V.z, A.m[0][1] * V.x + A.m[1][1] * V.y + A.m[1][2] * V.z,
            A.m[0][2] * V.x + A.m[1][2] * V.y + A.m[2][2] * V.z);
    double m00 = U.x * AU.x + U.y * AU.y + U.z * AU.z - eval1;
    double m01 = U.x * AV.x + U.y * AV.y + U.z * AV.z;
    double m11 = V.x * AV.x + V.y * AV.y + V.z * AV.z - eval1;
    double absM00 = std::fabs(m00), absM01 = std::fabs(m01), absM11 = std::fabs(m11);
    double max_abs_comp;
    if (absM00 >= absM11) {
        max_abs_comp = std::max(absM00, absM01);
        if (max_abs_comp > 0) {
            if (absM00 >= absM01) { m01 /= m00; m00 = 1 / std::sqrt(1 + m01 * m01); m01 *= m00; }
            else { m00 /= m01; m01 = 1 / std::sqrt(1 + m00 * m00); m00 *= m01; }
            return m01 * U - m00 * V;
        }
        return U;
    } else {
        max_abs_comp = std::max(absM11, absM01);
        if (max_abs_comp > 0) {
            if (absM11 >= absM01) { m01 /= m11; m11 = 1 / std::sqrt(1 + m01 * m01); m01 *= m11; }
            else { m11 /= m01; m01 = 1 / std::sqrt(1 + m11 * m11); m11 *= m01; }
            return m11 * U - m01 * V;
        }
        return U;
    }
}
Vec3 FastEigen3x3(Mat3 A) {
    double max_coeff = A.m[0][0];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) max_coeff = std::max(max_coeff, A.m[i][j]);
    if (max_coeff == 0) return Vec3(0, 0, 0);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) A.m[i][j] /= max_coeff;
    double norm = A.m[0][1] * A.m[0][1] + A.m[0][2] * A.m[0][2] + A.m[1][2] * A.m[1][2];
    if (norm > 0) {
        double q = (A.m[0][0] + A.m[1][1] + A.m[2][2]) / 3;
        double b00 = A.m[0][0] - q, b11 = A.m[1][1] - q, b22 = A.m[2][2] - q;
        double p = std::sqrt((b00 * b00 + b11 * b11 + b22 * b22 + norm * 2) / 6);
        double c00 = b11 * b22 - A.m[1][2] * A.m[1][2];
        double c01 = A.m[0][1] * b22 - A.m[1][2] * A.m[0][2];
        double c02 = A.m[0][1] * A.m[1][2] - b11 * A.m[0][2];
        double det = (b00 * c00 - A.m[0][1] * c01 + A.m[0][2] * c02) / (p * p * p);
        double half_det = det * 0.5;
        half_det = std::min(std::max(half_det, -1.0), 1.0);
        double angle = std::acos(half_det) / (double)3;
        const double two_thirds_pi = 2.09439510239319549;
        double beta2 = std::cos(angle) * 2;
        double beta0 = std::cos(angle + two_thirds_pi) * 2;
        double beta1 = -(beta0 + beta2);
        double eval0 = q + p * beta0, eval1 = q + p * beta1, eval2 = q + p * beta2;
        if (half_det >= 0) {
            Vec3 evec2 = ComputeEigenvector0(A, eval2);
            if (eval2 < eval0 && eval2 < eval1) return evec2;
            Vec3 evec1 = ComputeEigenvector1(A, evec2, eval1);
            if (eval1 < eval0 && eval1 < eval2) return evec1;
            return cross(evec1, evec2);
        } else {
            Vec3 evec0 = ComputeEigenvector0(A, eval0);
            if (eval0 < eval1 && eval0 < eval2) return evec0;
            Vec3 evec1 = ComputeEigenvector1(A, evec0, eval1);
            if (eval1 < eval0 && eval1 < eval2) return evec1;
            return cross(evec0, evec1);
        }
    }
    if (A.m[0][0] < A.m[1][1] && A.m[0][0] < A.m[2][2]) return Vec3(1, 0, 0);
    if (A.m[1][1] < A.m[0][0] && A.m[1][1] < A.m[2][2]) return Vec3(0, 1, 0);
    return Vec3(0, 0, 1);
}

// ------------------------------------------------ [3P] Eigen::JacobiSVD<Matrix3d> (for umeyama)
// One-sided Jacobi; singular values sorted descending like Eigen.
void svd3(const Mat3& A, Mat3& U, double s[3], Mat3& V) {
    double b[3][3];
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) b[i][j] = A.m[i][j];
    double v[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int sweep = 0; sweep < 64; sweep++) {
        bool rotated = false;
        static const int P[3] = {0, 0, 1}, Q[3] = {1, 2, 2};
        for (int r = 0; r < 3; r++) {
            int p = P[r], q = Q[r];
            double al = 0, be = 0, ga = 0;
            for (int i = 0; i < 3; i++) { al += b[i][p] * b[i][p]; be += b[i][q] * b[i][q]; ga += b[i][p] * b[i][q]; }
            if (ga == 0.0 || std::fabs(ga) <= 1e-17 * std::sqrt(al * be)) continue;
            rotated = true;
            double zeta = (be - al) / (2.0 * ga);
            double t = (zeta >= 0 ? 1.0 : -1.0) / (std::fabs(zeta) + std::sqrt(1.0 + zeta * zeta));
            double c = 1.0 / std::sqrt(1.0 + t * t), sn = c * t;
            for (int i = 0; i < 3; i++) {
                double bp = b[i][p], bq = b[i][q];
                b[i][p] = c * bp - sn * bq;
                b[i][q] = sn * bp + c * bq;
                double vp = v[i][p], vq = v[i][q];
                v[i][p] = c * vp - sn * vq;
                v[i][q] = sn * vp + c * vq;
            }
        }
        if (!rotated) break;
    }
    double sv[3];
    for (int j = 0; j < 3; j++) sv[j] = std::sqrt(b[0][j] * b[0][j] + b[1][j] * b[1][j] + b[2][j] * b[2][j]);
    int ord[3] = {0, 1, 2};
    std::sort(ord, ord + 3, [&](int i, int j) { return sv[i] > sv[j]; });
    Vec3 u[3];
    for (int c = 0; c < 3; c++) {
        int j = ord[c];
        s[c] = sv[j];
        for (int i = 0; i < 3; i++) V.m[i][c] = v[i][j];
        u[c] = Vec3(b[0][j], b[1][j], b[2][j]);
    }
    double tiny = 1e-300 + s[0] * 1e-15;
    for (int c = 0; c < 3; c++) {
        if (s[c] > tiny) {
            u[c] = (1.0 / s[c]) * u[c];
        } else if (c == 2) {
            u[2] = cross(u[0], u[1]);
        } else {  // rank <= 1: complete an orthonormal basis
            Vec3 a = u[0];
            Vec3 e = std::fabs(a.x) < 0.9 ? Vec3(1, 0, 0) : Vec3(0, 1, 0);
            Vec3 t = cross(a, e);
            u[1] = (1.0 / norm(t)) * t;
            u[2] = cross(u[0], u[1]);
            break;
        }
    }
    for (int c = 0; c < 3; c++)
        for (int i = 0; i < 3; i++) U.m[i][c] = u[c][i];
}
double det3(const Mat3& a) {
    return a.m[0][0] * (a.m[1][1] * a.m[2][2] - a.m[1][2] * a.m[2][1]) -
           a.m[0][1] * (a.m[1][0] * a.m[2][2] - a.m[1][2] * a.m[2][0]) +
           a.m[0][2] * (a.m[1][0] * a.m[2][1] - a.m[1][1] * a.m[2][0]);
}
// [3P] Eigen 3x3 inverse via cofactors.
Mat3 inverse3(const Mat3& a) {
    Mat3 c;
    c.m[0][0] = a.m[1][1] * a.m[2][2] - a.m[1][2] * a.m[2][1];
    c.m[0][1] = a.m[0][2] * a.m[2][1] - a.m[0][1] * a.m[2][2];
    c.m[0][2] = a.m[0][1] * a.m[1][2] - a.m[0][2] * a.m[1][1];
    c.m[1][0] = a.m[1][2] * a.m[2][0] - a.m[1][0] * a.m[2][2];
    c.m[1][1] = a.m[0][0] * a.m[2][2] - a.m[0][2] * a.m[2][0];
    c.m[1][2] = a.m[0][2] * a.m[1][0] - a.m[0][0] * a.m[1][2];
    c.m[2][0] = a.m[1][0] * a.m[2][1] - a.m[1][1] * a.m[2][0];
    c.m[2][1] = a.m[0][1] * a.m[2][0] - a.m[0][0] * a.m[2][1];
    c.m[2][2] = a.m[0][0] * a.m[1][1] - a.m[0][1] * a.m[1][0];
    double det = a.m[0][0] * c.m[0][0] + a.m[0][1] * c.m[1][0] + a.m[0][2] * c.m[2][0];
    double inv = 1.0 / det;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) c.m[i][j] *= inv;
    return c;
}
// [3P] Eigen MatrixFunctions .sqrt() of a symmetric PD matrix: V sqrt(L) V^T.
Mat3 sqrt_spd(const Mat3& a) {
    double w[3];
    Mat3 V;
    sym_eig3(a, w, V);
    Mat3 r;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int k = 0; k < 3; k++) s += V.m[i][k] * std::sqrt(std::max(w[k], 0.0)) * V.m[j][k];
            r.m[i][j] = s;
        }
    return r;
}

// ------------------------------------------------ [3P] Eigen LDLT<Matrix6d> solve (with pivoting)
// Open3D SolveLinearSystemPSD -> A.ldlt().solve(b); zero pivots act as a
// pseudo-inverse (Eigen LDLT::_solve_impl).
void ldlt_solve6(const double Ain[6][6], const double b[6], double x[6]) {
    const int n = 6;
    double a[6][6];
    for (int i = 0; i < n; i++)
        for (int j = 0; j < n; j++) a[i][j] = Ain[i][j];
    int tr[6];
    for (int k = 0; k < n; k++) {
        int p = k;
        double best = std::fabs(a[k][k]);
        for (int i = k + 1; i < n; i++)
            if (std::fabs(a[i][i]) > best) { best = std::fabs(a[i][i]); p = i; }
        tr[k] = p;
        if (p != k) {
            for (int j = 0; j < n; j++) std::swap(a[k][j], a[p][j]);
            for (int i = 0; i < n; i++) std::swap(a[i][k], a[i][p]);
        }
        // a[k][0..k-1] holds L(k, j); a[j][j] holds D(j)
        double temp[6];
        for (int j = 0; j < k; j++) temp[j] = a[j][j] * a[k][j];
        double s = 0;
        for (int j = 0; j < k; j++) s += a[k][j] * temp[j];
        a[k][k] -= s;
        for (int i = k + 1; i < n; i++) {
            double t = 0;
            for (int j = 0; j < k; j++) t += a[i][j] * temp[j];
            a[i][k] -= t;
        }
        double akk = a[k][k];
        if (std::fabs(akk) > 0.0) {
            for (int i = k + 1; i < n; i++) a[i][k] /= akk;
        }
        for (int i = k + 1; i < n; i++) a[k][i] = a[i][k];  // keep symmetric view for later swaps
    }
    double y[6];
    for (int i = 0; i < n; i++) y[i] = b[i];
    for (int k = 0; k < n; k++) std::swap(y[k], y[tr[k]]);
    for (int i = 0; i < n; i++)  // L y = Pb
        for (int j = 0; j < i; j++) y[i] -= a[i][j] * y[j];
    const double tol = std::numeric_limits<double>::min();
    for (int i = 0; i < n; i++) y[i] = (std::fabs(a[i][i]) > tol) ? y[i] / a[i][i] : 0.0;
    for (int i = n - 1; i >= 0; i--)  // L^T z = y
        for (int j = i + 1; j < n; j++) y[i] -= a[j][i] * y[j];
    for (int k = n - 1; k >= 0; k--) std::swap(y[k], y[tr[k]]);
    for (int i = 0; i < n; i++) x[i] = y[i];
}

// [3P] open3d::utility::TransformVector6dToMatrix4d: R = (AngleAxis(z)*AngleAxis(y)*AngleAxis(x)).matrix()
Mat4 vec6_to_mat4(const double x6[6]) {
    struct Q { double w, x, y, z; };
    auto qmul = [](Q a, Q b) {
        return Q{a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
                 a.w * b.y + a.y * b.w + a.z * b.x - a.x * b.z, a.w * b.z + a.z * b.w + a.x * b.y - a.y * b.x};
    };
    Q qz{std::cos(0.5 * x6[2]), 0, 0, std::sin(0.5 * x6[2])};
    Q qy{std::cos(0.5 * x6[1]), 0, std::sin(0.5 * x6[1]), 0};
    Q qx{std::cos(0.5 * x6[0]), std::sin(0.5 * x6[0]), 0, 0};
    Q q = qmul(qmul(qz, qy), qx);
    double tx = 2 * q.x, ty = 2 * q.y, tz = 2 * q.z;
    double twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
    double txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
    double tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
    Mat4 T = Mat4::I();
    T.m[0][0] = 1 - (tyy + tzz); T.m[0][1] = txy - twz;       T.m[0][2] = txz + twy;
    T.m[1][0] = txy + twz;       T.m[1][1] = 1 - (txx + tzz); T.m[1][2] = tyz - twx;
    T.m[2][0] = txz - twy;       T.m[2][1] = tyz + twx;       T.m[2][2] = 1 - (txx + tyy);
    T.m[0][3] = x6[3]; T.m[1][3] = x6[4]; T.m[2][3] = x6[5];
    return T;
}

// ------------------------------------------------ [3P] nanoflann (Open3D KDTreeFlann backend)
// L2_Adaptor::evalMetric: groups of 4 components, ((d0^2+d1^2)+d2^2)+d3^2 added to
// the running result, then the 0-3 trailing components one at a time.
inline double l2_nanoflann(const double* a, const double* b, int D) {
    double result = 0.0;
    int d = 0;
    for (; d + 3 < D; d += 4) {
        const double d0 = a[d] - b[d], d1 = a[d + 1] - b[d + 1], d2 = a[d + 2] - b[d + 2], d3 = a[d + 3] - b[d + 3];
        result += d0 * d0 + d1 * d1 + d2 * d2 + d3 * d3;
    }
    for (; d < D; d++) {
        const double df = a[d] - b[d];
        result += df * df;
    }
    return result;
}

// Exact kd-tree (leaf size 15 like Open3D's KDTreeFlann).  Structure differs from
// nanoflann's middle split, which changes only speed; the returned neighbours are
// the exact (d2, index)-lexicographic k smallest under l2_nanoflann (nanoflann's
// own tie order is unspecified; ties here go to the lowest index).
class KDTree {
  public:
    KDTree(const double* data, int n, int dim, int leaf = 15) : data_(data), n_(n), D_(dim), leaf_(leaf) {
        ind_.resize(n);
        std::iota(ind_.begin(), ind_.end(), 0);
        lo_.assign(D_, 0.0);
        hi_.assign(D_, 0.0);
        if (n > 0) {
            for (int d = 0; d < D_; d++) { lo_[d] = hi_[d] = pt(0)[d]; }
            for (int i = 1; i < n; i++)
                for (int d = 0; d < D_; d++) { lo_[d] = std::min(lo_[d], pt(i)[d]); hi_[d] = std::max(hi_[d], pt(i)[d]); }
            nodes_.reserve(2 * (n / leaf + 1) + 8);
            root_ = build(0, n);
        }
    }
    // k nearest of q, sorted ascending by (d2, idx).  Returns count (min(k, n)).
    int knn(const double* q, int k, int* oidx, double* od2) const {
        if (n_ == 0 || k <= 0) return 0;
        Result r{k, 0, oidx, od2};
        std::vector<double> dists(D_);
        double mind = 0;
        for (int d = 0; d < D_; d++) {
            double v = 0;
            if (q[d] < lo_[d]) v = lo_[d] - q[d];
            else if (q[d] > hi_[d]) v = q[d] - hi_[d];
            dists[d] = v * v;
            mind += dists[d];
        }
        search(root_, q, r, dists.data(), mind);
        return r.count;
    }

  private:
    struct Node { int left, right, begin, end, cutfeat; double divlow, divhigh; };
    struct Result {
        int cap, count;
        int* idx;
        double* d2;
        double worst() const { return count < cap ? std::numeric_limits<double>::infinity() : d2[cap - 1]; }
        void add(double d, int i) {
            if (count == cap && !(d < d2[cap - 1] || (d == d2[cap - 1] && i < idx[cap - 1]))) return;
            int j = count < cap ? count++ : cap - 1;
            while (j > 0 && (d2[j - 1] > d || (d2[j - 1] == d && idx[j - 1] > i))) {
                d2[j] = d2[j - 1];
                idx[j] = idx[j - 1];
                --j;
            }
            d2[j] = d;
            idx[j] = i;
        }
    };
    const double* pt(int i) const { return data_ + (size_t)i * D_; }
    int build(int begin, int end) {
        int id = (int)nodes_.size();
        nodes_.push_back(Node{-1, -1, begin, end, 0, 0, 0});
        if (end - begin <= leaf_) return id;
        int best = 0;
        double spread = -1;
        for (int d = 0; d < D_; d++) {
            double mn = pt(ind_[begin])[d], mx = mn;
            for (int i = begin + 1; i < end; i++) { double v = pt(ind_[i])[d]; mn = std::min(mn, v); mx = std::max(mx, v); }
            if (mx - mn > spread) { spread = mx - mn; best = d; }
        }
        int mid = (begin + end) / 2;
        std::nth_element(ind_.begin() + begin, ind_.begin() + mid, ind_.begin() + end,
                         [&](int a, int b) { return pt(a)[best] < pt(b)[best]; });
        double divlow = -std::numeric_limits<double>::infinity(), divhigh = std::numeric_limits<double>::infinity();
        for (int i = begin; i < mid; i++) divlow = std::max(divlow, pt(ind_[i])[best]);
        for (int i = mid; i < end; i++) divhigh = std::min(divhigh, pt(ind_[i])[best]);
        int l = build(begin, mid);
        int r = build(mid, end);
        nodes_[id].left = l;
        nodes_[id].right = r;
        nodes_[id].cutfeat = best;
        nodes_[id].divlow = divlow;
        nodes_[id].divhigh = divhigh;
        return id;
    }
    void search(int nid, const double* q, Result& r, double* dists, double mind) const {
        const Node& nd = nodes_[nid];
        if (nd.left < 0) {
            for (int i = nd.begin; i < nd.end; i++) {
                int id = ind_[i];
                r.add(l2_nanoflann(q, pt(id), D_), id);
            }
            return;
        }
        int f = nd.cutfeat;
        double v = q[f];
        double diff1 = v - nd.divlow, diff2 = v - nd.divhigh;
        int first, second;
        double cut;
        if (diff1 + diff2 < 0) { first = nd.left; second = nd.right; cut = diff2 * diff2; }
        else { first = nd.right; second = nd.left; cut = diff1 * diff1; }
        search(first, q, r, dists, mind);
        double saved = dists[f];
        // far side: along f the distance is at least |v - div|; recompute the
        // lower bound from scratch (no cancellation) and keep a 1e-12 slack so
        // rounding never prunes a node that holds an exact-distance tie.
        double lb_f = std::max(saved, cut);
        dists[f] = lb_f;
        double m2 = 0;
        for (int d = 0; d < D_; d++) m2 += dists[d];
        if (m2 * (1.0 - 1e-12) <= r.worst()) search(second, q, r, dists, m2);
        dists[f] = saved;
        (void)mind;
    }
    const double* data_;
    int n_, D_, leaf_;
    std::vector<int> ind_;
    std::vector<Node> nodes_;
    std::vector<double> lo_, hi_;
    int root_ = 0;
};

// ------------------------------------------------ point cloud (Open3D PointCloud subset)
struct Cloud {
    std::vector<Vec3> points;
    std::vector<Vec3> normals;
    std::vector<Mat3> covariances;
    const double* raw() const { return reinterpret_cast<const double*>(points.data()); }
};
static_assert(sizeof(Vec3) == 24, "Vec3 must be packed xyz");

// [3P] PointCloud::GetCenter (arithmetic mean, std::accumulate order)
Vec3 get_center(const Cloud& c) {
    Vec3 s(0, 0, 0);
    for (const auto& p : c.points) s += p;
    if (c.points.empty()) return s;
    const double n = (double)c.points.size();
    return Vec3(s.x / n, s.y / n, s.z / n);
}
// ISR.cpp:112-119
double largest_distance(const Vec3& ref, const Cloud& c) {
    double cur = -1.0;
    for (const auto& p : c.points) { double d = norm(p - ref); if (d > cur) cur = d; }
    return cur;
}
// [3P] PointCloud::Translate(t, relative=true) then Scale(s, center=0): p' = ((p + t) - 0)*s + 0
void translate(Cloud& c, const Vec3& t) { for (auto& p : c.points) p += t; }
void scale(Cloud& c, double s) { for (auto& p : c.points) p = Vec3(p.x * s, p.y * s, p.z * s); }

// [3P] PointCloud::Transform (TransformPoints / TransformNormals / TransformCovariances)
void transform(Cloud& c, const Mat4& T) {
    const int n = (int)c.points.size();
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; i++) {
        Vec3 p = c.points[i];
        c.points[i] = Vec3(((T.m[0][0] * p.x + T.m[0][1] * p.y) + T.m[0][2] * p.z) + T.m[0][3],
                           ((T.m[1][0] * p.x + T.m[1][1] * p.y) + T.m[1][2] * p.z) + T.m[1][3],
                           ((T.m[2][0] * p.x + T.m[2][1] * p.y) + T.m[2][2] * p.z) + T.m[2][3]);
    }
    Mat3 R;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R.m[i][j] = T.m[i][j];
    const int nn = (int)c.normals.size();
#pragma omp parallel for schedule(static)
    for (int i = 0; i < nn; i++) c.normals[i] = mul(R, c.normals[i]);
    const int nc = (int)c.covariances.size();
    Mat3 Rt = transpose(R);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < nc; i++) c.covariances[i] = mul(mul(R, c.covariances[i]), Rt);
}

// ------------------------------------------------ TOLDI LRF  (ISR.cpp:241-316, 318-331)
Mat4 toldi_frame(const Cloud& cloud, const KDTree& tree, const Vec3& central_point, int knn_pts) {
    std::vector<int> indices(knn_pts);
    std::vector<double> d2(knn_pts);
    double q[3] = {central_point.x, central_point.y, central_point.z};
    int cnt = tree.knn(q, knn_pts, indices.data(), d2.data());
    indices.resize(cnt);
    const auto& P = cloud.points;
    // ISR.cpp:256 radius = distance to the farthest of the k neighbours
    double computed_radius = norm(central_point - P[indices.back()]);
    // ISR.cpp:259-265 centroid quirk: sums i = 1 .. size/3 - 1 but divides by size/3
    Vec3 centroid(0, 0, 0);
    for (int i = 1; i < (int)(indices.size() / 3); i++) centroid += P[indices[i]];
    int rz_size = (int)(indices.size() / 3);
    centroid = Vec3(centroid.x / (double)rz_size, centroid.y / (double)rz_size, centroid.z / (double)rz_size);
    // ISR.cpp:268-272 covariance over i = 1 .. rz_size (inclusive)
    Mat3 cov;
    for (int i = 1; i < rz_size + 1; i++) {
        Vec3 v = P[indices[i]] - centroid;
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) cov.m[r][c] += v[r] * v[c];
    }
    // ISR.cpp:275-281 eigenvector of the smallest eigenvalue
    double w[3];
    Mat3 V;
    sym_eig3(cov, w, V);
    Vec3 n(V.m[0][0], V.m[1][0], V.m[2][0]);
    // ISR.cpp:286-298
    Vec3 acc(0, 0, 0), acc_s(0, 0, 0);
    for (int i = 1; i < (int)indices.size(); i++) {
        Vec3 v = P[indices[i]] - central_point;
        acc += v;
        double dn = dot(n, v);
        double vn = norm(v);
        double wi1 = (computed_radius - vn) * (computed_radius - vn);
        double wi2 = dn * dn;
        acc_s += (wi1 * wi2) * v;
    }
    if (dot(n, acc) < 0.0) n = -n;
    // ISR.cpp:300-306 (no guard for |x| == 0, as in the reference)
    Vec3 z = n;
    Vec3 x = acc_s - dot(acc_s, z) * z;
    x = (1 / norm(x)) * x;
    Vec3 y = cross(z, x);
    Mat4 F = Mat4::I();
    for (int r = 0; r < 3; r++) { F.m[r][0] = x[r]; F.m[r][1] = y[r]; F.m[r][2] = z[r]; F.m[r][3] = central_point[r]; }
    return F;
}
void toldi_all(const Cloud& cloud, const KDTree& tree, int k, std::vector<Mat4>& out) {
    out.resize(cloud.points.size());
    const int n = (int)cloud.points.size();
#pragma omp parallel for schedule(dynamic, 256)
    for (int i = 0; i < n; i++) out[i] = toldi_frame(cloud, tree, cloud.points[i], k);
}

// ------------------------------------------------ [3P] Open3D EstimateNormals (KNN, fast)
// EstimatePerPointCovariances -> ComputeCovariance (cumulants, incl. self) ->
// FastEigen3x3; zero normal -> (0,0,1); no prior normals => no orientation.
void estimate_normals(Cloud& c, int knn) {
    const int n = (int)c.points.size();
    KDTree tree(c.raw(), n, 3);
    c.normals.assign(n, Vec3(0, 0, 0));
#pragma omp parallel for schedule(dynamic, 256)
    for (int i = 0; i < n; i++) {
        std::vector<int> idx(knn);
        std::vector<double> d2(knn);
        const double q[3] = {c.points[i].x, c.points[i].y, c.points[i].z};
        int cnt = tree.knn(q, knn, idx.data(), d2.data());
        Mat3 cov = Mat3::I();
        if (cnt >= 3) {
            double cu[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            for (int j = 0; j < cnt; j++) {
                const Vec3& p = c.points[idx[j]];
                cu[0] += p.x; cu[1] += p.y; cu[2] += p.z;
                cu[3] += p.x * p.x; cu[4] += p.x * p.y; cu[5] += p.x * p.z;
                cu[6] += p.y * p.y; cu[7] += p.y * p.z; cu[8] += p.z * p.z;
            }
            for (int j = 0; j < 9; j++) cu[j] /= (double)cnt;
            cov.m[0][0] = cu[3] - cu[0] * cu[0];
            cov.m[1][1] = cu[6] - cu[1] * cu[1];
            cov.m[2][2] = cu[8] - cu[2] * cu[2];
            cov.m[0][1] = cov.m[1][0] = cu[4] - cu[0] * cu[1];
            cov.m[0][2] = cov.m[2][0] = cu[5] - cu[0] * cu[2];
            cov.m[1][2] = cov.m[2][1] = cu[7] - cu[1] * cu[2];
        }
        Vec3 nrm = FastEigen3x3(cov);
        if (norm(nrm) == 0.0) nrm = Vec3(0, 0, 1);
        c.normals[i] = nrm;
    }
}

// ISR.cpp:4-14 GetRotationFromE1ToX
Mat3 rotation_e1_to_x(const Vec3& x) {
    const Vec3 e1(1, 0, 0);
    Vec3 v = cross(e1, x);
    double cth = dot(e1, x);
    if (cth < -0.99) return Mat3::I();
    Mat3 sv = skew(v);
    double factor = 1 / (1 + cth);
    Mat3 sv2 = mul(sv, sv);
    Mat3 r = add(Mat3::I(), sv);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) r.m[i][j] += sv2.m[i][j] * factor;
    return r;
}
// ISR.cpp:33-52 InitializePointCloudForGeneralizedICP_modified
void init_gicp(Cloud& c, double eps) {
    if (!c.covariances.empty()) return;
    if (c.normals.empty()) estimate_normals(c, 20);
    const int n = (int)c.points.size();
    c.covariances.resize(n);
    Mat3 C;
    C.m[0][0] = eps; C.m[1][1] = 1; C.m[2][2] = 1;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < n; i++) {
        Mat3 Rx = rotation_e1_to_x(c.normals[i]);
        c.covariances[i] = mul(mul(Rx, C), transpose(Rx));
    }
}

// ------------------------------------------------ correspondences (pcl::Correspondence subset)
struct Corr { int q, m; float dist; };

// [3P] PCL CorrespondenceRejectorTrimmed::getRemainingCorrespondences (float ratio,
// nvalid = max(floor(ratio*N), nr_min_correspondences_ = 0)).  When nvalid >= N the input
// is copied unchanged (query order: the estimator then sums in query order); otherwise it
// is sorted by distance and cut to nvalid.  Unstable-sort ties are broken by query index.
std::vector<Corr> trim(const std::vector<Corr>& in, double overlap) {
    float ratio = std::min(1.0f, std::max(0.0f, (float)overlap));
    std::vector<Corr> out = in;
    if (in.empty()) return out;
    const unsigned nr_min_correspondences = 0;  // PCL's default, never set at ISR.cpp:634-635
    const unsigned nvalid = std::max((unsigned)std::floor(ratio * (float)in.size()), nr_min_correspondences);
    if (nvalid >= out.size()) return out;
    std::sort(out.begin(), out.end(), [](const Corr& a, const Corr& b) {
        return a.dist < b.dist || (a.dist == b.dist && a.q < b.q);
    });
    out.resize(nvalid);
    return out;
}

// deterministic parallel reduction: fixed 64 chunks summed in order
template <int NV, class F>
void chunked_sum(int n, double* out, F&& f) {
    const int NCH = 64;
    std::vector<double> part((size_t)NCH * NV, 0.0);
#pragma omp parallel for schedule(static)
    for (int c = 0; c < NCH; c++) {
        int b = (int)((long long)n * c / NCH), e = (int)((long long)n * (c + 1) / NCH);
        double* acc = &part[(size_t)c * NV];
        for (int i = b; i < e; i++) f(i, acc);
    }
    for (int v = 0; v < NV; v++) out[v] = 0;
    for (int c = 0; c < NCH; c++)
        for (int v = 0; v < NV; v++) out[v] += part[(size_t)c * NV + v];
}

// [3P] TransformationEstimationPointToPoint = Eigen::umeyama(src, dst, false)
Mat4 est_pt2pt(const Cloud& s, const Cloud& t, const std::vector<Corr>& c) {
    if (c.empty()) return Mat4::I();
    const int n = (int)c.size();
    double sums[6];
    chunked_sum<6>(n, sums, [&](int i, double* a) {
        const Vec3& ps = s.points[c[i].q];
        const Vec3& pt = t.points[c[i].m];
        a[0] += ps.x; a[1] += ps.y; a[2] += ps.z; a[3] += pt.x; a[4] += pt.y; a[5] += pt.z;
    });
    double one_over_n = 1.0 / (double)n;
    Vec3 ms(sums[0] * one_over_n, sums[1] * one_over_n, sums[2] * one_over_n);
    Vec3 md(sums[3] * one_over_n, sums[4] * one_over_n, sums[5] * one_over_n);
    double cs[9];
    chunked_sum<9>(n, cs, [&](int i, double* a) {
        Vec3 ps = s.points[c[i].q] - ms;
        Vec3 pt = t.points[c[i].m] - md;
        for (int r = 0; r < 3; r++)
            for (int k = 0; k < 3; k++) a[r * 3 + k] += pt[r] * ps[k];
    });
    Mat3 sigma;
    for (int r = 0; r < 3; r++)
        for (int k = 0; k < 3; k++) sigma.m[r][k] = one_over_n * cs[r * 3 + k];
    Mat3 U, V;
    double sv[3];
    svd3(sigma, U, sv, V);
    double S[3] = {1, 1, 1};
    if (det3(U) * det3(V) < 0) S[2] = -1;
    Mat3 R;
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) R.m[i][j] = U.m[i][0] * S[0] * V.m[j][0] + U.m[i][1] * S[1] * V.m[j][1] + U.m[i][2] * S[2] * V.m[j][2];
    Vec3 tr = md - mul(R, ms);
    Mat4 T = Mat4::I();
    for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++) T.m[i][j] = R.m[i][j];
        T.m[i][3] = tr[i];
    }
    return T;
}

// [3P] ComputeJTJandJTr + SolveJacobianSystemAndObtainExtrinsicMatrix
Mat4 solve_jtj(const double* acc /* 21 upper JTJ + 6 JTr */) {
    double JTJ[6][6], JTr[6];
    int k = 0;
    for (int i = 0; i < 6; i++)
        for (int j = i; j < 6; j++) { JTJ[i][j] = JTJ[j][i] = acc[k++]; }
    for (int i = 0; i < 6; i++) JTr[i] = -acc[21 + i];
    double x[6];
    ldlt_solve6(JTJ, JTr, x);
    for (int i = 0; i < 6; i++)
        if (!std::isfinite(x[i])) return Mat4::I();
    return vec6_to_mat4(x);
}
inline void acc_row(double* a, const double J[6], double r) {
    int k = 0;
    for (int i = 0; i < 6; i++)
        for (int j = i; j < 6; j++) a[k++] += J[i] * J[j];
    for (int i = 0; i < 6; i++) a[21 + i] += J[i] * r;
}

// [3P] TransformationEstimationPointToPlane::ComputeTransformation
Mat4 est_pt2pl(const Cloud& s, const Cloud& t, const std::vector<Corr>& c) {
    if (c.empty() || t.normals.empty()) return Mat4::I();
    double acc[27];
    chunked_sum<27>((int)c.size(), acc, [&](int i, double* a) {
        const Vec3& vs = s.points[c[i].q];
        const Vec3& vt = t.points[c[i].m];
        const Vec3& nt = t.normals[c[i].m];
        double r = dot(vs - vt, nt);
        Vec3 cr = cross(vs, nt);
        double J[6] = {cr.x, cr.y, cr.z, nt.x, nt.y, nt.z};
        acc_row(a, J, r);
    });
    return solve_jtj(acc);
}

// [3P] TransformationEstimationForGeneralizedICP::ComputeTransformation and
// ISR.cpp:57-110 optimize_generalizedICP_manual (W = w_i * (Ct+Cs)^-1/2, ISR.cpp:78)
Mat4 est_gicp(const Cloud& s, const Cloud& t, const std::vector<Corr>& c, const std::vector<double>* weights) {
    if (c.empty() || t.covariances.empty() || s.covariances.empty()) return Mat4::I();
    double acc[27];
    chunked_sum<27>((int)c.size(), acc, [&](int i, double* a) {
        const Vec3& vs = s.points[c[i].q];
        const Mat3& Cs = s.covariances[c[i].q];
        const Vec3& vt = t.points[c[i].m];
        const Mat3& Ct = t.covariances[c[i].m];
        Vec3 d = vs - vt;
        Mat3 M = add(Ct, Cs);
        Mat3 W = sqrt_spd(inverse3(M));
        if (weights) {
            double w = (*weights)[i];
            for (int r = 0; r < 3; r++)
                for (int k = 0; k < 3; k++) W.m[r][k] *= w;
        }
        Mat3 S = skew(vs);
        for (int row = 0; row < 3; row++) {
            double J[6];
            for (int col = 0; col < 3; col++) {
                J[col] = -(W.m[row][0] * S.m[0][col] + W.m[row][1] * S.m[1][col] + W.m[row][2] * S.m[2][col]);
                J[3 + col] = W.m[row][col];
            }
            double r = W.m[row][0] * d.x + W.m[row][1] * d.y + W.m[row][2] * d.z;
            acc_row(a, J, r);
        }
    });
    return solve_jtj(acc);
}

// ISR.cpp:16-30 (min_depth, not min_depth^2, in the numerator — as written)
double lounge_point_confidence(const Vec3& v) {
    double depth = v.z;
    double p1 = 0.002203, p2 = -0.001028, p3 = 0.0005351, min_depth = 0.4;
    double error = p1 * depth * depth + p2 * depth + p3;
    return (p1 * min_depth + p2 * min_depth + p3) / error;
}

// 12-vector of an SE(3) element as the reference packs it (ISR.cpp:450-453, 613-624):
// [R00 R10 R20 R01 R11 R21 R02 R12 R22 t0 t1 t2]
inline void se3_vec(const Mat4& M, double* v) {
    v[0] = M.m[0][0]; v[1] = M.m[1][0]; v[2] = M.m[2][0];
    v[3] = M.m[0][1]; v[4] = M.m[1][1]; v[5] = M.m[2][1];
    v[6] = M.m[0][2]; v[7] = M.m[1][2]; v[8] = M.m[2][2];
    v[9] = M.m[0][3]; v[10] = M.m[1][3]; v[11] = M.m[2][3];
}

double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ------------------------------------------------ the registration object (ISR.hpp:27-99)
struct Registration {
    refcpu_params prm;
    Cloud source_, source_moving_, target_;
    std::vector<Mat4> source_se3_cloud_, target_se3_cloud_;
    Mat4 T = Mat4::I();
    int num_iterations_ = 0, num_pure_se3_iterations_ = -1;
    double scaling_factor = 1.0;
    double t_setup = 0, t_loop = 0, t_nn = 0;
    // phase breakdown: TOLDI frames (kNN + LRF, ISR.cpp:590-591), normals /
    // GICP covariances (:642-648), trimming (:669-671), estimator + pose / cloud updates (:689-716)
    double t_toldi = 0, t_normals = 0, t_trim = 0, t_solve = 0;
    refcpu_trace* trace = nullptr;

    void record(int it, const Mat4& Ti, double mse, int nkept, const std::vector<Corr>& raw) {
        if (!trace || it >= trace->max_trace_iters) return;
        if (trace->Ti)
            for (int i = 0; i < 4; i++)
                for (int j = 0; j < 4; j++) trace->Ti[(size_t)it * 16 + i * 4 + j] = Ti.m[i][j];
        if (trace->mse) trace->mse[it] = mse;
        if (trace->n_kept) trace->n_kept[it] = nkept;
        const size_t ns = raw.size();
        for (size_t i = 0; i < ns; i++) {
            if (trace->corr_idx) trace->corr_idx[(size_t)it * ns + i] = raw[i].m;
            if (trace->corr_dist) trace->corr_dist[(size_t)it * ns + i] = raw[i].dist;
            if (trace->corr_d2 && i < nn_d2a.size()) trace->corr_d2[(size_t)it * ns + i] = nn_d2a[i];
            if (trace->corr_idx2 && i < nn_idx2.size()) trace->corr_idx2[(size_t)it * ns + i] = nn_idx2[i];
            if (trace->corr_d2b && i < nn_d2b.size()) trace->corr_d2b[(size_t)it * ns + i] = nn_d2b[i];
        }
    }
    // margins of the last search (filled only while a trace asks for them)
    std::vector<double> nn_d2a, nn_d2b;
    std::vector<int> nn_idx2;
    bool want_margin() const { return trace && (trace->corr_d2 || trace->corr_idx2 || trace->corr_d2b); }
    // the search of one query: 1-NN, or 2-NN (same first result) when margins are traced
    void search1(const KDTree& tree, const double* q, int i, int& idx, double& d2) {
        if (!want_margin()) {
            tree.knn(q, 1, &idx, &d2);
            return;
        }
        int ii[2] = {-1, -1};
        double dd[2] = {0, std::numeric_limits<double>::infinity()};
        tree.knn(q, 2, ii, dd);
        idx = ii[0];
        d2 = dd[0];
        nn_d2a[i] = dd[0];
        nn_idx2[i] = ii[1];
        nn_d2b[i] = dd[1];
    }
    void margins(int n) {
        if (!want_margin()) return;
        nn_d2a.assign(n, 0.0);
        nn_idx2.assign(n, -1);
        nn_d2b.assign(n, std::numeric_limits<double>::infinity());
    }

    // ISR.cpp:402-416
    void nn_xyz(const KDTree& tree, std::vector<Corr>& corr) {
        const int n = (int)source_moving_.points.size();
        corr.resize(n);
        margins(n);
#pragma omp parallel for schedule(dynamic, 512)
        for (int i = 0; i < n; i++) {
            const double q[3] = {source_moving_.points[i].x, source_moving_.points[i].y, source_moving_.points[i].z};
            int idx = -1;
            double d2 = 0;
            search1(tree, q, i, idx, d2);
            corr[i] = Corr{i, idx, float(std::sqrt(d2))};
        }
    }
    // ISR.cpp:444-470 (R3 distance stored, f64 -> float)
    void nn_se3(const KDTree& tree, std::vector<Corr>& corr) {
        const int n = (int)source_se3_cloud_.size();
        corr.resize(n);
        margins(n);
#pragma omp parallel for schedule(dynamic, 512)
        for (int i = 0; i < n; i++) {
            double q[12];
            se3_vec(source_se3_cloud_[i], q);
            int idx = -1;
            double d2 = 0;
            search1(tree, q, i, idx, d2);
            const Mat4& Mt = target_se3_cloud_[idx];
            Vec3 dv(source_se3_cloud_[i].m[0][3] - Mt.m[0][3], source_se3_cloud_[i].m[1][3] - Mt.m[1][3],
                    source_se3_cloud_[i].m[2][3] - Mt.m[2][3]);
            corr[i] = Corr{i, idx, float(norm(dv))};
        }
    }
    // ISR.cpp:379-387
    static double mse_of(const std::vector<Corr>& c) {
        double m = 0;
        int N = 0;
        for (const auto& x : c) { m += x.dist; N++; }
        return m / N;
    }
    // ISR.cpp:390-400
    double mse_euclid(const std::vector<Corr>& c) const {
        double m = 0;
        int N = 0;
        for (const auto& x : c) { m += norm(source_moving_.points[x.q] - target_.points[x.m]); N++; }
        return m / N;
    }

    Mat4 estimate(int variant, const std::vector<Corr>& c) {
        if (variant == REFCPU_PT2PT) return est_pt2pt(source_moving_, target_, c);
        if (variant == REFCPU_PT2PL) return est_pt2pl(source_moving_, target_, c);
        return est_gicp(source_moving_, target_, c, nullptr);
    }

    // ISR.cpp:568-626 (and 786-838 for cf): normalization, TOLDI, alpha/beta, 12-D target
    void se3_setup(bool cf, std::vector<double>& tgt12, Vec3& cs, Vec3& ct) {
        cs = get_center(source_);
        ct = get_center(target_);
        double rs = largest_distance(cs, source_), rt = largest_distance(ct, target_);
        double rmax = std::max(rs, rt);
        scaling_factor = prm.scale_preprocessing * (1.0 / rmax);
        translate(source_, -cs);
        translate(source_moving_, -cs);
        translate(target_, -ct);
        scale(source_, scaling_factor);
        scale(source_moving_, scaling_factor);
        scale(target_, scaling_factor);
        KDTree ts(source_.raw(), (int)source_.points.size(), 3), tt(target_.raw(), (int)target_.points.size(), 3);
        const double tl = now_ms();
        toldi_all(source_, ts, prm.number_of_nn_for_LRF, source_se3_cloud_);
        toldi_all(target_, tt, prm.number_of_nn_for_LRF, target_se3_cloud_);
        t_toldi = now_ms() - tl;
        for (auto* cl : {&source_se3_cloud_, &target_se3_cloud_})
            for (auto& M : *cl) {
                for (int i = 0; i < 3; i++)
                    for (int j = 0; j < 3; j++) M.m[i][j] *= prm.alpha_rot;
                for (int i = 0; i < 3; i++) M.m[i][3] *= prm.beta_transl;
            }
        const size_t nt = target_se3_cloud_.size();
        tgt12.resize(nt * 12);
        for (size_t i = 0; i < nt; i++) {
            se3_vec(target_se3_cloud_[i], &tgt12[i * 12]);
            if (cf) {  // ISR.cpp:834-836: translation rows from target_.points_
                tgt12[i * 12 + 9] = target_.points[i].x;
                tgt12[i * 12 + 10] = target_.points[i].y;
                tgt12[i * 12 + 11] = target_.points[i].z;
            }
        }
    }

    // ISR.cpp:555-739 run_se3_icp, 742-959 run_se3_icp_with_cf, 962-1127 run_se3_pure
    void run_se3(int variant, bool cf, bool pure) {
        double t0 = now_ms();
        std::vector<double> conf_s, conf_t;
        if (cf) {  // ISR.cpp:756-769 confidences on raw depth
            conf_s.resize(source_.points.size());
            conf_t.resize(target_.points.size());
            for (size_t i = 0; i < source_.points.size(); i++) conf_s[i] = lounge_point_confidence(source_.points[i]);
            for (size_t i = 0; i < target_.points.size(); i++) conf_t[i] = lounge_point_confidence(target_.points[i]);
        }
        Vec3 cs, ct;
        std::vector<double> tgt12;
        se3_setup(cf, tgt12, cs, ct);
        KDTree tree_se3(tgt12.data(), (int)target_se3_cloud_.size(), 12);
        KDTree tree_xyz(target_.raw(), (int)target_.points.size(), 3);
        T = Mat4::I();
        Mat4 Tprev = Mat4::I();
        double mse_prev = 1e7, mse_cur = 1e7, mse_rel = 1e7, change = 1e7;
        num_iterations_ = 0;
        num_pure_se3_iterations_ = 0;
        const double tnr = now_ms();
        if (cf || variant == REFCPU_GICP) {
            init_gicp(source_moving_, 1e-3);
            init_gicp(target_, 1e-3);
        } else if (variant == REFCPU_PT2PL) {
            estimate_normals(target_, 30);
        }
        t_normals = now_ms() - tnr;
        t_setup = now_ms() - t0;
        double t1 = now_ms();
        bool sw = false;
        std::vector<Corr> raw;
        while (true) {
            num_iterations_++;
            double tn = now_ms();
            if (!sw || pure) {
                num_pure_se3_iterations_++;
                nn_se3(tree_se3, raw);
            } else {
                nn_xyz(tree_xyz, raw);
            }
            t_nn += now_ms() - tn;
            const double tt0 = now_ms();
            std::vector<Corr> kept = trim(raw, prm.estimated_overlap);
            const double tt1 = now_ms();
            t_trim += tt1 - tt0;
            mse_prev = mse_cur;
            mse_cur = cf ? mse_euclid(kept) : mse_of(kept);
            mse_rel = std::fabs(mse_cur - mse_prev);
            Mat4 Ti;
            if (cf) {  // ISR.cpp:904-921 (the "kept" filter at :915 is unused: all trimmed corrs weighted)
                std::vector<double> w(kept.size());
                for (size_t i = 0; i < kept.size(); i++) w[i] = (conf_s[kept[i].q] + conf_t[kept[i].m]) / 2.0;
                Ti = est_gicp(source_moving_, target_, kept, &w);
            } else {
                Ti = estimate(variant, kept);
            }
            transform(source_moving_, Ti);
            Tprev = T;
            T = mul(Ti, T);
            change = frob_diff(Tprev, T);
            const int ns = (int)source_se3_cloud_.size();
#pragma omp parallel for schedule(static)
            for (int k = 0; k < ns; k++) source_se3_cloud_[k] = mul(Ti, source_se3_cloud_[k]);
            t_solve += now_ms() - tt1;
            record(num_iterations_ - 1, Ti, mse_cur, (int)kept.size(), raw);
            if (pure) {
                if (num_iterations_ == prm.max_num_se3_iterations || mse_rel < scaling_factor * prm.mse) break;
            } else if (!sw) {
                if (num_iterations_ == prm.max_num_se3_iterations || change < prm.mse_switch_error) sw = true;
            } else {
                if (num_iterations_ == prm.max_num_iterations || mse_rel < scaling_factor * prm.mse) break;
            }
            if (num_iterations_ >= 100000) break;  // guard: the reference loops forever here
        }
        // ISR.cpp:735-738
        Mat3 R;
        for (int i = 0; i < 3; i++)
            for (int j = 0; j < 3; j++) R.m[i][j] = T.m[i][j];
        Vec3 tp(T.m[0][3], T.m[1][3], T.m[2][3]);
        Vec3 Rc = mul(R, cs);
        Vec3 tog = Vec3((1.0 / scaling_factor) * tp.x - Rc.x + ct.x, (1.0 / scaling_factor) * tp.y - Rc.y + ct.y,
                        (1.0 / scaling_factor) * tp.z - Rc.z + ct.z);
        T.m[0][3] = tog.x; T.m[1][3] = tog.y; T.m[2][3] = tog.z;
        t_loop = now_ms() - t1;
    }

    // ISR.cpp:473-552 run_icp
    void run_icp(int variant) {
        double t0 = now_ms();
        KDTree tree_xyz(target_.raw(), (int)target_.points.size(), 3);
        T = Mat4::I();
        double mse_prev = 1e7, mse_cur = 1e7, mse_rel = 1e7;
        const double tnr = now_ms();
        if (variant == REFCPU_PT2PL) estimate_normals(target_, 30);
        if (variant == REFCPU_GICP) { init_gicp(source_moving_, 1e-3); init_gicp(target_, 1e-3); }
        t_normals = now_ms() - tnr;
        num_iterations_ = 0;
        t_setup = now_ms() - t0;
        double t1 = now_ms();
        std::vector<Corr> raw;
        while (true) {
            double tn = now_ms();
            nn_xyz(tree_xyz, raw);
            t_nn += now_ms() - tn;
            const double tt0 = now_ms();
            std::vector<Corr> kept = trim(raw, prm.estimated_overlap);
            const double tt1 = now_ms();
            t_trim += tt1 - tt0;
            mse_prev = mse_cur;
            mse_cur = mse_of(kept);
            mse_rel = std::fabs(mse_cur - mse_prev);
            Mat4 Ti = estimate(variant, kept);
            transform(source_moving_, Ti);
            T = mul(Ti, T);
            t_solve += now_ms() - tt1;
            record(num_iterations_, Ti, mse_cur, (int)kept.size(), raw);
            num_iterations_++;
            if (num_iterations_ == prm.max_num_iterations || mse_rel < prm.mse) break;
            if (num_iterations_ >= 100000) break;
        }
        t_loop = now_ms() - t1;
    }
};

Cloud make_cloud(const double* xyz, int64_t n) {
    Cloud c;
    c.points.resize(n);
    for (int64_t i = 0; i < n; i++) c.points[i] = Vec3(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
    return c;
}

}  // namespace

// ====================================================================== C API
extern "C" {

void refcpu_default_params(refcpu_params* p) {
    std::memset(p, 0, sizeof(*p));
    p->max_num_iterations = 150;
    p->max_num_se3_iterations = 20;
    p->number_of_nn_for_LRF = 30;
    p->mse = 0.00001;
    p->mse_switch_error = 0.001;
    p->estimated_overlap = 1.0;
    p->alpha_rot = 3.0;
    p->beta_transl = 1.0;
    p->scale_preprocessing = 3.0;
}

int refcpu_num_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
void refcpu_set_num_threads(int n) {
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
#else
    (void)n;
#endif
}

int refcpu_register(const double* src, int64_t n_src, const double* tgt, int64_t n_tgt, int run_kind, int variant,
                    const refcpu_params* params, refcpu_result* out, refcpu_trace* trace) {
    if (!src || !tgt || !out || n_src <= 0 || n_tgt <= 0) return -1;
    if (variant < 0 || variant > 2) return -2;
    Registration R;
    if (params) R.prm = *params; else refcpu_default_params(&R.prm);
    R.trace = trace;
    // ISR.cpp:358-376 setSourceCloud / setTargetCloud (copies)
    R.source_ = make_cloud(src, n_src);
    R.source_moving_ = R.source_;
    R.target_ = make_cloud(tgt, n_tgt);
    switch (run_kind) {
        case REFCPU_RUN_ICP: R.run_icp(variant); break;
        case REFCPU_RUN_SE3_ICP: R.run_se3(variant, false, false); break;
        case REFCPU_RUN_SE3_ICP_CF: R.run_se3(REFCPU_GICP, true, false); break;
        case REFCPU_RUN_SE3_PURE: R.run_se3(variant, false, true); break;
        default: return -3;
    }
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) out->T[i * 4 + j] = R.T.m[i][j];
    out->num_iterations = R.num_iterations_;
    out->num_pure_se3_iterations = R.num_pure_se3_iterations_;
    out->scaling_factor = R.scaling_factor;
    out->time_setup_ms = R.t_setup;
    out->time_loop_ms = R.t_loop;
    out->time_nn_ms = R.t_nn;
    out->time_toldi_ms = R.t_toldi;
    out->time_normals_ms = R.t_normals;
    out->time_trim_ms = R.t_trim;
    out->time_solve_ms = R.t_solve;
    return 0;
}

int refcpu_knn_self(const double* pts, int64_t n, int k, int32_t* idx, double* d2) {
    if (n <= 0 || k <= 0) return -1;
    KDTree tree(pts, (int)n, 3);
    const int kk = (int)std::min<int64_t>(k, n);
#pragma omp parallel for schedule(dynamic, 256)
    for (int64_t i = 0; i < n; i++) {
        std::vector<int> ii(kk);
        std::vector<double> dd(kk);
        tree.knn(pts + 3 * i, kk, ii.data(), dd.data());
        for (int j = 0; j < k; j++) {
            idx[i * k + j] = j < kk ? ii[j] : -1;
            d2[i * k + j] = j < kk ? dd[j] : std::numeric_limits<double>::infinity();
        }
    }
    return 0;
}

int refcpu_toldi_frames(const double* pts, int64_t n, int k, double* frames) {
    if (n <= 0 || k <= 0) return -1;
    Cloud c = make_cloud(pts, n);
    KDTree tree(c.raw(), (int)n, 3);
    std::vector<Mat4> F;
    toldi_all(c, tree, k, F);
    for (int64_t i = 0; i < n; i++)
        for (int r = 0; r < 4; r++)
            for (int q = 0; q < 4; q++) frames[i * 16 + r * 4 + q] = F[i].m[r][q];
    return 0;
}

int refcpu_estimate_normals(const double* pts, int64_t n, int k, double* normals) {
    if (n <= 0 || k <= 0) return -1;
    Cloud c = make_cloud(pts, n);
    estimate_normals(c, k);
    for (int64_t i = 0; i < n; i++) {
        normals[3 * i] = c.normals[i].x;
        normals[3 * i + 1] = c.normals[i].y;
        normals[3 * i + 2] = c.normals[i].z;
    }
    return 0;
}

int refcpu_gicp_covariances(const double* normals, int64_t n, double eps, double* cov) {
    Mat3 C;
    C.m[0][0] = eps; C.m[1][1] = 1; C.m[2][2] = 1;
    for (int64_t i = 0; i < n; i++) {
        Mat3 Rx = rotation_e1_to_x(Vec3(normals[3 * i], normals[3 * i + 1], normals[3 * i + 2]));
        Mat3 r = mul(mul(Rx, C), transpose(Rx));
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) cov[i * 9 + a * 3 + b] = r.m[a][b];
    }
    return 0;
}

int refcpu_nn(const double* query, int64_t nq, const double* data, int64_t nd, int dim, int32_t* idx, double* d2) {
    if (nd <= 0 || dim <= 0) return -1;
    KDTree tree(data, (int)nd, dim);
#pragma omp parallel for schedule(dynamic, 512)
    for (int64_t i = 0; i < nq; i++) {
        int id = -1;
        double dd = 0;
        tree.knn(query + i * dim, 1, &id, &dd);
        idx[i] = id;
        d2[i] = dd;
    }
    return 0;
}

int refcpu_estimate(int variant, const double* src_pts, const double* src_cov, const double* tgt_pts,
                    const double* tgt_normals, const double* tgt_cov, const int32_t* pairs, int64_t k,
                    const double* weights, double* Tout) {
    int64_t ns = 0, nt = 0;
    for (int64_t i = 0; i < k; i++) { ns = std::max<int64_t>(ns, pairs[2 * i] + 1); nt = std::max<int64_t>(nt, pairs[2 * i + 1] + 1); }
    Cloud s = make_cloud(src_pts, ns), t = make_cloud(tgt_pts, nt);
    if (tgt_normals) {
        t.normals.resize(nt);
        for (int64_t i = 0; i < nt; i++) t.normals[i] = Vec3(tgt_normals[3 * i], tgt_normals[3 * i + 1], tgt_normals[3 * i + 2]);
    }
    auto load_cov = [](const double* c, int64_t n, std::vector<Mat3>& out) {
        out.resize(n);
        for (int64_t i = 0; i < n; i++)
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) out[i].m[a][b] = c[i * 9 + a * 3 + b];
    };
    if (src_cov) load_cov(src_cov, ns, s.covariances);
    if (tgt_cov) load_cov(tgt_cov, nt, t.covariances);
    std::vector<Corr> c(k);
    for (int64_t i = 0; i < k; i++) c[i] = Corr{pairs[2 * i], pairs[2 * i + 1], 0.f};
    Mat4 T;
    if (variant == REFCPU_PT2PT) T = est_pt2pt(s, t, c);
    else if (variant == REFCPU_PT2PL) T = est_pt2pl(s, t, c);
    else if (variant == REFCPU_GICP) {
        std::vector<double> w;
        if (weights) w.assign(weights, weights + k);
        T = est_gicp(s, t, c, weights ? &w : nullptr);
    } else return -2;
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++) Tout[i * 4 + j] = T.m[i][j];
    return 0;
}

int64_t refcpu_trim(const float* dist, int64_t n, double overlap_ratio, int32_t* kept_query) {
    std::vector<Corr> in(n);
    for (int64_t i = 0; i < n; i++) in[i] = Corr{(int)i, 0, dist[i]};
    std::vector<Corr> out = trim(in, overlap_ratio);
    for (size_t i = 0; i < out.size(); i++) kept_query[i] = out[i].q;
    return (int64_t)out.size();
}

}  // extern "C"
