// hostmath.cpp — host f64 solves of one ICP iteration (see hostmath.hpp).
#include "hostmath.hpp"

#include <algorithm>
#include <cmath>
#include <limits>
#include <utility>

namespace se3icp {

M4 M4::eye() {
    M4 r{};
    for (int i = 0; i < 4; ++i) r.m[i][i] = 1.0;
    return r;
}

M4 mul4(const M4& a, const M4& b) {
    M4 r{};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = 0;
            for (int k = 0; k < 4; ++k) s += a.m[i][k] * b.m[k][j];
            r.m[i][j] = s;
        }
    return r;
}

double frob_diff4(const M4& a, const M4& b) {
    double s = 0;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) s += (a.m[i][j] - b.m[i][j]) * (a.m[i][j] - b.m[i][j]);
    return std::sqrt(s);
}

// Two-sided Jacobi SVD of a 3x3 matrix.  Each (p,q) step first symmetrises the
// 2x2 block with a left rotation, then diagonalises it with a symmetric Jacobi
// rotation applied on both sides.
void svd3(const double A[3][3], double U[3][3], double s[3], double V[3][3]) {
    double B[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            B[i][j] = A[i][j];
            U[i][j] = V[i][j] = (i == j) ? 1.0 : 0.0;
        }
    auto rot_left = [&](int p, int q, double c, double sn) {  // rows p,q of B; cols of U
        for (int k = 0; k < 3; ++k) {
            const double bp = B[p][k], bq = B[q][k];
            B[p][k] = c * bp + sn * bq;
            B[q][k] = -sn * bp + c * bq;
        }
        for (int k = 0; k < 3; ++k) {  // U <- U L^T
            const double up = U[k][p], uq = U[k][q];
            U[k][p] = c * up + sn * uq;
            U[k][q] = -sn * up + c * uq;
        }
    };
    auto rot_right = [&](int p, int q, double c, double sn) {  // cols p,q of B and V
        for (int k = 0; k < 3; ++k) {
            const double bp = B[k][p], bq = B[k][q];
            B[k][p] = c * bp - sn * bq;
            B[k][q] = sn * bp + c * bq;
            const double vp = V[k][p], vq = V[k][q];
            V[k][p] = c * vp - sn * vq;
            V[k][q] = sn * vp + c * vq;
        }
    };
    for (int sweep = 0; sweep < 100; ++sweep) {
        double dmax = 0;
        for (int i = 0; i < 3; ++i) dmax = std::max(dmax, std::fabs(B[i][i]));
        const double thr = std::max(std::numeric_limits<double>::min(), 2e-16 * dmax);
        bool done = true;
        for (int p = 0; p < 3; ++p)
            for (int q = p + 1; q < 3; ++q) {
                if (std::fabs(B[p][q]) <= thr && std::fabs(B[q][p]) <= thr) continue;
                done = false;
                // 1) left rotation making the block symmetric
                const double a = B[p][p], b = B[p][q], c = B[q][p], d = B[q][q];
                const double th1 = std::atan2(c - b, a + d);
                rot_left(p, q, std::cos(th1), std::sin(th1));
                // 2) symmetric Jacobi on [[x, y], [y, z]]
                const double x = B[p][p], y = 0.5 * (B[p][q] + B[q][p]), z = B[q][q];
                if (y != 0.0) {
                    const double th2 = 0.5 * std::atan2(2.0 * y, z - x);
                    const double c2 = std::cos(th2), s2 = std::sin(th2);
                    rot_left(p, q, c2, -s2);  // J^T from the left (J = [[c,s],[-s,c]] on the right)
                    rot_right(p, q, c2, s2);
                }
            }
        if (done) break;
    }
    double sv[3];
    for (int i = 0; i < 3; ++i) {
        sv[i] = B[i][i];
        if (sv[i] < 0) {
            sv[i] = -sv[i];
            for (int k = 0; k < 3; ++k) U[k][i] = -U[k][i];
        }
    }
    int ord[3] = {0, 1, 2};
    std::sort(ord, ord + 3, [&](int i, int j) { return sv[i] > sv[j]; });
    double U2[3][3], V2[3][3];
    for (int c = 0; c < 3; ++c) {
        s[c] = sv[ord[c]];
        for (int k = 0; k < 3; ++k) {
            U2[k][c] = U[k][ord[c]];
            V2[k][c] = V[k][ord[c]];
        }
    }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) { U[i][j] = U2[i][j]; V[i][j] = V2[i][j]; }
}

static double det3(const double a[3][3]) {
    return a[0][0] * (a[1][1] * a[2][2] - a[1][2] * a[2][1]) - a[0][1] * (a[1][0] * a[2][2] - a[1][2] * a[2][0]) +
           a[0][2] * (a[1][0] * a[2][1] - a[1][1] * a[2][0]);
}

M4 umeyama_from_moments(const double* s, double n) {
    if (!(n > 0)) return M4::eye();
    const double inv = 1.0 / n;
    const double ms[3] = {s[0] * inv, s[1] * inv, s[2] * inv};
    const double md[3] = {s[3] * inv, s[4] * inv, s[5] * inv};
    double sigma[3][3];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) sigma[a][b] = s[6 + 3 * a + b] * inv - md[a] * ms[b];
    double U[3][3], V[3][3], sv[3];
    svd3(sigma, U, sv, V);
    const double S2 = (det3(U) * det3(V) < 0) ? -1.0 : 1.0;
    M4 T = M4::eye();
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) T.m[i][j] = U[i][0] * V[j][0] + U[i][1] * V[j][1] + S2 * U[i][2] * V[j][2];
    for (int i = 0; i < 3; ++i)
        T.m[i][3] = md[i] - (T.m[i][0] * ms[0] + T.m[i][1] * ms[1] + T.m[i][2] * ms[2]);
    return T;
}

// LDL^T with symmetric diagonal pivoting: P A P^T = L D L^T.
void ldlt_solve6(const double Ain[6][6], const double b[6], double x[6]) {
    constexpr int n = 6;
    double a[n][n];
    int perm[n];
    for (int i = 0; i < n; ++i) {
        perm[i] = i;
        for (int j = 0; j < n; ++j) a[i][j] = Ain[i][j];
    }
    double L[n][n] = {}, D[n] = {};
    for (int k = 0; k < n; ++k) {
        // pivot on the largest remaining |diagonal| of the Schur complement
        int p = k;
        for (int i = k + 1; i < n; ++i)
            if (std::fabs(a[i][i]) > std::fabs(a[p][p])) p = i;
        if (p != k) {
            std::swap(perm[k], perm[p]);
            for (int j = 0; j < n; ++j) std::swap(a[k][j], a[p][j]);
            for (int i = 0; i < n; ++i) std::swap(a[i][k], a[i][p]);
            for (int j = 0; j < k; ++j) std::swap(L[k][j], L[p][j]);
        }
        D[k] = a[k][k];
        L[k][k] = 1.0;
        for (int i = k + 1; i < n; ++i) L[i][k] = (D[k] != 0.0) ? a[i][k] / D[k] : 0.0;
        for (int i = k + 1; i < n; ++i)
            for (int j = k + 1; j < n; ++j) a[i][j] -= L[i][k] * D[k] * L[j][k];
    }
    double y[n];
    for (int i = 0; i < n; ++i) y[i] = b[perm[i]];
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < i; ++j) y[i] -= L[i][j] * y[j];
    const double tiny = std::numeric_limits<double>::min();
    for (int i = 0; i < n; ++i) y[i] = (std::fabs(D[i]) > tiny) ? y[i] / D[i] : 0.0;
    for (int i = n - 1; i >= 0; --i)
        for (int j = i + 1; j < n; ++j) y[i] -= L[j][i] * y[j];
    for (int i = 0; i < n; ++i) x[perm[i]] = y[i];
}

M4 vec6_to_mat4(const double x[6]) {
    struct Q { double w, x, y, z; };
    auto qm = [](const Q& a, const Q& b) {
        return Q{a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
                 a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x, a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w};
    };
    const Q q = qm(qm(Q{std::cos(0.5 * x[2]), 0, 0, std::sin(0.5 * x[2])}, Q{std::cos(0.5 * x[1]), 0, std::sin(0.5 * x[1]), 0}),
                   Q{std::cos(0.5 * x[0]), std::sin(0.5 * x[0]), 0, 0});
    M4 T = M4::eye();
    const double xx = q.x * q.x, yy = q.y * q.y, zz = q.z * q.z;
    const double xy = q.x * q.y, xz = q.x * q.z, yz = q.y * q.z, wx = q.w * q.x, wy = q.w * q.y, wz = q.w * q.z;
    T.m[0][0] = 1 - 2 * (yy + zz); T.m[0][1] = 2 * (xy - wz);     T.m[0][2] = 2 * (xz + wy);
    T.m[1][0] = 2 * (xy + wz);     T.m[1][1] = 1 - 2 * (xx + zz); T.m[1][2] = 2 * (yz - wx);
    T.m[2][0] = 2 * (xz - wy);     T.m[2][1] = 2 * (yz + wx);     T.m[2][2] = 1 - 2 * (xx + yy);
    T.m[0][3] = x[3]; T.m[1][3] = x[4]; T.m[2][3] = x[5];
    return T;
}

M4 solve_normal_equations(const double* acc) {
    double A[6][6], b[6], x[6];
    int k = 0;
    for (int i = 0; i < 6; ++i)
        for (int j = i; j < 6; ++j) { A[i][j] = A[j][i] = acc[k++]; }
    for (int i = 0; i < 6; ++i) b[i] = -acc[21 + i];
    ldlt_solve6(A, b, x);
    for (int i = 0; i < 6; ++i)
        if (!std::isfinite(x[i])) return M4::eye();
    return vec6_to_mat4(x);
}

}  // namespace se3icp
