// pairmath.hpp — the per-iteration small f64 solves of one pair (umeyama 3x3 SVD,
// 6x6 LDLT, RzRyRx pose) and the reference's switch / convergence state machine.
// Header-only and __host__ __device__: k_reduce_final (k_loop.hip) runs them on the GPU
// after the correspondence reduction, so the loop never waits for the host.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "common.hpp"

#define SE3ICP_HD __host__ __device__ inline

namespace se3icp {

struct M4 {
    double m[4][4];
    SE3ICP_HD static M4 eye() {
        M4 r{};
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) r.m[i][j] = (i == j) ? 1.0 : 0.0;
        return r;
    }
};

SE3ICP_HD M4 mul4(const M4& a, const M4& b) {
    M4 r{};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            double s = 0;
            for (int k = 0; k < 4; ++k) s += a.m[i][k] * b.m[k][j];
            r.m[i][j] = s;
        }
    return r;
}

SE3ICP_HD double frob_diff4(const M4& a, const M4& b) {
    double s = 0;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) s += (a.m[i][j] - b.m[i][j]) * (a.m[i][j] - b.m[i][j]);
    return sqrt(s);
}

// A = U diag(s) V^T, s descending (two-sided Jacobi).  Each (p,q) step first
// symmetrises the 2x2 block with a left rotation, then diagonalises it with a
// symmetric Jacobi rotation applied on both sides.
SE3ICP_HD void svd3_rot_left(double B[3][3], double U[3][3], int p, int q, double c, double sn) {
    for (int k = 0; k < 3; ++k) {  // rows p,q of B
        const double bp = B[p][k], bq = B[q][k];
        B[p][k] = c * bp + sn * bq;
        B[q][k] = -sn * bp + c * bq;
    }
    for (int k = 0; k < 3; ++k) {  // U <- U L^T
        const double up = U[k][p], uq = U[k][q];
        U[k][p] = c * up + sn * uq;
        U[k][q] = -sn * up + c * uq;
    }
}
SE3ICP_HD void svd3_rot_right(double B[3][3], double V[3][3], int p, int q, double c, double sn) {
    for (int k = 0; k < 3; ++k) {  // cols p,q of B and V
        const double bp = B[k][p], bq = B[k][q];
        B[k][p] = c * bp - sn * bq;
        B[k][q] = sn * bp + c * bq;
        const double vp = V[k][p], vq = V[k][q];
        V[k][p] = c * vp - sn * vq;
        V[k][q] = sn * vp + c * vq;
    }
}
SE3ICP_HD void svd3(const double A[3][3], double U[3][3], double s[3], double V[3][3]) {
    double B[3][3];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            B[i][j] = A[i][j];
            U[i][j] = V[i][j] = (i == j) ? 1.0 : 0.0;
        }
    constexpr double kMinNormal = 2.2250738585072014e-308;  // DBL_MIN
    for (int sweep = 0; sweep < 100; ++sweep) {
        double dmax = 0;
        for (int i = 0; i < 3; ++i) dmax = fmax(dmax, fabs(B[i][i]));
        const double thr = fmax(kMinNormal, 2e-16 * dmax);
        bool done = true;
#pragma unroll
        for (int p = 0; p < 3; ++p)
#pragma unroll
            for (int q = p + 1; q < 3; ++q) {
                if (fabs(B[p][q]) <= thr && fabs(B[q][p]) <= thr) continue;
                done = false;
                // 1) left rotation making the block symmetric: the angle atan2(c - b, a + d),
                //    its cosine and sine from the hypotenuse (no trigonometric calls: the
                //    serial solve of k_reduce_final spent most of its time in them)
                const double a = B[p][p], b = B[p][q], c = B[q][p], d = B[q][q];
                {
                    const double h = hypot(a + d, c - b);  // (no overflow at ~1e154, no underflow at ~1e-160)
                    const double c1 = h > 0.0 ? (a + d) / h : 1.0, s1 = h > 0.0 ? (c - b) / h : 0.0;
                    svd3_rot_left(B, U, p, q, c1, s1);
                }
                // 2) symmetric Jacobi on [[x, y], [y, z]]: the angle 0.5 atan2(2y, z - x) in
                //    (-pi/2, pi/2], its cosine and sine by the half-angle formulas (the
                //    well-conditioned one of the two for the sign of cos 2t)
                const double x = B[p][p], y = 0.5 * (B[p][q] + B[q][p]), z = B[q][q];
                if (y != 0.0) {
                    const double h = hypot(2.0 * y, z - x);
                    const double c2t = (z - x) / h, s2t = 2.0 * y / h;
                    double c2, s2;
                    if (c2t >= 0.0) {
                        c2 = sqrt(0.5 * (1.0 + c2t));
                        s2 = s2t / (2.0 * c2);
                    } else {
                        s2 = copysign(sqrt(0.5 * (1.0 - c2t)), s2t);
                        c2 = s2t / (2.0 * s2);
                    }
                    svd3_rot_left(B, U, p, q, c2, -s2);  // J^T from the left (J = [[c,s],[-s,c]] on the right)
                    svd3_rot_right(B, V, p, q, c2, s2);
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
    // stable descending order of the three singular values (insertion network with
    // compile-time column indices: no dynamically indexed arrays, so the device keeps
    // everything in registers)
    auto cswap = [&](int i, int j) {
        if (sv[j] > sv[i]) {
            const double t = sv[i]; sv[i] = sv[j]; sv[j] = t;
            for (int k = 0; k < 3; ++k) {
                const double tu = U[k][i]; U[k][i] = U[k][j]; U[k][j] = tu;
                const double tv = V[k][i]; V[k][i] = V[k][j]; V[k][j] = tv;
            }
        }
    };
    cswap(0, 1);
    cswap(1, 2);
    cswap(0, 1);
    for (int c = 0; c < 3; ++c) s[c] = sv[c];
}

SE3ICP_HD double det3(const double a[3][3]) {
    return a[0][0] * (a[1][1] * a[2][2] - a[1][2] * a[2][1]) - a[0][1] * (a[1][0] * a[2][2] - a[1][2] * a[2][0]) +
           a[0][2] * (a[1][0] * a[2][1] - a[1][1] * a[2][0]);
}

// Eigen::umeyama(src, dst, false) (TransformationEstimationPointToPoint, ISR.cpp:692)
// from the one-pass moments of the kept correspondences:
//   s[0..2] = sum vs, s[3..5] = sum vt, s[6..14] = sum vt vs^T (row-major), n = count.
SE3ICP_HD M4 umeyama_from_moments(const double* s, double n) {
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
    for (int i = 0; i < 3; ++i) T.m[i][3] = md[i] - (T.m[i][0] * ms[0] + T.m[i][1] * ms[1] + T.m[i][2] * ms[2]);
    return T;
}

// A x = b for symmetric 6x6 A with Eigen LDLT semantics (diagonal pivoting, zero
// pivots treated as a pseudo-inverse) — Open3D SolveLinearSystemPSD.
// LDL^T with symmetric diagonal pivoting: P A P^T = L D L^T.
SE3ICP_HD void ldlt_solve6(const double Ain[6][6], const double b[6], double x[6]) {
    // every loop has compile-time bounds and the pivot swaps are predicated per
    // candidate row, so no array is indexed by a run-time value (registers on the GPU)
    constexpr int n = 6;
    double a[n][n];
    int perm[n];
#pragma unroll
    for (int i = 0; i < n; ++i) {
        perm[i] = i;
#pragma unroll
        for (int j = 0; j < n; ++j) a[i][j] = Ain[i][j];
    }
    double L[n][n] = {}, D[n] = {};
#pragma unroll
    for (int k = 0; k < n; ++k) {
        // pivot on the largest remaining |diagonal| of the Schur complement (first one on ties)
        int p = k;
        double best = fabs(a[k][k]);
#pragma unroll
        for (int i = k + 1; i < n; ++i)
            if (fabs(a[i][i]) > best) {
                best = fabs(a[i][i]);
                p = i;
            }
#pragma unroll
        for (int i = k + 1; i < n; ++i) {
            if (i != p) continue;
            { const int t = perm[k]; perm[k] = perm[i]; perm[i] = t; }
#pragma unroll
            for (int j = 0; j < n; ++j) { const double t = a[k][j]; a[k][j] = a[i][j]; a[i][j] = t; }
#pragma unroll
            for (int r = 0; r < n; ++r) { const double t = a[r][k]; a[r][k] = a[r][i]; a[r][i] = t; }
#pragma unroll
            for (int j = 0; j < k; ++j) { const double t = L[k][j]; L[k][j] = L[i][j]; L[i][j] = t; }
        }
        D[k] = a[k][k];
        L[k][k] = 1.0;
#pragma unroll
        for (int i = k + 1; i < n; ++i) L[i][k] = (D[k] != 0.0) ? a[i][k] / D[k] : 0.0;
#pragma unroll
        for (int i = k + 1; i < n; ++i)
#pragma unroll
            for (int j = k + 1; j < n; ++j) a[i][j] -= L[i][k] * D[k] * L[j][k];
    }
    double y[n];
#pragma unroll
    for (int i = 0; i < n; ++i) {
        y[i] = 0.0;
#pragma unroll
        for (int j = 0; j < n; ++j)
            if (perm[i] == j) y[i] = b[j];
    }
#pragma unroll
    for (int i = 0; i < n; ++i)
#pragma unroll
        for (int j = 0; j < i; ++j) y[i] -= L[i][j] * y[j];
    constexpr double tiny = 2.2250738585072014e-308;  // DBL_MIN
#pragma unroll
    for (int i = 0; i < n; ++i) y[i] = (fabs(D[i]) > tiny) ? y[i] / D[i] : 0.0;
#pragma unroll
    for (int i = n - 1; i >= 0; --i)
#pragma unroll
        for (int j = i + 1; j < n; ++j) y[i] -= L[j][i] * y[j];
#pragma unroll
    for (int i = 0; i < n; ++i)
#pragma unroll
        for (int j = 0; j < n; ++j)
            if (perm[i] == j) x[j] = y[i];
}

// TransformVector6dToMatrix4d: R = AngleAxis(x2,Z)*AngleAxis(x1,Y)*AngleAxis(x0,X), t = x3..5
struct Quat {
    double w, x, y, z;
};
SE3ICP_HD Quat qmul(const Quat& a, const Quat& b) {
    return Quat{a.w * b.w - a.x * b.x - a.y * b.y - a.z * b.z, a.w * b.x + a.x * b.w + a.y * b.z - a.z * b.y,
                a.w * b.y - a.x * b.z + a.y * b.w + a.z * b.x, a.w * b.z + a.x * b.y - a.y * b.x + a.z * b.w};
}
SE3ICP_HD M4 vec6_to_mat4(const double x[6]) {
    const Quat q = qmul(qmul(Quat{cos(0.5 * x[2]), 0, 0, sin(0.5 * x[2])}, Quat{cos(0.5 * x[1]), 0, sin(0.5 * x[1]), 0}),
                        Quat{cos(0.5 * x[0]), sin(0.5 * x[0]), 0, 0});
    M4 T = M4::eye();
    const double xx = q.x * q.x, yy = q.y * q.y, zz = q.z * q.z;
    const double xy = q.x * q.y, xz = q.x * q.z, yz = q.y * q.z, wx = q.w * q.x, wy = q.w * q.y, wz = q.w * q.z;
    T.m[0][0] = 1 - 2 * (yy + zz); T.m[0][1] = 2 * (xy - wz);     T.m[0][2] = 2 * (xz + wy);
    T.m[1][0] = 2 * (xy + wz);     T.m[1][1] = 1 - 2 * (xx + zz); T.m[1][2] = 2 * (yz - wx);
    T.m[2][0] = 2 * (xz - wy);     T.m[2][1] = 2 * (yz + wx);     T.m[2][2] = 1 - 2 * (xx + yy);
    T.m[0][3] = x[3]; T.m[1][3] = x[4]; T.m[2][3] = x[5];
    return T;
}

// Open3D SolveJacobianSystemAndObtainExtrinsicMatrix from the packed normal
// equations (21 upper-triangular JTJ entries then 6 JTr): x = -(JTJ)^-1 JTr,
// T = TransformVector6dToMatrix4d(x).  Identity when the solution is not finite.
SE3ICP_HD M4 solve_normal_equations(const double* acc) {
    double A[6][6], b[6], x[6];
    int k = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i)
#pragma unroll
        for (int j = i; j < 6; ++j) {
            A[i][j] = A[j][i] = acc[k++];
        }
    for (int i = 0; i < 6; ++i) b[i] = -acc[21 + i];
    ldlt_solve6(A, b, x);
    for (int i = 0; i < 6; ++i)
        if (!__builtin_isfinite(x[i])) return M4::eye();
    return vec6_to_mat4(x);
}

// ---- per-pair loop state: the reference's run_* locals (ISR.cpp:629-651, 654-732)
enum Kind : int32_t { KIND_ICP = 0, KIND_SE3 = 1, KIND_CF = 2, KIND_PURE = 3 };

struct PairState {
    M4 T;                  // current_estimated_T_ (normalized frame)
    double mse_prev, mse_cur, rel;
    double sf;             // scale of the preprocessing (1 for run_icp)
    double K;              // correspondences of the mean: nkeep when trimmed, else ns
    double mse, mse_switch;
    int32_t iter, pure, sw, done;
    int32_t kind, max_iter, max_se3, phase, phase_start;
    int32_t _pad[3];
};

// Close the iteration just run (ISR.cpp:684-732) from the pair's 28 reduced values.
// Sets S.done when the pair is finished, S.sw at the SE(3) -> R3 switch.
SE3ICP_HD void pair_close_iteration(PairState& S, int est, const double* acc) {
    // ISR.cpp:684-686 (mean of the kept distances; NaN when nothing is kept, as the reference)
    S.mse_prev = S.mse_cur;
    S.mse_cur = acc[27] / S.K;
    S.rel = fabs(S.mse_cur - S.mse_prev);
    // ISR.cpp:689-703 estimator
    M4 Ti;
    if (S.K <= 0) Ti = M4::eye();
    else if (est == EST_PT2PT) Ti = umeyama_from_moments(acc, acc[15]);
    else Ti = solve_normal_equations(acc);
    // ISR.cpp:706-716: the source cloud and its SE(3) elements follow T on the fly
    const M4 Tprev = S.T;
    S.T = mul4(Ti, S.T);
    const double change = frob_diff4(Tprev, S.T);
    if (S.kind == KIND_ICP) {  // ISR.cpp:547-550
        if (S.iter == S.max_iter || S.rel < S.mse) S.done = 1;
    } else if (S.kind == KIND_PURE) {  // ISR.cpp:1118-1119
        if (S.iter == S.max_se3 || S.rel < S.sf * S.mse) S.done = 1;
    } else if (!S.sw) {  // ISR.cpp:718-723
        if (S.iter == S.max_se3 || change < S.mse_switch) S.sw = 1;
    } else {  // ISR.cpp:724-729
        if (S.iter == S.max_iter || S.rel < S.sf * S.mse) S.done = 1;
    }
    if (S.iter >= 100000) S.done = 1;  // the reference would loop forever
}

// Open the next iteration (ISR.cpp:654-662): the phase of its correspondence search and
// the pose the kernels apply on the fly.  Writes the pair's PairDev fields that change.
SE3ICP_HD void pair_open_iteration(PairState& S, PairDev& P) {
    if (S.done) {
        P.phase = PHASE_IDLE;
        return;
    }
    S.iter++;                                                   // ISR.cpp:656
    const bool se3_nn = (S.kind == KIND_PURE) || (S.kind != KIND_ICP && !S.sw);
    if (se3_nn) S.pure++;                                       // ISR.cpp:660
    P.phase = se3_nn ? PHASE_SE3 : PHASE_R3;
    if (P.phase != S.phase) {  // NN certificates of the other metric are void
        S.phase = P.phase;
        S.phase_start = S.iter;
    }
    P.iter = S.iter;
    P.phase_start = S.phase_start;
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 4; ++c) P.T[r * 4 + c] = S.T.m[r][c];
}

}  // namespace se3icp
