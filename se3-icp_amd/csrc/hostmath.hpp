// hostmath.hpp — the per-iteration small solves, run on the host in f64 after the
// GPU has reduced the correspondences to moments / normal equations.
#pragma once

namespace se3icp {

struct M4 {
    double m[4][4];
    static M4 eye();
};
M4 mul4(const M4& a, const M4& b);
double frob_diff4(const M4& a, const M4& b);

// Eigen::umeyama(src, dst, false) (TransformationEstimationPointToPoint, ISR.cpp:692)
// from the one-pass moments of the kept correspondences:
//   s[0..2] = sum vs, s[3..5] = sum vt, s[6..14] = sum vt vs^T (row-major), n = count.
M4 umeyama_from_moments(const double* s, double n);

// A x = b for symmetric 6x6 A with Eigen LDLT semantics (diagonal pivoting, zero
// pivots treated as a pseudo-inverse) — Open3D SolveLinearSystemPSD.
void ldlt_solve6(const double A[6][6], const double b[6], double x[6]);

// Open3D SolveJacobianSystemAndObtainExtrinsicMatrix from the packed normal
// equations (21 upper-triangular JTJ entries then 6 JTr): x = -(JTJ)^-1 JTr,
// T = TransformVector6dToMatrix4d(x).  Identity when the solution is not finite.
M4 solve_normal_equations(const double* acc27);

// TransformVector6dToMatrix4d: R = AngleAxis(x2,Z)*AngleAxis(x1,Y)*AngleAxis(x0,X), t = x3..5
M4 vec6_to_mat4(const double x[6]);

// A = U diag(s) V^T, s descending (two-sided Jacobi).
void svd3(const double A[3][3], double U[3][3], double s[3], double V[3][3]);

}  // namespace se3icp
