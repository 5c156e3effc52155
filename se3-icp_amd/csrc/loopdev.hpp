// loopdev.hpp — device helpers shared by the per-iteration kernels (k_nn.hip, k_loop.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>
#include <cmath>

#include "tree.hpp"
#include "view.hpp"
#include "wave.hpp"

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
// in the cf variant) and the 3-D NN distance in the R3 phase (ISR.cpp:411-413), f64 -> float.
// The match's anchor: its translation row (SE(3) phase) or its point (R3 phase).
__device__ __forceinline__ void match_anchor(const View& v, int phase, const CloudDev& ct, int j, double* t) {
    const int gt = ct.off + j;
    if (phase == PHASE_SE3) {
        t[0] = v.fr64[(size_t)gt * 12 + 9];
        t[1] = v.fr64[(size_t)gt * 12 + 10];
        t[2] = v.fr64[(size_t)gt * 12 + 11];
    } else {
        t[0] = v.xyz64[gt];
        t[1] = v.xyz64[v.ld + gt];
        t[2] = v.xyz64[2 * (size_t)v.ld + gt];
    }
}
// q: the query's translation part (SE(3)) or point (R3); no FMA contraction (the
// reference's x86 arithmetic)
__device__ __forceinline__ float anchor_dist(const double* q, const double* t) {
#pragma clang fp contract(off)
    const double d0 = q[0] - t[0], d1 = q[1] - t[1], d2 = q[2] - t[2];
    return (float)sqrt((d0 * d0 + d1 * d1) + d2 * d2);
}
// Q: the query vector of the phase (12-D: translation part in Q[9..11]; 3-D: Q[0..2])
__device__ __forceinline__ float stored_dist(const View& v, int phase, const CloudDev& ct, const double* Q, int j) {
    double t[3];
    match_anchor(v, phase, ct, j, t);
    return anchor_dist(phase == PHASE_SE3 ? Q + 9 : Q, t);
}

__device__ __forceinline__ bool key_less(double da, int ia, double db, int ib) {
    return da < db || (da == db && ia < ib);
}

// ------------------------------------------------------------------ recheck (exact f64)
// One wavefront per flagged query: exact f64 1-NN over the target kd-tree of the phase.
// The f32 node boxes were inflated to bound the f64 vectors (k_tree.hip), so a box
// lower bound computed in f64 against the f64 query prunes exactly; boxes whose bound
// equals the best distance are still opened (a lower index may tie).  Seeded with the
// f32 winner of the search (`seed`, a target index).  All 64 lanes of the wave take part;
// lane 0 writes the query's corr_idx / corr_dist.
template <int D>
__device__ __forceinline__ void recheck_one(const View& v, const PairDev* P, const CloudDev& ct, int g, int seed,
                                            int lane) {
    const bool cf = P->cf != 0;
    const TreeRef TR = (D == 12) ? v.t12 : v.t3;
    double T[12], Q[D], qs[D];
    load_T(P, T);
    query_f64<D>(v, T, g, Q);
#pragma unroll
    for (int r = 0; r < D; ++r) qs[r] = (D == 3) ? Q[r] - P->f32_center[r] : Q[r];
    auto dist = [&](int j) __attribute__((always_inline)) {
        if constexpr (D == 12) {
            double b[12];
            target12(v, ct, cf, j, b);
            return l2_nanoflann12(Q, b);
        } else {
            const int gt = ct.off + j;
            const double b[3] = {v.xyz64[gt], v.xyz64[v.ld + gt], v.xyz64[2 * (size_t)v.ld + gt]};
            return l2_nanoflann3(Q, b);
        }
    };
    const float* box_lo = TR.lo + (size_t)P->tgt * TR.nnodes * D;
    const float* box_hi = TR.hi + (size_t)P->tgt * TR.nnodes * D;
    auto lbound = [&](int h) __attribute__((always_inline)) {
        double s = 0.0;
#pragma unroll
        for (int r = 0; r < D; ++r) {
            const double e = fmax(fmax((double)box_lo[h * D + r] - qs[r], qs[r] - (double)box_hi[h * D + r]), 0.0);
            s += e * e;
        }
        return s * (1.0 - 1e-12);
    };
    int bi = seed;  // (the f32 winner)
    if (bi < 0 || bi >= ct.n) bi = 0;
    double bd = dist(bi);
    const int first_leaf = (1 << TR.L) - 1;
    // Lane-parallel box tests (64 nodes per instruction): the nodes of level A = L - 6
    // (<= 64 leaves below each), then the leaves under each node that can still hold a
    // point at or below the best distance (<=: a lower index may tie); open leaves are
    // swept a point per lane.  Seeded with the f32 winner, few boxes stay open.
    const int sh = TR.L > 6 ? 6 : TR.L;
    const int A = TR.L - sh, nA = 1 << A, firstA = nA - 1;
    for (int c0 = 0; c0 < nA; c0 += 64) {
        const int ai = c0 + lane;
        const double lbA = ai < nA ? lbound(firstA + ai) : DBL_MAX;
        unsigned long long mA = __ballot(lbA <= bd);
        while (mA) {
            const int j = __builtin_ctzll(mA);
            mA &= mA - 1ull;
            if (!(__shfl(lbA, j, 64) <= bd)) continue;
            const int l0 = (c0 + j) << sh;
            const int li = l0 + lane;
            const double lbL = lane < (1 << sh) ? lbound(first_leaf + li) : DBL_MAX;
            unsigned long long mL = __ballot(lbL <= bd);
            while (mL) {
                const int t = __builtin_ctzll(mL);
                mL &= mL - 1ull;
                if (!(__shfl(lbL, t, 64) <= bd)) continue;
                const int ta = tree_first(ct.n, TR.L, l0 + t), tb = tree_first(ct.n, TR.L, l0 + t + 1);
                double d = DBL_MAX;
                int jj = INT_MAX;
                if (lane < tb - ta) {
                    jj = TR.perm[ct.off + ta + lane];
                    d = dist(jj);
                }
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) {
                    const double od = xor_lane(d, o);
                    const int oj = xor_lane(jj, o);
                    const bool tk = (bool)((int)(od < d) | ((int)(od == d) & (int)(oj < jj)));
                    d = tk ? od : d;
                    jj = tk ? oj : jj;
                }
                if ((int)(d < bd) | ((int)(d == bd) & (int)(jj < bi))) { bd = d; bi = jj; }
            }
        }
    }
    if (lane == 0) {
        v.corr_idx[g] = bi;
        v.corr_dist[g] = stored_dist(v, P->phase, ct, Q, bi);
    }
}

}  // namespace loopdev
}  // namespace se3icp
