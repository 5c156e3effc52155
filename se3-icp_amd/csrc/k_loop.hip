// k_loop.hip — kernels of one ICP iteration (gfx950), batched over every active pair.
//
//   sweep_se3   brute-force 1-NN under the weighted SE(3) metric (12-D L2),
//               update_correspondences_raw_flann_SE3 ISR.cpp:444-470.  f32, LDS-tiled
//               targets (broadcast ds_read_b128), per query the best (d1,i1) and the
//               second-best distance d2 for the certification below.
//   sweep_r3    same in 3-D, update_correspondences_kd_tree_XYZ ISR.cpp:402-416.
//   finalize    merges target splits, computes the stored R3 distance in f64
//               (ISR.cpp:465-468, 411-413) and certifies the f32 arg-min: when the gap
//               d2-d1 is below twice a rigorous f32 error bound the query is queued for
//   recheck     an exact f64 sweep in nanoflann's arithmetic (ties -> lowest index).
//   trim        PCL CorrespondenceRejectorTrimmed: the floor(ratio*N)-th smallest
//               (float dist, query) key by MSB radix select (ISR.cpp:669-671).
//   reduce      per-correspondence Jacobian terms of the estimator, summed per block:
//               pt2pt moments (umeyama, ISR.cpp:692), pt2pl JTJ/JTr (ISR.cpp:695),
//               GICP JTJ/JTr with M^-1 = (Ct+Cs)^-1 (ISR.cpp:698, 57-110), MSE sum
//               (ISR.cpp:379-400).  A second kernel sums the partials of each pair in
//               a fixed order (deterministic).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>
#include <cmath>

#include "view.hpp"

namespace se3icp {

namespace {

constexpr int kTile = 256;  // targets staged per LDS tile

// query = T * M0 for the 12-vector packing [R(:,0) R(:,1) R(:,2) t] (ISR.cpp:713-716).
__device__ __forceinline__ void pose_frame(const double* T, const double* m, double* q) {
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r)
            q[c * 3 + r] = T[r * 4 + 0] * m[c * 3 + 0] + T[r * 4 + 1] * m[c * 3 + 1] + T[r * 4 + 2] * m[c * 3 + 2];
#pragma unroll
    for (int r = 0; r < 3; ++r) q[9 + r] = T[r * 4 + 0] * m[9] + T[r * 4 + 1] * m[10] + T[r * 4 + 2] * m[11] + T[r * 4 + 3];
}
__device__ __forceinline__ void pose_point(const double* T, double x, double y, double z, double* q) {
#pragma unroll
    for (int r = 0; r < 3; ++r) q[r] = T[r * 4 + 0] * x + T[r * 4 + 1] * y + T[r * 4 + 2] * z + T[r * 4 + 3];
}

__device__ __forceinline__ void load_T(const PairDev* P, double* T) {
#pragma unroll
    for (int i = 0; i < 12; ++i) T[i] = P->T[i];
}

// f64 query vector of source point g of pair P in the current phase.
template <int D>
__device__ __forceinline__ void query_f64(const View& v, const double* T, int g, double* q) {
    if constexpr (D == 12) {
        double m[12];
#pragma unroll
        for (int r = 0; r < 12; ++r) m[r] = v.fr64[(size_t)r * v.ld + g];
        pose_frame(T, m, q);
    } else {
        pose_point(T, v.xyz64[g], v.xyz64[v.ld + g], v.xyz64[2 * (size_t)v.ld + g], q);
    }
}

// ------------------------------------------------------------------ sweeps
template <int D>
__global__ __launch_bounds__(256) void k_sweep(View v) {
    constexpr int NV = (D + 3) / 4;  // float4 per target
    __shared__ float4 tile[kTile * NV];
    const BlockWork w = v.work[blockIdx.x];
    const PairDev* P = v.pairs + w.pair;
    if (P->phase != (D == 12 ? PHASE_SE3 : PHASE_R3)) return;
    const CloudDev cs = v.clouds[P->src], ct = v.clouds[P->tgt];
    const int split = blockIdx.y, S = gridDim.y;
    const int tb = (int)((long long)ct.n * split / S), te = (int)((long long)ct.n * (split + 1) / S);
    const int qi = w.q0 + threadIdx.x;
    const bool valid = qi < cs.n;
    float q[D];
    {
        double T[12], Q[D];
        load_T(P, T);
        query_f64<D>(v, T, cs.off + (valid ? qi : 0), Q);
        if constexpr (D == 3) {
            Q[0] -= P->f32_center[0]; Q[1] -= P->f32_center[1]; Q[2] -= P->f32_center[2];
        }
#pragma unroll
        for (int r = 0; r < D; ++r) q[r] = (float)Q[r];
    }
    const float* src = (D == 12) ? v.fr32 : v.xyz32;
    float d1 = INFINITY, d2 = INFINITY;
    int i1 = -1;
    for (int t0 = tb; t0 < te; t0 += kTile) {
        {
            const int t = t0 + (int)threadIdx.x;
            float a[NV * 4];
#pragma unroll
            for (int r = 0; r < NV * 4; ++r) a[r] = 0.f;
            if (t < te) {
                const int gt = ct.off + t;
#pragma unroll
                for (int r = 0; r < D; ++r) a[r] = src[(size_t)r * v.ld + gt];
            } else {
#pragma unroll
                for (int r = 0; r < D; ++r) a[r] = 1e18f;  // padding: never the nearest
            }
#pragma unroll
            for (int k = 0; k < NV; ++k) tile[threadIdx.x * NV + k] = make_float4(a[4 * k], a[4 * k + 1], a[4 * k + 2], a[4 * k + 3]);
        }
        __syncthreads();
#pragma unroll 4
        for (int j = 0; j < kTile; ++j) {
            float acc;
            if constexpr (D == 12) {
                const float4 A = tile[j * 3], B = tile[j * 3 + 1], C = tile[j * 3 + 2];
                float e;
                e = q[0] - A.x; acc = e * e;
                e = q[1] - A.y; acc = fmaf(e, e, acc);
                e = q[2] - A.z; acc = fmaf(e, e, acc);
                e = q[3] - A.w; acc = fmaf(e, e, acc);
                e = q[4] - B.x; acc = fmaf(e, e, acc);
                e = q[5] - B.y; acc = fmaf(e, e, acc);
                e = q[6] - B.z; acc = fmaf(e, e, acc);
                e = q[7] - B.w; acc = fmaf(e, e, acc);
                e = q[8] - C.x; acc = fmaf(e, e, acc);
                e = q[9] - C.y; acc = fmaf(e, e, acc);
                e = q[10] - C.z; acc = fmaf(e, e, acc);
                e = q[11] - C.w; acc = fmaf(e, e, acc);
            } else {
                const float4 A = tile[j];
                float e;
                e = q[0] - A.x; acc = e * e;
                e = q[1] - A.y; acc = fmaf(e, e, acc);
                e = q[2] - A.z; acc = fmaf(e, e, acc);
            }
            const bool lt = acc < d1;
            d2 = __builtin_amdgcn_fmed3f(d1, d2, acc);
            d1 = lt ? acc : d1;
            i1 = lt ? (t0 + j) : i1;
        }
        __syncthreads();
    }
    if (valid) v.cand[(size_t)split * v.ld + cs.off + qi] = Cand{d1, i1, d2};
}

// ------------------------------------------------------------------ finalize
// Rigorous bound on |f32 distance - exact distance of the f64 vectors| (DESIGN.md
// "Certified f32 arg-min"): inputs rounded to f32 (u = 2^-24), D differences and a
// D-term FMA chain.  na, nb bound the norms of the query and target vectors.
__device__ __forceinline__ float f32_err(float d, float na, float nb, int D) {
    const float u = 5.9604645e-08f;
    const float s = na + nb;
    return 1.25f * (2.f * u * s * sqrtf(fmaxf(d, 0.f)) + (float)(D + 3) * u * d + 4.f * u * u * s * s) + 1e-30f;
}

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

// target search vector j (12-D: alpha-weighted rotation rows + translation rows;
// for run_se3_icp_with_cf the translation rows are the points, ISR.cpp:834-836)
__device__ __forceinline__ void target12(const View& v, const CloudDev& ct, bool cf, int j, double* b) {
    const int gt = ct.off + j;
#pragma unroll
    for (int r = 0; r < 9; ++r) b[r] = v.fr64[(size_t)r * v.ld + gt];
    if (cf) {
        b[9] = v.xyz64[gt]; b[10] = v.xyz64[v.ld + gt]; b[11] = v.xyz64[2 * (size_t)v.ld + gt];
    } else {
        b[9] = v.fr64[9 * (size_t)v.ld + gt]; b[10] = v.fr64[10 * (size_t)v.ld + gt]; b[11] = v.fr64[11 * (size_t)v.ld + gt];
    }
}

// stored distance: R3 distance between the translation parts (ISR.cpp:465: uses the
// beta-weighted target_se3_cloud_ translation even in the cf variant) or the 3-D NN distance
__device__ __forceinline__ float stored_dist(const View& v, int phase, const CloudDev& ct, const double* Q, int j) {
    const int gt = ct.off + j;
    if (phase == PHASE_SE3) {
        const double dx = Q[9] - v.fr64[9 * (size_t)v.ld + gt];
        const double dy = Q[10] - v.fr64[10 * (size_t)v.ld + gt];
        const double dz = Q[11] - v.fr64[11 * (size_t)v.ld + gt];
        return (float)sqrt((dx * dx + dy * dy) + dz * dz);
    }
    const double b[3] = {v.xyz64[gt], v.xyz64[v.ld + gt], v.xyz64[2 * (size_t)v.ld + gt]};
    return (float)sqrt(l2_nanoflann3(Q, b));
}

__global__ __launch_bounds__(256) void k_finalize(View v) {
    const BlockWork w = v.work[blockIdx.x];
    const PairDev* P = v.pairs + w.pair;
    const int phase = P->phase;
    if (phase == PHASE_IDLE) return;
    const CloudDev cs = v.clouds[P->src], ct = v.clouds[P->tgt];
    const int qi = w.q0 + threadIdx.x;
    if (qi >= cs.n) return;
    const int g = cs.off + qi;
    Cand c = v.cand[g];
    float d1 = c.d1, d2 = c.d2;
    int i1 = c.i1;
    for (int s = 1; s < v.nsplit; ++s) {
        const Cand o = v.cand[(size_t)s * v.ld + g];
        if (o.d1 < d1 || (o.d1 == d1 && o.i1 >= 0 && (i1 < 0 || o.i1 < i1))) {
            d2 = fminf(d1, o.d2);
            d1 = o.d1;
            i1 = o.i1;
        } else {
            d2 = fminf(d2, o.d1);
        }
    }
    double T[12], Q[12];
    load_T(P, T);
    float na;
    int D;
    float nb;
    if (phase == PHASE_SE3) {
        query_f64<12>(v, T, g, Q);
        double n2 = 0;
#pragma unroll
        for (int r = 0; r < 12; ++r) n2 += Q[r] * Q[r];
        na = (float)sqrt(n2) * 1.000001f;
        nb = P->tgt_norm12;
        D = 12;
    } else {
        query_f64<3>(v, T, g, Q);
        const double fx = Q[0] - P->f32_center[0], fy = Q[1] - P->f32_center[1], fz = Q[2] - P->f32_center[2];
        na = (float)sqrt(fx * fx + fy * fy + fz * fz) * 1.000001f;
        nb = P->tgt_norm3;
        D = 3;
    }
    const bool flag = (i1 < 0) || !(d2 - d1 > 2.f * f32_err(d2, na, nb, D));
    if (flag && ct.n > 1) {
        const int at = atomicAdd(v.flag_count, 1);
        v.flag_list[at] = g;
        atomicAdd(&v.pair_rechecked[w.pair], 1);
    }
    if (i1 < 0) i1 = 0;  // NaN query: the reference's zero-initialised result index
    v.corr_idx[g] = i1;
    v.corr_dist[g] = stored_dist(v, phase, ct, Q, i1);
}

// ------------------------------------------------------------------ recheck (exact f64)
__device__ __forceinline__ bool key_less(double da, int ia, double db, int ib) {
    return da < db || (da == db && ia < ib);
}

__global__ __launch_bounds__(256) void k_recheck(View v) {
    __shared__ double s_d[4];
    __shared__ int s_i[4];
    const int cnt = *v.flag_count;
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    for (int f = blockIdx.x; f < cnt; f += gridDim.x) {
        const int g = v.flag_list[f];
        const int pair = v.cloud_of[g] >> 1;
        const PairDev* P = v.pairs + pair;
        const int phase = P->phase;
        const CloudDev ct = v.clouds[P->tgt];
        const bool cf = P->cf != 0;
        double T[12], Q[12];
        load_T(P, T);
        double bd = DBL_MAX;
        int bi = INT_MAX;
        if (phase == PHASE_SE3) {
            query_f64<12>(v, T, g, Q);
            for (int j = threadIdx.x; j < ct.n; j += blockDim.x) {
                double b[12];
                target12(v, ct, cf, j, b);
                const double d = l2_nanoflann12(Q, b);
                if (key_less(d, j, bd, bi)) { bd = d; bi = j; }
            }
        } else {
            query_f64<3>(v, T, g, Q);
            for (int j = threadIdx.x; j < ct.n; j += blockDim.x) {
                const int gt = ct.off + j;
                const double b[3] = {v.xyz64[gt], v.xyz64[v.ld + gt], v.xyz64[2 * (size_t)v.ld + gt]};
                const double d = l2_nanoflann3(Q, b);
                if (key_less(d, j, bd, bi)) { bd = d; bi = j; }
            }
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            const double od = __shfl_xor(bd, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            if (key_less(od, oi, bd, bi)) { bd = od; bi = oi; }
        }
        if (lane == 0) { s_d[wid] = bd; s_i[wid] = bi; }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int k = 1; k < 4; ++k)
                if (key_less(s_d[k], s_i[k], bd, bi)) { bd = s_d[k]; bi = s_i[k]; }
            if (bi == INT_MAX) bi = 0;
            v.corr_idx[g] = bi;
            v.corr_dist[g] = stored_dist(v, phase, ct, Q, bi);
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------ trim
__device__ __forceinline__ unsigned long long trim_key_of(const float* dist, int base, int i) {
    return ((unsigned long long)__float_as_uint(dist[base + i]) << 32) | (unsigned)i;
}

// One 1024-thread block per trimming pair: MSB radix select (8-bit digits) of the
// nkeep-th smallest key.  High digits are counted with wave-aggregated atomics
// (distances of neighbouring queries share their exponent byte).
__global__ __launch_bounds__(1024) void k_trim(View v) {
    __shared__ unsigned int hist[256];
    __shared__ unsigned long long s_prefix, s_mask;
    __shared__ int s_k;
    const PairDev* P = v.pairs + blockIdx.x;
    if (P->phase == PHASE_IDLE || !P->trim) return;
    const CloudDev cs = v.clouds[P->src];
    const int n = cs.n;
    if (P->nkeep <= 0) {
        if (threadIdx.x == 0) v.trim_key[blockIdx.x] = 0ull;  // keep none (handled by reduce)
        return;
    }
    if (threadIdx.x == 0) { s_prefix = 0; s_mask = 0; s_k = P->nkeep; }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    for (int shift = 56; shift >= 0; shift -= 8) {
        if (threadIdx.x < 256) hist[threadIdx.x] = 0;
        __syncthreads();
        const unsigned long long prefix = s_prefix, mask = s_mask;
        const bool aggregate = shift >= 48;
        for (int i0 = 0; i0 < n; i0 += blockDim.x) {
            const int i = i0 + threadIdx.x;
            bool act = false;
            unsigned dig = 0;
            if (i < n) {
                const unsigned long long key = trim_key_of(v.corr_dist, cs.off, i);
                act = (key & mask) == prefix;
                dig = (unsigned)(key >> shift) & 255u;
            }
            if (aggregate) {
                unsigned long long am = __ballot(act);
                while (am) {
                    const int leader = __ffsll((long long)am) - 1;
                    const unsigned ld = __shfl(dig, leader, 64);
                    const unsigned long long same = __ballot(act && dig == ld);
                    if (lane == leader) atomicAdd(&hist[ld], (unsigned)__popcll(same));
                    if (dig == ld) act = false;
                    am &= ~same;
                }
            } else if (act) {
                atomicAdd(&hist[dig], 1u);
            }
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            unsigned cum = 0;
            int k = s_k;
            int sel = 255;
            for (int b = 0; b < 256; ++b) {
                if (cum + hist[b] >= (unsigned)k) { sel = b; break; }
                cum += hist[b];
            }
            s_k = k - (int)cum;
            s_prefix = prefix | ((unsigned long long)sel << shift);
            s_mask = mask | (255ull << shift);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) v.trim_key[blockIdx.x] = s_prefix;
}

// ------------------------------------------------------------------ reduce
template <typename T>
__device__ __forceinline__ T wsum(T x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

__global__ __launch_bounds__(256) void k_reduce(View v) {
    __shared__ double red[4][kRedVals];
    const BlockWork w = v.work[blockIdx.x];
    const PairDev* P = v.pairs + w.pair;
    double acc[kRedVals];
#pragma unroll
    for (int i = 0; i < kRedVals; ++i) acc[i] = 0.0;
    if (P->phase == PHASE_IDLE) return;
    const CloudDev cs = v.clouds[P->src], ct = v.clouds[P->tgt];
    const int qi = w.q0 + threadIdx.x;
    bool kept = qi < cs.n;
    if (kept && P->trim) {
        kept = P->nkeep > 0 && trim_key_of(v.corr_dist, cs.off, qi) <= v.trim_key[w.pair];
    }
    if (kept) {
        double T[12];
        load_T(P, T);
        const int g = cs.off + qi;
        const int j = v.corr_idx[g];
        const int gt = ct.off + j;
        double vs[3];
        pose_point(T, v.xyz64[g], v.xyz64[v.ld + g], v.xyz64[2 * (size_t)v.ld + g], vs);
        const double vt[3] = {v.xyz64[gt], v.xyz64[v.ld + gt], v.xyz64[2 * (size_t)v.ld + gt]};
        const double dist = (double)v.corr_dist[g];
        const int est = P->est;
        if (est == EST_PT2PT) {
#pragma unroll
            for (int a = 0; a < 3; ++a) { acc[a] = vs[a]; acc[3 + a] = vt[a]; }
#pragma unroll
            for (int a = 0; a < 3; ++a)
#pragma unroll
                for (int b = 0; b < 3; ++b) acc[6 + a * 3 + b] = vt[a] * vs[b];
            acc[15] = 1.0;
            acc[27] = dist;
        } else {
            double J[3][6], r[3];
            int nrows;
            double wgt = 1.0;
            if (est == EST_PT2PL) {
                const double n[3] = {v.nrm64[gt], v.nrm64[v.ld + gt], v.nrm64[2 * (size_t)v.ld + gt]};
                r[0] = (vs[0] - vt[0]) * n[0] + (vs[1] - vt[1]) * n[1] + (vs[2] - vt[2]) * n[2];
                J[0][0] = vs[1] * n[2] - vs[2] * n[1];
                J[0][1] = vs[2] * n[0] - vs[0] * n[2];
                J[0][2] = vs[0] * n[1] - vs[1] * n[0];
                J[0][3] = n[0]; J[0][4] = n[1]; J[0][5] = n[2];
                nrows = 1;
            } else {
                // Cs = R Cs0 R^T (PointCloud::Transform on covariances, ISR.cpp:706)
                double C0[3][3];
                {
                    const double* cv = v.cov64;
                    const size_t ld = v.ld;
                    C0[0][0] = cv[g]; C0[0][1] = C0[1][0] = cv[ld + g]; C0[0][2] = C0[2][0] = cv[2 * ld + g];
                    C0[1][1] = cv[3 * ld + g]; C0[1][2] = C0[2][1] = cv[4 * ld + g]; C0[2][2] = cv[5 * ld + g];
                }
                double RC[3][3], M[3][3];
#pragma unroll
                for (int a = 0; a < 3; ++a)
#pragma unroll
                    for (int b = 0; b < 3; ++b) RC[a][b] = T[a * 4] * C0[0][b] + T[a * 4 + 1] * C0[1][b] + T[a * 4 + 2] * C0[2][b];
                {
                    const double* cv = v.cov64;
                    const size_t ld = v.ld;
                    const double Ct[6] = {cv[gt], cv[ld + gt], cv[2 * ld + gt], cv[3 * ld + gt], cv[4 * ld + gt], cv[5 * ld + gt]};
                    const int map[3][3] = {{0, 1, 2}, {1, 3, 4}, {2, 4, 5}};
#pragma unroll
                    for (int a = 0; a < 3; ++a)
#pragma unroll
                        for (int b = 0; b < 3; ++b)
                            M[a][b] = Ct[map[a][b]] + (RC[a][0] * T[b * 4] + RC[a][1] * T[b * 4 + 1] + RC[a][2] * T[b * 4 + 2]);
                }
                // M^-1 by cofactors (M is SPD)
                double Mi[3][3];
                Mi[0][0] = M[1][1] * M[2][2] - M[1][2] * M[2][1];
                Mi[0][1] = M[0][2] * M[2][1] - M[0][1] * M[2][2];
                Mi[0][2] = M[0][1] * M[1][2] - M[0][2] * M[1][1];
                Mi[1][0] = M[1][2] * M[2][0] - M[1][0] * M[2][2];
                Mi[1][1] = M[0][0] * M[2][2] - M[0][2] * M[2][0];
                Mi[1][2] = M[0][2] * M[1][0] - M[0][0] * M[1][2];
                Mi[2][0] = M[1][0] * M[2][1] - M[1][1] * M[2][0];
                Mi[2][1] = M[0][1] * M[2][0] - M[0][0] * M[2][1];
                Mi[2][2] = M[0][0] * M[1][1] - M[0][1] * M[1][0];
                const double det = M[0][0] * Mi[0][0] + M[0][1] * Mi[1][0] + M[0][2] * Mi[2][0];
                const double idet = 1.0 / det;
                // J^T J = G^T M^-1 G and J^T r = G^T M^-1 d are invariant to the choice of
                // W with W^T W = M^-1; the reference uses W = M^-1/2 (ISR.cpp:78), here
                // W = L^T with M^-1 = L L^T (Cholesky), which needs no matrix square root.
                double A[3][3];
#pragma unroll
                for (int a = 0; a < 3; ++a)
#pragma unroll
                    for (int b = 0; b < 3; ++b) A[a][b] = 0.5 * (Mi[a][b] + Mi[b][a]) * idet;
                // Cholesky A = L L^T; rows of L^T G are 3 weighted Jacobian rows
                const double l00 = sqrt(A[0][0]);
                const double l10 = A[1][0] / l00, l20 = A[2][0] / l00;
                const double l11 = sqrt(A[1][1] - l10 * l10);
                const double l21 = (A[2][1] - l20 * l10) / l11;
                const double l22 = sqrt(A[2][2] - l20 * l20 - l21 * l21);
                const double Lt[3][3] = {{l00, l10, l20}, {0, l11, l21}, {0, 0, l22}};
                // G = [-[vs]x, I]
                const double G[3][6] = {{0, vs[2], -vs[1], 1, 0, 0}, {-vs[2], 0, vs[0], 0, 1, 0}, {vs[1], -vs[0], 0, 0, 0, 1}};
                const double d[3] = {vs[0] - vt[0], vs[1] - vt[1], vs[2] - vt[2]};
#pragma unroll
                for (int a = 0; a < 3; ++a) {
#pragma unroll
                    for (int b = 0; b < 6; ++b) J[a][b] = Lt[a][0] * G[0][b] + Lt[a][1] * G[1][b] + Lt[a][2] * G[2][b];
                    r[a] = Lt[a][0] * d[0] + Lt[a][1] * d[1] + Lt[a][2] * d[2];
                }
                nrows = 3;
                if (P->cf) {
                    const double wc = (v.conf64[g] + v.conf64[gt]) / 2.0;  // ISR.cpp:913
                    wgt = wc * wc;
                }
            }
            for (int rr = 0; rr < nrows; ++rr) {
                int k = 0;
#pragma unroll
                for (int a = 0; a < 6; ++a)
#pragma unroll
                    for (int b = a; b < 6; ++b) acc[k++] += wgt * J[rr][a] * J[rr][b];
#pragma unroll
                for (int a = 0; a < 6; ++a) acc[21 + a] += wgt * J[rr][a] * r[rr];
            }
            if (P->cf) {  // estimate_current_mse_compute_euclidean, ISR.cpp:390-400
                acc[27] = sqrt(((vs[0] - vt[0]) * (vs[0] - vt[0]) + (vs[1] - vt[1]) * (vs[1] - vt[1])) +
                               (vs[2] - vt[2]) * (vs[2] - vt[2]));
            } else {
                acc[27] = dist;
            }
        }
    }
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < kRedVals; ++i) {
        const double s = wsum(acc[i]);
        if (lane == 0) red[wid][i] = s;
    }
    __syncthreads();
    if (threadIdx.x < kRedVals) {
        const int i = threadIdx.x;
        v.red_partial[(size_t)blockIdx.x * kRedVals + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
    }
}

// Sum each pair's block partials in block order (deterministic); the block list of
// pair p is the contiguous work-table range where work[b].pair == p.
__global__ __launch_bounds__(256) void k_reduce_final(View v, const int32_t* pair_wb, const int32_t* pair_wn) {
    const int p = blockIdx.x;
    if (v.pairs[p].phase == PHASE_IDLE) return;
    __shared__ double part[8][kRedVals];
    const int i = threadIdx.x % kRedVals, s = threadIdx.x / kRedVals;
    const int wb = pair_wb[p], wn = pair_wn[p];
    if (s < 8) {
        double sum = 0;
        for (int b = s; b < wn; b += 8) sum += v.red_partial[(size_t)(wb + b) * kRedVals + i];
        part[s][i] = sum;
    }
    __syncthreads();
    if (threadIdx.x < kRedVals) {
        double sum = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) sum += part[k][threadIdx.x];
        v.red_out[(size_t)p * kRedVals + threadIdx.x] = sum;
    }
}

}  // namespace

void launch_sweep_se3(const View& v, hipStream_t s) {
    hipLaunchKernelGGL(k_sweep<12>, dim3(v.nwork, v.nsplit), dim3(256), 0, s, v);
}
void launch_sweep_r3(const View& v, hipStream_t s) {
    hipLaunchKernelGGL(k_sweep<3>, dim3(v.nwork, v.nsplit), dim3(256), 0, s, v);
}
void launch_finalize(const View& v, hipStream_t s) {
    hipLaunchKernelGGL(k_finalize, dim3(v.nwork), dim3(256), 0, s, v);
}
void launch_recheck(const View& v, int nblocks, hipStream_t s) {
    hipLaunchKernelGGL(k_recheck, dim3(nblocks), dim3(256), 0, s, v);
}
void launch_trim(const View& v, hipStream_t s) {
    hipLaunchKernelGGL(k_trim, dim3(v.npairs), dim3(1024), 0, s, v);
}
void launch_reduce(const View& v, const int32_t* pair_wb, const int32_t* pair_wn, hipStream_t s) {
    hipLaunchKernelGGL(k_reduce, dim3(v.nwork), dim3(256), 0, s, v);
    hipLaunchKernelGGL(k_reduce_final, dim3(v.npairs), dim3(256), 0, s, v, pair_wb, pair_wn);
}

}  // namespace se3icp
