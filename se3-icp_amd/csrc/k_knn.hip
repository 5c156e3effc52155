// k_knn.hip — exact k nearest neighbours of every point in its own cloud
// (KDTreeFlann::SearchKNN, ISR.cpp:253 for TOLDI and Open3D EstimateNormals for the
// normals), one wavefront per query point, over the cloud's 3-D kd-tree (k_tree.hip).
//
// The wave first scans the query's own leaf, then walks the tree depth first
// (nearer child first) and visits a node only while the node's box can still hold a
// point at or below the current k-th distance.  Candidates are kept as (d2, index)
// keys in f64 with nanoflann's arithmetic; the top list (<= 128) and a staging area
// share one 256-entry LDS buffer that a register bitonic network re-sorts when full.
// Ties go to the lowest index.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>

#include "tree.hpp"
#include "view.hpp"

namespace se3icp {

namespace {

constexpr int kWaves = 4;
constexpr int kBuf = 256;
constexpr int kStack = 64;

__device__ __forceinline__ double l2_3(double ax, double ay, double az, double bx, double by, double bz) {
#pragma clang fp contract(off)
    const double d0 = ax - bx, d1 = ay - by, d2 = az - bz;
    return (d0 * d0 + d1 * d1) + d2 * d2;
}

__device__ __forceinline__ bool key_less(double da, int ia, double db, int ib) {
    return da < db || (da == db && ia < ib);
}

// ascending sort of the wave's 256 (d2, idx) keys: 4 keys per lane, bitonic network,
// cross-lane stages through __shfl
__device__ __forceinline__ void wave_bitonic256(double* bd, int* bi, int lane, int cnt) {
    double kd[4];
    int ki[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int e = lane * 4 + s;
        kd[s] = e < cnt ? bd[e] : DBL_MAX;
        ki[s] = e < cnt ? bi[e] : INT_MAX;
    }
#pragma unroll
    for (int k = 2; k <= 256; k <<= 1) {
#pragma unroll
        for (int jd = k >> 1; jd > 0; jd >>= 1) {
            if (jd >= 4) {
                const int pl = lane ^ (jd >> 2);
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int e = lane * 4 + s;
                    const double pd = __shfl(kd[s], pl, 64);
                    const int pi = __shfl(ki[s], pl, 64);
                    const bool up = (e & k) == 0;
                    const bool lower = (e & jd) == 0;
                    const bool take = (lower == up) ? key_less(pd, pi, kd[s], ki[s]) : key_less(kd[s], ki[s], pd, pi);
                    if (take) { kd[s] = pd; ki[s] = pi; }
                }
            } else {
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    if ((s & jd) == 0) {
                        const int t = s | jd;
                        const bool up = ((lane * 4 + s) & k) == 0;
                        const bool sw = up ? key_less(kd[t], ki[t], kd[s], ki[s]) : key_less(kd[s], ki[s], kd[t], ki[t]);
                        if (sw) {
                            const double td = kd[s]; kd[s] = kd[t]; kd[t] = td;
                            const int ti = ki[s]; ki[s] = ki[t]; ki[t] = ti;
                        }
                    }
                }
            }
        }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        bd[lane * 4 + s] = kd[s];
        bi[lane * 4 + s] = ki[s];
    }
}

// squared distance from q to a 3-D box (f32, conservative)
__device__ __forceinline__ float box_lb3(const float* lo, const float* hi, float qx, float qy, float qz) {
    const float dx = fmaxf(fmaxf(lo[0] - qx, qx - hi[0]), 0.f);
    const float dy = fmaxf(fmaxf(lo[1] - qy, qy - hi[1]), 0.f);
    const float dz = fmaxf(fmaxf(lo[2] - qz, qz - hi[2]), 0.f);
    return dx * dx + dy * dy + dz * dz;
}

__global__ __launch_bounds__(256) void k_knn_tree(View v) {
    __shared__ double s_d[kWaves][kBuf];
    __shared__ int s_i[kWaves][kBuf];
    __shared__ int s_stack[kWaves][kStack];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int g = blockIdx.x * kWaves + wid;
    if (g >= v.npts) return;
    const int c = v.cloud_of[g];
    const int K = v.setup[c].k_knn;
    if (K == 0) return;
    const CloudDev cl = v.clouds[c];
    const TreeRef T = v.t3;
    double* bd = s_d[wid];
    int* bi = s_i[wid];
    int* stk = s_stack[wid];
    const double qx = v.xyz64[g], qy = v.xyz64[v.ld + g], qz = v.xyz64[2 * (size_t)v.ld + g];
    const float fx = v.xyz32[g], fy = v.xyz32[v.ld + g], fz = v.xyz32[2 * (size_t)v.ld + g];
    const float* box_lo = T.lo + (size_t)c * T.nnodes * 3;
    const float* box_hi = T.hi + (size_t)c * T.nnodes * 3;
    const int Kw = min(K, cl.n);
    const int first_leaf = (1 << T.L) - 1;
    const int own = first_leaf + tree_node_of(T.pos[g], cl.n, T.L);
    int nTop = 0, nStg = 0;
    double thr = DBL_MAX;
    int thr_i = INT_MAX;

    auto merge = [&]() {
        __builtin_amdgcn_wave_barrier();
        wave_bitonic256(bd, bi, lane, nTop + nStg);
        __builtin_amdgcn_wave_barrier();
        nTop = min(Kw, nTop + nStg);
        nStg = 0;
        if (nTop == Kw) { thr = bd[Kw - 1]; thr_i = bi[Kw - 1]; }
    };
    auto leaf = [&](int h) {
        const int i = h - first_leaf;
        const int a = tree_first(cl.n, T.L, i), b = tree_first(cl.n, T.L, i + 1);
        bool acc = false;
        double d = DBL_MAX;
        int li = INT_MAX;
        if (lane < b - a) {
            li = T.perm[cl.off + a + lane];
            const int gp = cl.off + li;
            d = l2_3(qx, qy, qz, v.xyz64[gp], v.xyz64[v.ld + gp], v.xyz64[2 * (size_t)v.ld + gp]);
            acc = (nTop < Kw) || key_less(d, li, thr, thr_i);
        }
        const unsigned long long m = __ballot(acc);
        if (acc) {
            const int at = nTop + nStg + __popcll(m & ((1ull << lane) - 1ull));
            bd[at] = d;
            bi[at] = li;
        }
        nStg += __popcll(m);
        if (nTop + nStg > kBuf - kLeafMax) merge();
    };

    leaf(own);
    int sp = 0;
    if (lane == 0) stk[0] = 0;
    sp = 1;
    while (sp > 0) {
        __builtin_amdgcn_wave_barrier();
        const int h = __builtin_amdgcn_readfirstlane(stk[sp - 1]);
        --sp;
        if (h >= first_leaf) {
            if (h != own) leaf(h);
            continue;
        }
        const int hl = 2 * h + 1, hr = 2 * h + 2;
        const float ll = box_lb3(box_lo + 3 * hl, box_hi + 3 * hl, fx, fy, fz);
        const float lr = box_lb3(box_lo + 3 * hr, box_hi + 3 * hr, fx, fy, fz);
        // conservative: the f32 bound may exceed the true f64 distance by a few ulps
        const bool vl = (nTop < Kw) || (double)ll * (1.0 - 1e-6) <= thr;
        const bool vr = (nTop < Kw) || (double)lr * (1.0 - 1e-6) <= thr;
        const int nearh = ll <= lr ? hl : hr, farh = ll <= lr ? hr : hl;
        const bool vnear = ll <= lr ? vl : vr, vfar = ll <= lr ? vr : vl;
        if (lane == 0) {
            if (vfar) stk[sp] = farh;
            if (vnear) stk[sp + (vfar ? 1 : 0)] = nearh;
        }
        sp += (vfar ? 1 : 0) + (vnear ? 1 : 0);
    }
    if (nStg > 0) merge();
    int* out = v.knn + (size_t)g * v.kmax;
    for (int j = lane; j < K; j += 64) out[j] = j < nTop ? bi[j] : -1;
}

}  // namespace

void launch_knn(const View& v, hipStream_t s) {
    hipLaunchKernelGGL(k_knn_tree, dim3((v.npts + kWaves - 1) / kWaves), dim3(64 * kWaves), 0, s, v);
}

}  // namespace se3icp
