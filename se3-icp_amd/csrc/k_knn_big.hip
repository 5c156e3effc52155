// k_knn_big.hip — kNN + TOLDI frame + normals for neighbourhoods the LDS kernels cannot
// hold: Kw = min(number_of_nn_for_LRF_, n) > kSmallK.  The reference's field is unbounded
// (include/iterative_SE3_registration.hpp:80) and goes straight to KDTreeFlann::SearchKNN
// (ISR.cpp:253), so this path has no cap but device memory.
//
// One wavefront (a 64-thread block) per query, grid-strided over the queries; each block
// owns a candidate buffer of `cap` (d2, tree slot) entries in global memory (L2-resident).
// The search is the exact kernel's (k_knn.hip k_lrf): own leaf, tree-order neighbours until
// Kw candidates exist, then level-A boxes 64 per instruction and the leaves of every open
// node, re-tested as the bound shrinks.  The bound is the Kw-th smallest f32-rounded-up
// distance (a bisection over the f32 bit patterns with ballot counts), so it never drops
// a member of the exact top-Kw; massive ties at the bound are cut exactly by (d, index).
// The survivors are sorted by (f64 d, point index) — nanoflann's order, ties by the lower
// index — in registers up to 512 entries, by a bitonic network in the buffer beyond.
// The neighbour sums, eigen-solves and frame use the same loops, lane assignment and
// arithmetic as k_lrf's epilogue (lanes 0-7 of the wave play one query's eight-lane group),
// so a query routed here gets k_lrf's result bit for bit (tests/test_gpu_parity.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <climits>

#include "devmath.hpp"
#include "knn_util.hpp"
#include "tree.hpp"
#include "view.hpp"
#include "wave.hpp"

namespace se3icp {

namespace {

using namespace knn;

// one compare-exchange stage (block K, distance J) of an ascending bitonic network over the
// wave's 64 * PER (d, index) keys, entry e = lane * PER + s in register s (compile-time
// indices: template recursion, so nothing goes to scratch)
template <int PER, int K, int J>
__device__ __forceinline__ void big_stage(double (&kd)[PER], int (&ki)[PER], int lane) {
    if constexpr (J >= PER) {
#pragma unroll
        for (int s = 0; s < PER; ++s) {
            const int e = lane * PER + s;
            const double pd = xor_lane(kd[s], J / PER);
            const int pi = xor_lane(ki[s], J / PER);
            const bool up = (e & K) == 0, lower = (e & J) == 0;
            const bool take = key_less(pd, pi, kd[s], ki[s]) != (lower != up);
            kd[s] = take ? pd : kd[s];
            ki[s] = take ? pi : ki[s];
        }
    } else {
#pragma unroll
        for (int s = 0; s < PER; ++s) {
            if ((s & J) == 0) {
                const int t = s | J;
                const bool up = ((lane * PER + s) & K) == 0;
                const bool sw = key_less(kd[t], ki[t], kd[s], ki[s]) != !up;
                const double ds = kd[s], dt = kd[t];
                const int is = ki[s], it = ki[t];
                kd[s] = sw ? dt : ds; kd[t] = sw ? ds : dt;
                ki[s] = sw ? it : is; ki[t] = sw ? is : it;
            }
        }
    }
}
template <int PER, int N, int K = 2, int J = 1>
__device__ __forceinline__ void big_net(double (&kd)[PER], int (&ki)[PER], int lane) {
    big_stage<PER, K, J>(kd, ki, lane);
    if constexpr (J > 1) big_net<PER, N, K, J / 2>(kd, ki, lane);
    else if constexpr (K < N) big_net<PER, N, K * 2, K>(kd, ki, lane);
}
// ascending (f64 d, point index) sort of entries [0, n) of the buffer, n <= 64 * PER, in registers
template <int PER>
__device__ __forceinline__ void reg_sort(double* bd, int* bi, int n, int lane) {
    double kd[PER];
    int ki[PER];
#pragma unroll
    for (int s = 0; s < PER; ++s) {
        const int e = lane * PER + s;
        kd[s] = e < n ? bd[e] : DBL_MAX;
        ki[s] = e < n ? bi[e] : INT_MAX;
    }
    big_net<PER, 64 * PER>(kd, ki, lane);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < PER; ++s) {
        const int e = lane * PER + s;
        if (e < n) {
            bd[e] = kd[s];
            bi[e] = ki[s];
        }
    }
    __syncthreads();
}

// the same order for any n <= cap (cap a power of two): bitonic network in the buffer
__device__ void mem_sort(double* bd, int* bi, int n, int cap, int lane) {
    if (n <= 64) { reg_sort<1>(bd, bi, n, lane); return; }
    if (n <= 128) { reg_sort<2>(bd, bi, n, lane); return; }
    if (n <= 256) { reg_sort<4>(bd, bi, n, lane); return; }
    if (n <= 512) { reg_sort<8>(bd, bi, n, lane); return; }
    int N = 1024;
    while (N < n) N <<= 1;  // <= cap
    for (int e = n + lane; e < N; e += 64) { bd[e] = DBL_MAX; bi[e] = INT_MAX; }
    __syncthreads();
    for (int k = 2; k <= N; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = lane; i < N; i += 64) {
                const int p = i ^ j;
                if (p > i) {
                    const double di = bd[i], dp = bd[p];
                    const int ii = bi[i], ip = bi[p];
                    const bool up = (i & k) == 0;
                    if (key_less(dp, ip, di, ii) == up) {
                        bd[i] = dp; bd[p] = di;
                        bi[i] = ip; bi[p] = ii;
                    }
                }
            }
            __syncthreads();
        }
    }
    (void)cap;
}

__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_knn_big(View v, int write_knn, int k_min, const int32_t* __restrict__ qlist,
                                                const int32_t* __restrict__ qcount, double* __restrict__ scratch_d,
                                                int32_t* __restrict__ scratch_i, int cap) {
    const int lane = threadIdx.x;
    const TreeRef T = v.t3;
    const double* TX = T.tvec64;
    const double* TY = T.tvec64 + v.ld;
    const double* TZ = T.tvec64 + 2 * (size_t)v.ld;
    const int first_leaf = (1 << T.L) - 1;
    double* bd = scratch_d + (size_t)blockIdx.x * cap;
    int* bi = scratch_i + (size_t)blockIdx.x * cap;
    const int nvq = qlist ? *qcount : v.npts;
    for (int qi = blockIdx.x; qi < nvq; qi += gridDim.x) {
        const int w = qlist ? qlist[qi] : qi;  // the query's tree slot
        const int c = v.cloud_of[w];
        const CloudSetup st = v.setup[c];
        const int K = st.k_knn;
        const CloudDev cl = v.clouds[c];
        const int n = cl.n;
        const int Kw = min(K, n);
        if (K == 0 || Kw <= k_min) continue;  // (k_lrf's queries)
        const double qx = TX[w], qy = TY[w], qz = TZ[w];
        const float fx = T.tvec[w], fy = T.tvec[v.ld + w], fz = T.tvec[2 * (size_t)v.ld + w];
        const float* box_lo = T.lo + (size_t)c * T.nnodes * 3;
        const float* box_hi = T.hi + (size_t)c * T.nnodes * 3;
        const int own = first_leaf + tree_node_of(w - cl.off, n, T.L);

        // ------------------------------------------------------------ kNN (k_lrf's search)
        int nb = 0;
        bool have_thr = false;
        double thr = DBL_MAX;
        int thr_i = INT_MAX;  // < INT_MAX only after an exact truncation (ties by point index)
        float thr_f = INFINITY;
        auto set_thr_f = [&]() { thr_f = __uint_as_float(f32_up_bits(thr * (1.0 + 2e-6))); };
        // exact (d, point index) sort of the buffer, truncated to Kw: the bound of massive ties
        auto exact_cut = [&]() {
            __syncthreads();
            for (int e = lane; e < nb; e += 64) bi[e] = T.perm[bi[e]];  // slots -> point indices
            __syncthreads();
            mem_sort(bd, bi, nb, cap, lane);
            nb = min(nb, Kw);
            thr = bd[nb - 1];
            thr_i = bi[nb - 1];
            for (int e = lane; e < nb; e += 64) bi[e] = cl.off + T.pos[cl.off + bi[e]];  // and back
            __syncthreads();
            set_thr_f();
        };
        auto select_thr = [&]() {
            __syncthreads();
            // smallest f32 pattern u with count(f32_up(d) <= u) >= Kw
            unsigned lo = 0, hi = 0x7f800000u;
            while (lo < hi) {
                const unsigned mid = lo + ((hi - lo) >> 1);
                int cnt = 0;
                for (int e0 = 0; e0 < nb; e0 += 64) {
                    const int e = e0 + lane;
                    cnt += __popcll(__ballot(e < nb && f32_up_bits(bd[e]) <= mid));
                }
                if (cnt >= Kw) hi = mid; else lo = mid + 1;
            }
            const double t = (double)__uint_as_float(lo);
            if (t < thr) { thr = t; thr_i = INT_MAX; set_thr_f(); }
            // stable compaction in place: entries (d, index) <= (thr, thr_i)
            int base = 0;
            for (int e0 = 0; e0 < nb; e0 += 64) {
                const int e = e0 + lane;
                double d = DBL_MAX;
                int id = 0;
                bool keep = false;
                if (e < nb) {
                    d = bd[e];
                    id = bi[e];
                    keep = d < thr;
                    if (d == thr) keep = thr_i == INT_MAX || T.perm[id] <= thr_i;
                }
                const unsigned long long m = __ballot(keep);
                if (keep) {
                    const int at = base + __popcll(m & ((1ull << lane) - 1ull));
                    bd[at] = d;
                    bi[at] = id;
                }
                base += __popcll(m);
            }
            nb = base;
            have_thr = true;
            __syncthreads();
            if (nb > cap - kLeafMax) exact_cut();
        };
        auto leaf = [&](int h) {
            const int i = h - first_leaf;
            const int a = tree_first(n, T.L, i), b = tree_first(n, T.L, i + 1);
            bool acc = false;
            double d = DBL_MAX;
            const int slot = cl.off + a + lane;
            if (lane < b - a) {
                d = l2_3(qx, qy, qz, TX[slot], TY[slot], TZ[slot]);
                bool eq = d == thr;
                if (thr_i != INT_MAX) eq = eq && T.perm[slot] <= thr_i;
                acc = !have_thr || d < thr || eq;
            }
            const unsigned long long m = __ballot(acc);
            if (acc) {
                const int at = nb + __popcll(m & ((1ull << lane) - 1ull));
                bd[at] = d;
                bi[at] = slot;
            }
            nb += __popcll(m);
            if ((!have_thr && nb >= Kw) || nb > cap - kLeafMax) select_thr();
        };
        auto open = [&](float lb) { return !have_thr || lb <= thr_f; };

        leaf(own);
        const int nleaf = 1 << T.L;
        const int own_i = own - first_leaf;
        int s_lo = own_i, s_hi = own_i;
        while (!have_thr && (s_lo > 0 || s_hi < nleaf - 1)) {
            if (s_hi < nleaf - 1) leaf(first_leaf + (++s_hi));
            if (!have_thr && s_lo > 0) leaf(first_leaf + (--s_lo));
        }
        {
            const int sh = T.L > 6 ? 6 : T.L;
            const int nA = 1 << (T.L - sh), firstA = nA - 1;
            for (int c0 = 0; c0 < nA; c0 += 64) {
                const int ai = c0 + lane;
                float lbA = INFINITY;
                if (ai < nA) lbA = box_lb3(box_lo + 3 * (firstA + ai), box_hi + 3 * (firstA + ai), fx, fy, fz);
                OutwardBits itA(__ballot(ai < nA && open(lbA)), (own_i >> sh) - c0);
                for (int j; (j = itA.next()) >= 0;) {
                    if (!open(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(lbA), j)))) continue;
                    const int l0 = (c0 + j) << sh;
                    const int li = l0 + lane;
                    float lbL = INFINITY;
                    if (lane < (1 << sh) && (li < s_lo || li > s_hi))
                        lbL = box_lb3(box_lo + 3 * (first_leaf + li), box_hi + 3 * (first_leaf + li), fx, fy, fz);
                    OutwardBits itL(__ballot(open(lbL)), own_i - l0);
                    for (int t; (t = itL.next()) >= 0;) {
                        if (!open(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(lbL), t)))) continue;
                        leaf(first_leaf + l0 + t);
                    }
                }
            }
        }
        if (nb > Kw + kLeafMax) select_thr();
        // exact (f64 d, point index) order of the survivors; the list keeps tree slots
        __syncthreads();
        for (int e = lane; e < nb; e += 64) bi[e] = T.perm[bi[e]];
        __syncthreads();
        mem_sort(bd, bi, nb, cap, lane);
        for (int e = lane; e < nb; e += 64) bi[e] = cl.off + T.pos[cl.off + bi[e]];
        __syncthreads();
        const int nTop = min(Kw, nb);
        const int gp = cl.off + T.perm[w];
        if (write_knn) {
            int* out = v.knn + (size_t)gp * v.kmax;
            for (int r = lane; r < K; r += 64) out[r] = r < nTop ? T.perm[bi[r]] : -1;
        }

        // ------------------------------------------------------------ sums (k_lrf's epilogue)
        // lanes 0-7 are the query's eight-lane group: lane qs takes ranks = qs (mod 8)
        const int qs = lane;
        const bool grp = lane < 8;
        const bool want_t = st.k_lrf > 0, want_n = st.k_nrm > 0;
        const int kk = min(st.k_lrf, nTop);
        double x[kSums];
#pragma unroll
        for (int i = 0; i < kSums; ++i) x[i] = 0.0;
        if (grp && want_t) {
            const int rz = kk / 3;
            const int hi = min(rz, kk - 1);
            for (int rk = 1 + qs; rk <= hi; rk += 8) {
                const int q = bi[rk];
                const double vx = TX[q] - qx, vy = TY[q] - qy, vz = TZ[q] - qz;
                if (rk < rz) { x[0] += vx; x[1] += vy; x[2] += vz; }
                x[3] += vx; x[4] += vy; x[5] += vz;
                x[6] += vx * vx; x[7] += vx * vy; x[8] += vx * vz;
                x[9] += vy * vy; x[10] += vy * vz; x[11] += vz * vz;
            }
        }
        if (grp && want_n) {
            const int kn = min(st.k_nrm, nTop);
            for (int r = qs; r < kn; r += 8) {
                const int q = bi[r];
                const double px = TX[q], py = TY[q], pz = TZ[q];
                x[12] += px; x[13] += py; x[14] += pz;
                x[15] += px * px; x[16] += px * py; x[17] += px * pz;
                x[18] += py * py; x[19] += py * pz; x[20] += pz * pz;
            }
        }
#pragma unroll
        for (int i = 0; i < kSums; ++i) {
            x[i] += xor_lane(x[i], 1);
            x[i] += xor_lane(x[i], 2);
            x[i] += xor_lane(x[i], 4);
        }
        // ------------------------------------------------------------ eigen-solves (lane 0)
        double Rf = 0.0;
        d3 zn{0, 0, 0};
        if (lane == 0 && want_t) {
            const int far = bi[kk - 1];
            const double fdx = qx - TX[far], fdy = qy - TY[far], fdz = qz - TZ[far];
            Rf = sqrt(fdx * fdx + fdy * fdy + fdz * fdz);  // ISR.cpp:256
            const double rz = (double)(kk / 3);
            const double q3[3] = {qx, qy, qz};
            double cq[3], S[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                cq[a] = (x[a] - q3[a]) / rz;
                S[a] = x[3 + a];
            }
            const double* M = x + 6;
            const int ia[6] = {0, 0, 0, 1, 1, 2}, ib[6] = {0, 1, 2, 1, 2, 2};
            double c6[6];
#pragma unroll
            for (int k = 0; k < 6; ++k)
                c6[k] = M[k] - S[ia[k]] * cq[ib[k]] - cq[ia[k]] * S[ib[k]] + rz * cq[ia[k]] * cq[ib[k]];
            zn = jacobi_smallest_evec(c6[0], c6[1], c6[2], c6[3], c6[4], c6[5]);
        }
        if (lane == 0 && want_n) {
            const int knb = min(st.k_nrm, nTop);
            double n6[6] = {1, 0, 0, 1, 0, 1};
            if (knb >= 3) {
                double cu[9];
#pragma unroll
                for (int i = 0; i < 9; ++i) cu[i] = x[12 + i] / (double)knb;
                n6[0] = cu[3] - cu[0] * cu[0];
                n6[1] = cu[4] - cu[0] * cu[1];
                n6[2] = cu[5] - cu[0] * cu[2];
                n6[3] = cu[6] - cu[1] * cu[1];
                n6[4] = cu[7] - cu[1] * cu[2];
                n6[5] = cu[8] - cu[2] * cu[2];
            }
            d3 nm = fast_eigen3x3(n6[0], n6[1], n6[2], n6[3], n6[4], n6[5]);
            if (sqrt(dot3(nm, nm)) == 0.0) nm = d3{0, 0, 1};
            v.nrm64[gp] = nm.x;
            v.nrm64[v.ld + gp] = nm.y;
            v.nrm64[2 * (size_t)v.ld + gp] = nm.z;
        }
        // ------------------------------------------------------------ TOLDI axes (ISR.cpp:286-306)
        const double nx = __shfl(zn.x, 0, 64), ny = __shfl(zn.y, 0, 64), nz = __shfl(zn.z, 0, 64);
        const double R = __shfl(Rf, 0, 64);
        double x6[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        if (grp && want_t) {
            for (int r = 1 + qs; r < kk; r += 8) {  // ranks 1 .. kk-1
                const int slot = bi[r];
                const double vx = TX[slot] - qx, vy = TY[slot] - qy, vz = TZ[slot] - qz;
                x6[0] += vx; x6[1] += vy; x6[2] += vz;
                const double an = nx * vx + ny * vy + nz * vz;
                const double rr = R - sqrt(vx * vx + vy * vy + vz * vz);
                const double wgt = (rr * rr) * (an * an);
                x6[3] += wgt * vx; x6[4] += wgt * vy; x6[5] += wgt * vz;
            }
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            x6[i] += xor_lane(x6[i], 1);
            x6[i] += xor_lane(x6[i], 2);
            x6[i] += xor_lane(x6[i], 4);
        }
        if (lane == 0 && want_t) {  // the frame (ISR.cpp:298-307, 597-607)
            d3 nrm = zn;
            if (nrm.x * x6[0] + nrm.y * x6[1] + nrm.z * x6[2] < 0.0) nrm = d3{-nrm.x, -nrm.y, -nrm.z};  // ISR.cpp:298
            const d3 zax = nrm;
            const d3 accs{x6[3], x6[4], x6[5]};
            d3 xax = accs - dot3(accs, zax) * zax;  // ISR.cpp:302-303 (no |x| = 0 guard, as the reference)
            xax = (1.0 / sqrt(dot3(xax, xax))) * xax;
            const d3 yax = cross3(zax, xax);  // ISR.cpp:306
            const double al = st.alpha, be = st.beta;
            const double f12[12] = {al * xax.x, al * xax.y, al * xax.z, al * yax.x, al * yax.y, al * yax.z,
                                    al * zax.x, al * zax.y, al * zax.z, be * qx, be * qy, be * qz};
            store_frame_rows(v.fr64, v.fr32, gp, f12, st.cf_target, qx, qy, qz);
        }
        __syncthreads();  // (the next query reuses the buffer)
    }
}

}  // namespace

int knn_big_cap(int kw_max) {
    int cap = 2048;
    while (cap < 2 * kw_max + 4 * kLeafMax) cap <<= 1;
    return cap;
}

int knn_big_blocks(int cap, int nq) {
    const size_t budget = (size_t)768 << 20;  // scratch bytes
    const int by_mem = (int)std::max<size_t>(64, budget / ((size_t)cap * 12));
    return std::max(1, std::min({nq, 4096, by_mem}));
}

void launch_knn_big(const View& v, int write_knn, int k_min, const int32_t* qlist, const int32_t* qcount, int nblocks,
                    double* scratch_d, int32_t* scratch_i, int cap, hipStream_t s) {
    hipLaunchKernelGGL(k_knn_big, dim3(nblocks), dim3(64), 0, s, v, write_knn, k_min, qlist, qcount, scratch_d,
                       scratch_i, cap);
}

}  // namespace se3icp
