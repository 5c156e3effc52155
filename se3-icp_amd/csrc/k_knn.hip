// k_knn.hip — per-point local geometry from the k nearest neighbours, fused:
//   * exact kNN of the point in its own cloud (KDTreeFlann::SearchKNN, ISR.cpp:253),
//   * the TOLDI local reference frame -> alpha/beta-weighted SE(3) 12-vector
//     (computeSingleTOLDISE3Frame ISR.cpp:241-316, weights ISR.cpp:597-607),
//   * Open3D EstimateNormals on the k_nrm nearest (ISR.cpp:643, :43) and the GICP
//     covariance Rx diag(eps,1,1) Rx^T (ISR.cpp:33-52).
// One wavefront per point, points taken in kd-tree order so that neighbouring waves
// touch the same leaves.  The wave scans the point's own leaf, then tests node boxes
// lane-parallel (64 per instruction: the nodes of the level with <= 64 leaves below
// each, then the leaves under each open one) and scans the leaves that can still hold
// a point at or below the current k-th distance.  Candidates are
// (d2, index) keys in f64 with nanoflann's arithmetic (ties -> lowest index), kept in
// a 256-entry LDS buffer re-sorted by a register bitonic network.  The TOLDI and
// normal sums over neighbour ranks are then wave reductions (the reference sums them
// sequentially; the difference is rounding only).
#include <hip/hip_runtime.h>

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

constexpr int kWaves = 4;
constexpr int kBuf = 256;
constexpr int kQ = 8;  // queries per wave (consecutive tree positions)

// SE3ICP_PROF builds (make prof): per-section shader-clock cycles into stats columns 8..11
#ifdef SE3ICP_PROF
#define PROF_NOW(t) const unsigned long long t = __builtin_readcyclecounter()
#define PROF_ADD(acc, a, b) acc += (b) - (a)
#else
#define PROF_NOW(t) do {} while (0)
#define PROF_ADD(acc, a, b) do {} while (0)
#endif

// Fast path of the final order: one 64-bit key per candidate, (f32 bits of d rounded
// up) << 32 | idx.  Distinct f32 keys are in the f64 order (f32_up_bits is monotone), so
// the order is the exact (f64 d, idx) order unless two of the first `lim` entries share
// an f32 key; that is detected after the network and the caller falls back to the exact
// (f64, idx) sort (bd / bi untouched).  On success bi[] holds the sorted indices and bd[]
// the f32-rounded-up distances (upper bounds, used only to seed the next query's bound).
template <int PER>
__device__ __forceinline__ bool wave_sort_u64(double* bd, int* bi, int lane, int cnt, int lim) {
    constexpr int N = 64 * PER;
    unsigned long long k[PER];
#pragma unroll
    for (int s = 0; s < PER; ++s) {
        const int e = lane * PER + s;
        k[s] = e < cnt ? ((unsigned long long)f32_up_bits(bd[e]) << 32) | (unsigned)bi[e] : ~0ull;
    }
#pragma unroll
    for (int kk = 2; kk <= N; kk <<= 1) {
#pragma unroll
        for (int jd = kk >> 1; jd > 0; jd >>= 1) {
            if (jd >= PER) {
#pragma unroll
                for (int s = 0; s < PER; ++s) {
                    const int e = lane * PER + s;
                    const unsigned long long pk = xor_lane(k[s], jd / PER);
                    // keys are distinct except identical padding (see wave_bitonic)
                    const bool take = (pk < k[s]) != (((e & jd) == 0) != ((e & kk) == 0));
                    k[s] = take ? pk : k[s];
                }
            } else {
#pragma unroll
                for (int s = 0; s < PER; ++s) {
                    if ((s & jd) == 0) {
                        const int t = s | jd;
                        const bool up = ((lane * PER + s) & kk) == 0;
                        const bool sw = (k[t] < k[s]) != !up;
                        const unsigned long long ks = k[s], kt = k[t];
                        k[s] = sw ? kt : ks;
                        k[t] = sw ? ks : kt;
                    }
                }
            }
        }
    }
    bool tie = false;
#pragma unroll
    for (int s = 0; s + 1 < PER; ++s) {
        const int e = lane * PER + s;
        tie |= (bool)((int)(e + 1 < lim) & (int)((unsigned)(k[s] >> 32) == (unsigned)(k[s + 1] >> 32)));
    }
    {
        const unsigned nxt = __shfl_down((unsigned)(k[0] >> 32), 1, 64);
        const int e = lane * PER + PER - 1;
        tie |= (bool)((int)(e + 1 < lim) & (int)(lane < 63) & (int)((unsigned)(k[PER - 1] >> 32) == nxt));
    }
    if (__ballot(tie) != 0ull) return false;
#pragma unroll
    for (int s = 0; s < PER; ++s) {
        const int e = lane * PER + s;
        if (e < cnt) {
            bi[e] = (int)(unsigned)k[s];
            bd[e] = (double)__uint_as_float((unsigned)(k[s] >> 32));
        }
    }
    return true;
}

// ascending sort of the wave's first 64*PER (d2, idx) keys (PER per lane, entry
// lane*PER+s; entries >= cnt are padding): register bitonic network, cross-lane stages
// through __shfl
template <int PER>
__device__ __forceinline__ void wave_bitonic(double* bd, int* bi, int lane, int cnt) {
    constexpr int N = 64 * PER;
    double kd[PER];
    int ki[PER];
#pragma unroll
    for (int s = 0; s < PER; ++s) {
        const int e = lane * PER + s;
        kd[s] = e < cnt ? bd[e] : DBL_MAX;
        ki[s] = e < cnt ? bi[e] : INT_MAX;
    }
#pragma unroll
    for (int k = 2; k <= N; k <<= 1) {
#pragma unroll
        for (int jd = k >> 1; jd > 0; jd >>= 1) {
            if (jd >= PER) {
#pragma unroll
                for (int s = 0; s < PER; ++s) {
                    const int e = lane * PER + s;
                    const double pd = xor_lane(kd[s], jd / PER);
                    const int pi = xor_lane(ki[s], jd / PER);
                    const bool up = (e & k) == 0;
                    const bool lower = (e & jd) == 0;
                    // keys are distinct except identical padding, so "mine < partner" is
                    // !(partner < mine): one comparison, no divergent select
                    const bool take = key_less(pd, pi, kd[s], ki[s]) != (lower != up);
                    kd[s] = take ? pd : kd[s];
                    ki[s] = take ? pi : ki[s];
                }
            } else {
#pragma unroll
                for (int s = 0; s < PER; ++s) {
                    if ((s & jd) == 0) {
                        const int t = s | jd;
                        const bool up = ((lane * PER + s) & k) == 0;
                        const bool sw = key_less(kd[t], ki[t], kd[s], ki[s]) != !up;
                        const double ds = kd[s], dt = kd[t];
                        const int is = ki[s], it = ki[t];
                        kd[s] = sw ? dt : ds; kd[t] = sw ? ds : dt;
                        ki[s] = sw ? it : is; ki[t] = sw ? is : it;
                    }
                }
            }
        }
    }
#pragma unroll
    for (int s = 0; s < PER; ++s) {
        bd[lane * PER + s] = kd[s];
        bi[lane * PER + s] = ki[s];
    }
}

// The per-cloud records and node boxes are also passed as restrict-qualified arguments:
// with no possible aliasing store the compiler can serve their wave-uniform reads from
// the scalar cache (s_load) instead of vector loads.
// (5 waves per SIMD)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5))) void k_lrf(View v, int write_knn, const int32_t* __restrict__ cloud_of,
                                             const CloudSetup* __restrict__ setup,
                                             const CloudDev* __restrict__ clouds, const float* __restrict__ tlo,
                                             const float* __restrict__ thi, const int32_t* __restrict__ qlist,
                                             const int32_t* __restrict__ qcount, int qpw) {
    __shared__ double s_d[kWaves][kBuf];
    __shared__ int s_i[kWaves][kBuf];
    // the queries' sorted neighbour lists: dynamic LDS, kQ x v.kmax ints per wave, sized to
    // the batch's largest k so that five 4-wave blocks fit a CU's 160 KB
    extern __shared__ int s_dyn[];
    __shared__ double s_park[kWaves][kQ][PK_N];
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // first global slot (3-D tree order) of the wave's kQ queries; wave-uniform so that
    // the per-cloud records and the node boxes are scalar loads
    const int bid = xcd_block(blockIdx.x, gridDim.x);  // neighbouring blocks (tree order) share an XCD's L2
    // queries: tree slots 0 .. npts-1, or (list mode, the queries k_lrf8 hands over) the
    // slots qlist[0 .. *qcount-1], the grid striding over them
    const int nvq = qlist ? *qcount : v.npts;
    auto qslot = [&](int i) __attribute__((always_inline)) { return qlist ? qlist[i] : i; };
    // (list mode: qpw <= kQ queries per wave, the slots j >= qpw of a wave left empty, so
    // that the few handed-over queries spread over more waves)
    for (int vb = bid; vb * kWaves * qpw < nvq; vb += (int)gridDim.x) {
    const int w0 = __builtin_amdgcn_readfirstlane((vb * kWaves + wid) * qpw);
    const TreeRef T = v.t3;
    double* bd = s_d[wid];
    int* bi = s_i[wid];
    const double* TX = T.tvec64;  // tree-ordered f64 coordinates: one coalesced load per leaf
    const double* TY = T.tvec64 + v.ld;
    const double* TZ = T.tvec64 + 2 * (size_t)v.ld;
    const int first_leaf = (1 << T.L) - 1;
    double* park = &s_park[wid][0][0];
    const int ks = min(v.kmax, kSmallK);  // list stride: k_knn_big.hip takes Kw > kSmallK
    int* s_nbw = s_dyn + (size_t)wid * kQ * ks;
    if (lane < kQ) park[lane * PK_N + PK_FLAGS] = 0.0;
    // previous query of the wave (same cloud): its k-th distance bounds the next one's
    int prev_c = -1, prev_K = 0;
    double prev_kth = 0.0, pqx = 0.0, pqy = 0.0, pqz = 0.0;
    unsigned n_queries = 0, n_leaves = 0, n_sel = 0, n_box = 0, n_cand = 0;
#define LRF_COUNT(x) x
#ifdef SE3ICP_PROF
    unsigned long long c_knn = 0, c_sort = 0, c_sum = 0, c_fin = 0;
#endif

    for (int j = 0; j < kQ; ++j) {
        if ((j >= qpw) | (w0 + j >= nvq)) break;
        const int w = qslot(w0 + j);
        const int c = cloud_of[w];
        const CloudSetup st = setup[c];
        const int K = st.k_knn;
        if (K == 0) continue;
        const CloudDev cl = clouds[c];
        const int n = cl.n;
        const int gp = cl.off + T.perm[w];
        const double qx = TX[w], qy = TY[w], qz = TZ[w];
        const float fx = T.tvec[w], fy = T.tvec[v.ld + w], fz = T.tvec[2 * (size_t)v.ld + w];
        const float* box_lo = tlo + (size_t)c * T.nnodes * 3;
        const float* box_hi = thi + (size_t)c * T.nnodes * 3;
        const int Kw = min(K, n);
        if (Kw > kSmallK) continue;  // (k_knn_big.hip)
        const int own = first_leaf + tree_node_of(w - cl.off, n, T.L);
        ++n_queries;
        PROF_NOW(t_q0);

        // ------------------------------------------------------------ kNN
        // Candidates accepted by the current bound are appended, unsorted, to the wave's
        // buffer.  Once Kw candidates exist (and whenever the buffer is full) the bound is
        // tightened to the Kw-th smallest f32-rounded-up distance, found by bisection
        // over the f32 bit patterns with ballot counts, and the buffer is compacted; the
        // survivors are sorted exactly, once, at the end.  The bound always stays >= the
        // true Kw-th distance, so no member of the exact top-Kw is dropped.  The previous
        // query's k-th distance plus the distance between the two queries (triangle
        // inequality) is such a bound from the start.
        int nb = 0;
        bool have_thr = false;
        double thr = DBL_MAX;
        float thr_f = INFINITY;  // f32 bound >= thr * (1 + 2e-6): box pruning in f32 (never prunes more)
        auto set_thr_f = [&]() __attribute__((always_inline)) {
            thr_f = __uint_as_float(f32_up_bits(thr * (1.0 + 2e-6)));
        };
        int thr_i = INT_MAX;  // < INT_MAX only after an exact truncation (ties resolved by index)
        bool tight = false;   // a bound from this query's own candidates exists
        if (prev_c == c && prev_K == K) {
            const double dx = qx - pqx, dy = qy - pqy, dz = qz - pqz;
            const double r = sqrt(prev_kth) + sqrt(dx * dx + dy * dy + dz * dz);
            thr = r * r * (1.0 + 1e-12);
            have_thr = true;
            set_thr_f();
        }
        auto select_thr = [&]() __attribute__((always_inline)) {
            __builtin_amdgcn_wave_barrier();
            LRF_COUNT(++n_sel);
            double dk[4];
            int ik[4];
            unsigned u[4];
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int e = s * 64 + lane;
                dk[s] = e < nb ? bd[e] : DBL_MAX;
                ik[s] = e < nb ? bi[e] : INT_MAX;
                u[s] = e < nb ? f32_up_bits(dk[s]) : 0xffffffffu;
            }
            unsigned lo = 0, hi = 0x7f800000u;  // count(u <= hi) = nb >= Kw
            while (lo < hi) {
                const unsigned mid = lo + ((hi - lo) >> 1);
                int cnt = 0;
#pragma unroll
                for (int s = 0; s < 4; ++s) cnt += __popcll(__ballot(u[s] <= mid));
                if (cnt >= Kw) hi = mid; else lo = mid + 1;
            }
            const double t = (double)__uint_as_float(lo);
            if (t < thr) { thr = t; thr_i = INT_MAX; set_thr_f(); }
            __builtin_amdgcn_wave_barrier();
            int base = 0;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                // (d, point index) <= (thr, thr_i); the buffer holds tree slots, so the point
                // index is looked up only after an exact truncation (thr_i set, rare)
                bool keep = dk[s] < thr;
                if (thr_i != INT_MAX) {
                    const int li = (s * 64 + lane < nb) ? T.perm[ik[s]] : INT_MAX;
                    keep |= (bool)((int)(dk[s] == thr) & (int)(li <= thr_i));
                } else {
                    keep |= dk[s] == thr;
                }
                const unsigned long long m = __ballot(keep);
                if (keep) {
                    const int at = base + __popcll(m & ((1ull << lane) - 1ull));
                    bd[at] = dk[s];
                    bi[at] = ik[s];
                }
                base += __popcll(m);
            }
            nb = base;
            have_thr = true;
            tight = true;
            if (nb > kBuf - kLeafMax) {  // massive ties at the bound: exact sort and truncation
                __builtin_amdgcn_wave_barrier();
                for (int e = lane; e < nb; e += 64) bi[e] = T.perm[bi[e]];  // slots -> point indices
                __builtin_amdgcn_wave_barrier();
                wave_bitonic<4>(bd, bi, lane, nb);
                __builtin_amdgcn_wave_barrier();
                nb = Kw;
                thr = bd[Kw - 1];
                thr_i = bi[Kw - 1];
                for (int e = lane; e < nb; e += 64) bi[e] = cl.off + T.pos[cl.off + bi[e]];  // and back
                set_thr_f();
            }
            __builtin_amdgcn_wave_barrier();
        };
        auto leaf = [&](int h) __attribute__((always_inline)) {
            // (wave-uniform: readfirstlane keeps the leaf range arithmetic on the scalar unit)
            const int i = __builtin_amdgcn_readfirstlane(h - first_leaf);
            LRF_COUNT(++n_leaves);
            const int a = __builtin_amdgcn_readfirstlane(tree_first(n, T.L, i));
            const int b = __builtin_amdgcn_readfirstlane(tree_first(n, T.L, i + 1));
            bool acc = false;
            double d = DBL_MAX;
            const int slot = cl.off + a + lane;
            if (lane < b - a) {
                d = l2_3(qx, qy, qz, TX[slot], TY[slot], TZ[slot]);
                // (d, point index) <= (thr, thr_i): the index matters only at d == thr after an
                // exact truncation (rare), so the candidate is kept as its tree slot
                bool eq = d == thr;
                if (thr_i != INT_MAX) eq = (bool)((int)eq & (int)(T.perm[slot] <= thr_i));
                acc = (bool)((int)!have_thr | (int)(d < thr) | (int)eq);
            }
            const unsigned long long m = __ballot(acc);
            if (acc) {
                const int at = nb + __popcll(m & ((1ull << lane) - 1ull));
                bd[at] = d;
                bi[at] = slot;
            }
            nb += __popcll(m);
            // the first bound from Kw candidates (a seeded bound is loose), then whenever the buffer fills
            if ((!tight && nb >= Kw && !have_thr) || nb > kBuf - kLeafMax) select_thr();
        };
        auto open = [&](float lb) __attribute__((always_inline)) {  // may a box at lb hold a candidate?
            return !have_thr || lb <= thr_f;
        };

        // Own leaf first.  Without a bound yet (first query of the wave or of a cloud) the
        // leaves next to it in tree order follow until Kw candidates give one.  Then the
        // boxes are tested lane-parallel, 64 nodes per VALU instruction: all nodes of the
        // level A = L - 6 (<= 64 leaves below each), and the leaves of each level-A node
        // that can still hold a point within the bound; open leaves are scanned in order,
        // re-tested against the bound as it tightens.  Every leaf whose box lies within
        // the bound is scanned, so no member of the exact top-Kw is missed.
        leaf(own);
        const int nleaf = 1 << T.L;
        const int own_i = own - first_leaf;
        int s_lo = own_i, s_hi = own_i;  // leaves scanned so far: [s_lo, s_hi]
        while (!have_thr && (s_lo > 0 || s_hi < nleaf - 1)) {
            if (s_hi < nleaf - 1) leaf(first_leaf + (++s_hi));
            if (!have_thr && s_lo > 0) leaf(first_leaf + (--s_lo));
        }
        {
            const int sh = T.L > 6 ? 6 : T.L;  // leaves per level-A node: 2^sh <= 64
            const int A = T.L - sh;
            const int nA = 1 << A, firstA = nA - 1;
            for (int c0 = 0; c0 < nA; c0 += 64) {
                const int ai = c0 + lane;
                float lbA = INFINITY;
                if (ai < nA) lbA = box_lb3(box_lo + 3 * (firstA + ai), box_hi + 3 * (firstA + ai), fx, fy, fz);
                LRF_COUNT(++n_box);
                OutwardBits itA(__ballot((int)(ai < nA) & (int)open(lbA)), (own_i >> sh) - c0);
                for (int j; (j = itA.next()) >= 0;) {
                    if (!open(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(lbA), j)))) continue;
                    const int l0 = (c0 + j) << sh;  // first leaf of the level-A node
                    const int li = l0 + lane;
                    float lbL = INFINITY;
                    if ((int)(lane < (1 << sh)) & ((int)(li < s_lo) | (int)(li > s_hi)))
                        lbL = box_lb3(box_lo + 3 * (first_leaf + li), box_hi + 3 * (first_leaf + li), fx, fy, fz);
                    LRF_COUNT(++n_box);
                    OutwardBits itL(__ballot(open(lbL)), own_i - l0);
                    for (int t; (t = itL.next()) >= 0;) {
                        if (!open(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(lbL), t)))) continue;
                        leaf(first_leaf + l0 + t);
                    }
                }
            }
        }
        // exact order of the survivors
        PROF_NOW(t_q1);
        PROF_ADD(c_knn, t_q0, t_q1);
        LRF_COUNT(n_cand += nb);
        if (nb > 128) select_thr();
        __builtin_amdgcn_wave_barrier();
        {
            const int lim = min(nb, Kw + 1);  // ranks whose order matters (top-Kw and its boundary)
            const bool done = nb <= 128 ? wave_sort_u64<2>(bd, bi, lane, nb, lim) : wave_sort_u64<4>(bd, bi, lane, nb, lim);
            __builtin_amdgcn_wave_barrier();
            if (!done) {  // exact (f64 d, point index) order; the lists keep tree slots
                for (int e = lane; e < nb; e += 64) bi[e] = T.perm[bi[e]];
                __builtin_amdgcn_wave_barrier();
                if (nb <= 128) wave_bitonic<2>(bd, bi, lane, nb);
                else wave_bitonic<4>(bd, bi, lane, nb);
                __builtin_amdgcn_wave_barrier();
                for (int e = lane; e < nb; e += 64) bi[e] = cl.off + T.pos[cl.off + bi[e]];
            }
        }
        __builtin_amdgcn_wave_barrier();
        const int nTop = min(Kw, nb);
        if (nTop == Kw) {
            prev_c = c;
            prev_K = K;
            prev_kth = bd[Kw - 1];
            pqx = qx; pqy = qy; pqz = qz;
        } else {
            prev_c = -1;
        }
        // the sorted list stays in LDS (the epilogue below reads it); nothing is stored to
        // global memory inside this loop, which lets the compiler keep the per-cloud
        // records and node boxes on the scalar path
        {
            int* nbl = (s_nbw + j * ks);
            for (int r = lane; r < nTop; r += 64) nbl[r] = bi[r];
        }
        if (lane == 0) {
            double* pj = park + j * PK_N;
            pj[PK_GP] = (double)gp;
            pj[PK_K] = (double)K;
            pj[PK_NTOP] = (double)nTop;
            pj[PK_FLAGS] = (double)((st.k_lrf > 0 ? 1 : 0) | (st.k_nrm > 0 ? 2 : 0) | (write_knn ? 4 : 0));
        }
        __builtin_amdgcn_wave_barrier();
        PROF_NOW(t_q2);
        PROF_ADD(c_sort, t_q1, t_q2);
    }
    PROF_NOW(t_s0);

    // ---------------------------------------------------------------- per-query sums
    // (a separate pass over the parked neighbour lists keeps the kNN loop's live state small)
    // Eight lanes per query, the wave's kQ = 8 queries at once: lane qs of group qj takes the
    // neighbour ranks = qs (mod 8), and the group's partial sums are combined by a three-stage
    // butterfly (DPP / swizzle exchanges).  21 values per query:
    //   [0..2]  S' = sum of v over ranks 1 .. rz-1   (v = p - q, local coordinates)
    //   [3..5]  S  = sum of v over ranks 1 .. rz
    //   [6..11] M  = sum of v v^T over ranks 1 .. rz (xx xy xz yy yz zz)
    //   [12..20] Open3D cumulants of the raw coordinates over ranks 0 .. kn-1
    // The TOLDI covariance about the quirk centroid (ISR.cpp:259-272) is assembled from
    // S', S, M in the eigen pass; the reference sums the products sequentially, so
    // both differ from it by rounding only.
    static_assert(kQ * 8 == 64, "eight lanes per query");
    const int qj = lane >> 3, qs = lane & 7;
    {
        double* pj = park + qj * PK_N;
        const int flags = (int)pj[PK_FLAGS];
        double x[kSums];
#pragma unroll
        for (int i = 0; i < kSums; ++i) x[i] = 0.0;
        if (flags & 3) {
            const int w = qslot(w0 + qj);
            const int c = cloud_of[w];
            const double* X = TX;  // the lists hold tree slots: tree-ordered coordinates
            const double* Y = TY;
            const double* Z = TZ;
            const double qx = TX[w], qy = TY[w], qz = TZ[w];
            const int nTop = (int)pj[PK_NTOP];
            const int* nbl = s_nbw + qj * ks;
            if (flags & 1) {
                const int kk = min(setup[c].k_lrf, nTop);
                const int rz = kk / 3;
                const int hi = min(rz, kk - 1);
                for (int rk = 1 + qs; rk <= hi; rk += 8) {
                    const int q = nbl[rk];
                    const double vx = X[q] - qx, vy = Y[q] - qy, vz = Z[q] - qz;
                    if (rk < rz) { x[0] += vx; x[1] += vy; x[2] += vz; }
                    x[3] += vx; x[4] += vy; x[5] += vz;
                    x[6] += vx * vx; x[7] += vx * vy; x[8] += vx * vz;
                    x[9] += vy * vy; x[10] += vy * vz; x[11] += vz * vz;
                }
                if (qs == 0) {
                    const int far = nbl[kk - 1];
                    const double fdx = qx - X[far], fdy = qy - Y[far], fdz = qz - Z[far];
                    pj[PK_R] = sqrt(fdx * fdx + fdy * fdy + fdz * fdz);  // ISR.cpp:256
                    pj[PK_KK] = (double)kk;
                }
            }
            if (flags & 2) {  // EstimateNormals (ISR.cpp:643, :43): ranks 0 .. kn-1, self included
                const int kn = min(setup[c].k_nrm, nTop);
                for (int r = qs; r < kn; r += 8) {
                    const int q = nbl[r];
                    const double px = X[q], py = Y[q], pz = Z[q];
                    x[12] += px; x[13] += py; x[14] += pz;
                    x[15] += px * px; x[16] += px * py; x[17] += px * pz;
                    x[18] += py * py; x[19] += py * pz; x[20] += pz * pz;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < kSums; ++i) {
            x[i] += xor_lane(x[i], 1);
            x[i] += xor_lane(x[i], 2);
            x[i] += xor_lane(x[i], 4);
        }
        __builtin_amdgcn_wave_barrier();
        if ((int)(qs == 0) & (int)((flags & 3) != 0)) {
#pragma unroll
            for (int i = 0; i < kSums; ++i) pj[PK_SUM + i] = x[i];
        }
        __builtin_amdgcn_wave_barrier();
    }
    PROF_NOW(t_s1);
    PROF_ADD(c_sum, t_s0, t_s1);
    unsigned long long* ctr = v.stats + kStatCols * ((w0 / kQ) & 63);
    if (lane == 0) {  // work counters (bench diagnostics)
        atomicAdd(ctr + 0, (unsigned long long)n_queries);
        atomicAdd(ctr + 1, (unsigned long long)n_leaves);
        atomicAdd(ctr + 2, (unsigned long long)n_sel);
        atomicAdd(ctr + 3, (unsigned long long)n_box);
        atomicAdd(ctr + 4, (unsigned long long)n_cand);
    }

    // ---------------------------------------------------------------- batched eigen-solves
    // The 3x3 problems of the block's kWaves * kQ = 32 queries, lane wq * kQ + j for query
    // j of wave wq: wave 0 the TOLDI ones, wave 1 the normals at the same time (one solve
    // per 32 queries instead of one per kQ queries on each wave).
    __builtin_amdgcn_wave_barrier();
    if (write_knn) {  // se3icp_knn_self: the sorted lists
        for (int j = 0; j < kQ; ++j) {
            const double* pj = park + j * PK_N;
            if (!((int)pj[PK_FLAGS] & 4)) continue;
            const int K = (int)pj[PK_K], nTop = (int)pj[PK_NTOP];
            int* out = v.knn + (size_t)(int)pj[PK_GP] * v.kmax;
            for (int r = lane; r < K; r += 64) out[r] = r < nTop ? T.perm[s_nbw[j * ks + r]] : -1;
        }
    }
    __syncthreads();
    if (wid <= 1) {  // wave 0: the TOLDI problems, wave 1 the normals, side by side
        static_assert(kWaves * kQ <= 64, "one lane per query of the block");
        double* pb = &s_park[lane < kWaves * kQ ? lane / kQ : 0][lane % kQ][0];
        const int b_flags = lane < kWaves * kQ ? (int)pb[PK_FLAGS] : 0;
        const int wb = b_flags ? qslot((vb * kWaves + lane / kQ) * qpw + lane % kQ) : 0;  // the query's tree slot
        d3 zn{0, 0, 0};
        if ((b_flags & 1) && wid == 0) {
            // C = sum over ranks 1..rz of (v - cl)(v - cl)^T with the quirk centroid
            // cl = c - q = (S' - q) / rz  (c = (ranks 1..rz-1 summed) / rz, ISR.cpp:259-265)
            const double rz = (double)((int)pb[PK_KK] / 3);
            const double q3[3] = {TX[wb], TY[wb], TZ[wb]};
            double cl[3], S[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                cl[a] = (pb[PK_SUM + a] - q3[a]) / rz;
                S[a] = pb[PK_SUM + 3 + a];
            }
            const double* M = pb + PK_SUM + 6;
            const int ia[6] = {0, 0, 0, 1, 1, 2}, ib[6] = {0, 1, 2, 1, 2, 2};
            double c6[6];
#pragma unroll
            for (int k = 0; k < 6; ++k)
                c6[k] = M[k] - S[ia[k]] * cl[ib[k]] - cl[ia[k]] * S[ib[k]] + rz * cl[ia[k]] * cl[ib[k]];
            zn = jacobi_smallest_evec(c6[0], c6[1], c6[2], c6[3], c6[4], c6[5]);
        }
        if ((b_flags & 2) && wid == 1) {
            const int c = v.cloud_of[wb];
            const int kn = min(v.setup[c].k_nrm, (int)pb[PK_NTOP]);
            double n6[6] = {1, 0, 0, 1, 0, 1};
            if (kn >= 3) {
                double cu[9];
#pragma unroll
                for (int i = 0; i < 9; ++i) cu[i] = pb[PK_SUM + 12 + i] / (double)kn;
                n6[0] = cu[3] - cu[0] * cu[0];
                n6[1] = cu[4] - cu[0] * cu[1];
                n6[2] = cu[5] - cu[0] * cu[2];
                n6[3] = cu[6] - cu[1] * cu[1];
                n6[4] = cu[7] - cu[1] * cu[2];
                n6[5] = cu[8] - cu[2] * cu[2];
            }
            d3 nm = fast_eigen3x3(n6[0], n6[1], n6[2], n6[3], n6[4], n6[5]);
            if (sqrt(dot3(nm, nm)) == 0.0) nm = d3{0, 0, 1};
            const int gp = (int)pb[PK_GP];
            v.nrm64[gp] = nm.x;
            v.nrm64[v.ld + gp] = nm.y;
            v.nrm64[2 * (size_t)v.ld + gp] = nm.z;
        }
        if ((b_flags & 1) && wid == 0) {
            pb[PK_ZN] = zn.x;
            pb[PK_ZN + 1] = zn.y;
            pb[PK_ZN + 2] = zn.z;
        }
    }
    __syncthreads();

    // ---------------------------------------------------------------- TOLDI axes (ISR.cpp:286-306)
    __builtin_amdgcn_wave_barrier();  // (the eigen pass has read PK_SUM; the axis sums reuse it)
    {  // eight lanes per query again (see the sums pass)
        double* pj = park + qj * PK_N;
        const int flags = (int)pj[PK_FLAGS];
        const double nx = pj[PK_ZN], ny = pj[PK_ZN + 1], nz = pj[PK_ZN + 2];
        double x6[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        if (flags & 1) {
            const int w = qslot(w0 + qj);
            const double* X = TX;  // (tree slots, see the sums pass)
            const double* Y = TY;
            const double* Z = TZ;
            const double qx = TX[w], qy = TY[w], qz = TZ[w];
            const double R = pj[PK_R];
            const int kk = (int)pj[PK_KK];
            const int* nbl = s_nbw + qj * ks;
            for (int r = 1 + qs; r < kk; r += 8) {
                const int q = nbl[r];
                const double vx = X[q] - qx, vy = Y[q] - qy, vz = Z[q] - qz;
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
        __builtin_amdgcn_wave_barrier();
        if ((int)(qs == 0) & (int)((flags & 1) != 0)) {
#pragma unroll
            for (int i = 0; i < 6; ++i) pj[PK_SUM + i] = x6[i];
        }
    }
    // the frames, again on wave 0 for the block's 32 queries
    __syncthreads();
    if (wid == 0) {
        const double* pb = &s_park[lane < kWaves * kQ ? lane / kQ : 0][lane % kQ][0];
        const int b_flags = lane < kWaves * kQ ? (int)pb[PK_FLAGS] : 0;
        if (b_flags & 1) {
            const int w = qslot((vb * kWaves + lane / kQ) * qpw + lane % kQ);
            const CloudSetup st = v.setup[v.cloud_of[w]];
            const double qx = TX[w], qy = TY[w], qz = TZ[w];
            d3 nrm{pb[PK_ZN], pb[PK_ZN + 1], pb[PK_ZN + 2]};
            if (nrm.x * pb[PK_SUM] + nrm.y * pb[PK_SUM + 1] + nrm.z * pb[PK_SUM + 2] < 0.0)
                nrm = d3{-nrm.x, -nrm.y, -nrm.z};  // ISR.cpp:298
            const d3 zax = nrm;
            const d3 accs{pb[PK_SUM + 3], pb[PK_SUM + 4], pb[PK_SUM + 5]};
            d3 xax = accs - dot3(accs, zax) * zax;  // ISR.cpp:302-303 (no |x| = 0 guard, as the reference)
            xax = (1.0 / sqrt(dot3(xax, xax))) * xax;
            const d3 yax = cross3(zax, xax);  // ISR.cpp:306
            const double al = st.alpha, be = st.beta;
            const double f12[12] = {al * xax.x, al * xax.y, al * xax.z, al * yax.x, al * yax.y, al * yax.z,
                                    al * zax.x, al * zax.y, al * zax.z, be * qx, be * qy, be * qz};
            // (f32 copy: 12-D search vectors of targets and the kd-tree grouping of sources)
            store_frame_rows(v.fr64, v.fr32, (int)pb[PK_GP], f12, st.cf_target, qx, qy, qz);
        }
    }
#ifdef SE3ICP_PROF
    PROF_NOW(t_f1);
    PROF_ADD(c_fin, t_s1, t_f1);
    if (lane == 0) {
        atomicAdd(ctr + 8, c_knn);
        atomicAdd(ctr + 9, c_sort);
        atomicAdd(ctr + 10, c_sum);
        atomicAdd(ctr + 11, c_fin);
    }
#endif
    if (!qlist) break;  // (one round per block over the whole point range)
    __syncthreads();    // (the next round reuses the LDS lists and park)
    }
}

}  // namespace

void launch_lrf(const View& v, int write_knn, hipStream_t s) {
    const int nw = (v.npts + kQ - 1) / kQ;
    const size_t lds = sizeof(int) * (size_t)kWaves * kQ * std::min(v.kmax, kSmallK);
    hipLaunchKernelGGL(k_lrf, dim3((nw + kWaves - 1) / kWaves), dim3(64 * kWaves), lds, s, v, write_knn, v.cloud_of,
                       v.setup, v.clouds, v.t3.lo, v.t3.hi, nullptr, nullptr, kQ);
}

// The hand-over pass: queries per wave and its grid (strided).  1,280 4-wave blocks are one
// resident round at 5 waves per SIMD; two queries per wave then cover C4's ~9.9k hand-overs
// in that round (same-box A/B at C4, k_lrf8 + k_lrf: 4.01 ms at 4 per wave / 1,024 blocks,
// 3.92 at 2 / 1,280, 3.95 at 3 / 1,024, 4.02 at 2 / 2,048; round 3: 1 and 8 per wave slower)
constexpr int kListQpw = 2;
constexpr int kListBlocks = 1280;
void launch_lrf_list(const View& v, const int32_t* qlist, const int32_t* qcount, hipStream_t s, int qpw) {
    const size_t lds = sizeof(int) * (size_t)kWaves * kQ * std::min(v.kmax, kSmallK);
    const int nblk = std::max(1, std::min(kListBlocks, (v.npts + kWaves * kQ - 1) / (kWaves * kQ)));
    hipLaunchKernelGGL(k_lrf, dim3(nblk), dim3(64 * kWaves), lds, s, v, 0, v.cloud_of, v.setup, v.clouds, v.t3.lo,
                       v.t3.hi, qlist, qcount, qpw > 0 ? std::min(qpw, kQ) : kListQpw);
}

}  // namespace se3icp
