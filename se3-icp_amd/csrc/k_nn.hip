// k_nn.hip — the correspondence search of one ICP iteration, batched over every active pair.
//
//   SE(3) phase: exact 1-NN of each source SE(3) element under the weighted SE(3) metric
//                (12-D L2), update_correspondences_raw_flann_SE3 ISR.cpp:444-470;
//   R3 phase:    exact 3-D 1-NN, update_correspondences_kd_tree_XYZ ISR.cpp:402-416.
//
// Certificates (k_nn_prep).  A search leaves each query a certificate: the exact distance
// to its match is <= D1 and to every other target >= L2.  The query moves with the pose
// only (q = T M0), so at a later iteration of the same phase, with delta = |q_now - q_then|
// computed in f64 from the two poses, D1 + delta < L2 - delta proves the match unchanged
// (triangle inequality) and the query is settled without a search.  As ICP converges the
// per-iteration displacement shrinks geometrically and most queries settle this way.
// To make certificates useful the search widens its radius to the smaller of
// (sqrt(d1) + 2m)^2 and the second-best distance d2, m = the query's displacement in
// this iteration (so the extra work is at most that of an exact 2-NN search).
//
// Search (k_nn_search, group part).  The queries k_nn_prep could not settle are compacted per chunk
// (<= 1024 consecutive source tree positions, i.e. close together in the search space;
// the pose acts on the vectors as an isometry, so they stay close as the source moves)
// and swept 64 per wavefront.  The wave walks the TARGET kd-tree depth first; a node is
// entered when some lane's f32 box bound is below that lane's pruning threshold, and a
// leaf's <= 64 targets are staged through LDS and swept with broadcast ds_read_b128 (or
// by compacted lane groups) while each lane keeps (d1, i1, d2).  The previous
// iteration's match seeds the threshold.  The f32 arg-min is then certified
// (k_loop.hip recheck handles the rest):
//   thr >= d1 + 3 err(d1)  => every unvisited target is > 2 err farther than the winner,
//   and among the visited ones the gap d2 - d1 must exceed 2 err(d2).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>

#include "loopdev.hpp"
#include "wave.hpp"
#include "tree.hpp"

namespace se3icp {

namespace {

using namespace loopdev;

// Tuned constants (A/B on the bench's C4 batch; the rejected alternatives are listed in
// DESIGN.md's measurement log):
//   k_nn_search blocks are ONE wave: a block's LDS is released when its last wave ends, so
//   4-wave blocks whose waves ended at different times stranded LDS (a CU held at most five
//   28.7 KB blocks): SE(3) NN -9 %.
constexpr int kTPL = 4;        // targets per lane in the compacted leaf sweeps (kept in registers across queries)
#ifndef SE3ICP_NN_COMPACT
#define SE3ICP_NN_COMPACT 40
#endif
constexpr int kCompact = SE3ICP_NN_COMPACT;  // a leaf wanted by at most this many lanes takes the compacted sweep (12-D and 3-D)
#ifndef SE3ICP_NN_KEYMERGE
#define SE3ICP_NN_KEYMERGE 1
#endif
#ifndef SE3ICP_SEED_TARGETS
#define SE3ICP_SEED_TARGETS 1
#endif
constexpr int kSeedTargets = SE3ICP_SEED_TARGETS;  // first searches: seeded by a greedy tree descent and this many leaf targets

// packed f32 pairs: v_pk_add_f32 / v_pk_fma_f32 issue two lanes' worth of f32 math per
// instruction (the f32 vector peak of gfx950 assumes them)
typedef float f32x2 __attribute__((ext_vector_type(2)));

template <int D>
__device__ __forceinline__ float box_lb(const float* lo, const float* hi, const float* q) {
    float s = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        const float e = fmaxf(fmaxf(lo[d] - q[d], q[d] - hi[d]), 0.f);
        s = fmaf(e, e, s);
    }
    return s;
}

// 12-D: dimensions in pairs on the packed f32 path (v_pk_add_f32 with the box corners
// read as scalar pairs), max(lo - q, q - hi, 0) per dimension (v_max3_f32), v_pk_fma_f32
// chains: 5 instead of 7 VALU per two dimensions
__device__ __forceinline__ float box_lb12(const float* lo, const float* hi, const f32x2* q2) {
    f32x2 s2;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        const f32x2 a = f32x2{lo[2 * r], lo[2 * r + 1]} - q2[r];
        const f32x2 b = q2[r] - f32x2{hi[2 * r], hi[2 * r + 1]};
        const f32x2 e = f32x2{fmaxf(fmaxf(a.x, b.x), 0.f), fmaxf(fmaxf(a.y, b.y), 0.f)};
        s2 = (r == 0) ? e * e : __builtin_elementwise_fma(e, e, s2);
    }
    return s2.x + s2.y;
}

// box_lb12 for a wave-uniform box (the group walk's nodes): read through the constant
// address space, so the two 48-byte corners come in as scalar loads -- no vector-memory
// address processing for 64 identical addresses, and the scalar cache's latency
typedef const __attribute__((address_space(4))) float cfloat;
__device__ __forceinline__ float box_lb12_u(const float* lo_, const float* hi_, const f32x2* q2) {
    cfloat* lo = (cfloat*)lo_;
    cfloat* hi = (cfloat*)hi_;
    f32x2 s2;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        const f32x2 a = f32x2{lo[2 * r], lo[2 * r + 1]} - q2[r];
        const f32x2 b = q2[r] - f32x2{hi[2 * r], hi[2 * r + 1]};
        const f32x2 e = f32x2{fmaxf(fmaxf(a.x, b.x), 0.f), fmaxf(fmaxf(a.y, b.y), 0.f)};
        s2 = (r == 0) ? e * e : __builtin_elementwise_fma(e, e, s2);
    }
    return s2.x + s2.y;
}
template <int D>
__device__ __forceinline__ float box_lb_u(const float* lo_, const float* hi_, const float* q) {
    cfloat* lo = (cfloat*)lo_;
    cfloat* hi = (cfloat*)hi_;
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < D; ++r) {
        const float e = fmaxf(fmaxf(lo[r] - q[r], q[r] - hi[r]), 0.f);
        s = fmaf(e, e, s);
    }
    return s;
}

// min / max of values the compiler cannot prove canonical (DPP moves, LDS reads): fminf /
// fmaxf would quiet a possible signalling NaN first (a v_max_f32 x, x, x per operand); the
// distances here are finite or quiet NaNs, for which the raw instructions agree
__device__ __forceinline__ float fmin_raw(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float fmax_raw(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float fmin3_raw(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}

// f32 squared 12-D distance of a query (dimension pairs) to a staged target: two
// interleaved FMA chains (even / odd dimensions) and one add, within the D-term chain
// bound f32_err assumes
__device__ __forceinline__ float dist12(const f32x2* q2, const float4* t) {
    const float4 A = t[0], B = t[1], C = t[2];
    f32x2 e, s2;
    e = q2[0] - f32x2{A.x, A.y}; s2 = e * e;
    e = q2[1] - f32x2{A.z, A.w}; s2 = __builtin_elementwise_fma(e, e, s2);
    e = q2[2] - f32x2{B.x, B.y}; s2 = __builtin_elementwise_fma(e, e, s2);
    e = q2[3] - f32x2{B.z, B.w}; s2 = __builtin_elementwise_fma(e, e, s2);
    e = q2[4] - f32x2{C.x, C.y}; s2 = __builtin_elementwise_fma(e, e, s2);
    e = q2[5] - f32x2{C.z, C.w}; s2 = __builtin_elementwise_fma(e, e, s2);
    return s2.x + s2.y;
}

// One leaf against its w wanting queries (list wl): LPQ lanes per query, targets
// sub, sub+LPQ, sub+2LPQ, sub+3LPQ per lane (LPQ * 4 >= cnt), the group's top-2 into
// r1/r2/rb[query].  The lane's 4 targets are loop-invariant over the queries: the
// compiler keeps them in registers (4 waves/SIMD; measured faster than re-reading at 5).
template <int D, int LPQ, int TPL = kTPL>
__device__ __forceinline__ void compact_sweep(const float4* tile, const float4* sq, const int* wl, float* r1, float* r2,
                                              int* rb, int w, int cnt, int ta, int lane) {
    constexpr int NV = (D + 3) / 4;
    constexpr int QPI = 64 / LPQ;  // queries per pass
    const int sub = lane & (LPQ - 1);
    for (int it = 0; it < w; it += QPI) {
        const int slot = it + lane / LPQ;
        const int qi = wl[slot < w ? slot : it];
        f32x2 qq[6];
        float4 Q3;
        if constexpr (D == 12) {
            const float4 QA = sq[qi * 3], QB = sq[qi * 3 + 1], QC = sq[qi * 3 + 2];
            qq[0] = f32x2{QA.x, QA.y}; qq[1] = f32x2{QA.z, QA.w}; qq[2] = f32x2{QB.x, QB.y};
            qq[3] = f32x2{QB.z, QB.w}; qq[4] = f32x2{QC.x, QC.y}; qq[5] = f32x2{QC.z, QC.w};
        } else {
            Q3 = sq[qi];
        }
        float a1 = INFINITY, a2 = INFINITY;
        int b1 = 0;
#pragma unroll
        for (int u = 0; u < TPL; ++u) {
            const int j = sub + LPQ * u;
            float acc;
            if constexpr (D == 12) {
                acc = dist12(qq, tile + NV * (j < cnt ? j : 0));
            } else {  // the broadcast sweep's arithmetic (f32_err bound)
                const float4 A = tile[j < cnt ? j : 0];
                float e;
                e = Q3.x - A.x; acc = e * e;
                e = Q3.y - A.y; acc = fmaf(e, e, acc);
                e = Q3.z - A.z; acc = fmaf(e, e, acc);
            }
            acc = j < cnt ? acc : INFINITY;
            const bool lt = acc < a1;
            a2 = __builtin_amdgcn_fmed3f(a1, a2, acc);
            a1 = lt ? acc : a1;
            b1 = lt ? j : b1;
        }
#if SE3ICP_NN_KEYMERGE
        // the group's top-2: the best as one u64 key (f32 distance bits | target: the lowest
        // index among equal distances), then the second-best distance as a plain minimum of
        // every lane's best except the winner's, whose own second counts instead -- two
        // butterflies of 5 + 2 VALU per step instead of one of ~12
        {
            const unsigned long long mine = ((unsigned long long)__float_as_uint(a1) << 32) | (unsigned)b1;
            unsigned long long key = mine;
#pragma unroll
            for (int m = 1; m < LPQ; m <<= 1) {
                const unsigned long long pk = xor_lane(key, m);
                key = pk < key ? pk : key;
            }
            float c = key == mine ? a2 : a1;
#pragma unroll
            for (int m = 1; m < LPQ; m <<= 1) c = fmin_raw(c, xor_lane(c, m));
            a1 = __uint_as_float((unsigned)(key >> 32));
            b1 = (int)(unsigned)key;
            a2 = c;
        }
#else
#pragma unroll
        for (int m = 1; m < LPQ; m <<= 1) {
            const float p1 = xor_lane(a1, m), p2 = xor_lane(a2, m);
            const int pb = xor_lane(b1, m);
            const bool lt = (bool)((int)(p1 < a1) | ((int)(p1 == a1) & (int)(pb < b1)));
            a2 = fmin3_raw(fmax_raw(a1, p1), a2, p2);
            b1 = lt ? pb : b1;
            a1 = fmin_raw(a1, p1);
        }
#endif
        if ((int)(sub == 0) & (int)(slot < w)) {
            r1[qi] = a1;
            r2[qi] = a2;
            rb[qi] = ta + b1;
        }
    }
}

// A chunk with at least dense_min searched queries is searched 64 per wave, a sparser one
// one query per wave (k_nn_search's first kSingleWaves blocks).  A wave-per-query search costs
// far more wave time per query than a group's lane (C4 64 pairs, make prof: ~10 us against
// ~0.6 us in the 3-D search), but its latency is short, and with few groups a group wave's
// latency bounds the launch.  The single-query list is served by a fixed 4,096 waves, so the
// threshold scales down with the batch: dense_min = kDense * 1024 / nchunks in [kDenseMin,
// kDense] -- 256 for 8 KITTI pairs (1,024 chunks), 32 for 64.  Same-box A/B at a fixed
// threshold (iter/s): 64 pairs 256 / 128 / 64 / 32 = 13,500 / 13,870 / 14,060 / 14,080;
// 8 pairs 10,570 / 10,420 / 10,340 / 10,180.
#ifndef SE3ICP_NN_DENSE
#define SE3ICP_NN_DENSE 256
#endif
#ifndef SE3ICP_NN_DENSE_MIN
#define SE3ICP_NN_DENSE_MIN 32
#endif
constexpr int kDense = SE3ICP_NN_DENSE, kDenseMin = SE3ICP_NN_DENSE_MIN;
__device__ __forceinline__ int dense_min(int nchunks) {
    return max(kDenseMin, min(kDense, (int)(((long long)kDense * 1024) / max(nchunks, 1))));
}
constexpr int kWpe = 4;        // waves per SIMD of k_nn_search (its natural 128 VGPRs; 5 measured +8 %)
// the 3-D search at 6 waves per SIMD (79 VGPRs, no scratch): same-box A/B x2, C2 (72 R3
// iterations) 25,957 -> 26,257 iter/s, C4 within noise; 8 (64 VGPRs, 52 B of scratch) +0.8 %
constexpr int kWpe3 = 6;
constexpr int kXcdRun = 256;   // group blocks per XCD run (16 chunks; runs dealt round-robin over the XCDs:
                               // neighbouring chunks share target leaves in one L2, SE(3) NN -3 %)
__device__ __forceinline__ int group_xcd(int g, int nb) {
    const int whole = nb / (8 * kXcdRun) * (8 * kXcdRun);
    return g < whole ? (g / kXcdRun) & 7 : g & 7;
}
#ifndef SE3ICP_KSMALL
#define SE3ICP_KSMALL 4
#endif
constexpr int kSmall = SE3ICP_KSMALL;  // groups of at most this many queries are searched one query at a time
// one-query-per-wave blocks at the front of the search grid (grid-strided; 4,096 measured
// faster than 16,384 at C4: fewer empty waves to dispatch in iterations without sparse chunks)
constexpr int kSingleWaves = 4096;
#ifndef SE3ICP_SINGLE_BATCH
#define SE3ICP_SINGLE_BATCH 16
#endif
constexpr int kSingleBatch = SE3ICP_SINGLE_BATCH;  // single-list entries set up together (1: one at a time)
static_assert(kSingleBatch >= 1 && kSingleBatch <= 64, "one lane per entry");
static_assert(kSingleWaves % 8 == 0, "single_list deals the list to the 8 XCDs in whole eighths of its waves");
#ifndef SE3ICP_NN_THB
#define SE3ICP_NN_THB 1
#endif
constexpr float kBoxScale = SE3ICP_NN_THB ? 1.0000025f : 1.0f;  // (group search box tests, see thb)
constexpr float kBoxMul = SE3ICP_NN_THB ? 1.0f : (1.f - 2e-6f);
#ifndef SE3ICP_EXPAND
#define SE3ICP_EXPAND 1.0
#endif
constexpr double kExpand = SE3ICP_EXPAND;  // search widening, in units of the query's displacement this iteration
// First iteration of the SE(3) phase whose searches are widened for certificates (a run's
// first search has no displacement yet and is a plain 1-NN search either way).  A widened
// search costs more now and settles more queries in the next iterations: a large batch
// (throughput-bound) gains from widening early, a small one (latency-bound: its longest
// waves set the launches) loses.  Same-box A/B of the start iteration 4 / 3 / 2 (iter/s):
// C4 KITTI 8 pairs 10,580 / 10,440 / 10,310, 16 pairs 11,700 / 11,820 / 11,770, 32 pairs
// 13,270 / 13,500 / 13,490, 64 pairs 14,100 / 14,360 / 14,340; C3 (32 RGB-D pairs) 41,910 /
// 42,870 / 41,310; C5 (256 RGB-D pairs) 55,220 / 57,330 / 58,350; C2 (8 bunny cases) 26,460 /
// 26,240 / 26,030 -- the batch's pair count orders them (its chunk count does not: C3 and 8
// KITTI pairs both have 1,024 chunks).  SE3ICP_WIDEN_FROM > 0 fixes it.
#ifndef SE3ICP_WIDEN_FROM
#define SE3ICP_WIDEN_FROM 0
#endif
__device__ __forceinline__ int widen_from(int npairs) {
    if (SE3ICP_WIDEN_FROM > 0) return SE3ICP_WIDEN_FROM;
    return npairs >= 128 ? 2 : (npairs > 8 ? 3 : 4);
}

// Cost-ordered dispatch of the SE(3) group waves: k_nn_prep files each group under its XCD
// (the block -> XCD map of the run-dealt order) and a cost class (its wave's duration in the
// previous search, half-octaves, longest first, unknown first); a group block then takes the
// i-th item of its XCD's lists in class order, so the long waves start first and the
// launch's tail is short waves (C2, two group waves per slot: SE(3) NN 8.4 -> 7.6 ms per
// step; C4 within noise).  The R3 searches of small batches keep the run order (ordered,
// 8 KITTI pairs' R3 NN was 10 % slower: their short waves gain less than the L2 locality of
// the run order); from 64 pairs they are ordered too (order3 below).
constexpr int kClsHead = 2 * 8 * 16;  // counts [phase][XCD][class]
// The 3-D group waves take the same cost-ordered dispatch in batches of at least
// SE3ICP_NN_ORDER3 pairs (0: never): same-box A/B, ordered against the run order: C4 64
// pairs +0.5 %, C5 (256 pairs) +1.0 %, C4 8 pairs -2.3 %, C2 -6 % (a small batch's short R3
// waves gain less than the run order's L2 locality).
#ifndef SE3ICP_NN_ORDER3
#define SE3ICP_NN_ORDER3 64
#endif
__host__ __device__ inline bool order3(int npairs) { return (SE3ICP_NN_ORDER3 > 0) & (npairs >= SE3ICP_NN_ORDER3); }
__host__ __device__ inline int cls_cap(int nchunks) { return nchunks * 16 / 8 + 1; }
__device__ __forceinline__ int cost_class(unsigned t) {
    if (t == 0u) return 0;
    const int b = 31 - __clz((int)t);
    const int b2 = 2 * b + (b >= 1 ? (int)((t >> (b - 1)) & 1u) : 0);
    return min(15, max(1, 33 - b2));
}

template <int D>
__device__ __forceinline__ double dist_f64(const double* a, const double* b) {
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < D; ++r) s += (a[r] - b[r]) * (a[r] - b[r]);
    return sqrt(s);
}
template <int D>
__device__ __forceinline__ double norm_f64(const double* a) {
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < D; ++r) s += a[r] * a[r];
    return sqrt(s);
}
__device__ __forceinline__ void load_hist(const View& v, int iter, int pair, double* T) {
    const double* h = v.hist + ((size_t)(iter % kHist) * v.npairs + pair) * 12;
#pragma unroll
    for (int i = 0; i < 12; ++i) T[i] = h[i];
}

// f64 source element / point at global tree slot gx (the tree-ordered f64 copy: queries of
// a chunk read contiguous memory)
template <int D>
__device__ __forceinline__ void load_m0(const View& v, const TreeRef& TR, int gx, int g, double* m) {
    if constexpr (D == 12) {  // the point's 96-B frame row (the 12-D tree keeps only the translation rows in tree order)
        const double2* r2 = reinterpret_cast<const double2*>(v.fr64 + (size_t)g * 12);
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const double2 x = r2[k];
            m[2 * k] = x.x;
            m[2 * k + 1] = x.y;
        }
    } else {
#pragma unroll
        for (int r = 0; r < D; ++r) m[r] = TR.tvec64[(size_t)r * v.ld + gx];
    }
}
template <int D>
__device__ __forceinline__ void pose_m0(const double* T, const double* m, double* q) {
    if constexpr (D == 12) pose_frame(T, m, q);
    else pose_point(T, m[0], m[1], m[2], q);
}

// Only the translation rows of a source element are loaded here.  Its rotation columns are
// alpha times an orthonormal TOLDI frame X, so for two poses T, T':
//   |T M0 - T' M0|^2 = alpha^2 |(R - R') X|_F^2 + |(R - R') m_t + t - t'|^2
//                    = alpha^2 |R - R'|_F^2     + |(R - R') m_t + t - t'|^2
// and |T M0|^2 = 3 alpha^2 + |R m_t + t|^2 (X orthonormal to f64 rounding; padded below).
// The 3-D phase is the translation part alone (alpha = 0).
__device__ __forceinline__ double rot_frob2(const double* A, const double* B) {
    double s = 0.0;
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) s += (A[r * 4 + c] - B[r * 4 + c]) * (A[r * 4 + c] - B[r * 4 + c]);
    return s;
}
__device__ __forceinline__ double dist3_f64(const double* a, const double* b) {
    return sqrt((a[0] - b[0]) * (a[0] - b[0]) + (a[1] - b[1]) * (a[1] - b[1]) + (a[2] - b[2]) * (a[2] - b[2]));
}

// Settle the query at source tree slot gx (point g) from its certificate (true: corr_idx
// stays, corr_dist refreshed for the moved query) or prepare its search (false: nn_margin).
template <int D>
__device__ __forceinline__ bool prep_settle(const View& v, const TreeRef& TR, const PairDev* P, int pair,
                                            const CloudDev& ct, int gx, int g, double a2) {
    double mt[3], T[12], Qt[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) mt[r] = TR.tvec64[(size_t)r * v.ld + gx];  // (3 rows: points / translations)
    load_T(P, T);
    pose_point(T, mt[0], mt[1], mt[2], Qt);
    const double rot2 = 3.0 * a2 * (1.0 + 1e-12);  // |rotation columns|^2 (12-D), 0 (3-D)
    const int it = P->iter;
    NNCert* cp = v.cert + gx;  // (the phase's tree slot: coalesced)
    const float4 c0 = reinterpret_cast<const float4*>(cp)[0];
    const int ci = __float_as_int(c0.z);
    const double qn = sqrt(rot2 + Qt[0] * Qt[0] + Qt[1] * Qt[1] + Qt[2] * Qt[2]);
    if ((int)(ci >= P->phase_start) & (int)(ci < it) & (int)(it - ci < kHist)) {
        double Tr[12], Qr[3];
        load_hist(v, ci, pair, Tr);
        pose_point(Tr, mt[0], mt[1], mt[2], Qr);
        const double qr = sqrt(rot2 + Qr[0] * Qr[0] + Qr[1] * Qr[1] + Qr[2] * Qr[2]);
        const double dt = dist3_f64(Qt, Qr);
        // |q_now - q_then|, padded for the frame's orthonormality and the rounding of the
        // two f64 queries the searches used
        const double dl = sqrt(a2 * rot_frob2(T, Tr) * (1.0 + 1e-12) + dt * dt) * (1.0 + 1e-12) + 2e-15 * (qn + qr);
        const double a = (double)c0.y - dl, b = (double)c0.x + dl;
        // margin for the f64 rounding of the reference's own squared distances (|q| + |target| <= M)
        const double M = 2.0 * qn + b;
        if ((int)(a > b) & (int)((a - b) * (a + b) > 1e-14 * M * M)) {
            // settled: corr_idx[g] (= the record's j) stays; the distance to its anchor
            const double t[3] = {cp->t[0], cp->t[1], cp->t[2]};
            v.corr_dist[g] = anchor_dist(Qt, t);
            return true;
        }
    }
    float m = 0.f;
    if ((int)(it >= 2) & ((int)(D == 3) | (int)(it - P->phase_start + 1 >= widen_from(v.npairs)))) {
        double Tp[12], Qp[3];
        load_hist(v, it - 1, pair, Tp);
        pose_point(Tp, mt[0], mt[1], mt[2], Qp);
        const double dt = dist3_f64(Qt, Qp);
        m = (float)(kExpand * sqrt(a2 * rot_frob2(T, Tp) + dt * dt));
    }
    cp->margin = m;
    return false;
}

// No previous match (a pair's first search, it == 1): seed one from a greedy descent of the
// target tree (the child whose f32 box bound is smaller, down to a leaf; a target of that
// leaf).  The search only uses it for its first pruning threshold, so any target is valid;
// a near one spares the group walk the nodes an infinite threshold opens.  One descent per
// kSeedShare consecutive source tree positions (close together in the search space), by the
// block's first threads: the chunk's 1,024 per-query descents -- a chain of 2L dependent box
// loads each -- made the first k_nn_prep ~4x the cost of a later one (C4 64 pairs, same-box
// A/B: one seed per 16 positions saved 0.4 ms/step of k_nn_prep but cost the first search
// as much).
#ifndef SE3ICP_SEED_SHARE
#define SE3ICP_SEED_SHARE 4
#endif
constexpr int kSeedShare = SE3ICP_SEED_SHARE;
template <int D>
__device__ __forceinline__ int seed_descent(const View& v, const TreeRef& TR, const PairDev* P, const CloudDev& ct,
                                            int gx, int g) {
    double T[12], m0[D], Q[D];
    load_T(P, T);
    load_m0<D>(v, TR, gx, g, m0);
    pose_m0<D>(T, m0, Q);
    float qf[D];
#pragma unroll
    for (int r = 0; r < D; ++r) qf[r] = (float)((D == 3) ? Q[r] - P->f32_center[r] : Q[r]);
    const float* lo = TR.lo + (size_t)P->tgt * TR.nnodes * D;
    const float* hi = TR.hi + (size_t)P->tgt * TR.nnodes * D;
    int h = 0;
    for (int lv = 0; lv < TR.L; ++lv) {
        const int a = 2 * h + 1;
        const float la = box_lb<D>(lo + (size_t)a * D, hi + (size_t)a * D, qf);
        const float lb = box_lb<D>(lo + (size_t)(a + 1) * D, hi + (size_t)(a + 1) * D, qf);
        h = la <= lb ? a : a + 1;
    }
    const int li = h - ((1 << TR.L) - 1);
    const int ta = min(tree_first(ct.n, TR.L, li), ct.n - 1);
    const int cnt = max(tree_first(ct.n, TR.L, li + 1) - ta, 1);
    // the nearest of kSeedTargets targets spread over the leaf
    const float* tv = TR.tvec + tree_tv_ix<D>(0, ct.off, 0);  // (the cloud's first slot)
    int best = ta;
    float bd = INFINITY;
    for (int k = 0; k < kSeedTargets; ++k) {
        const int t = ta + (2 * k + 1) * cnt / (2 * kSeedTargets);
        float d = 0.f;
#pragma unroll
        for (int r = 0; r < D; ++r) {
            const float e = qf[r] - tv[tree_tv_ix<D>(v.ld, t, r)];
            d = fmaf(e, e, d);
        }
        best = d < bd ? t : best;
        bd = fminf(d, bd);
    }
    return TR.perm[ct.off + best];
}

// One 1024-thread block per chunk (a node of level CL = GL - 4 of the source tree: 16
// query leaves of level GL).  Settles what the certificates allow and packs the rest
// for k_nn_search: consecutive leaves' remaining queries share a 64-lane group as long as
// they fit, a leaf is never split (with every query searched, a group is one leaf).
// qlist[c][j][lane] = local tree position, qcount[c][j] = lanes of group j.
#ifdef SE3ICP_PROF
// k_nn_prep block phases (100 MHz clock), summed over blocks: settle, pack, lists; blocks;
// and the span of each launch (latest end - earliest start), summed over launches
__device__ unsigned long long g_prep_prof[6];
__device__ unsigned long long g_prep_span[2] = {~0ull, 0ull};
// SE(3) group waves by duration (25 us bins, the last open): count and summed ticks; and
// the launch span (earliest wave start, latest wave end)
__device__ unsigned long long g_wave_hist[2][41];
__device__ unsigned long long g_wave_span[2] = {~0ull, 0ull};
// SE(3) group waves per hardware XCD (HW_REG_XCC_ID): summed wave time, latest wave end, waves
__device__ unsigned long long g_xcd_prof[8][3];
// SE(3) ordered group blocks per hardware XCD: summed lifetime (kernel entry to exit) of the
// blocks that ran a group, of the empty ones, and the empty ones' count
__device__ unsigned long long g_xcd_life[8][3];
// 3-D search waves per launch: [0] group waves, [1] single-query-list waves: count, summed
// ticks, longest wave (ticks), queries
__device__ unsigned long long g_r3_prof[2][4];
#endif
// (8 waves per SIMD: two 1024-thread blocks per CU, <= 64 VGPRs)
// publish (may be null): the host's ring slot of the previous iteration, which receives
// every pair's phase in this one (its k_reduce_final opened it).  Written first thing by
// block 0, so the host-memory write completes inside this launch instead of delaying the
// end of k_reduce_final (a fine-grained host write held the next launch back ~6 us).
__global__ __launch_bounds__(1024) __attribute__((amdgpu_waves_per_eu(8))) void k_nn_prep(View v, int32_t* publish) {
#ifdef SE3ICP_PROF
    const unsigned long long tp0 = __builtin_amdgcn_s_memrealtime();
#endif
    if ((int)(blockIdx.x == 0) & (int)(publish != nullptr))
        for (int p = threadIdx.x; p < v.npairs; p += blockDim.x) publish[p] = v.pairs[p].phase;
    constexpr int NL = kChunkQ / 64;  // leaves (groups) per chunk
    __shared__ int s_cnt[NL], s_slot[NL], s_base[NL], s_wc[NL], s_single;
    const int c = xcd_block_runs(blockIdx.x, gridDim.x, kXcdRun / 16);  // (k_nn_search's chunk runs)
    const int pair = c >> v.chunk_level;
    const PairDev* P = v.pairs + pair;
    const int phase = P->phase;
    // a finished pair's chunks have nothing to settle or list: the searches skip its groups
    // by its phase, so its stale qcount rows are never read (block-uniform exit; the loop's
    // last iterations run with few pairs left)
    if (phase == PHASE_IDLE) return;
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if (threadIdx.x < NL) s_cnt[threadIdx.x] = 0;
    __syncthreads();
    bool active = false;
    int x = 0, l = 0;
    if (phase != PHASE_IDLE) {
        const CloudDev cs = v.clouds[P->src], ct = v.clouds[P->tgt];
        const TreeRef TR = (phase == PHASE_SE3) ? v.t12 : v.t3;
        const int ci = c & ((1 << v.chunk_level) - 1);
        const int a = tree_first(cs.n, v.chunk_level, ci), b = tree_first(cs.n, v.chunk_level, ci + 1);
        x = a + (int)threadIdx.x;
        if (x < b) {
            const int gx = cs.off + x, g = cs.off + TR.perm[gx];
            const double al = v.setup[P->src].alpha;
            active = (phase == PHASE_SE3) ? !prep_settle<12>(v, TR, P, pair, ct, gx, g, al * al)
                                          : !prep_settle<3>(v, TR, P, pair, ct, gx, g, 0.0);
            l = tree_node_of(x, cs.n, TR.GL) - (ci << (TR.GL - v.chunk_level));
            if (active) atomicAdd(&s_cnt[l], 1);
        }
    }
    // a run's first search: shared seeds (seed_descent), one per kSeedShare positions
    if ((int)(phase != PHASE_IDLE) & (int)(P->iter == 1)) {  // (block-uniform)
        static_assert(kSeedShare >= 1 && kChunkQ % kSeedShare == 0, "a thread per seed");
        __shared__ int s_seed[kChunkQ / kSeedShare];
        const CloudDev cs = v.clouds[P->src], ct = v.clouds[P->tgt];
        const TreeRef TR = (phase == PHASE_SE3) ? v.t12 : v.t3;
        const int ci = c & ((1 << v.chunk_level) - 1);
        const int a = tree_first(cs.n, v.chunk_level, ci), b = tree_first(cs.n, v.chunk_level, ci + 1);
        if ((int)threadIdx.x < kChunkQ / kSeedShare) {
            const int xr = a + kSeedShare * (int)threadIdx.x;
            int sd = -1;
            if ((int)(xr < b) & (int)(ct.n > 0)) {
                const int gxr = cs.off + xr, gr = cs.off + TR.perm[gxr];
                sd = (phase == PHASE_SE3) ? seed_descent<12>(v, TR, P, ct, gxr, gr) : seed_descent<3>(v, TR, P, ct, gxr, gr);
            }
            s_seed[threadIdx.x] = sd;
        }
        __syncthreads();
        if ((int)active & (int)(ct.n > 0)) {
            const int g = cs.off + TR.perm[cs.off + x];
            if (v.corr_idx[g] < 0) v.corr_idx[g] = s_seed[(x - a) / kSeedShare];
        }
    }
    const unsigned long long m = __ballot(active);
    if (lane == 0) s_wc[wid] = __popcll(m);
    __syncthreads();
#ifdef SE3ICP_PROF
    const unsigned long long tp1 = __builtin_amdgcn_s_memrealtime();
#endif
    if (wid == 0) {
        // greedy packing of whole leaves into groups of <= 64: the 16 leaf counts in a VGPR,
        // the sequential pass in scalar registers (no LDS round trip per leaf)
        const int cnt_l = lane < NL ? s_cnt[lane] : 0;
        int cur = 0, grp = 0, base = 0;
        int slot_l = 0, base_l = 0, gcnt_l = 0;
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int n = __builtin_amdgcn_readlane(cnt_l, j);
            if (cur + n > 64) { ++grp; cur = 0; }
            if (lane == j) { slot_l = 64 * grp + cur; base_l = base; }
            if (lane == grp) gcnt_l += n;
            cur += n;
            base += n;
        }
        const int total = base;
        // a sparse chunk goes to the one-query-per-wave kernel instead (SE(3) list from the
        // front of sq_list, R3 from the back)
        const bool dense = total >= dense_min(v.nchunks);
        if (lane < NL) {
            s_slot[lane] = slot_l;
            s_base[lane] = base_l;
            v.qcount[c * NL + lane] = dense ? gcnt_l : 0;
        }
        if ((int)dense & (int)(total > 0) & (int)(lane <= grp) & ((int)(phase == PHASE_SE3) | ((int)order3(v.npairs) & (int)(phase == PHASE_R3)))) {
            const int g = c * NL + lane;
            const int ph = phase == PHASE_SE3 ? 0 : 1;
            // the group's last wave time: one row for both phases, so a pair's first R3
            // searches are ordered by its groups' SE(3) times (the same source queries against
            // the same target cloud) until its R3 waves have written their own.  Round 6
            // measured separate rows per phase: SE(3) NN 18.40 -> 19.02 ms per
            // step at C4 64 pairs, same box -- the shared row stays, deliberately
            const int row = (ph * 8 + group_xcd(g, v.nchunks * NL)) * 16 + cost_class(v.gcost[g]);
            const int at = atomicAdd(&v.cls[row], 1);
            v.cls[kClsHead + (size_t)row * cls_cap(v.nchunks) + at] = g;
        }
        if (lane == 0) {
            s_single = ((int)!dense & (int)(total > 0)) ? atomicAdd(&v.flag_count[phase == PHASE_SE3 ? 1 : 2], total) : -1;
            if (phase != PHASE_IDLE) {  // work counters: queries / searched queries per phase
                unsigned long long* st = v.stats + kStatCols * (c & 63) + (phase == PHASE_SE3 ? 4 : 6);
                const CloudDev cs = v.clouds[P->src];
                const int ci = c & ((1 << v.chunk_level) - 1);
                atomicAdd(st, (unsigned long long)(tree_first(cs.n, v.chunk_level, ci + 1) - tree_first(cs.n, v.chunk_level, ci)));
                atomicAdd(st + 1, (unsigned long long)total);
            }
        }
    }
    __syncthreads();
#ifdef SE3ICP_PROF
    const unsigned long long tp2 = __builtin_amdgcn_s_memrealtime();
#endif
    if (active) {
        int r = __builtin_amdgcn_mbcnt_hi((unsigned)(m >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m, 0u));
        for (int w = 0; w < wid; ++w) r += s_wc[w];
        const int sb = s_single;
        if (sb < 0) {
            v.qlist[(size_t)c * kChunkQ + s_slot[l] + (r - s_base[l])] = x;
        } else {
            const int gxs = v.clouds[P->src].off + x;
            if (phase == PHASE_SE3) v.sq_list[sb + r] = gxs;
            else v.sq_list[v.ld - 1 - (sb + r)] = gxs;
        }
    }
#ifdef SE3ICP_PROF
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long tp3 = __builtin_amdgcn_s_memrealtime();
        atomicAdd(&g_prep_prof[0], tp1 - tp0);
        atomicAdd(&g_prep_prof[1], tp2 - tp1);
        atomicAdd(&g_prep_prof[2], tp3 - tp2);
        atomicAdd(&g_prep_prof[3], 1ull);
        atomicMin(&g_prep_span[0], tp0);
        atomicMax(&g_prep_span[1], tp3);
    }
#endif
}

// Results of a searched query (one lane): the recheck flag, the certificate, the
// correspondence and its stored distance.
// A flagged query (uncertified f32 arg-min) is re-resolved in f64 by the calling wave right
// after (recheck_one), which then writes its corr_idx / corr_dist.
template <int D>
__device__ __forceinline__ void nn_finish(const View& v, const PairDev* P, int pair, const TreeRef& TR,
                                          const CloudDev& ct, int gx, int g, bool flag, float d1, float d2, int i1,
                                          float thr, float na, float nb) {
    const bool rc = (bool)((int)flag & (int)(ct.n > 1));
    if (rc) atomicAdd(&v.pair_rechecked[pair], 1);
    // certificate for the next iterations (k_nn_prep), at the source tree slot gx: exact
    // match distance <= sqrt(d1 + err), every other target >= min(d2 - err(d2), thr):
    // visited ones by the top-2, unvisited ones because every box skipped had a bound >= thr
    // at the time (thr only decreases); the match and its anchor (the margin slot is dead
    // once the search has read it)
    float4* cw = reinterpret_cast<float4*>(v.cert + gx);
    const bool nocert = (bool)((int)flag | (int)(i1 < 0));
    if (nocert) cw[0] = make_float4(0.f, 0.f, __int_as_float(-1), __int_as_float(0));
    if (rc) return;
    // tree position -> target index; a NaN query keeps the reference's zero-initialised index
    const int j = (i1 < 0) ? 0 : TR.perm[ct.off + i1];
    v.corr_idx[g] = j;
    // the stored distance needs the translation part of the query only (ISR.cpp:465-468)
    double Tm[12], Qt[3], t[3];
    load_T(P, Tm);
    const double* m = TR.tvec64 + gx;  // (3 rows: points / translations)
    pose_point(Tm, m[0], m[v.ld], m[2 * (size_t)v.ld], Qt);
    match_anchor(v, D == 12 ? PHASE_SE3 : PHASE_R3, ct, j, t);
    v.corr_dist[g] = anchor_dist(Qt, t);
    if (!nocert) {
        const float l2 = fminf(d2 - f32_err(d2, na, nb, D), thr * (1.f - 4e-6f));
        cw[0] = make_float4(sqrtf(d1 + f32_err(d1, na, nb, D)) * (1.f + 1e-6f), sqrtf(fmaxf(l2, 0.f)) * (1.f - 1e-6f),
                            __int_as_float(P->iter), __int_as_float(j));
        double* tw = reinterpret_cast<double*>(cw + 1);
        tw[0] = t[0];
        tw[1] = t[1];
        tw[2] = t[2];
    }
}

template <int D>
__device__ __forceinline__ void single_one(const View& v, const PairDev* P, int pair, const TreeRef& TR,
                                           const CloudDev& ct, int gx, int g, int lane, unsigned* n_eval,
                                           unsigned* n_box, unsigned* n_use, int tp_pre = -2, float mrg_pre = 0.f);

template <int D>
__device__ __forceinline__ void single_list(const View& v, int bw);

// One launch per phase and iteration: blocks [0, kSingleWaves) are one-query-per-wave
// searches of the phase's single-query list (single_list, dispatched first: they are the
// launch's latency tail), the rest one 64-query group each.  (Round 3 ran the two parts as
// two grids on two streams, joined by events: two extra launches and two cross-stream
// waits per iteration.)
// ORD: the group waves take the cost-ordered lists (always for D = 12; for D = 3 in batches
// of order3() pairs -- its own instantiation, so the run-order 3-D search keeps its registers)
template <int D, bool ORD>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(D == 12 ? kWpe : kWpe3))) void k_nn_search(View v) {
    if (blockIdx.x < (unsigned)kSingleWaves) {
        single_list<D>(v, (int)blockIdx.x);
        return;
    }
    constexpr int NV = (D + 3) / 4;
    __shared__ float4 s_tile[kLeafMax * NV];
    // compacted leaf sweeps (12-D): the wave's query vectors, the list of lanes that want
    // the current leaf, and the per-query top-2 of the leaf
    __shared__ float4 s_q[64 * NV];
    __shared__ int s_wl[64];
    __shared__ float s_r1[64], s_r2[64];
    __shared__ int s_rb[64];
    const int lane = threadIdx.x & 63;
    // wave-uniform work item: group gi & 15 (64 listed queries) of chunk c; the pair record,
    // node boxes and leaf ranges become scalar loads (blocks of one XCD take runs of
    // consecutive chunks: a pair's target tree stays in that XCD's L2)
    // (kSingleWaves is a multiple of 8: block b and b - kSingleWaves share an XCD)
    auto group = [&](const int gq) __attribute__((always_inline)) {
        if ((gq >> 4) >= v.nchunks) return;
        const int c = gq >> 4;
        const int gi = gq;
        const int pair = c >> v.chunk_level;
        const PairDev* P = v.pairs + pair;
        const int phase = P->phase;
        if (phase != (D == 12 ? PHASE_SE3 : PHASE_R3)) return;
        const int cnt_q = __builtin_amdgcn_readfirstlane(v.qcount[gi]);
        if (cnt_q <= 0) return;
        const CloudDev cs = v.clouds[P->src], ct = v.clouds[P->tgt];
        const TreeRef TR = (D == 12) ? v.t12 : v.t3;
        if (cnt_q <= kSmall) {
            // a group of a few queries (a chunk's leftovers): each searched by all 64 lanes in
            // turn (single_one's lane-parallel search) -- a lone query with a wide ball would
            // otherwise walk the tree one node per step and set the launch's time
            unsigned n_eval = 0, n_box = 0, n_use = 0;
            for (int q = 0; q < cnt_q; ++q) {
                const int gxq = __builtin_amdgcn_readfirstlane(cs.off + v.qlist[(size_t)gi * 64 + q]);
                const int gq = __builtin_amdgcn_readfirstlane(cs.off + TR.perm[gxq]);
                single_one<D>(v, P, pair, TR, ct, gxq, gq, lane, &n_eval, &n_box, &n_use);
            }
            if (lane == 0) {
                unsigned long long* st = v.stats + kStatCols * (gi & 63) + (D == 12 ? 0 : 2);
                atomicAdd(st, 64ull * n_eval);
                atomicAdd(st + 1, 64ull * n_box);
                atomicAdd(v.stats + kStatCols * (gi & 63) + (D == 12 ? kStatUseSe3 : kStatUseR3), (unsigned long long)n_use);
            }
            return;
        }
        const bool valid = lane < cnt_q;
        const int gx = cs.off + v.qlist[(size_t)gi * 64 + (valid ? lane : 0)];  // source tree slot
        const int g = cs.off + TR.perm[gx];
        const float mrg = valid ? v.cert[gx].margin : 0.f;

        // query: f64 pose applied to the source element, rounded to f32
        float q[D];
        float na;
        {  // (the f64 query is recomputed at the end rather than held through the traversal)
            double Tm[12], Q[D];
            load_T(P, Tm);
            double m0[D];
            load_m0<D>(v, TR, gx, g, m0);
            pose_m0<D>(Tm, m0, Q);
            double n2 = 0;
    #pragma unroll
            for (int r = 0; r < D; ++r) {
                const double c = (D == 3) ? Q[r] - P->f32_center[r] : Q[r];
                q[r] = (float)c;
                n2 += c * c;
            }
            na = (float)sqrt(n2) * 1.000001f;
        }
        const float nb = (D == 12) ? P->tgt_norm12 : P->tgt_norm3;
        f32x2 q2[(D + 1) / 2];
    #pragma unroll
        for (int r = 0; r < D / 2; ++r) q2[r] = f32x2{q[2 * r], q[2 * r + 1]};
        const float* tv = TR.tvec + tree_tv_ix<D>(0, ct.off, 0);  // (the cloud's first slot)
        const size_t ld = v.ld;
        if constexpr (D == 12) {
            s_q[lane * 3 + 0] = make_float4(q[0], q[1], q[2], q[3]);
            s_q[lane * 3 + 1] = make_float4(q[4], q[5], q[6], q[7]);
            s_q[lane * 3 + 2] = make_float4(q[8], q[9], q[10], q[11]);
        } else {
            s_q[lane] = make_float4(q[0], q[1], q[2], 0.f);
        }

        // pruning threshold for the best / second-best f32 distances a1 <= a2: the certified
        // radius a1 + 3 err, widened by the margin up to (sqrt(a1) + 2 mrg)^2 but never past a2
        auto widen = [&](float a1, float a2) __attribute__((always_inline)) {
            const float e = sqrtf(a1) + 2.f * mrg;
            const float t = fmaxf(a1, fminf(e * e, a2));
            return t + 3.f * f32_err(t, na, nb, D);
        };
        float d1 = INFINITY, d2 = INFINITY;
        int i1 = -1;  // target tree position of the best candidate
        float thr = valid ? INFINITY : -1.f;
        // box tests compare against thb = thr * kBoxScale instead of lb * (1 - 2e-6) < thr
        // (one multiply per bound update instead of one per box): kBoxScale >= 1 / ((1 - 2e-6)
        // (1 - 2^-24)^2), so every box the scaled form admits is still admitted (more visits at
        // worst, never fewer)
        float thb = thr;
        if (valid) {  // seed the pruning threshold with the previous match
            const int prev = v.corr_idx[g];
            if (prev >= 0 && prev < ct.n) {
                const int tp = TR.pos[ct.off + prev];
                float s = 0.f;
    #pragma unroll
                for (int r = 0; r < D; ++r) {
                    const float e = q[r] - tv[tree_tv_ix<D>(ld, tp, r)];
                    s = fmaf(e, e, s);
                }
                thr = widen(s, INFINITY);
            }
        }
        thb = thr * kBoxScale;

        const float* box_lo = TR.lo + (size_t)P->tgt * TR.nnodes * D;
        const float* box_hi = TR.hi + (size_t)P->tgt * TR.nnodes * D;
        const int first_leaf = (1 << TR.L) - 1;
        float4* tile = s_tile;
        int stk = 0;  // DFS stack in a VGPR: lane i holds entry i (depth <= 2L+1 < 64)
        int sp = 1;
        unsigned n_eval = 0, n_box = 0;  // wave-uniform work counters (roofline accounting)
        unsigned n_use = 0;  // occupied (query, target) distance evaluations
        const unsigned long long vmask = __ballot(valid);
    #ifdef SE3ICP_PROF
        unsigned n_want = 0, n_leafv = 0;
        unsigned long long c_leaf = 0, c_lload = 0;  // shader-clock cycles in leaf visits / their target loads
        const unsigned long long c_w0 = __builtin_amdgcn_s_memtime();
        const unsigned n_valid = (unsigned)__popcll(__ballot(valid));
        const unsigned long long t_w0 = __builtin_amdgcn_s_memrealtime();
    #endif
        // a near leaf is swept right after its parent's box tests, with the lanes those tests
        // admitted (no bound changed in between): no stack round trip, no box re-test
        int pend = -1;
        unsigned long long pendW = 0ull;
        while ((int)(sp > 0) | (int)(pend >= 0)) {
            int h;
            const bool known = pend >= 0;
            if (known) {
                h = pend;
                pend = -1;
            } else {
                h = __builtin_amdgcn_readlane(stk, sp - 1);
                --sp;
            }
            if (h >= first_leaf) {
                const int li = h - first_leaf;
                const int ta = tree_first(ct.n, TR.L, li), tb = tree_first(ct.n, TR.L, li + 1);
                const int cnt = tb - ta;
                if (cnt <= 0) continue;
                // lanes whose own bound admits this leaf (box re-tested: the bounds shrank since the push)
                unsigned long long W = pendW;
                int w = 64;
                {
                    if (!known) {
                        float lbh;
                        if constexpr (D == 12) lbh = box_lb12_u(box_lo + (size_t)h * D, box_hi + (size_t)h * D, q2);
                        else lbh = box_lb_u<D>(box_lo + (size_t)h * D, box_hi + (size_t)h * D, q);
                        W = __ballot(lbh * kBoxMul < thb);
                    }
                    if (W == 0ull) continue;
                    w = __popcll(W);
                }
                n_use += (unsigned)__popcll(W & vmask) * (unsigned)cnt;
    #ifdef SE3ICP_PROF
                n_want += __popcll(W & __ballot(valid));
                ++n_leafv;
                const unsigned long long c_l0 = __builtin_amdgcn_s_memtime();
    #endif
                __builtin_amdgcn_wave_barrier();
                if (lane < cnt) {
                    if constexpr (D == 12) {  // the leaf's rows: one contiguous run, three 16-B loads per lane
                        const float4* r = reinterpret_cast<const float4*>(tv + (size_t)(ta + lane) * 12);
                        const float4 a = r[0], b = r[1], c = r[2];
                        tile[lane * 3] = a;
                        tile[lane * 3 + 1] = b;
                        tile[lane * 3 + 2] = c;
                    } else {
                        tile[lane] = make_float4(tv[ta + lane], tv[ld + ta + lane], tv[2 * ld + ta + lane], 0.f);
                    }
                }
                __builtin_amdgcn_wave_barrier();
    #ifdef SE3ICP_PROF
                __builtin_amdgcn_s_waitcnt(0);
                const unsigned long long c_l1 = __builtin_amdgcn_s_memtime();
                c_lload += c_l1 - c_l0;
    #endif
                if (w > kCompact) {
                    // every lane sweeps every target (broadcast LDS reads)
                    for (int j = 0; j < cnt; ++j) {
                        float acc;
                        if constexpr (D == 12) {
                            acc = dist12(q2, tile + j * 3);
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
                        i1 = lt ? (ta + j) : i1;  // target tree position
                    }
                    n_eval += cnt;
                } else {
                    // compacted: LPQ lanes per wanting query (8 for leaves of <= 32 targets, 16
                    // up to 64), 4 targets per lane, then a top-2 merge over the LPQ lanes and
                    // into the query's own lane
                    if ((W >> lane) & 1ull)
                        s_wl[__builtin_amdgcn_mbcnt_hi((unsigned)(W >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)W, 0u))] = lane;
                    __builtin_amdgcn_wave_barrier();
                    constexpr int kL32 = 32 / kTPL, kL64 = 64 / kTPL;  // lanes per query
                    if (cnt <= 32) compact_sweep<D, kL32>(tile, s_q, s_wl, s_r1, s_r2, s_rb, w, cnt, ta, lane);
                    else compact_sweep<D, kL64>(tile, s_q, s_wl, s_r1, s_r2, s_rb, w, cnt, ta, lane);
                    __builtin_amdgcn_wave_barrier();
                    if ((W >> lane) & 1ull) {
                        const float r1 = s_r1[lane], r2 = s_r2[lane];
                        const int rb = s_rb[lane];
                        d2 = fmin3_raw(fmax_raw(d1, r1), d2, r2);
                        i1 = r1 < d1 ? rb : i1;
                        d1 = fmin_raw(d1, r1);
                    }
                    __builtin_amdgcn_wave_barrier();
                    {  // 64-lane evaluation slots issued
                        const int qpi = 64 / (cnt <= 32 ? 32 / kTPL : 64 / kTPL);
                        n_eval += kTPL * ((w + qpi - 1) / qpi);
                    }
                }
                if ((int)valid & (int)(d1 < INFINITY)) {
                    thr = fminf(thr, widen(d1, d2));
                    thb = thr * kBoxScale;
                }
    #ifdef SE3ICP_PROF
                c_leaf += __builtin_amdgcn_s_memtime() - c_l0;
    #endif
                continue;
            }
            n_box += 2;
            const int hl = 2 * h + 1, hr = 2 * h + 2;
            float ll, lr;
            if constexpr (D == 12) {
                ll = box_lb12_u(box_lo + (size_t)hl * D, box_hi + (size_t)hl * D, q2);
                lr = box_lb12_u(box_lo + (size_t)hr * D, box_hi + (size_t)hr * D, q2);
            } else {
                ll = box_lb_u<D>(box_lo + (size_t)hl * D, box_hi + (size_t)hl * D, q);
                lr = box_lb_u<D>(box_lo + (size_t)hr * D, box_hi + (size_t)hr * D, q);
            }
            // the f32 bound is within (D+2) ulps of the exact distance to the (inflated) box
            const unsigned long long Wl = __ballot(ll * kBoxMul < thb);
            const unsigned long long Wr = __ballot(lr * kBoxMul < thb);
            const bool vl = Wl != 0ull, vr = Wr != 0ull;
            const bool left_first = __builtin_amdgcn_readfirstlane(ll <= lr ? 1 : 0) != 0;
            const int nearh = left_first ? hl : hr, farh = left_first ? hr : hl;
            const bool vnear = left_first ? vl : vr, vfar = left_first ? vr : vl;
            if (vfar) { stk = (lane == sp) ? farh : stk; ++sp; }
            if (vnear) {
                if (hl >= first_leaf) {  // (children are leaves)
                    pend = nearh;
                    pendW = left_first ? Wl : Wr;
                } else {
                    stk = (lane == sp) ? nearh : stk;
                    ++sp;
                }
            }
        }

        if (lane == 0) {  // 64 lanes per evaluation; 64 counter slots against contention
            unsigned long long* st = v.stats + kStatCols * (gi & 63) + (D == 12 ? 0 : 2);
            atomicAdd(st, 64ull * n_eval);
            atomicAdd(st + 1, 64ull * n_box);
            atomicAdd(v.stats + kStatCols * (gi & 63) + (D == 12 ? kStatUseSe3 : kStatUseR3), (unsigned long long)n_use);
            // the wave's work (box-test steps + leaf sweeps): the chunk's cost for k_nn_order
    #ifdef SE3ICP_PROF
            if (D == 12) {
                atomicAdd(v.stats + kStatCols * (gi & 63) + 8, (unsigned long long)n_want);
                atomicAdd(v.stats + kStatCols * (gi & 63) + 9, (unsigned long long)n_leafv);
                const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t_w0;
                // longest wave, with its leaf visits, box-test steps and valid queries
                atomicMax(v.stats + 10, (dt << 40) | ((unsigned long long)min(n_box, 0xfffffu) << 20) |
                                            ((unsigned long long)min(n_leafv, 0x3fffu) << 6) | (n_valid % 64u));
                atomicAdd(v.stats + kStatCols + 10, dt * dt);                      // (spread)
                atomicAdd(v.stats + kStatCols * (gi & 63) + 11, (1ull << 44) + dt);  // waves, wave time
                const int hb = min((int)(dt / 2500ull), 40);
                atomicAdd(&g_wave_hist[0][hb], 1ull);
                atomicAdd(&g_wave_hist[1][hb], dt);
                atomicMin(&g_wave_span[0], t_w0);
                atomicMax(&g_wave_span[1], t_w0 + dt);
                {
                    const int xcc = (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u);  // HW_REG_XCC_ID
                    atomicAdd(&g_xcd_prof[xcc][0], dt);
                    atomicMax(&g_xcd_prof[xcc][1], t_w0 + dt);
                    atomicAdd(&g_xcd_prof[xcc][2], 1ull);
                }
                atomicAdd(v.stats + kStatCols * (gi & 63) + 12, c_leaf);   // shader cycles in leaf visits,
                atomicAdd(v.stats + kStatCols * (gi & 63) + 14, c_lload);  // in their target loads,
                atomicAdd(v.stats + kStatCols * (gi & 63) + 13, __builtin_amdgcn_s_memtime() - c_w0);  // in the wave
            } else {
                const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t_w0;
                atomicAdd(&g_r3_prof[0][0], 1ull);
                atomicAdd(&g_r3_prof[0][1], dt);
                atomicMax(&g_r3_prof[0][2], dt);
                atomicAdd(&g_r3_prof[0][3], (unsigned long long)n_valid);
            }
    #endif
        }
        // certification (see the header) and the stored distance; the uncertified queries are
        // re-resolved in f64 by the whole wave, one after the other (few: ~0.4 % of queries)
        const bool flag = (bool)((int)valid & ((int)(i1 < 0) | (int)!(d2 - d1 > 2.f * f32_err(d2, na, nb, D))));
        if (valid) nn_finish<D>(v, P, pair, TR, ct, gx, g, flag, d1, d2, i1, thr, na, nb);
        unsigned long long fm = __ballot((int)flag & (int)(ct.n > 1));
        const int seed = i1 < 0 ? 0 : TR.perm[ct.off + i1];
        while (fm) {
            const int j = __builtin_ctzll(fm);
            fm &= fm - 1ull;
            recheck_one<D>(v, P, ct, __shfl(g, j, 64), __shfl(seed, j, 64), lane);
        }
    };
    if constexpr (ORD) {
#ifdef SE3ICP_PROF
        const unsigned long long t_entry = __builtin_amdgcn_s_memrealtime();
        auto life = [&](int slot) {
            if ((int)(D == 12) & (int)(lane == 0)) {
                const int xcc = (int)(__builtin_amdgcn_s_getreg((3 << 11) | 20) & 7u);
                atomicAdd(&g_xcd_life[xcc][slot], __builtin_amdgcn_s_memrealtime() - t_entry);
                if (slot == 1) atomicAdd(&g_xcd_life[xcc][2], 1ull);
            }
        };
#else
        auto life = [](int) {};
#endif
        const int bb = (int)blockIdx.x - kSingleWaves, x = bb & 7, i = bb >> 3;
        const int row0 = ((D == 12 ? 0 : 1) * 8 + x) * 16;
        int acc = 0, k = -1, lo = 0;
        for (int j = 0; j < 16; ++j) {
            const int cj = __builtin_amdgcn_readfirstlane(v.cls[row0 + j]);
            if ((int)(k < 0) & (int)(i < acc + cj)) { k = j; lo = acc; }
            acc += cj;
        }
        // (no group of this XCD timed yet -- the SE(3) phase's first search; an R3 phase starts
        // with the SE(3) times, see k_nn_prep: the run order, whose
        // neighbouring chunks share target leaves in the XCD's L2)
        const int known = acc - __builtin_amdgcn_readfirstlane(v.cls[row0]);
        if (known == 0) {
            const int gs = __builtin_amdgcn_readfirstlane(xcd_block_runs(bb, (int)gridDim.x - kSingleWaves, kXcdRun));
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            group(gs);
            const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
            if ((int)(lane == 0) & (int)((gs >> 4) < v.nchunks)) v.gcost[gs] = (unsigned)min(t1 - t0, 0xffffffffull) | 1u;
            life(0);
            return;
        }
        if (k < 0) {
            life(1);
            return;
        }
        const int gq = __builtin_amdgcn_readfirstlane(v.cls[kClsHead + (size_t)(row0 + k) * cls_cap(v.nchunks) + (i - lo)]);
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        group(gq);
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        if (lane == 0) v.gcost[gq] = (unsigned)min(t1 - t0, 0xffffffffull) | 1u;
        life(0);
        return;
    }
    const int gq = __builtin_amdgcn_readfirstlane(
        xcd_block_runs((int)blockIdx.x - kSingleWaves, (int)gridDim.x - kSingleWaves, kXcdRun));
    group(gq);
}

// ------------------------------------------------------------------ one wavefront per query
// For the queries of sparse chunks (k_nn_prep): a wave's latency, not its lanes, bounds
// the group kernel when few queries remain, so here the 64 lanes work on ONE query:
// lane-parallel box tests (the nodes of level A = L - 6, then the 64 leaves under each
// open one) and a target per lane in the leaf sweeps; each lane keeps the top-2 of the
// targets it evaluated, the wave's (d1, d2) are two wave minima per leaf.
template <int D>
// tp_pre: the previous match's target tree position (-1 none) and mrg_pre the query's margin,
// when the caller fetched them already (single_list); -2: load them here.
__device__ __forceinline__ void single_one(const View& v, const PairDev* P, int pair, const TreeRef& TR,
                                           const CloudDev& ct, int gx, int g, int lane, unsigned* n_eval,
                                           unsigned* n_box, unsigned* n_use, int tp_pre, float mrg_pre) {
    float q[D];
    float na;
    {
        double Tm[12], m0[D], Q[D];
        load_T(P, Tm);
        load_m0<D>(v, TR, gx, g, m0);
        pose_m0<D>(Tm, m0, Q);
        double n2 = 0;
#pragma unroll
        for (int r = 0; r < D; ++r) {
            const double c = (D == 3) ? Q[r] - P->f32_center[r] : Q[r];
            q[r] = (float)c;
            n2 += c * c;
        }
        na = (float)sqrt(n2) * 1.000001f;
    }
    const float nb = (D == 12) ? P->tgt_norm12 : P->tgt_norm3;
    f32x2 q2[(D + 1) / 2];
#pragma unroll
    for (int r = 0; r < D / 2; ++r) q2[r] = f32x2{q[2 * r], q[2 * r + 1]};
    const float mrg = tp_pre == -2 ? v.cert[gx].margin : mrg_pre;
    auto widen = [&](float a1, float a2) __attribute__((always_inline)) {
        const float e = sqrtf(a1) + 2.f * mrg;
        const float t = fmaxf(a1, fminf(e * e, a2));
        return t + 3.f * f32_err(t, na, nb, D);
    };
    const float* tv = TR.tvec + tree_tv_ix<D>(0, ct.off, 0);  // (the cloud's first slot)
    const size_t ld = v.ld;
    float thr = INFINITY;
    {  // seed with the previous match
        int tp = tp_pre;
        if (tp_pre == -2) {
            const int prev = v.corr_idx[g];
            tp = (prev >= 0 && prev < ct.n) ? TR.pos[ct.off + prev] : -1;
        }
        if (tp >= 0) {
            float s = 0.f;
#pragma unroll
            for (int r = 0; r < D; ++r) {
                const float e = q[r] - tv[tree_tv_ix<D>(ld, tp, r)];
                s = fmaf(e, e, s);
            }
            thr = widen(s, INFINITY);
        }
    }
    const float* box_lo = TR.lo + (size_t)P->tgt * TR.nnodes * D;
    const float* box_hi = TR.hi + (size_t)P->tgt * TR.nnodes * D;
    auto lbound = [&](int h) __attribute__((always_inline)) {
        if constexpr (D == 12) return box_lb12_u(box_lo + (size_t)h * D, box_hi + (size_t)h * D, q2);
        else return box_lb_u<D>(box_lo + (size_t)h * D, box_hi + (size_t)h * D, q);
    };
    const int L = TR.L;
    const int sh = L > 6 ? 6 : L;
    const int A = L - sh, nA = 1 << A, firstA = nA - 1, first_leaf = (1 << L) - 1;
    float a1 = INFINITY, a2 = INFINITY, d1 = INFINITY, d2 = INFINITY;
    int b1 = -1;
    for (int c0 = 0; c0 < nA; c0 += 64) {
        const int ai = c0 + lane;
        const float lbA = ai < nA ? lbound(firstA + ai) : INFINITY;
        *n_box += 1;
        unsigned long long mA = __ballot(lbA * (1.f - 2e-6f) < thr);
        while (mA) {
            const int j = __builtin_ctzll(mA);
            mA &= mA - 1ull;
            if (!(__shfl(lbA, j, 64) * (1.f - 2e-6f) < thr)) continue;
            const int l0 = (c0 + j) << sh;
            const float lbL = lane < (1 << sh) ? lbound(first_leaf + l0 + lane) : INFINITY;
            *n_box += 1;
            unsigned long long mL = __ballot(lbL * (1.f - 2e-6f) < thr);
            while (mL) {
                const int t = __builtin_ctzll(mL);
                mL &= mL - 1ull;
                if (!(__shfl(lbL, t, 64) * (1.f - 2e-6f) < thr)) continue;
                const int ta = tree_first(ct.n, L, l0 + t), tb = tree_first(ct.n, L, l0 + t + 1);
                float d = INFINITY;
                if (lane < tb - ta) {
                    const int x = ta + lane;
                    if constexpr (D == 12) {  // the target's 48-B row (the broadcast sweep's arithmetic)
                        d = dist12(q2, reinterpret_cast<const float4*>(tv + (size_t)x * 12));
                    } else {
                        float e, acc;
                        e = q[0] - tv[x]; acc = e * e;
                        e = q[1] - tv[ld + x]; acc = fmaf(e, e, acc);
                        e = q[2] - tv[2 * ld + x]; acc = fmaf(e, e, acc);
                        d = acc;
                    }
                }
                *n_eval += 1;
                *n_use += (unsigned)(tb - ta);  // (the one query against every target of the leaf)
                const bool lt = d < a1;
                a2 = __builtin_amdgcn_fmed3f(a1, a2, d);
                b1 = lt ? ta + lane : b1;
                a1 = lt ? d : a1;
                // the pruning threshold needs only the wave's best: one wave minimum per leaf;
                // the second-best (which could cap the widened radius below (sqrt(d1) + 2m)^2)
                // is left out here -- a wider ball, never a wrong answer -- and the wave's
                // top-2 is formed once, after the search, from the lanes' own top-2
                d1 = wave_minf(a1);
                if (d1 < INFINITY) thr = fminf(thr, widen(d1, INFINITY));
            }
        }
    }
    {  // wave top-2: the smallest lane best, then the smallest of the other lanes' bests and
       // the winner's second (ties between lanes: d2 = d1)
        d1 = wave_minf(a1);
        const unsigned long long win = __ballot(a1 == d1);
        const float other = wave_minf(a1 == d1 ? a2 : a1);
        d2 = __popcll(win) > 1 ? d1 : other;
    }
    int i1 = -1;
    {
        const unsigned long long win = __ballot((int)(a1 == d1) & (int)(b1 >= 0));
        if (win) i1 = __shfl(b1, __builtin_ctzll(win), 64);
    }
    const bool flag = (bool)((int)(i1 < 0) | (int)!(d2 - d1 > 2.f * f32_err(d2, na, nb, D)));  // (wave-uniform)
    if (lane == 0) nn_finish<D>(v, P, pair, TR, ct, gx, g, flag, d1, d2, i1, thr, na, nb);
    if ((int)flag & (int)(ct.n > 1)) recheck_one<D>(v, P, ct, g, i1 < 0 ? 0 : TR.perm[ct.off + i1], lane);
}

// grid-stride over the single-query list of the phase: SE(3) entries from the front,
// R3 entries from the back (counters flag_count[1], [2]).  The list holds each sparse
// chunk's queries together (nearby points: they read the same target leaves), so every XCD
// takes one contiguous eighth of it (blocks are dealt to the XCDs round-robin): neighbouring
// queries' leaf reads meet in one L2 instead of being fetched by all eight.  bw: the wave's
// block, < kSingleWaves.
template <int D>
__device__ __forceinline__ void single_list(const View& v, int bw) {
    const int lane = threadIdx.x & 63;
    const int nq = __builtin_amdgcn_readfirstlane(v.flag_count[D == 12 ? 1 : 2]);
    if (nq <= 0) return;
    constexpr int nbx = kSingleWaves >> 3;  // waves per XCD
#ifdef SE3ICP_PROF
    const unsigned long long t_s0 = __builtin_amdgcn_s_memrealtime();
    unsigned n_sq = 0;
#endif
    const int xcd = bw & 7;
    const int seg = (nq + 7) >> 3;
    const int f_end = min(nq, (xcd + 1) * seg);
    const int w0 = __builtin_amdgcn_readfirstlane(xcd * seg + (bw >> 3));
    unsigned n_eval = 0, n_box = 0, n_use = 0;
    const TreeRef TR = (D == 12) ? v.t12 : v.t3;
    // The wave's next kSingleBatch list entries are set up together, one per lane (list entry
    // -> point -> pair -> clouds -> previous match -> its tree position, and the margin: a
    // chain of dependent loads each query otherwise waited for in turn), then searched one
    // after the other by the whole wave.
    for (int f0 = w0; f0 < f_end; f0 += kSingleBatch * nbx) {
        const int fj = f0 + lane * nbx;
        int gxj = 0, gj = 0, pj = 0, tpj = -1;
        float mj = 0.f;
        if ((int)(lane < kSingleBatch) & (int)(fj < f_end)) {
            gxj = D == 12 ? v.sq_list[fj] : v.sq_list[v.ld - 1 - fj];
            pj = v.cloud_of[gxj] >> 1;
            const PairDev* Pj = v.pairs + pj;
            const CloudDev csj = v.clouds[Pj->src], ctj = v.clouds[Pj->tgt];
            gj = csj.off + TR.perm[gxj];
            const int prev = v.corr_idx[gj];
            tpj = (prev >= 0 && prev < ctj.n) ? TR.pos[ctj.off + prev] : -1;
            mj = v.cert[gxj].margin;
        }
        const int nbq = min(kSingleBatch, (f_end - f0 + nbx - 1) / nbx);
        for (int j = 0; j < nbq; ++j) {
            const int gx = __builtin_amdgcn_readlane(gxj, j), g = __builtin_amdgcn_readlane(gj, j);
            const int pair = __builtin_amdgcn_readlane(pj, j), tp = __builtin_amdgcn_readlane(tpj, j);
            const float mrg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(mj), j));
            const PairDev* P = v.pairs + pair;
            const CloudDev ct = v.clouds[P->tgt];
            single_one<D>(v, P, pair, TR, ct, gx, g, lane, &n_eval, &n_box, &n_use, kSingleBatch > 1 ? tp : -2, mrg);
#ifdef SE3ICP_PROF
            ++n_sq;
#endif
        }
    }
#ifdef SE3ICP_PROF
    if ((int)(D == 3) & (int)(lane == 0) & (int)(n_sq > 0)) {
        const unsigned long long dt = __builtin_amdgcn_s_memrealtime() - t_s0;
        atomicAdd(&g_r3_prof[1][0], 1ull);
        atomicAdd(&g_r3_prof[1][1], dt);
        atomicMax(&g_r3_prof[1][2], dt);
        atomicAdd(&g_r3_prof[1][3], (unsigned long long)n_sq);
    }
#endif
    if ((int)(lane == 0) & (int)(n_eval + n_box > 0)) {
        unsigned long long* st = v.stats + kStatCols * (w0 & 63) + (D == 12 ? 0 : 2);
        atomicAdd(st, 64ull * n_eval);
        atomicAdd(st + 1, 64ull * n_box);
        atomicAdd(v.stats + kStatCols * (w0 & 63) + (D == 12 ? kStatUseSe3 : kStatUseR3), (unsigned long long)n_use);
    }
}

}  // namespace

void nn_prof_report() {
#ifdef SE3ICP_PROF
    unsigned long long h[6];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_prep_prof), sizeof(h)) != hipSuccess) return;
    if (h[3])
        std::fprintf(stderr, "[prof] k_nn_prep per block: settle %.2f pack %.2f lists %.2f us (%llu blocks)\n",
                     h[0] / 100.0 / h[3], h[1] / 100.0 / h[3], h[2] / 100.0 / h[3], h[3]);
    const unsigned long long z[6] = {0, 0, 0, 0, 0, 0};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_prep_prof), z, sizeof(z));
#endif
}
#ifdef SE3ICP_PROF
// the SE(3) group waves since the last call: duration histogram (25 us bins: count, share of
// the summed wave time) and the span from the first wave start to the last wave end; reset
void nn_wave_report(int it) {
    unsigned long long h[2][41], sp[2];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_wave_hist), sizeof(h)) != hipSuccess) return;
    if (hipMemcpyFromSymbol(sp, HIP_SYMBOL(g_wave_span), sizeof(sp)) != hipSuccess) return;
    double tot = 0, n = 0;
    for (int b = 0; b < 41; ++b) { tot += (double)h[1][b]; n += (double)h[0][b]; }
    std::fprintf(stderr, "[nn] iter %d: %.0f group waves, span %.1f us; summed wave time / 4096 slots %.1f us; "
                 "durations (25 us bins):", it, n, sp[1] > sp[0] ? (sp[1] - sp[0]) / 100.0 : 0.0, tot / 100.0 / 4096.0);
    for (int b = 0; b < 41; ++b)
        if (h[0][b]) std::fprintf(stderr, " %d:%llu/%.1f%%", 25 * b, h[0][b], 100.0 * (double)h[1][b] / std::max(tot, 1.0));
    std::fprintf(stderr, "\n");
    unsigned long long xp[8][3];
    if (hipMemcpyFromSymbol(xp, HIP_SYMBOL(g_xcd_prof), sizeof(xp)) == hipSuccess && sp[1] > sp[0]) {
        std::fprintf(stderr, "[nn] iter %d: per XCD summed wave time / 512 slots, last wave end after the first start, waves (us):", it);
        for (int x = 0; x < 8; ++x)
            std::fprintf(stderr, " %d:%.1f/%.1f/%llu", x, xp[x][0] / 100.0 / 512.0,
                         xp[x][1] > sp[0] ? (xp[x][1] - sp[0]) / 100.0 : 0.0, xp[x][2]);
        std::fprintf(stderr, "\n");
        const unsigned long long zx[8][3] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_xcd_prof), zx, sizeof(zx));
        unsigned long long xl[8][3];
        if (hipMemcpyFromSymbol(xl, HIP_SYMBOL(g_xcd_life), sizeof(xl)) == hipSuccess) {
            std::fprintf(stderr, "[nn] iter %d: per XCD block lifetimes / 512 slots: working, empty (count) (us):", it);
            for (int x = 0; x < 8; ++x)
                std::fprintf(stderr, " %d:%.1f,%.1f(%llu)", x, xl[x][0] / 100.0 / 512.0, xl[x][1] / 100.0 / 512.0, xl[x][2]);
            std::fprintf(stderr, "\n");
            (void)hipMemcpyToSymbol(HIP_SYMBOL(g_xcd_life), zx, sizeof(zx));
        }
    }
    unsigned long long r3[2][4];
    if (hipMemcpyFromSymbol(r3, HIP_SYMBOL(g_r3_prof), sizeof(r3)) == hipSuccess && (r3[0][0] | r3[1][0])) {
        std::fprintf(stderr, "[nn] iter %d: R3 group waves %llu (%llu queries), mean %.1f us, longest %.1f us; single-list waves "
                     "%llu (%llu queries), mean %.1f us, longest %.1f us\n", it, r3[0][0], r3[0][3],
                     r3[0][0] ? r3[0][1] / 100.0 / r3[0][0] : 0.0, r3[0][2] / 100.0, r3[1][0], r3[1][3],
                     r3[1][0] ? r3[1][1] / 100.0 / r3[1][0] : 0.0, r3[1][2] / 100.0);
        const unsigned long long z3[2][4] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_r3_prof), z3, sizeof(z3));
    }
    unsigned long long z[2][41] = {};
    const unsigned long long zs[2] = {~0ull, 0ull};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wave_hist), z, sizeof(z));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_wave_span), zs, sizeof(zs));
}
// span of the last k_nn_prep launch (us), reset for the next
double nn_prep_span() {
    unsigned long long h[2];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_prep_span), sizeof(h)) != hipSuccess) return 0.0;
    const unsigned long long z[2] = {~0ull, 0ull};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_prep_span), z, sizeof(z));
    return h[1] > h[0] ? (h[1] - h[0]) / 100.0 : 0.0;
}
#endif
size_t nn_cls_words(int nchunks) { return (size_t)kClsHead + (size_t)kClsHead * cls_cap(nchunks); }
void launch_nn_prep(const View& v, int32_t* publish, hipStream_t s) {
    hipLaunchKernelGGL(k_nn_prep, dim3(v.nchunks), dim3(kChunkQ), 0, s, v, publish);
}
// kSingleWaves single-query waves, then 16 groups of 64 per chunk, one wave each
void launch_nn(const View& v, int D, hipStream_t s) {
    const dim3 grid(kSingleWaves + v.nchunks * (kChunkQ / 64));
    if (D == 12) hipLaunchKernelGGL((k_nn_search<12, true>), grid, dim3(64), 0, s, v);
    else if (order3(v.npairs)) hipLaunchKernelGGL((k_nn_search<3, true>), grid, dim3(64), 0, s, v);
    else hipLaunchKernelGGL((k_nn_search<3, false>), grid, dim3(64), 0, s, v);
}

}  // namespace se3icp
