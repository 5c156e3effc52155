// k_lrf8.hip — the setup's per-point local geometry, eight queries per wavefront:
//   exact kNN-k of every point in its own cloud (KDTreeFlann::SearchKNN, ISR.cpp:253),
//   the TOLDI frame -> alpha/beta-weighted SE(3) 12-vector (ISR.cpp:241-316, 597-607),
//   Open3D EstimateNormals (ISR.cpp:643, :43) and the GICP covariance (ISR.cpp:33-52).
//
// A wavefront takes 8 consecutive points of the 3-D kd-tree order (one cloud).  They lie
// in one or two leaves and share almost all of their neighbourhoods, so the leaves are
// scanned once for all eight: each lane holds one point of the leaf and computes its
// distance to the eight queries (f64, nanoflann arithmetic), and every query appends the
// points within its own bound to its LDS candidate list.  The ordering work that a
// one-query-per-wave kernel spends 64 lanes on is done by eight lanes per query, for the
// eight queries at once, with key-only bitonic networks that run mostly inside registers:
//   * key = f32 bits of the squared distance rounded up (monotone in the f64 distance);
//     the lists hold it cut to its top 20 bits, packed with a 12-bit candidate id;
//   * bound: the Kw-th smallest packed key with the id bits set (sort of the candidates of
//     the first leaves, again whenever a list would overflow), then only candidates at or
//     below it are kept (a cut key keeps a few extra candidates, never loses one);
//   * the TOLDI / normal sums are sums over rank SETS (ranks 1..rz-1, 1..rz, 1..kk-1,
//     0..kn-1; the reference sums them sequentially, the order changes rounding only),
//     so the final pass needs the keys at the set boundaries, not a sorted list: a sort
//     of the full keys (recomputed from the points) gives them, and each candidate is
//     classified by comparing its key with them.
// A boundary whose two keys are equal (an f32 tie, or duplicate points at distance 0)
// cannot be resolved from keys: that query is handed to the exact one-query-per-wave
// kernel (k_knn.hip k_lrf over a list), as are a cloud's last, partial, wave, clouds with
// k > kCap - 64, and waves that scan more than kLeaves leaves.  Waves are aligned to the
// start of each cloud, so a point's result does not depend on the batch around its cloud.  Every other query gets exactly the
// reference's neighbour sets (ties by lowest index never arise: its boundaries are strict).
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

#ifndef SE3ICP_LRF8_WAVES
#define SE3ICP_LRF8_WAVES 4
#endif
constexpr int kW = SE3ICP_LRF8_WAVES;  // waves per block
constexpr int kQ = 8;     // queries per wave (eight lanes each in the group phases)
#ifndef SE3ICP_LRF8_CAP
#define SE3ICP_LRF8_CAP 192
#endif
// candidates buffered per query (u32: cut key | candidate id); round 5, C4 64 pairs: 224
// (5 waves per SIMD) +7 %, 256 (4 waves) +22 % k_lrf8 time -- occupancy beats the tighter
// first bound a larger accept-all fill gives
constexpr int kCap = SE3ICP_LRF8_CAP;
#ifndef SE3ICP_LRF8_FILL
#define SE3ICP_LRF8_FILL SE3ICP_LRF8_CAP
#endif
// the accept-all fill stops before a leaf would pass this (round 5, C4 64 pairs: 128 or 160
// instead of 192 -- a cheaper first tightening from fewer points -- made k_lrf8 8 % slower:
// the looser first bound opens more leaves and costs more tightenings later)
constexpr int kFill = SE3ICP_LRF8_FILL;
// LDS stride of the lists: 196 entries = 49 16-B slots, odd, so that the lane-major
// ds_read_b128 of a 128-entry run (lane l of group g: entries 16 l .. 16 l + 15) puts every
// 16-lane bank group on 16 distinct slots of the 256-B bank row (conflict-free), and the
// lane-major ds_read_b32 of an unaligned run is 4-way instead of 16-way
constexpr int kStride = kCap + 4;
static_assert(((kStride / 4) & 1) == 1, "an odd number of 16-B slots per list");
constexpr int kLeaves = 64;              // leaves one wave may scan: candidate id = (list index << 6) | lane
constexpr unsigned kIdBits = 0xfffu;     // low bits of a list entry: the candidate id
// bound of the accept-all phase: every finite key (a lane past the leaf's end carries an
// infinite distance, so its entry is above every bound)
constexpr unsigned kAll = 0x7f7fffffu;
constexpr unsigned kPad = 0xffffffffu;   // sort padding (> every entry)

// park slots per query (doubles)
enum Park8 {
    P8_SUM = 0,     // 21 neighbour sums, later the 6 TOLDI axis sums
    P8_R = 21, P8_KK = 22, P8_GP = 23, P8_FLAGS = 24, P8_K = 25, P8_NTOP = 26, P8_ZN = 27,
    P8_W = 30,                // the query's tree slot
    P8_N = 31
};
constexpr int kParkAt = 128;  // list entry where the park starts (8-byte aligned)
static_assert(kCap >= kParkAt + 2 * P8_N && kStride >= kCap, "the park overlays the list tail");

// lane ^ m within a group of eight lanes (m = 1..7 as used by the networks)
__device__ __forceinline__ unsigned gx(unsigned x, int m) {
    switch (m) {
    case 1: return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);   // quad_perm [1,0,3,2]
    case 2: return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);   // quad_perm [2,3,0,1]
    case 3: return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x1B, 0xF, 0xF, true);   // quad_perm [3,2,1,0]
    case 4: return (unsigned)__builtin_amdgcn_ds_swizzle((int)x, 0x101F);                      // xor 4
    case 7: return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x141, 0xF, 0xF, true);  // row_half_mirror
    default: return (unsigned)__shfl_xor((int)x, m, 64);
    }
}
__device__ __forceinline__ double gxd(double x, int m) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(x);
    const unsigned lo = gx((unsigned)u, m), hi = gx((unsigned)(u >> 32), m);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// the median of (a, b, x): min(a, b) for x = 0, max(a, b) for x = ~0u -- a cross-lane
// compare-exchange in one instruction after the partner's value is fetched (instead of a
// min, a max and a lane select)
__device__ __forceinline__ unsigned med3u(unsigned a, unsigned b, unsigned x) {
    unsigned r;
    asm("v_med3_u32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(x));
    return r;
}

// Ascending bitonic sort of the 8*PER keys of a group of eight lanes (element e =
// l*PER + s in k[s] of group lane l), every comparator ascending (each merge starts with
// the "flip" step e <-> e ^ (KK-1)): an in-register compare-exchange is a min and a max,
// a cross-lane one the partner's value (DPP / swizzle) and a med3 against 0 (the lower
// lane keeps the min) or ~0 (the upper lane keeps the max).
// Stages are instantiated at compile time (template recursion) so that every register
// index is a constant.
template <int PER, int KK, int JD>
__device__ __forceinline__ void stage8(unsigned (&k)[PER], int l) {
    if constexpr (JD == 0) {  // flip
        if constexpr (KK <= PER) {
#pragma unroll
            for (int s = 0; s < PER; ++s) {
                const int t = s ^ (KK - 1);
                if (s < t) {
                    const unsigned a = k[s], b = k[t];
                    k[s] = min(a, b);
                    k[t] = max(a, b);
                }
            }
        } else {
            constexpr int lm = KK / PER - 1;
            const unsigned x = (l & (KK / PER / 2)) == 0 ? 0u : ~0u;  // lower lane: min
#pragma unroll
            for (int s = 0; s < PER / 2; ++s) {
                const int t = PER - 1 - s;
                const unsigned a = gx(k[t], lm), b = gx(k[s], lm);
                k[s] = med3u(k[s], a, x);
                k[t] = med3u(k[t], b, x);
            }
        }
    } else if constexpr (JD < PER) {
#pragma unroll
        for (int s = 0; s < PER; ++s) {
            if ((s & JD) == 0) {
                const int t = s | JD;
                const unsigned a = k[s], b = k[t];
                k[s] = min(a, b);
                k[t] = max(a, b);
            }
        }
    } else {
        constexpr int lm = JD / PER;
        const unsigned x = (l & lm) == 0 ? 0u : ~0u;  // lower lane: min
#pragma unroll
        for (int s = 0; s < PER; ++s) k[s] = med3u(k[s], gx(k[s], lm), x);
    }
}
template <int PER, int N, int KK = 2, int JD = 0>
__device__ __forceinline__ void net8(unsigned (&k)[PER], int l) {
    stage8<PER, KK, JD>(k, l);
    constexpr int next_jd = JD == 0 ? KK / 4 : JD / 2;
    if constexpr (next_jd > 0) net8<PER, N, KK, next_jd>(k, l);
    else if constexpr (KK < N) net8<PER, N, KK * 2, 0>(k, l);
}
template <int PER>
__device__ __forceinline__ void sort8(unsigned (&k)[PER], int l) {
    net8<PER, 8 * PER>(k, l);
}

// Lane-major access of a run at a 16-B aligned list base: entry e = l * PER + s in k[s],
// one ds_read_b128 / ds_write_b128 per four entries.  Entries past len read as kPad; a
// store writes whole quads (a quad's entries past len land in free list space: the aligned
// runs are the list's head, and a head that is followed by a tail is exactly 128 long).
template <int PER>
__device__ __forceinline__ void load_head(const unsigned* list, int len, int l, unsigned (&k)[PER]) {
#pragma unroll
    for (int q = 0; q < PER / 4; ++q) {
        const int e0 = l * PER + 4 * q;
        uint4 x = make_uint4(kPad, kPad, kPad, kPad);
        if (e0 < len) x = *reinterpret_cast<const uint4*>(list + e0);
        k[4 * q] = x.x;
        k[4 * q + 1] = e0 + 1 < len ? x.y : kPad;
        k[4 * q + 2] = e0 + 2 < len ? x.z : kPad;
        k[4 * q + 3] = e0 + 3 < len ? x.w : kPad;
    }
}
template <int PER>
__device__ __forceinline__ void store_head(unsigned* list, int len, int l, const unsigned (&k)[PER], unsigned add = 0u) {
#pragma unroll
    for (int q = 0; q < PER / 4; ++q) {
        const int e0 = l * PER + 4 * q;
        if (e0 < len)
            *reinterpret_cast<uint4*>(list + e0) =
                make_uint4(k[4 * q] + add, k[4 * q + 1] + add, k[4 * q + 2] + add, k[4 * q + 3] + add);
    }
}
// sort the head run list[0 .. len) (len <= 8 * PER, list 16-B aligned) in place
template <int PER = 16>
__device__ __forceinline__ void sort_head(unsigned* list, int len, int l) {
    unsigned k[PER];
    load_head<PER>(list, len, l, k);
    sort8<PER>(k, l);
    __builtin_amdgcn_wave_barrier();
    store_head<PER>(list, len, l, k);
    __builtin_amdgcn_wave_barrier();
}
// sort the run list[0 .. len) (len <= 8 * PER, any alignment) in place
template <int PER = 16>
__device__ __forceinline__ void sort_run(unsigned* list, int len, int l) {
    unsigned k[PER];
#pragma unroll
    for (int s = 0; s < PER; ++s) {
        const int e = l * PER + s;
        k[s] = e < len ? list[e] : kPad;
    }
    sort8<PER>(k, l);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int s = 0; s < PER; ++s) {
        const int e = l * PER + s;
        if (e < len) list[e] = k[s];
    }
    __builtin_amdgcn_wave_barrier();
}
// |f32 squared distance of the f32-rounded points - exact squared distance of the f64
// points| for distances <= d (loopdev.hpp f32_err, D = 3); S bounds the sum of the norms
__device__ __forceinline__ float f32_err3(float d, float S) {
    const float u = 5.9604645e-08f;
    return 1.25f * (2.f * u * S * sqrtf(fmaxf(d, 0.f)) + 6.f * u * d + 4.f * u * u * S * S) + 1e-30f;
}
// the list bound from the Kw-th smallest entry t (f32 keys): every point whose exact
// distance is within the Kw-th smallest exact distance has an f32 key <= the value of t
// plus two errors
__device__ __forceinline__ unsigned widen_bound(unsigned t, float S) {
    if (t >= 0x7f800000u) return kAll;
    const float b = __uint_as_float(t);
    return min((__float_as_uint(fmaf(2.02f, f32_err3(b, S), b)) + 2u) | kIdBits, kAll);
}
// number of entries <= t in the sorted run A[0 .. n)
__device__ __forceinline__ int upper_count(const unsigned* A, int n, unsigned t) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int m = (lo + hi) >> 1;
        if (A[m] <= t) lo = m + 1; else hi = m;
    }
    return lo;
}
// entry of rank r of the union of two sorted runs A (na) and B (nb) (distinct entries):
// i entries of A and r+1-i of B are the r+1 smallest; binary search on i
__device__ __forceinline__ unsigned kth_of_two(const unsigned* A, int na, const unsigned* B, int nb, int r) {
    int lo = max(0, r + 1 - nb), hi = min(r + 1, na);
    while (lo < hi) {
        const int i = (lo + hi) >> 1;
        if (A[i] < B[r - i]) lo = i + 1; else hi = i;
    }
    const int j = r + 1 - lo;
    return max(lo > 0 ? A[lo - 1] : 0u, j > 0 ? B[j - 1] : 0u);
}
// Bound tightening over a list whose first mv entries are already sorted (the kept set of
// the previous tightening): only the tail appended since is sorted, the Kw-th entry is
// found by a merge-path search of the two runs, and the kept parts of both runs are merged
// by a bitonic half-cleaner network (A ascending, padding, B descending: one bitonic
// sequence of 128), so the kept list stays sorted for the next tightening.
//   presort (wave-uniform): some list has no sorted prefix (the first tightening) or a
//           tail over 128: list[0 .. min(nbg, 128)) is sorted first;
//   tail_per (wave-uniform): 0 every tail empty, 8 every tail <= 64 entries, else 16.
// Returns (bound, kept, new sorted prefix) for the group; kept sets over 128 entries (ties
// at the bound) are compacted unmerged (prefix 0).
__device__ __forceinline__ uint3 tighten_group_sorted(unsigned* lists, int g, int l, int nbg, int mv, int nmax, int Kw,
                                                      bool presort, int tail_per, float S) {
    unsigned* list = lists + g * kStride;
    if (presort) {
        mv = min(nbg, 128);
        sort_head<16>(list, mv, l);
    }
    const int nb = nbg - mv;
    unsigned* B = list + mv;
    if (tail_per == 8) sort_run<8>(B, nb, l);
    else if (tail_per == 16) sort_run<16>(B, nb, l);
    const unsigned tg = nbg >= Kw ? widen_bound(kth_of_two(list, mv, B, nb, Kw - 1) | kIdBits, S) : kAll;
    const int ka = upper_count(list, mv, tg), kb = upper_count(B, nb, tg);
    const int kept = ka + kb;
    if (__ballot(kept > 128) == 0ull) {
        unsigned k[16];
        load_head<16>(list, ka, l, k);
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const int e = l * 16 + s;
            if (e >= 128 - kb) k[s] = B[127 - e];
        }
        __builtin_amdgcn_wave_barrier();
        stage8<16, 128, 64>(k, l);
        stage8<16, 128, 32>(k, l);
        stage8<16, 128, 16>(k, l);
        stage8<16, 128, 8>(k, l);
        stage8<16, 128, 4>(k, l);
        stage8<16, 128, 2>(k, l);
        stage8<16, 128, 1>(k, l);
        store_head<16>(list, kept, l, k);
        __builtin_amdgcn_wave_barrier();
        return make_uint3(tg, (unsigned)kept, (unsigned)kept);
    }
    // (rare) stable compaction in place, as tighten_group
    unsigned keep_n = 0;
    for (int r0 = 0; r0 < nmax; r0 += 8) {
        const int e = r0 + l;
        const unsigned ent = e < nbg ? list[e] : kPad;
        const bool keep = ent <= tg;
        const unsigned long long m = __ballot(keep);
        const unsigned gm = (unsigned)(m >> (8 * g)) & 0xffu;
        __builtin_amdgcn_wave_barrier();
        if (keep) list[(int)keep_n + __popc(gm & ((1u << l) - 1u))] = ent;
        keep_n += (unsigned)__popc(gm);
        __builtin_amdgcn_wave_barrier();
    }
    return make_uint3(tg, keep_n, 0u);
}

// the f64 point of tree slot i from its (x, y, z, 0) record: one 16-B and one 8-B load of
// one cache line (the unused fourth word is not loaded)
struct p3 { double x, y, z; };
__device__ __forceinline__ p3 ld3(const double4* __restrict__ P4, int i) {
    const double2 xy = *reinterpret_cast<const double2*>(P4 + i);
    const double z = reinterpret_cast<const double*>(P4 + i)[2];
    return p3{xy.x, xy.y, z};
}

// The final list of the group's query (nbg <= 128 entries) in rank order.  The list
// entries (cut key | id) sorted as u32 give the rank order up to runs whose full keys the
// cut does not separate; the full keys ((f32 of the exact f64 distance, nanoflann's
// arithmetic) << 32 | tree slot) of that order are put right by three odd-even
// transposition passes and checked, and the tree slots are written back over the list in
// rank order.  Two adjacent ranks the sums use that share an f32 key are put in the exact
// order -- (f64 distance, point index): the reference's kNN and the exact kernel's -- by a
// swap when no neighbouring rank shares their key.  Returns false (the query goes to the
// exact kernel) when the order is still wrong, or when a run of three or more ranks shares
// an f32 key and is not already in the exact order.
__device__ __forceinline__ bool final_group(unsigned* lists, const int* leaf_slot, const double4* __restrict__ P4,
                                            const int32_t* __restrict__ perm, double qx, double qy, double qz, int off,
                                            int g, int l, int nbg, int mv, int fmode, int lim) {
    unsigned* list = lists + g * kStride;
    unsigned long long k[16];
    bool unsorted = false;
    {
        unsigned k32[16];
        // fmode (wave-uniform): 0 a full sort; 1 the sorted prefix list[0 .. mv) (the last
        // tightening's kept set) merged with the tail appended since (<= 64 entries, sorted
        // first), as tighten_group_sorted merges; 2 the tail is empty (already in order)
        if (fmode == 0) {
            load_head<16>(list, nbg, l, k32);
            sort8<16>(k32, l);
        } else {
            const int nb = nbg - mv;
            unsigned* B = list + mv;
            if (fmode == 1) sort_run<8>(B, nb, l);
            load_head<16>(list, mv, l, k32);
            if (fmode == 1) {
#pragma unroll
                for (int s = 0; s < 16; ++s) {
                    const int e = l * 16 + s;
                    if (e >= 128 - nb) k32[s] = B[127 - e];
                }
                __builtin_amdgcn_wave_barrier();
                stage8<16, 128, 64>(k32, l);
                stage8<16, 128, 32>(k32, l);
                stage8<16, 128, 16>(k32, l);
                stage8<16, 128, 8>(k32, l);
                stage8<16, 128, 4>(k32, l);
                stage8<16, 128, 2>(k32, l);
                stage8<16, 128, 1>(k32, l);
            }
        }
#pragma unroll
        for (int s = 0; s < 16; ++s) {
            const int e = l * 16 + s;
            unsigned long long x = ~0ull;
            if (e < nbg) {
                const unsigned id = k32[s] & kIdBits;
                const int slot = leaf_slot[id >> 6] + (int)(id & 63u);
                const p3 p = ld3(P4, slot);
                const unsigned key = __float_as_uint((float)l2_3(qx, qy, qz, p.x, p.y, p.z));
                x = ((unsigned long long)key << 32) | (unsigned)(slot - off);
            }
            k[s] = x;
        }
    }
    auto ce = [](unsigned long long& a, unsigned long long& b) __attribute__((always_inline)) {
        const bool sw = b < a;
        const unsigned long long lo = sw ? b : a, hi = sw ? a : b;
        a = lo;
        b = hi;
    };
    const int me = (int)(threadIdx.x & 63);
    auto next_first = [&]() __attribute__((always_inline)) {  // lane l + 1's k[0] (within the group for l < 7)
        return ((unsigned long long)(unsigned)__shfl((int)(unsigned)(k[0] >> 32), me + 1, 64) << 32) |
               (unsigned)__shfl((int)(unsigned)k[0], me + 1, 64);
    };
#pragma unroll
    for (int s = 0; s < 16; s += 2) ce(k[s], k[s + 1]);
    {
#pragma unroll
        for (int s = 1; s + 1 < 16; s += 2) ce(k[s], k[s + 1]);
        // (lane l's last, lane l+1's first) within the group of eight
        const unsigned long long nx = next_first();
        const unsigned long long pv = ((unsigned long long)(unsigned)__shfl((int)(unsigned)(k[15] >> 32), me - 1, 64) << 32) |
                                      (unsigned)__shfl((int)(unsigned)k[15], me - 1, 64);
        if (l < 7 && nx < k[15]) k[15] = nx;
        if (l > 0 && k[0] < pv) k[0] = pv;
    }
#pragma unroll
    for (int s = 0; s < 16; s += 2) ce(k[s], k[s + 1]);
    const unsigned long long nx = next_first();
#pragma unroll
    for (int s = 0; s + 1 < 16; ++s) unsorted |= k[s + 1] < k[s];
    unsorted |= (l < 7) && nx < k[15];
    // adjacent ranks sharing an f32 key (bit s: ranks l*16+s and +1): tall over the list,
    // tied among the first lim (the ranks the sums use, and the one after them)
    unsigned tall = 0u;
#pragma unroll
    for (int s = 0; s + 1 < 16; ++s) {
        const int e = l * 16 + s;
        if ((int)(e + 1 < nbg) & (int)((unsigned)(k[s] >> 32) == (unsigned)(k[s + 1] >> 32))) tall |= 1u << s;
    }
    {
        const int e = l * 16 + 15;
        if ((int)(l < 7) & (int)(e + 1 < nbg) & (int)((unsigned)(k[15] >> 32) == (unsigned)(nx >> 32))) tall |= 1u << 15;
    }
    const int nlim = lim - 1 - l * 16;  // bits s < nlim have e + 1 < lim
    unsigned tied = tall & (nlim >= 16 ? 0xffffu : nlim > 0 ? (1u << nlim) - 1u : 0u);
    // a pair is isolated when neither neighbouring pair is tied (across the lanes of the group too)
    const unsigned tprev = (unsigned)__shfl((int)tall, me - 1, 64), tnext = (unsigned)__shfl((int)tall, me + 1, 64);
    const unsigned tall_lo = (tall << 1) | (l > 0 ? (tprev >> 15) & 1u : 0u);   // bit s: pair s-1 tied
    const unsigned tall_hi = (tall >> 1) | (l < 7 ? (tnext & 1u) << 15 : 0u);   // bit s: pair s+1 tied
    const unsigned isolated = ~(tall_lo | tall_hi);
    __builtin_amdgcn_wave_barrier();
    {
        unsigned sl[16];
#pragma unroll
        for (int s = 0; s < 16; ++s) sl[s] = (unsigned)k[s];
        store_head<16>(list, nbg, l, sl, (unsigned)off);
    }
    __builtin_amdgcn_wave_barrier();
    bool bad = unsorted;
    while (tied) {  // rare: the tree slots of the tied ranks, now in rank order in the list
        const int sb = __builtin_ctz(tied);
        const int e = l * 16 + sb;
        tied &= tied - 1u;
        const int a = (int)list[e], b = (int)list[e + 1];
        const p3 pa = ld3(P4, a), pb = ld3(P4, b);
        const double da = l2_3(qx, qy, qz, pa.x, pa.y, pa.z), db = l2_3(qx, qy, qz, pb.x, pb.y, pb.z);
        // the exact order is (f64 distance, point index); an isolated pair is put right by a
        // swap (its neighbours' f32 keys differ, so their ranks are settled), a longer run of
        // equal f32 keys goes to the exact kernel
        const bool wrong = (bool)((int)(da > db) | ((int)(da == db) & (int)(perm[a] > perm[b])));
        // (a run that continues past the checked ranks: which of its members fall inside is
        // not settled here)
        bad |= (bool)((int)(e + 2 >= lim) & (int)((tall_hi >> sb) & 1u));
        if (wrong) {
            if ((isolated >> sb) & 1u) {
                list[e] = (unsigned)b;
                list[e + 1] = (unsigned)a;
            } else {
                bad = true;
            }
        } else if (!((isolated >> sb) & 1u)) {
            bad |= da != db;  // (a run of three or more with distinct f64 distances)
        }
    }
    const bool ok = !(bool)(unsigned)((__ballot(bad) >> (8 * g)) & 0xffull);
    return ok;
}

// SE3ICP_PROF builds (make prof): per-section shader-clock cycles into stats columns 8..11
#ifdef SE3ICP_PROF
#define PROF8_NOW(t) const unsigned long long t = __builtin_readcyclecounter()
#define PROF8_ADD(acc, a, b) acc += (b) - (a)
#else
#define PROF8_NOW(t) do {} while (0)
#define PROF8_ADD(acc, a, b) do {} while (0)
#endif

static_assert(kW >= 2 && kW * kQ <= 64, "the per-block epilogue: waves 0 and 1, a lane per query");

// waves per SIMD: 6 = the LDS limit (26.6 KB per block); A/B 4 -> 5 -> 6: 6.73 -> 6.45 -> 6.38 ms
__global__ __launch_bounds__(64 * kW) __attribute__((amdgpu_waves_per_eu(kCap <= 192 ? 6 : (kCap <= 224 ? 5 : 4)))) void k_lrf8(
    View v, const int32_t* __restrict__ cloud_of, const CloudSetup* __restrict__ setup,
    const CloudDev* __restrict__ clouds, const float* __restrict__ tlo, const float* __restrict__ thi,
    const double4* __restrict__ P4, const int32_t* __restrict__ wave_base, int w_lo, int nwaves,
    int32_t* __restrict__ fb_list, int32_t* __restrict__ fb_count) {
    // (a query's park overlays the tail of its list, free once the list is final: <= 128 entries)
    __shared__ __attribute__((aligned(16))) unsigned s_list[kW][kQ][kStride];
    auto park_of = [&](int w, int j) __attribute__((always_inline)) {
        return reinterpret_cast<double*>(&s_list[w][j][kParkAt]);
    };
    __shared__ int s_leaf[kW][kLeaves];  // first tree slot of each scanned leaf
    __shared__ __attribute__((aligned(16))) float s_q[kW][3 * kQ];  // the queries' f32 x[8] y[8] z[8]
    // (wid through readfirstlane: the wave's LDS bases become scalar, not per-lane registers)
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 3, l = lane & 7;  // query of the lane's group, lane within the group
    const int bid = xcd_block(blockIdx.x, gridDim.x);
    const TreeRef T = v.t3;
    const int first_leaf = (1 << T.L) - 1;
    unsigned* lists = &s_list[wid][0][0];
    int* leaves = s_leaf[wid];
    unsigned n_leaves = 0, n_sel = 0, n_cand = 0, n_q = 0;
#ifdef SE3ICP_PROF
    unsigned long long c_scan = 0, c_tight = 0, c_sums = 0, c_epi = 0;
    unsigned n_tover = 0, n_tend = 0;  // tightenings for an overflowing leaf / for the final <= 128
    unsigned long long fb_cause = 0;     // 16-bit fields: leaf table full, no room, > 128 at the end, f32/f64 ties
#define PROF8_FB(field) fb_cause += 1ull << (16 * (field))
#else
#define PROF8_FB(field) do {} while (0)
#endif
    PROF8_NOW(t_a0);

    // ---------------------------------------------------------------- the wave's queries
    // Wave wv covers local points 8*(wv - wave_base[c]) .. +7 of cloud c (waves aligned to
    // each cloud's start).  mode 0: nothing to do (no kNN wanted, past the end); 1: this
    // kernel; 2: its queries go to the exact kernel (partial wave, k too large for the lists).
    const int wv = __builtin_amdgcn_readfirstlane(w_lo + bid * kW + wid);
    int mode = 0, c = 0, w0 = 0, qn = 0;
    CloudSetup st{};
    CloudDev cl{0, 0};
    int K = 0, Kw = 0;
    if (wv < nwaves) {
        int lo = 0, hi = v.nclouds - 1;  // last cloud with wave_base <= wv
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (wave_base[mid] <= wv) lo = mid; else hi = mid - 1;
        }
        c = lo;
        cl = clouds[c];
        st = setup[c];
        K = st.k_knn;
        w0 = cl.off + kQ * (wv - wave_base[c]);
        qn = min(kQ, cl.off + cl.n - w0);
        if (K > 0 && qn > 0) {
            Kw = min(K, cl.n);
            mode = (qn == kQ && Kw <= 128) ? 1 : 2;  // (the final order holds <= 128 entries)
        }
    }
    bool fb_wave = mode == 2;
    // per-query state: bound (wave-uniform arrays) and list lengths; the length of the lane's
    // own group is picked from them only where the group phases need it (group_len)
    unsigned Tq[kQ], nbq[kQ];
#pragma unroll
    for (int j = 0; j < kQ; ++j) { Tq[j] = kAll; nbq[j] = 0u; }
    auto group_len = [&]() __attribute__((always_inline)) {
        // lane 8 j gets nbq[j] (v_writelane), every lane reads its group's first lane (a
        // select chain over the scalars is turned into a scratch array indexed by g)
        int x = 0;
#pragma unroll
        for (int j = 0; j < kQ; ++j) asm volatile("v_writelane_b32 %0, %1, %2" : "+v"(x) : "s"(nbq[j]), "n"(8 * j));
        return (unsigned)__shfl(x, lane & ~7, 64);
    };
    int mvv = 0;  // sorted prefix of the group's list
    float* qv = s_q[wid];
    float fqlo[3] = {0.f, 0.f, 0.f}, fqhi[3] = {0.f, 0.f, 0.f};
    int nlist = 0;
    const int n = cl.n;
    float s_norm = 0.f;  // bound on |q| + |p| over the cloud, from its root box (f32 scan error)
    if (mode == 1) {
        // f32 box of the eight queries (the node boxes' frame)
        const float fx = lane < kQ ? T.tvec[w0 + lane] : 0.f;
        const float fy = lane < kQ ? T.tvec[v.ld + w0 + lane] : 0.f;
        const float fz = lane < kQ ? T.tvec[2 * (size_t)v.ld + w0 + lane] : 0.f;
        if (lane < kQ) {
            qv[lane] = fx;
            qv[kQ + lane] = fy;
            qv[2 * kQ + lane] = fz;
        }
        {
            const float* rlo = tlo + (size_t)c * T.nnodes * 3;
            const float* rhi = thi + (size_t)c * T.nnodes * 3;
            float r2 = 0.f;
#pragma unroll
            for (int a = 0; a < 3; ++a) r2 += fmaxf(rlo[a] * rlo[a], rhi[a] * rhi[a]);
            s_norm = 2.f * sqrtf(r2) * 1.0001f;
        }
        __builtin_amdgcn_wave_barrier();
        fqlo[0] = fqhi[0] = __shfl(fx, 0, 64);
        fqlo[1] = fqhi[1] = __shfl(fy, 0, 64);
        fqlo[2] = fqhi[2] = __shfl(fz, 0, 64);
#pragma unroll
        for (int j = 1; j < kQ; ++j) {
            const float a = __shfl(fx, j, 64), b = __shfl(fy, j, 64), d = __shfl(fz, j, 64);
            fqlo[0] = fminf(fqlo[0], a); fqhi[0] = fmaxf(fqhi[0], a);
            fqlo[1] = fminf(fqlo[1], b); fqhi[1] = fmaxf(fqhi[1], b);
            fqlo[2] = fminf(fqlo[2], d); fqhi[2] = fmaxf(fqhi[2], d);
        }
        n_q = kQ;
    }

    // ---------------------------------------------------------------- bound tightening
    auto tighten = [&]() __attribute__((always_inline)) {
        ++n_sel;
        unsigned nmax = 0;
#pragma unroll
        for (int j = 0; j < kQ; ++j) nmax = max(nmax, nbq[j]);
        __builtin_amdgcn_wave_barrier();
        int dmax = 0;
        bool anyz = false;
#pragma unroll
        for (int j = 0; j < kQ; ++j) {
            const int mj = __builtin_amdgcn_readlane(mvv, 8 * j);
            dmax = max(dmax, (int)nbq[j] - mj);
            anyz |= mj == 0;
        }
        const bool presort = anyz || dmax > 128;
        const int tail_per = presort ? (nmax <= 128 ? 0 : (nmax <= 192 ? 8 : 16)) : (dmax == 0 ? 0 : dmax <= 64 ? 8 : 16);
        const uint3 r3 = tighten_group_sorted(lists, g, l, (int)group_len(), mvv, (int)nmax, Kw, presort, tail_per, s_norm);
        mvv = (int)r3.z;
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < kQ; ++j) {
            Tq[j] = (unsigned)__builtin_amdgcn_readlane((int)r3.x, 8 * j);
            nbq[j] = (unsigned)__builtin_amdgcn_readlane((int)r3.y, 8 * j);
        }
    };

    // ---------------------------------------------------------------- leaf scan
    // Each lane holds one point of leaf i; query j appends it when its entry (cut key |
    // id) <= Tq[j].  part: 0 the whole leaf, 1 / 2 its first / second 32 points (a leaf that
    // does not fit a list even after a tightening is appended in two halves).  Lanes past
    // the part carry an infinite distance: their entries exceed every bound.
    auto scan_leaf = [&](int i, int part) __attribute__((always_inline)) -> bool {
        if (nlist >= kLeaves) { fb_wave = true; PROF8_FB(0); return true; }
        const int li = nlist++;
        ++n_leaves;
        const int a = __builtin_amdgcn_readfirstlane(tree_first(n, T.L, i));
        const int b = __builtin_amdgcn_readfirstlane(tree_first(n, T.L, i + 1));
        if (lane == 0) leaves[li] = cl.off + a;
        const bool valid = (bool)((int)(lane < b - a) & (int)(part == 0 || (part == 1) == (lane < 32)));
        const int slot = cl.off + a + (valid ? lane : 0);
        const unsigned id = (unsigned)((li << 6) | lane);
        unsigned ent[kQ];
        unsigned long long m[kQ];
        bool over = false;
        // the list key: the f32 squared distance of the f32 points (two queries per packed
        // instruction); the bounds carry its error (widen_bound), the final order uses exact keys
        float dq[kQ];
        {
            typedef float f2 __attribute__((ext_vector_type(2)));
            const float px = valid ? T.tvec[slot] : INFINITY;
            const float py = valid ? T.tvec[v.ld + slot] : INFINITY;
            const float pz = valid ? T.tvec[2 * (size_t)v.ld + slot] : INFINITY;
            const f2* qf2 = reinterpret_cast<const f2*>(qv);
            const f2 pxx = f2{px, px}, pyy = f2{py, py}, pzz = f2{pz, pz};
            // a - b as one v_pk_add_f32 (the compiler splits a broadcast operand into two v_sub_f32)
            auto pk_sub = [](f2 a, f2 b) __attribute__((always_inline)) {
                f2 r;
                asm("v_pk_add_f32 %0, %1, %2 neg_lo:[0,1] neg_hi:[0,1]" : "=v"(r) : "v"(a), "v"(b));
                return r;
            };
#pragma unroll
            for (int jp = 0; jp < kQ / 2; ++jp) {
                const f2 ex = pk_sub(qf2[jp], pxx), ey = pk_sub(qf2[kQ / 2 + jp], pyy), ez = pk_sub(qf2[kQ + jp], pzz);
                f2 s2 = ex * ex;
                s2 = __builtin_elementwise_fma(ey, ey, s2);
                s2 = __builtin_elementwise_fma(ez, ez, s2);
                dq[2 * jp] = s2.x;
                dq[2 * jp + 1] = s2.y;
            }
        }
#pragma unroll
        for (int j = 0; j < kQ; ++j) {
            ent[j] = (__float_as_uint(dq[j]) & ~kIdBits) | id;
            m[j] = __ballot(ent[j] <= Tq[j]);
            over |= nbq[j] + (unsigned)__popcll(m[j]) > (unsigned)kCap;
        }
        if (over) {  // a list would overflow: the caller tightens the bounds and rescans the leaf
            --nlist;
            --n_leaves;
            return false;
        }
#pragma unroll
        for (int j = 0; j < kQ; ++j) {
            if (ent[j] <= Tq[j]) {  // (the ballot's own compare: the exec mask, no bit test of m)
                const int at = (int)nbq[j] + __builtin_amdgcn_mbcnt_hi((unsigned)(m[j] >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m[j], 0u));
                lists[j * kStride + at] = ent[j];
            }
            nbq[j] += (unsigned)__popcll(m[j]);
        }
        __builtin_amdgcn_wave_barrier();
        return true;
    };

    if (mode == 1) {
        // The leaves holding the eight queries, then their tree-order neighbours, every
        // point accepted, until each query has Kw candidates: the first bound.
        const int lf0 = tree_node_of(w0 - cl.off, n, T.L), lf1 = tree_node_of(w0 + kQ - 1 - cl.off, n, T.L);
        const int nleaf = 1 << T.L;
        int s_lo = lf0, s_hi = lf1;
        // Then every leaf whose box may hold a point within the largest bound of the
        // eight (squared box-to-box distance from the queries' f32 box, f32 boxes inflated
        // to bound the f64 points): level-A nodes 64 per instruction, then the leaves of
        // each open one, scanned outward from the queries and re-tested as bounds shrink.
        auto thr_f = [&]() __attribute__((always_inline)) {
            unsigned tm = 0u;
#pragma unroll
            for (int j = 0; j < kQ; ++j) tm = max(tm, Tq[j]);
            return __uint_as_float(f32_up_bits((double)__uint_as_float(tm) * (1.0 + 2e-6)));
        };
        auto box_lb = [&](int h) __attribute__((always_inline)) {
            const float* lo = tlo + ((size_t)c * T.nnodes + h) * 3;
            const float* hi = thi + ((size_t)c * T.nnodes + h) * 3;
            float s = 0.f;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                const float e = fmaxf(fmaxf(lo[a] - fqhi[a], fqlo[a] - hi[a]), 0.f);
                s += e * e;
            }
            return s;
        };
        const int sh = T.L > 6 ? 6 : T.L;
        const int nA = 1 << (T.L - sh), firstA = nA - 1;
        // one loop, one scan site: stage 0 the queries' own leaves, 1 their tree-order
        // neighbours until Kw candidates exist (accept-all), 2 level-A nodes, 3 the leaves
        // of the current level-A node
        // A leaf that does not fit a list: tighten and retry; then its two halves (each
        // after a tightening if needed); still no room (massive ties at the bound): the
        // exact kernel.  One tightening site keeps the kernel's code and registers small.
        int stage = 0, nxt = lf0, c0 = 0, l0 = 0;
        bool up = true, haveA = false;
        float lbA = INFINITY, lbL = INFINITY;
        OutwardBits itA(0ull, 0), itL(0ull, 0);
        int cur = -1, part = 0;
        bool do_tighten = false, retried = false;
        float tf = INFINITY;  // f32 box-test bound of the union of the eight (set with each tightening)
        while (!fb_wave) {
            if (do_tighten) {
                PROF8_NOW(t_t0);
                tighten();
                PROF8_NOW(t_t1);
                PROF8_ADD(c_tight, t_t0, t_t1);
                do_tighten = false;
                tf = thr_f();  // the box-test bound changes only here
#if defined(SE3ICP_LRF8_CUT) && SE3ICP_LRF8_CUT == 4
                if (stage == 2) break;  // (measurement build: stop after the first bound)
#endif
            }
            if (cur >= 0) {  // appending leaf cur (part)
#if defined(SE3ICP_LRF8_CUT) && SE3ICP_LRF8_CUT == 5
                if (stage >= 2) { cur = -1; part = 0; ++n_leaves; continue; }  // (measurement build: no scans after the first bound)
#endif
                if (scan_leaf(cur, part)) {
                    if (part == 1) part = 2;
                    else { cur = -1; part = 0; }
                    retried = false;
                } else if (!retried && (int)nbq[0] >= Kw) {
                    do_tighten = true;
                    retried = true;
#ifdef SE3ICP_PROF
                    ++n_tover;
#endif
                } else if (part == 0) {
                    part = 1;
                    retried = false;
                } else {
                    fb_wave = true;
                    PROF8_FB(1);
                }
                continue;
            }
            int leaf = -1;
            if (stage == 0) {
                leaf = nxt++;
                if (nxt > lf1) stage = 1;
            } else if (stage == 1) {
                // (filling the lists beyond Kw while a whole leaf still fits: the first
                // bound, the Kw-th of more nearby points, is tighter)
                const bool more_hi = s_hi < nleaf - 1, more_lo = s_lo > 0;
                const int cand = (more_hi && (up || !more_lo)) ? s_hi + 1 : s_lo - 1;
                const int csz = (more_hi || more_lo) ? tree_first(n, T.L, cand + 1) - tree_first(n, T.L, cand) : 0;
                if ((more_hi || more_lo) && ((int)nbq[0] < Kw || (int)nbq[0] + csz <= kFill)) {
                    leaf = cand;
                    if (cand > s_hi) s_hi = cand; else s_lo = cand;
                    up = !up;
                } else {
                    do_tighten = true;
                    stage = 2;
                    continue;
                }
            } else if (stage == 2) {
                if (!haveA) {
                    if (c0 >= nA) {  // done; the final sort takes lists of <= 128: tighten once more
                        unsigned nmax = 0;
#pragma unroll
                        for (int j = 0; j < kQ; ++j) nmax = max(nmax, nbq[j]);
                        if (nmax > 128 && !retried) {
#ifdef SE3ICP_PROF
                            ++n_tend;
#endif
                            do_tighten = true;
                            retried = true;
                            continue;
                        }
                        if (nmax > 128) { fb_wave = true; PROF8_FB(2); }  // (ties at the bound)
                        break;
                    }
                    const int ai = c0 + lane;
                    lbA = ai < nA ? box_lb(firstA + ai) : INFINITY;
                    itA = OutwardBits(__ballot(lbA <= tf), (lf0 >> sh) - c0);
                    haveA = true;
                }
                const int j = itA.next();
                if (j < 0) { haveA = false; c0 += 64; continue; }
                if (!(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(lbA), j)) <= tf)) continue;
                l0 = (c0 + j) << sh;
                const int li = l0 + lane;
                lbL = INFINITY;
                if ((int)(lane < (1 << sh)) & ((int)(li < s_lo) | (int)(li > s_hi))) lbL = box_lb(first_leaf + li);
                itL = OutwardBits(__ballot(lbL <= tf), lf0 - l0);
                stage = 3;
                continue;
            } else {
                const int t = itL.next();
                if (t < 0) { stage = 2; continue; }
                if (!(__int_as_float(__builtin_amdgcn_readlane(__float_as_int(lbL), t)) <= tf)) continue;
                leaf = l0 + t;
            }
            cur = leaf;
        }
    }
    __builtin_amdgcn_wave_barrier();

    PROF8_NOW(t_a1);
#if defined(SE3ICP_LRF8_CUT) && (SE3ICP_LRF8_CUT == 1 || SE3ICP_LRF8_CUT == 4 || SE3ICP_LRF8_CUT == 5)
    if (lane == 0 && n_leaves == 12345u) v.stats[0] = nlist;  // (measurement build: stop after the traversal)
    return;
#endif
    PROF8_ADD(c_scan, t_a0, t_a1);
    // ---------------------------------------------------------------- final sets
    // Each list in rank order by exact key (ties by point index); every set boundary must
    // be strict (else the query goes to the exact kernel).
    const int kl = st.k_lrf, kn_want = st.k_nrm;
    const bool want_t = kl > 0, want_n = kn_want > 0;
    bool fb_q = fb_wave;  // (group-uniform)
    const int nbg = (int)group_len();
    const int nTop = min(Kw, nbg);
    const int kk = min(kl, nTop), kn = min(kn_want, nTop);
    const int wq = w0 + g;
    // the group's f64 query (final order, sums)
    p3 qg{0.0, 0.0, 0.0};
    if (mode == 1) qg = ld3(P4, wq);
    if (mode == 1 && !fb_wave) {
        __builtin_amdgcn_wave_barrier();
        int fmode = 0;
        {
            int dmax = 0;
            bool anyz = false;
#pragma unroll
            for (int j = 0; j < kQ; ++j) {
                const int mj = __builtin_amdgcn_readlane(mvv, 8 * j);
                dmax = max(dmax, (int)nbq[j] - mj);
                anyz |= mj == 0;
            }
            fmode = anyz || dmax > 64 ? 0 : dmax == 0 ? 2 : 1;
        }
        const bool exact = final_group(lists, leaves, P4, T.perm, qg.x, qg.y, qg.z, cl.off, g, l, nbg, mvv, fmode,
                                       min(nbg, max(kk, kn) + 1));
        fb_q = (bool)((int)!exact | (int)(nTop < Kw));
        n_cand += (unsigned)nbg;
#ifdef SE3ICP_PROF
        fb_cause += (unsigned long long)__popcll(__ballot((int)fb_q & (int)(l == 0) & (int)(g < qn))) << 48;
#endif
    }
    // queries for the exact kernel
    if ((int)(mode != 0) & (int)fb_q & (int)(l == 0) & (int)(g < qn)) {
        const int at = atomicAdd(fb_count, 1);
        fb_list[at] = wq;
        atomicAdd(v.stats + kStatCols * (wv & 63) + 6, 1ull);  // (bench diagnostics: hand-overs)
    }
    const bool mine = (bool)((int)(mode == 1) & (int)!fb_q);

#if defined(SE3ICP_LRF8_CUT) && SE3ICP_LRF8_CUT == 2
    if (lane == 0 && n_cand == 12345u) v.stats[0] = n_cand;  // (measurement build: stop after the final order)
    return;
#endif
    // ---------------------------------------------------------------- per-query sums
    // (group g, list entries l, l+8, ...; see k_knn.hip for the 21 sums and the TOLDI
    // covariance about the quirk centroid, ISR.cpp:259-272).  The same loops, lane
    // assignment and arithmetic as k_knn.hip's sums pass, over the same rank order, so the
    // two kernels' frames agree bit for bit; the TOLDI and the normal sums are two passes
    // (their live registers do not add up).
    const unsigned* rl = lists + g * kStride;
    double* pj = park_of(wid, g);
    {
        double x[12];
#pragma unroll
        for (int i = 0; i < 12; ++i) x[i] = 0.0;
        double Rf = 0.0;
        if ((int)mine & (int)want_t) {
            const int rz = kk / 3;
            const int hi = min(rz, kk - 1);
            // (each iteration loads the next one's point first: the loads overlap the sums;
            // the last prefetch re-reads rank hi)
            p3 pn = ld3(P4, (int)rl[max(min(1 + l, hi), 0)]);
            for (int rk = 1 + l; rk <= hi; rk += 8) {
                const p3 p = pn;
                pn = ld3(P4, (int)rl[min(rk + 8, hi)]);
                const double vx = p.x - qg.x, vy = p.y - qg.y, vz = p.z - qg.z;
                if (rk < rz) { x[0] += vx; x[1] += vy; x[2] += vz; }
                x[3] += vx; x[4] += vy; x[5] += vz;
                x[6] += vx * vx; x[7] += vx * vy; x[8] += vx * vz;
                x[9] += vy * vy; x[10] += vy * vz; x[11] += vz * vz;
            }
            if (l == 0) {
                const p3 f = ld3(P4, (int)rl[kk - 1]);
                const double fdx = qg.x - f.x, fdy = qg.y - f.y, fdz = qg.z - f.z;
                Rf = sqrt(fdx * fdx + fdy * fdy + fdz * fdz);  // ISR.cpp:256
            }
        }
#pragma unroll
        for (int i = 0; i < 12; ++i) {
            x[i] += gxd(x[i], 1);
            x[i] += gxd(x[i], 2);
            x[i] += gxd(x[i], 4);
        }
        __builtin_amdgcn_wave_barrier();
        if ((int)(l == 0) & (int)mine) {
#pragma unroll
            for (int i = 0; i < 12; ++i) pj[P8_SUM + i] = x[i];
            pj[P8_R] = Rf;
        }
    }
    {
        double x[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) x[i] = 0.0;
        if ((int)mine & (int)want_n) {  // EstimateNormals (ISR.cpp:643, :43): ranks 0 .. kn-1, self included
            p3 pn = ld3(P4, (int)rl[max(min(l, kn - 1), 0)]);
            for (int r = l; r < kn; r += 8) {
                const p3 p = pn;
                pn = ld3(P4, (int)rl[min(r + 8, kn - 1)]);
                const double px = p.x, py = p.y, pz = p.z;
                x[0] += px; x[1] += py; x[2] += pz;
                x[3] += px * px; x[4] += px * py; x[5] += px * pz;
                x[6] += py * py; x[7] += py * pz; x[8] += pz * pz;
            }
        }
#pragma unroll
        for (int i = 0; i < 9; ++i) {
            x[i] += gxd(x[i], 1);
            x[i] += gxd(x[i], 2);
            x[i] += gxd(x[i], 4);
        }
        __builtin_amdgcn_wave_barrier();
        if (l == 0) {
            const int flags = mine ? ((want_t ? 1 : 0) | (want_n ? 2 : 0)) : 0;
            pj[P8_FLAGS] = (double)flags;
            if (mine) {
#pragma unroll
                for (int i = 0; i < 9; ++i) pj[P8_SUM + 12 + i] = x[i];
                pj[P8_KK] = (double)kk;
                pj[P8_GP] = (double)(cl.off + T.perm[wq]);
                pj[P8_K] = (double)K;
                pj[P8_NTOP] = (double)nTop;
                pj[P8_W] = (double)wq;
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    PROF8_NOW(t_a2);
    PROF8_ADD(c_sums, t_a1, t_a2);
    unsigned long long* ctr = v.stats + kStatCols * (wv & 63);
    if (lane == 0) {  // work counters (bench diagnostics): queries, leaf scans, bound sorts, candidates
        atomicAdd(ctr + 0, (unsigned long long)n_q);
        atomicAdd(ctr + 1, (unsigned long long)n_leaves);
        atomicAdd(ctr + 2, (unsigned long long)n_sel);
        atomicAdd(ctr + 4, (unsigned long long)n_cand);
    }

#if defined(SE3ICP_LRF8_CUT) && SE3ICP_LRF8_CUT == 3
    return;  // (measurement build: stop after the neighbour sums)
#endif
    // ---------------------------------------------------------------- eigen-solves
    // TOLDI: C about the quirk centroid cl = (S' - q) / rz (ISR.cpp:259-272, see k_knn.hip),
    // its smallest eigenvector by cyclic Jacobi; normals: FastEigen3x3 of the kn-point
    // covariance (Open3D EstimateNormals, ISR.cpp:643) and the GICP covariance from it.
    auto toldi_eig = [&](double* pb) __attribute__((always_inline)) {
        const p3 q = ld3(P4, (int)pb[P8_W]);  // the query's tree slot
        const double rz = (double)((int)pb[P8_KK] / 3);
        const double q3[3] = {q.x, q.y, q.z};
        double cq[3], S[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            cq[a] = (pb[P8_SUM + a] - q3[a]) / rz;
            S[a] = pb[P8_SUM + 3 + a];
        }
        const double* M = pb + P8_SUM + 6;
        const int ia[6] = {0, 0, 0, 1, 1, 2}, ib[6] = {0, 1, 2, 1, 2, 2};
        double c6[6];
#pragma unroll
        for (int k = 0; k < 6; ++k)
            c6[k] = M[k] - S[ia[k]] * cq[ib[k]] - cq[ia[k]] * S[ib[k]] + rz * cq[ia[k]] * cq[ib[k]];
        const d3 zn = jacobi_smallest_evec(c6[0], c6[1], c6[2], c6[3], c6[4], c6[5]);
        pb[P8_ZN] = zn.x;
        pb[P8_ZN + 1] = zn.y;
        pb[P8_ZN + 2] = zn.z;
    };
    auto normal_eig = [&](const double* pb) __attribute__((always_inline)) {
        const int wb = (int)pb[P8_W];
        const int cc = cloud_of[wb];
        const int knb = min(setup[cc].k_nrm, (int)pb[P8_NTOP]);
        double n6[6] = {1, 0, 0, 1, 0, 1};
        if (knb >= 3) {
            double cu[9];
#pragma unroll
            for (int i = 0; i < 9; ++i) cu[i] = pb[P8_SUM + 12 + i] / (double)knb;
            n6[0] = cu[3] - cu[0] * cu[0];
            n6[1] = cu[4] - cu[0] * cu[1];
            n6[2] = cu[5] - cu[0] * cu[2];
            n6[3] = cu[6] - cu[1] * cu[1];
            n6[4] = cu[7] - cu[1] * cu[2];
            n6[5] = cu[8] - cu[2] * cu[2];
        }
        d3 nm = fast_eigen3x3(n6[0], n6[1], n6[2], n6[3], n6[4], n6[5]);
        if (sqrt(dot3(nm, nm)) == 0.0) nm = d3{0, 0, 1};
        const int gp = (int)pb[P8_GP];
        v.nrm64[gp] = nm.x;
        v.nrm64[v.ld + gp] = nm.y;
        v.nrm64[2 * (size_t)v.ld + gp] = nm.z;
    };
    // The 3x3 problems of the block's 32 queries, one lane each: wave 0 the TOLDI ones
    // (cyclic Jacobi), wave 1 the normals at the same time.
    __syncthreads();
    if (wid <= 1) {
        double* pb = park_of(lane < kW * kQ ? lane / kQ : 0, lane % kQ);
        const int b_flags = lane < kW * kQ ? (int)pb[P8_FLAGS] : 0;
        if ((b_flags & 1) && wid == 0) toldi_eig(pb);
        if ((b_flags & 2) && wid == 1) normal_eig(pb);
    }
    __syncthreads();

    // ---------------------------------------------------------------- TOLDI axes (ISR.cpp:286-306)
    {
        const int flags = (int)pj[P8_FLAGS];
        double x6[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
        if (flags & 1) {
            const double nx = pj[P8_ZN], ny = pj[P8_ZN + 1], nz = pj[P8_ZN + 2];
            const double R = pj[P8_R];
            const int kkq = (int)pj[P8_KK];
            p3 pn = ld3(P4, (int)rl[max(min(1 + l, kkq - 1), 0)]);
            for (int r = 1 + l; r < kkq; r += 8) {  // ranks 1 .. kk-1
                const p3 p = pn;
                pn = ld3(P4, (int)rl[min(r + 8, kkq - 1)]);
                const double vx = p.x - qg.x, vy = p.y - qg.y, vz = p.z - qg.z;
                x6[0] += vx; x6[1] += vy; x6[2] += vz;
                const double an = nx * vx + ny * vy + nz * vz;
                const double rr = R - sqrt(vx * vx + vy * vy + vz * vz);
                const double wgt = (rr * rr) * (an * an);
                x6[3] += wgt * vx; x6[4] += wgt * vy; x6[5] += wgt * vz;
            }
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            x6[i] += gxd(x6[i], 1);
            x6[i] += gxd(x6[i], 2);
            x6[i] += gxd(x6[i], 4);
        }
        __builtin_amdgcn_wave_barrier();
        if ((int)(l == 0) & (int)((flags & 1) != 0)) {
#pragma unroll
            for (int i = 0; i < 6; ++i) pj[P8_SUM + i] = x6[i];
        }
    }
    // the frames (ISR.cpp:298-307, 597-607), on wave 0 for the block's 32 queries
    __syncthreads();
    if (wid == 0) {
        const double* pb = park_of(lane < kW * kQ ? lane / kQ : 0, lane % kQ);
        const int b_flags = lane < kW * kQ ? (int)pb[P8_FLAGS] : 0;
        if (b_flags & 1) {
            const int w = (int)pb[P8_W];
            const CloudSetup sw = setup[cloud_of[w]];
            const p3 q = ld3(P4, w);
            d3 nrm{pb[P8_ZN], pb[P8_ZN + 1], pb[P8_ZN + 2]};
            if (nrm.x * pb[P8_SUM] + nrm.y * pb[P8_SUM + 1] + nrm.z * pb[P8_SUM + 2] < 0.0)
                nrm = d3{-nrm.x, -nrm.y, -nrm.z};  // ISR.cpp:298
            const d3 zax = nrm;
            const d3 accs{pb[P8_SUM + 3], pb[P8_SUM + 4], pb[P8_SUM + 5]};
            d3 xax = accs - dot3(accs, zax) * zax;  // ISR.cpp:302-303 (no |x| = 0 guard, as the reference)
            xax = (1.0 / sqrt(dot3(xax, xax))) * xax;
            const d3 yax = cross3(zax, xax);  // ISR.cpp:306
            const double al = sw.alpha, be = sw.beta;
            const double f12[12] = {al * xax.x, al * xax.y, al * xax.z, al * yax.x, al * yax.y, al * yax.z,
                                    al * zax.x, al * zax.y, al * zax.z, be * q.x, be * q.y, be * q.z};
            store_frame_rows(v.fr64, v.fr32, (int)pb[P8_GP], f12, sw.cf_target, q.x, q.y, q.z);
        }
    }
#ifdef SE3ICP_PROF
    PROF8_NOW(t_a3);
    PROF8_ADD(c_epi, t_a2, t_a3);
    if (lane == 0) {
        atomicAdd(ctr + 8, c_scan - c_tight);
        atomicAdd(ctr + 9, c_tight);
        atomicAdd(ctr + 10, c_sums);
        atomicAdd(ctr + 11, c_epi);
        atomicAdd(ctr + 3, (unsigned long long)n_tover);
        atomicAdd(ctr + 7, (unsigned long long)n_tend);
        atomicAdd(ctr + 5, fb_cause);
    }
#endif
}

}  // namespace

void launch_lrf8(const View& v, const int32_t* wave_base, int w_lo, int w_hi, int32_t* fb_list, int32_t* fb_count,
                 hipStream_t s) {
    const int nb = (w_hi - w_lo + kW - 1) / kW;
    if (nb <= 0) return;
    hipLaunchKernelGGL(k_lrf8, dim3(nb), dim3(64 * kW), 0, s, v, v.cloud_of, v.setup, v.clouds, v.t3.lo, v.t3.hi,
                       v.t3.tpt64, wave_base, w_lo, w_hi, fb_list, fb_count);
}

}  // namespace se3icp
