// k_loop.hip — kernels of one ICP iteration (gfx950), batched over every active pair.
//
//   (the correspondence search itself is k_nn.hip)
//   recheck     queries whose f32 arg-min k_nn.hip could not certify: an exact f64 sweep
//               in nanoflann's arithmetic (ties -> lowest index).
//   trim        PCL CorrespondenceRejectorTrimmed: the floor(ratio*N)-th smallest
//               (float dist, query) key, from a window around the previous cut or by
//               MSB radix select (ISR.cpp:669-671).
//   reduce      per-correspondence Jacobian terms of the estimator, summed per block:
//               pt2pt moments (umeyama, ISR.cpp:692), pt2pl JTJ/JTr (ISR.cpp:695),
//               GICP JTJ/JTr with M^-1 = (Ct+Cs)^-1 (ISR.cpp:698, 57-110), MSE sum
//               (ISR.cpp:379-400).  A second kernel sums the partials of each pair in
//               a fixed order (deterministic), solves the pair's step and advances its
//               loop state on the device (pairmath.hpp).
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>
#include <cmath>
#include <cstdio>

#include "devmath.hpp"
#include "loopdev.hpp"
#include "pairmath.hpp"
#include "wave.hpp"
#include "tree.hpp"

namespace se3icp {

namespace {

using namespace loopdev;

// (recheck: the NN kernels re-resolve their uncertified queries in f64 inline,
// loopdev.hpp recheck_one)

// ------------------------------------------------------------------ trim
__device__ __forceinline__ unsigned long long trim_key_of(const float* dist, int base, int i) {
    return ((unsigned long long)__float_as_uint(dist[base + i]) << 32) | (unsigned)i;
}

// One wave finds the bin holding the k-th smallest element (k >= 1) of a histogram of
// 64*PER bins (lane l owns bins l*PER .. l*PER+PER-1); returns the bin and the count
// of elements in the bins before it.
template <int PER>
__device__ __forceinline__ void wave_find_bin(const unsigned* hist, unsigned k, int lane, int* bin,
                                              unsigned* before) {
    unsigned h[PER];
    unsigned t = 0;
#pragma unroll
    for (int j = 0; j < PER; ++j) { h[j] = hist[lane * PER + j]; t += h[j]; }
    unsigned incl = t;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const unsigned y = __shfl_up(incl, o, 64);
        if (lane >= o) incl += y;
    }
    const unsigned long long m = __ballot(incl >= k);
    const int owner = m ? __ffsll((long long)m) - 1 : 63;
    if (lane == owner) {
        unsigned cum = incl - t;
        int b = lane * PER + PER - 1;
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            if (cum + h[j] >= k) { b = lane * PER + j; break; }
            cum += h[j];
        }
        *bin = b;
        *before = cum;
    }
}

// wave-aggregated LDS histogram increment: lanes with equal digits add once
__device__ __forceinline__ void hist_add_aggregated(unsigned* hist, bool act, unsigned dig, int lane) {
    unsigned long long am = __ballot(act);
    while (am) {
        const int leader = __ffsll((long long)am) - 1;
        const unsigned ld = __shfl(dig, leader, 64);
        const unsigned long long same = __ballot(act && dig == ld);
        if (lane == leader) atomicAdd(&hist[ld], (unsigned)__popcll(same));
        if (dig == ld) act = false;
        am &= ~same;
    }
}

__device__ __forceinline__ unsigned wsum_u32(unsigned x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}


// PCL CorrespondenceRejectorTrimmed (ISR.cpp:669-671): the nkeep-th smallest 64-bit
// key (float distance bits << 32 | query index) of each trimming pair.
//  * Window (from the 2nd iteration of a phase on): the cut distance moves little between
//    ICP iterations, so k_trim_window (kTrimBlocks blocks per pair) counts the keys below
//    [d_prev(1-w), d_prev(1+w)] and appends the keys inside it to a global list; k_trim
//    ranks the list (each candidate counts the smaller ones, LDS broadcast reads) if the
//    cut rank falls inside.  w adapts toward a few hundred keys.
//  * Otherwise k_trim runs an MSB radix select: the first digit (top 12 bits) comes from
//    the histogram k_trim_window builds of every key; further 8-bit digits are counted
//    over all keys (global re-reads) until the selected bin holds at most kTrimList keys,
//    which are then compacted into LDS where the remaining digits are resolved.  A window
//    of more than kRankMax keys is resolved by the same digit passes inside LDS.
// Both give the same key.  Window state: trim_key[npairs + pair] (f32 d_prev bits << 32 |
// f32 w bits; 0 = none).  Per pair scratch: trim_cand[pair][kTrimList] and
// trim_ctr[pair][4] = {in-window count, below count, -, -} and trim_hist[pair][4096],
// reset by k_trim.
__device__ __forceinline__ unsigned long long trim_window_state(const View& v, const PairDev* P, int pair) {
    // the first iteration of a phase has no usable window (the R3 cut is far below the SE(3) one)
    return P->iter == P->phase_start ? 0ull : (unsigned long long)v.trim_key[v.npairs + pair];
}

__global__ __launch_bounds__(256) void k_trim_window(View v) {
    constexpr int kLoc = 2048;  // in-window keys a block collects before one global append
    __shared__ unsigned long long s_loc[kLoc];
    __shared__ unsigned s_hist[4096];  // top 12 key bits: the radix select's first digit
    __shared__ unsigned s_n, s_below, s_base;
    const int pair = blockIdx.x / kTrimBlocks, sub = blockIdx.x % kTrimBlocks;
    const PairDev* P = v.pairs + pair;
    if ((int)(P->phase == PHASE_IDLE) | (int)(P->trim == 0) | (int)(P->nkeep <= 0)) return;
    const unsigned long long wstate = trim_window_state(v, P, pair);
    const int lane = threadIdx.x & 63;
    for (int i = threadIdx.x; i < 4096; i += blockDim.x) s_hist[i] = 0u;
    const CloudDev cs = v.clouds[P->src];
    const int n = cs.n;
    const unsigned* dist = reinterpret_cast<const unsigned*>(v.corr_dist) + cs.off;
    unsigned* ctr = v.trim_ctr + 4 * pair;
    unsigned long long* cand = v.trim_cand + (size_t)pair * kTrimList;
    // no window: an empty one (lo > hi), the pass then only builds the histogram
    const float dprev = __uint_as_float((unsigned)(wstate >> 32));
    const float wv = __uint_as_float((unsigned)wstate);
    const unsigned lo = wstate ? __float_as_uint(dprev * (1.0f - wv)) : 0xffffffffu;
    const unsigned hi = wstate ? __float_as_uint(dprev * (1.0f + wv)) : 0u;
    const int per = ((n + kTrimBlocks - 1) / kTrimBlocks + 63) & ~63;
    const int i_beg = sub * per, i_end = min(n, i_beg + per);
    if (threadIdx.x == 0) { s_n = 0; s_below = 0; }
    __syncthreads();
    constexpr int U = 4;
    unsigned below = 0;
    for (int i0 = i_beg; i0 < i_end; i0 += U * blockDim.x) {
        unsigned u[U];
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int i = i0 + j * blockDim.x + threadIdx.x;
            u[j] = i < i_end ? dist[i] : 0xffffffffu;
        }
#pragma unroll
        for (int j = 0; j < U; ++j) {
            const int i = i0 + j * blockDim.x + threadIdx.x;
            if (i < i_end) atomicAdd(&s_hist[u[j] >> 20], 1u);
            below += (unsigned)((int)(i < i_end) & (int)(u[j] < lo));
            const bool sel = (int)(i < i_end) & (int)(u[j] >= lo) & (int)(u[j] <= hi);
            const unsigned long long m = __ballot(sel);
            if (m == 0) continue;
            unsigned base = 0;
            if (lane == 0) base = atomicAdd(&s_n, (unsigned)__popcll(m));
            base = __shfl(base, 0, 64);
            const unsigned at = base + (unsigned)__popcll(m & ((1ull << lane) - 1ull));
            if ((int)sel & (int)(at < (unsigned)kLoc)) s_loc[at] = ((unsigned long long)u[j] << 32) | (unsigned)i;
        }
    }
    below = wstate ? wsum_u32(below) : 0u;  // (no window: only the histogram is wanted)
    if ((int)(lane == 0) & (int)(below > 0)) atomicAdd(&s_below, below);
    __syncthreads();
    unsigned* gh = v.trim_hist + (size_t)pair * 4096;
    for (int i = threadIdx.x; i < 4096; i += blockDim.x)
        if (s_hist[i]) atomicAdd(&gh[i], s_hist[i]);
    // one global reservation per block (a block that overflowed its list forces a miss)
    const unsigned nloc = s_n;
    if (threadIdx.x == 0) {
        s_base = nloc ? atomicAdd(ctr, nloc <= (unsigned)kLoc ? nloc : (unsigned)kTrimList + 1u) : 0u;
        if (s_below) atomicAdd(ctr + 1, s_below);
    }
    __syncthreads();
    const unsigned base = s_base;
    if (nloc <= (unsigned)kLoc)
        for (unsigned e = threadIdx.x; e < nloc; e += blockDim.x)
            if (base + e < (unsigned)kTrimList) cand[base + e] = s_loc[e];
}

#ifdef SE3ICP_PROF
// k_trim phases summed over launches and pairs (100 MHz ticks): [0] whole block, [1] the
// window rank / first digit, [2] compaction passes, [3] global digit-count passes, [4] the
// LDS digit passes, [5] blocks, [6] blocks on the radix path
__device__ unsigned long long g_trim_prof[8];
#define TRIM_T(x) const unsigned long long x = __builtin_amdgcn_s_memrealtime()
#else
#define TRIM_T(x) do {} while (0)
#endif
// One 1024-thread block per trimming pair (see above).
__global__ __launch_bounds__(1024) void k_trim(View v) {
    __shared__ unsigned hist[4096];
    __shared__ unsigned long long s_list[kTrimList];
    __shared__ unsigned s_cnt;
    __shared__ int s_bin;
    __shared__ unsigned s_before;
    __shared__ unsigned long long s_found;
    const int pair = blockIdx.x;
    const PairDev* P = v.pairs + pair;
    if (P->phase == PHASE_IDLE || !P->trim) return;
    const CloudDev cs = v.clouds[P->src];
    const int n = cs.n;
    if (P->nkeep <= 0) {
        if (threadIdx.x == 0) v.trim_key[pair] = 0ull;  // keep none (handled by reduce)
        return;
    }
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    TRIM_T(tp0);
#ifdef SE3ICP_PROF
    unsigned long long c_comp = 0, c_gcount = 0, c_lds = 0;
#endif
    const unsigned* dist = reinterpret_cast<const unsigned*>(v.corr_dist) + cs.off;
    constexpr int U = 8;  // independent loads in flight per thread
    uint64_t* win = v.trim_key + v.npairs + pair;
    unsigned* ctr = v.trim_ctr + 4 * pair;
    const unsigned long long* cand = v.trim_cand + (size_t)pair * kTrimList;
    const unsigned long long wstate = trim_window_state(v, P, pair);
    float wv = wstate != 0ull ? __uint_as_float((unsigned)wstate) : 0.02f;
    unsigned* gh = v.trim_hist + (size_t)pair * 4096;  // k_trim_window's first-digit histogram
    constexpr unsigned kRankMax = 768;  // larger windows: LDS radix select instead of ranking
    unsigned win_cnt = 0, win_k = 0;
    if (wstate != 0ull) {
        const unsigned k = (unsigned)P->nkeep;  // rank (1-based) of the cut key
        const unsigned cnt = ctr[0], nb = ctr[1];
        const bool hit = cnt <= (unsigned)kTrimList && nb < k && k <= nb + cnt;
        // adapt the window: too full -> halve, missed -> x4, sparse -> x1.5
        if (cnt > 768u) wv *= 0.5f;
        else if (!hit) wv *= 4.0f;
        else if (cnt < 96u) wv *= 1.5f;
        wv = fminf(wv, 0.9f);
#ifdef SE3ICP_TRIM_TRACE  // (diagnostic build: window hits and sizes per pair and iteration)
        if (threadIdx.x == 0)
            printf("[trim] it %d pair %d hit %d cnt %u below %u k %u dprev %g w %g\n", P->iter, pair, (int)hit, cnt,
                   nb, k, (double)__uint_as_float((unsigned)(wstate >> 32)), (double)__uint_as_float((unsigned)wstate));
#endif
        constexpr unsigned R = 16;  // independent LDS reads in flight per rank count
        const unsigned cpad = (cnt + R - 1) & ~(R - 1);
        if (hit) {
            for (unsigned e = threadIdx.x; e < cpad; e += blockDim.x) s_list[e] = e < cnt ? cand[e] : ~0ull;
            __syncthreads();
            if (cnt > kRankMax) {  // a wide window: radix select inside the LDS list (below)
                win_cnt = cnt;
                win_k = k - nb;
            }
        }
        if ((int)hit & (int)(cnt <= kRankMax)) {
            const unsigned r = k - nb - 1;  // 0-based rank inside the window (keys are distinct)
            for (unsigned e = threadIdx.x; e < cnt; e += blockDim.x) {
                const unsigned long long key = s_list[e];
                unsigned less = 0;
                for (unsigned j = 0; j < cpad; j += R) {
                    unsigned long long t[R];
#pragma unroll
                    for (unsigned q = 0; q < R; ++q) t[q] = s_list[j + q];
#pragma unroll
                    for (unsigned q = 0; q < R; ++q) less += (unsigned)(t[q] < key);
                }
                if (less == r) {
                    v.trim_key[pair] = key;
                    *win = (key & 0xffffffff00000000ull) | __float_as_uint(wv);
                }
            }
            __syncthreads();
            if (threadIdx.x < 2) ctr[threadIdx.x] = 0u;
            for (int i = threadIdx.x; i < 4096; i += blockDim.x) gh[i] = 0u;
#ifdef SE3ICP_PROF
            if (threadIdx.x == 0) {
                TRIM_T(tpe);
                atomicAdd(&g_trim_prof[0], tpe - tp0);
                atomicAdd(&g_trim_prof[1], tpe - tp0);
                atomicAdd(&g_trim_prof[5], 1ull);
            }
#endif
            return;
        }
        __syncthreads();
        if (threadIdx.x < 2) ctr[threadIdx.x] = 0u;
    }
    unsigned long long prefix = 0, mask = 0;
    unsigned k = (unsigned)P->nkeep;  // rank (1-based) within the keys matching prefix/mask
    unsigned sel_count = (unsigned)n;
    int pos = 0;                      // key bits resolved (from the top)
    bool in_lds = false;
    unsigned cnt = 0;
    if (win_cnt) {  // the window's keys are in LDS: all digits resolved there
        in_lds = true;
        cnt = win_cnt;
        sel_count = win_cnt;
        k = win_k;
        for (int i = threadIdx.x; i < 4096; i += blockDim.x) gh[i] = 0u;
    } else {  // first digit (top 12 bits) from k_trim_window's histogram
        for (int i = threadIdx.x; i < 4096; i += blockDim.x) {
            hist[i] = gh[i];
            gh[i] = 0u;
        }
        __syncthreads();
        if (wid == 0) wave_find_bin<64>(hist, k, lane, &s_bin, &s_before);
        __syncthreads();
        const unsigned bin = (unsigned)s_bin;
        k -= s_before;
        sel_count = hist[bin];
        prefix = (unsigned long long)bin << 52;
        mask = 0xfffull << 52;
        pos = 12;
        __syncthreads();
    }
    TRIM_T(tp1);
    while (pos < 64) {
        const int w = pos == 0 ? 12 : min(8, 64 - pos);
        TRIM_T(tl0);
        const int sh = 64 - pos - w;
        const unsigned dmask = (1u << w) - 1u;
        if (!in_lds && sel_count <= (unsigned)kTrimList) {
            // compact the keys matching the prefix into LDS
            if (threadIdx.x == 0) s_cnt = 0;
            __syncthreads();
            for (int i0 = 0; i0 < n; i0 += U * blockDim.x) {
                unsigned u[U];
#pragma unroll
                for (int j = 0; j < U; ++j) {
                    const int i = i0 + j * blockDim.x + threadIdx.x;
                    u[j] = i < n ? dist[i] : 0xffffffffu;
                }
#pragma unroll
                for (int j = 0; j < U; ++j) {
                    const int i = i0 + j * blockDim.x + threadIdx.x;
                    const unsigned long long key = ((unsigned long long)u[j] << 32) | (unsigned)i;
                    const bool sel = i < n && (key & mask) == prefix;
                    const unsigned long long m = __ballot(sel);
                    if (m == 0) continue;
                    unsigned base = 0;
                    if (lane == 0) base = atomicAdd(&s_cnt, (unsigned)__popcll(m));
                    base = __shfl(base, 0, 64);
                    if (sel) s_list[base + (unsigned)__popcll(m & ((1ull << lane) - 1ull))] = key;
                }
            }
            __syncthreads();
            cnt = s_cnt;
            in_lds = true;
#ifdef SE3ICP_PROF
            c_comp += __builtin_amdgcn_s_memrealtime() - tl0;
#endif
        }
        TRIM_T(tl1);
#ifdef SE3ICP_PROF
        const bool lds_pass = in_lds;
#endif
        for (int i = threadIdx.x; i <= (int)dmask; i += blockDim.x) hist[i] = 0;
        __syncthreads();
        if (in_lds) {
            for (unsigned e = threadIdx.x; e < cnt; e += blockDim.x) {
                const unsigned long long key = s_list[e];
                if ((key & mask) == prefix) atomicAdd(&hist[(unsigned)(key >> sh) & dmask], 1u);
            }
        } else {
            for (int i0 = 0; i0 < n; i0 += U * blockDim.x) {
                unsigned u[U];
#pragma unroll
                for (int j = 0; j < U; ++j) {
                    const int i = i0 + j * blockDim.x + threadIdx.x;
                    u[j] = i < n ? dist[i] : 0xffffffffu;
                }
#pragma unroll
                for (int j = 0; j < U; ++j) {
                    const int i = i0 + j * blockDim.x + threadIdx.x;
                    const unsigned long long key = ((unsigned long long)u[j] << 32) | (unsigned)i;
                    if (i < n && (key & mask) == prefix) atomicAdd(&hist[(unsigned)(key >> sh) & dmask], 1u);
                }
            }
        }
        __syncthreads();
        if (wid == 0) {
            if (w == 12) wave_find_bin<64>(hist, k, lane, &s_bin, &s_before);
            else wave_find_bin<4>(hist, k, lane, &s_bin, &s_before);
        }
        __syncthreads();
        const unsigned bin = (unsigned)s_bin;
        k -= s_before;
        sel_count = hist[bin];
        prefix |= (unsigned long long)bin << sh;
        mask |= (unsigned long long)dmask << sh;
        pos += w;
        __syncthreads();
#ifdef SE3ICP_PROF
        if (lds_pass) c_lds += __builtin_amdgcn_s_memrealtime() - tl1;
        else c_gcount += __builtin_amdgcn_s_memrealtime() - tl1;
#endif
        if ((int)in_lds & (int)(sel_count == 1u) & (int)(pos < 64)) {
            // one key left with this prefix (the distance bits usually settle it): it is the cut
            for (unsigned e = threadIdx.x; e < cnt; e += blockDim.x)
                if ((s_list[e] & mask) == prefix) s_found = s_list[e];
            __syncthreads();
            prefix = s_found;
            break;
        }
    }
    if (threadIdx.x == 0) {
        v.trim_key[pair] = prefix;
        *win = (prefix & 0xffffffff00000000ull) | __float_as_uint(wv);
#ifdef SE3ICP_PROF
        TRIM_T(tpe);
        atomicAdd(&g_trim_prof[0], tpe - tp0);
        atomicAdd(&g_trim_prof[1], tp1 - tp0);
        atomicAdd(&g_trim_prof[2], c_comp);
        atomicAdd(&g_trim_prof[3], c_gcount);
        atomicAdd(&g_trim_prof[4], c_lds);
        atomicAdd(&g_trim_prof[5], 1ull);
        atomicAdd(&g_trim_prof[6], 1ull);
#endif
    }
}

// ------------------------------------------------------------------ reduce
template <typename T>
__device__ __forceinline__ T wsum(T x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o, 64);
    return x;
}

// One correspondence's terms (ISR.cpp:689-703, 57-110; MSE ISR.cpp:379-400) added to acc:
// vs the moved source point, vt the target point, ns0 / nt the source (initial frame) and
// target normals, w2 the cf weight squared (1 otherwise), dist the stored distance.
__device__ __forceinline__ void corr_terms(int est, bool cf, const double* T, const double* vs, const double* vt,
                                           const double* ns0, const double* nt, double w2, double dist, double* acc) {
    if (est == EST_PT2PT) {
#pragma unroll
        for (int a = 0; a < 3; ++a) { acc[a] += vs[a]; acc[3 + a] += vt[a]; }
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int b = 0; b < 3; ++b) acc[6 + a * 3 + b] += vt[a] * vs[b];
        acc[15] += 1.0;
        acc[27] += dist;
        return;
    }
    if (est == EST_PT2PL) {
        const double r = (vs[0] - vt[0]) * nt[0] + (vs[1] - vt[1]) * nt[1] + (vs[2] - vt[2]) * nt[2];
        const double J[6] = {vs[1] * nt[2] - vs[2] * nt[1], vs[2] * nt[0] - vs[0] * nt[2], vs[0] * nt[1] - vs[1] * nt[0],
                             nt[0], nt[1], nt[2]};
        int k = 0;
#pragma unroll
        for (int a = 0; a < 6; ++a)
#pragma unroll
            for (int b = a; b < 6; ++b) acc[k++] += J[a] * J[b];
#pragma unroll
        for (int a = 0; a < 6; ++a) acc[21 + a] += J[a] * r;
        acc[27] += dist;
        return;
    }
    // GICP: Cs = R Cs0 R^T (PointCloud::Transform on covariances, ISR.cpp:706); both
    // covariances from the stored normals (ISR.cpp:33-52: 3 loads instead of 6)
    double C0[3][3];
    {
        double c6[6];
        gicp_cov_from_normal(d3{ns0[0], ns0[1], ns0[2]}, 1e-3, c6);
        C0[0][0] = c6[0]; C0[0][1] = C0[1][0] = c6[1]; C0[0][2] = C0[2][0] = c6[2];
        C0[1][1] = c6[3]; C0[1][2] = C0[2][1] = c6[4]; C0[2][2] = c6[5];
    }
    double RC[3][3], M[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) RC[a][b] = T[a * 4] * C0[0][b] + T[a * 4 + 1] * C0[1][b] + T[a * 4 + 2] * C0[2][b];
    {
        double Ct[6];
        gicp_cov_from_normal(d3{nt[0], nt[1], nt[2]}, 1e-3, Ct);
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
    // J^T J = G^T M^-1 G and J^T r = G^T M^-1 d for every W with W^T W = M^-1 (the
    // reference's W = M^-1/2, ISR.cpp:78, is one of them), so the sums are formed from
    // A = w^2 M^-1 and G = [S | I], S = -[vs]x, without a matrix root or factor:
    // J^T J = [[S^T A S, S^T A], [A S, A]], J^T r = [S^T A d; A d].
    const double sc = w2 / det;
    double A[3][3];
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) A[a][b] = 0.5 * (Mi[a][b] + Mi[b][a]) * sc;
    const double S[3][3] = {{0, vs[2], -vs[1]}, {-vs[2], 0, vs[0]}, {vs[1], -vs[0], 0}};
    const double d[3] = {vs[0] - vt[0], vs[1] - vt[1], vs[2] - vt[2]};
    double B[3][3];  // A S
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) B[a][b] = A[a][0] * S[0][b] + A[a][1] * S[1][b] + A[a][2] * S[2][b];
    double H[6][6];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
#pragma unroll
        for (int b = a; b < 3; ++b) H[a][b] = S[0][a] * B[0][b] + S[1][a] * B[1][b] + S[2][a] * B[2][b];
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            H[a][3 + b] = B[b][a];  // (S^T A)[a][b] = (A S)[b][a]
            H[3 + a][3 + b] = A[a][b];
        }
    }
    double Ad[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) Ad[a] = A[a][0] * d[0] + A[a][1] * d[1] + A[a][2] * d[2];
    int k = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
        for (int b = a; b < 6; ++b) acc[k++] += H[a][b];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        acc[21 + a] += S[0][a] * Ad[0] + S[1][a] * Ad[1] + S[2][a] * Ad[2];
        acc[24 + a] += Ad[a];
    }
    // estimate_current_mse_compute_euclidean for cf (ISR.cpp:390-400), the stored distance else
    acc[27] += cf ? sqrt((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]) : dist;
}

// The target points' geometry rows for k_reduce's gathers (View::tgeo): one 64-B row per
// point of a target cloud -- a kept correspondence then touches one 128-B line of target
// data instead of up to seven (measured: every fabric read on gfx950 is a 128-B request,
// profiles/r05_fetch_calib.json).  A lane per row reads the SoA columns (coalesced), the
// wave's 64 rows are transposed through LDS so that every store instruction writes 1 KB of
// consecutive rows (four lanes per row end to end: 361 us per 64-pair batch against 300 us
// for one lane per row storing its own 64 B; source clouds are skipped, their rows are never
// read).
__global__ __launch_bounds__(256) void k_geo_rows(View v) {
    __shared__ double2 s_rows[4][64 * 4];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int r0 = (blockIdx.x * 4 + wv) * 64;  // the wave's first row
    const int i = r0 + lane;
    bool tgt = false;
    if (i < v.npts) {
        const CloudSetup* st = v.setup + v.cloud_of[i];
        tgt = st->is_target != 0;
        if (tgt) {
            const size_t ld = v.ld;
            double2* r = &s_rows[wv][lane * 4];
            r[0] = make_double2(v.xyz64[i], v.xyz64[ld + i]);
            r[1] = make_double2(v.xyz64[2 * ld + i], v.nrm64[i]);
            r[2] = make_double2(v.nrm64[ld + i], v.nrm64[2 * ld + i]);
            r[3] = make_double2(st->want_conf ? v.conf64[i] : 0.0, 0.0);
        }
    }
    const unsigned long long tm = __ballot(tgt);
    __builtin_amdgcn_wave_barrier();
    if (tm == 0ull) return;
    double2* out = reinterpret_cast<double2*>(v.tgeo) + (size_t)r0 * 4;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int e = k * 64 + lane;  // part e & 3 of row e >> 2
        if ((tm >> (e >> 2)) & 1ull) out[e] = s_rows[wv][e];
    }
}

// Block b sums the terms of its pair's queries q0 + threadIdx.x + kRedThreads u (u < kRedPer,
// below q1).  Every input of the thread's kRedPer correspondences is loaded before the
// first is used: a wave's latency is a few dependent round trips (work record -> index and
// distance -> target gathers), so the loads of several correspondences share them.
__global__ __launch_bounds__(kRedThreads) void k_reduce(View v) {
    constexpr int NW = kRedThreads / 64;
    __shared__ double red[NW][kRedVals];
    const BlockWork w = v.work[blockIdx.x];
    const PairDev* P = v.pairs + w.pair;
    double acc[kRedVals];
#pragma unroll
    for (int i = 0; i < kRedVals; ++i) acc[i] = 0.0;
    if (P->phase == PHASE_IDLE) return;
    const int est = P->est;
    const bool cf = P->cf != 0;
    // trimmed pairs keep the keys (float dist bits << 32 | query) up to the cut (none when nkeep = 0)
    const unsigned long long cut = P->trim ? (P->nkeep > 0 ? v.trim_key[w.pair] : 0ull) : ~0ull;
    const bool none = (int)(P->trim != 0) & (int)(P->nkeep <= 0);
    const size_t ld = v.ld;
    int g[kRedPer], gt[kRedPer];
    float dd[kRedPer];
    bool kept[kRedPer];
#pragma unroll
    for (int u = 0; u < kRedPer; ++u) {
        const int qi = w.q0 + (int)threadIdx.x + kRedThreads * u;
        kept[u] = qi < w.q1;
        g[u] = w.s_off + (kept[u] ? qi : w.q0);
        dd[u] = v.corr_dist[g[u]];
        gt[u] = w.t_off + v.corr_idx[g[u]];
        const unsigned long long key = ((unsigned long long)__float_as_uint(dd[u]) << 32) | (unsigned)qi;
        kept[u] = (bool)((int)kept[u] & (int)!none & (int)(key <= cut));
    }
    double xs[kRedPer][3], xt[kRedPer][3], n0[kRedPer][3], nt[kRedPer][3], w2[kRedPer];
#pragma unroll
    for (int u = 0; u < kRedPer; ++u) {
        // the target's point, normal and confidence: one 64-B geometry row (k_geo_rows)
        const double2* tr = reinterpret_cast<const double2*>(v.tgeo + (size_t)gt[u] * 8);
        const double2 t01 = tr[0], t23 = tr[1], t45 = tr[2];
        xt[u][0] = t01.x; xt[u][1] = t01.y; xt[u][2] = t23.x;
        nt[u][0] = t23.y; nt[u][1] = t45.x; nt[u][2] = t45.y;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            xs[u][a] = v.xyz64[a * ld + g[u]];
            n0[u][a] = est == EST_GICP ? v.nrm64[a * ld + g[u]] : 0.0;
        }
        if (cf) {
            const double wc = (v.conf64[g[u]] + tr[3].x) / 2.0;  // ISR.cpp:913
            w2[u] = wc * wc;
        } else {
            w2[u] = 1.0;
        }
    }
    {
        double T[12];
        load_T(P, T);
#pragma unroll
        for (int u = 0; u < kRedPer; ++u) {
            if (!kept[u]) continue;
            double vs[3];
            pose_point(T, xs[u][0], xs[u][1], xs[u][2], vs);
            corr_terms(est, cf, T, vs, xt[u], n0[u], nt[u], w2[u], (double)dd[u], acc);
        }
    }
    const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    {  // the 28 sums over the wave by recursive halving (wave.hpp)
        double x[32];
#pragma unroll
        for (int i = 0; i < 32; ++i) x[i] = i < kRedVals ? acc[i] : 0.0;
        const double sv = wave_sum32(x);
        if ((int)((lane & 1) == 0) & (int)((lane >> 1) < kRedVals)) red[wid][lane >> 1] = sv;
    }
    __syncthreads();
    if (threadIdx.x < kRedVals) {
        const int i = threadIdx.x;
        double s4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            s4[k] = red[k][i];
#pragma unroll
            for (int w2 = k + 4; w2 < NW; w2 += 4) s4[k] += red[w2][i];
        }
        v.red_partial[(size_t)blockIdx.x * kRedVals + i] = (s4[0] + s4[1]) + (s4[2] + s4[3]);
    }
}

// Sum each pair's block partials in block order (deterministic); the block list of
// pair p is the contiguous work-table range where work[b].pair == p.  Then one lane
// closes the pair's iteration `it` on the device (estimator solve, pose update,
// switch / convergence: pairmath.hpp) and opens iteration it+1 (PairDev, pose history
// row), so the next iteration's kernels are already queued behind this one.
// next_phase[p] receives pair p's phase in iteration it+1 (PHASE_IDLE once finished); it
// lives in coherent host memory, and the host polls it (engine.cpp spin_phases) and goes on
// as soon as every pair's slot is written -- possibly before this kernel has completed.
// So the slot is the only value the host may read without ordering: any host read of
// other device state after finish() must stay stream-ordered (an async copy on the stream,
// then a sync), as the engine's result copies are.
#ifdef SE3ICP_PROF
// k_reduce_final phases summed over launches and pairs (100 MHz ticks): [0] the block
// partials' sums, [1] the one-lane close / open of the iteration, [2] pair blocks
// (one slot per phase: [3] state load, [4] close, [5] open + stores; round 5 packed the
// three into 21-bit fields of one word, which overflowed over a large batch -- ADVICE r05)
__device__ unsigned long long g_fin_prof[6];
#endif
constexpr int kFinThreads = 512;                    // (the solve's ~220 VGPRs allow two waves per SIMD)
constexpr int kFinChunks = kFinThreads / kRedVals;  // 18 interleaved chunks of block partials
__global__ __launch_bounds__(kFinThreads) void k_reduce_final(View v, const int32_t* pair_wb, const int32_t* pair_wn,
                                                      PairState* state, double* hist, int32_t* next_phase) {
    const int p = blockIdx.x;
    if ((int)(p == 0) & (int)(threadIdx.x < 3)) v.flag_count[threadIdx.x] = 0;  // single-query lists
    if ((int)(p == 0) & (int)(threadIdx.x < 2 * 8 * 16)) v.cls[threadIdx.x] = 0;  // search cost-class counts
    PairDev* P = v.pairs + p;
    if (P->phase == PHASE_IDLE) {
        if ((int)(threadIdx.x == 0) & (int)(next_phase != nullptr)) next_phase[p] = PHASE_IDLE;
        return;
    }
    __shared__ double part[kFinChunks][kRedVals];
    __shared__ double tot[kRedVals];
#ifdef SE3ICP_PROF
    const unsigned long long tf0 = __builtin_amdgcn_s_memrealtime();
#endif
    const int i = threadIdx.x % kRedVals, s = threadIdx.x / kRedVals;
    const int wb = pair_wb[p], wn = pair_wn[p];
    // the pair's loop state, loaded by the closing lane before the sums (its round trip
    // overlaps them instead of following them)
    PairState S;
    if (threadIdx.x == 0) S = state[p];
    if (s < kFinChunks) {  // eight independent chains per lane: eight loads in flight
        constexpr int C = kFinChunks, U = 8;
        double s8[U];
#pragma unroll
        for (int u = 0; u < U; ++u) s8[u] = 0.0;
        const double* rp = v.red_partial + (size_t)wb * kRedVals + i;
        int b = s;
        for (; b + (U - 1) * C < wn; b += U * C) {
            double x[U];
#pragma unroll
            for (int u = 0; u < U; ++u) x[u] = rp[(size_t)(b + C * u) * kRedVals];
#pragma unroll
            for (int u = 0; u < U; ++u) s8[u] += x[u];
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (b + C * u < wn) s8[u] += rp[(size_t)(b + C * u) * kRedVals];
        part[s][i] = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
    }
    __syncthreads();
    if (threadIdx.x < kRedVals) {
        double sum = 0;
#pragma unroll
        for (int k = 0; k < kFinChunks; ++k) sum += part[k][threadIdx.x];
        v.red_out[(size_t)p * kRedVals + threadIdx.x] = sum;
        tot[threadIdx.x] = sum;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
#ifdef SE3ICP_PROF
        const unsigned long long tf1 = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef SE3ICP_PROF
        const int est_ = P->est;
        __builtin_amdgcn_s_waitcnt(0);
        asm volatile("" :: "v"(S.mse_cur), "s"(est_));
        const unsigned long long tfa = __builtin_amdgcn_s_memrealtime();
        pair_close_iteration(S, est_, tot);
        asm volatile("" :: "v"(S.T.m[0][0]), "v"(S.T.m[2][3]));
        const unsigned long long tfb = __builtin_amdgcn_s_memrealtime();
#else
        pair_close_iteration(S, P->est, tot);
#endif
        pair_open_iteration(S, *P);
        state[p] = S;
        if (!S.done) {
            double* h = hist + ((size_t)(S.iter % kHist) * v.npairs + p) * 12;
            for (int k = 0; k < 12; ++k) h[k] = P->T[k];
        }
        if (next_phase) next_phase[p] = P->phase;
#ifdef SE3ICP_PROF
        __builtin_amdgcn_s_waitcnt(0);
        const unsigned long long tf2 = __builtin_amdgcn_s_memrealtime();
        atomicAdd(&g_fin_prof[0], tf1 - tf0);
        atomicAdd(&g_fin_prof[1], tf2 - tf1);
        atomicAdd(&g_fin_prof[2], 1ull);
        atomicAdd(&g_fin_prof[3], tfa - tf1);
        atomicAdd(&g_fin_prof[4], tfb - tfa);
        atomicAdd(&g_fin_prof[5], tf2 - tfb);
#endif
    }
}

}  // namespace

void trim_prof_report() {
#ifdef SE3ICP_PROF
    unsigned long long h[8];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_trim_prof), sizeof(h)) != hipSuccess || !h[5]) return;
    std::fprintf(stderr, "[prof] k_trim per block (us): whole %.2f, window rank / first digit %.2f; radix-path blocks "
                 "%llu of %llu: compaction %.2f, global counts %.2f, LDS digits %.2f (per radix block)\n",
                 h[0] / 100.0 / h[5], h[1] / 100.0 / h[5], h[6], h[5], h[6] ? h[2] / 100.0 / h[6] : 0.0,
                 h[6] ? h[3] / 100.0 / h[6] : 0.0, h[6] ? h[4] / 100.0 / h[6] : 0.0);
    const unsigned long long z[8] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_trim_prof), z, sizeof(z));
    unsigned long long f[6];
    if (hipMemcpyFromSymbol(f, HIP_SYMBOL(g_fin_prof), sizeof(f)) == hipSuccess && f[2]) {
        std::fprintf(stderr, "[prof] k_reduce_final per pair block (us): partial sums %.2f, close/open %.2f (state load %.2f, "
                     "close %.2f, open + stores %.2f) (%llu)\n",
                     f[0] / 100.0 / f[2], f[1] / 100.0 / f[2], f[3] / 100.0 / f[2], f[4] / 100.0 / f[2],
                     f[5] / 100.0 / f[2], f[2]);
        const unsigned long long z6[6] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_fin_prof), z6, sizeof(f));
    }
#endif
}
void launch_trim(const View& v, hipStream_t s) {
    hipLaunchKernelGGL(k_trim_window, dim3(v.npairs * kTrimBlocks), dim3(256), 0, s, v);
    hipLaunchKernelGGL(k_trim, dim3(v.npairs), dim3(1024), 0, s, v);
}
void launch_geo_rows(const View& v, hipStream_t s) {
    if (v.npts > 0) hipLaunchKernelGGL(k_geo_rows, dim3((v.npts + 255) / 256), dim3(256), 0, s, v);
}
void launch_reduce(const View& v, const int32_t* pair_wb, const int32_t* pair_wn, PairState* state, double* hist,
                   int32_t* next_phase, hipStream_t s) {
    hipLaunchKernelGGL(k_reduce, dim3(v.nwork), dim3(kRedThreads), 0, s, v);
    hipLaunchKernelGGL(k_reduce_final, dim3(v.npairs), dim3(kFinThreads), 0, s, v, pair_wb, pair_wn, state, hist, next_phase);
}

}  // namespace se3icp
