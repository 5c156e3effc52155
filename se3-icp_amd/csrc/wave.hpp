// wave.hpp — cross-lane exchanges of a full wavefront (64 lanes) without LDS address
// traffic where gfx950 has a cheaper route:
//   lane ^ 1, ^ 2   DPP quad_perm            (a VALU move)
//   lane ^ 4, ^ 8   ds_swizzle bit-mask mode (no address VGPR)
//   lane ^ 16, ^ 32 v_permlane16/32_swap + a select
// All lanes of the wave must be active (DPP / swizzle read 0 from inactive lanes); the
// callers use them in wave-uniform code only.  `m` must fold to a constant (unrolled loops).
#pragma once
#include <hip/hip_runtime.h>

namespace se3icp {

__device__ __forceinline__ unsigned xor_lane(unsigned x, int m) {
    switch (m) {
    case 1: return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0xB1, 0xF, 0xF, true);  // quad_perm [1,0,3,2]
    case 2: return (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x4E, 0xF, 0xF, true);  // quad_perm [2,3,0,1]
    case 4: return (unsigned)__builtin_amdgcn_ds_swizzle((int)x, 0x101F);  // and 0x1f, xor 4
    case 8: return (unsigned)__builtin_amdgcn_ds_swizzle((int)x, 0x201F);
    case 16: {
        const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);
        return ((threadIdx.x >> 4) & 1) ? r[0] : r[1];
    }
    case 32: {
        const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);
        return ((threadIdx.x >> 5) & 1) ? r[0] : r[1];
    }
    default: return (unsigned)__shfl_xor((int)x, m, 64);
    }
}
__device__ __forceinline__ int xor_lane(int x, int m) { return (int)xor_lane((unsigned)x, m); }
__device__ __forceinline__ float xor_lane(float x, int m) { return __uint_as_float(xor_lane(__float_as_uint(x), m)); }
__device__ __forceinline__ unsigned long long xor_lane(unsigned long long x, int m) {
    const unsigned lo = xor_lane((unsigned)x, m), hi = xor_lane((unsigned)(x >> 32), m);
    return ((unsigned long long)hi << 32) | lo;
}
__device__ __forceinline__ double xor_lane(double x, int m) {
    return __longlong_as_double((long long)xor_lane((unsigned long long)__double_as_longlong(x), m));
}

// butterfly sum / min over the 64 lanes (every lane gets the result)
__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x += xor_lane(x, o);
    return x;
}
__device__ __forceinline__ float wave_minf(float x) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x = fminf(x, xor_lane(x, o));
    return x;
}

// Sums of 32 values over the 64 lanes by recursive halving (each exchange step sends
// half of the values still held): 32 f64 exchanges instead of 32 x 6 butterflies.
// Returns the total of value (lane >> 1) in every lane.
__device__ __forceinline__ double swap_add32(double a, double b) {
    // v_permlane32_swap on both dwords: lanes 0-31 get (own a) + (partner's a),
    // lanes 32-63 get (own b) + (partner's b)
    const unsigned long long ua = (unsigned long long)__double_as_longlong(a), ub = (unsigned long long)__double_as_longlong(b);
    const auto lo = __builtin_amdgcn_permlane32_swap((unsigned)ua, (unsigned)ub, false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
    const double na = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
    const double nb = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
    return na + nb;
}
__device__ __forceinline__ double swap_add16(double a, double b) {
    // v_permlane16_swap: rows 0/2 keep a and receive the odd row's a, rows 1/3 keep b
    // and receive the even row's b
    const unsigned long long ua = (unsigned long long)__double_as_longlong(a), ub = (unsigned long long)__double_as_longlong(b);
    const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)ua, (unsigned)ub, false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(ua >> 32), (unsigned)(ub >> 32), false, false);
    const double na = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
    const double nb = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
    return na + nb;
}
__device__ __forceinline__ double wave_sum32(const double (&x)[32]) {
    const int lane = threadIdx.x & 63;
    double y16[16], y8[8], y4[4], y2[2];
#pragma unroll
    for (int i = 0; i < 16; ++i) y16[i] = swap_add32(x[i], x[i + 16]);  // value i + 16*bit5
#pragma unroll
    for (int i = 0; i < 8; ++i) y8[i] = swap_add16(y16[i], y16[i + 8]);  // + 8*bit4
#pragma unroll
    for (int i = 0; i < 4; ++i) {  // lane ^ 8: keep the half of bit3, send the other
        const bool b = (lane >> 3) & 1;
        const double keep = b ? y8[i + 4] : y8[i], send = b ? y8[i] : y8[i + 4];
        y4[i] = keep + xor_lane(send, 8);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const bool b = (lane >> 2) & 1;
        const double keep = b ? y4[i + 2] : y4[i], send = b ? y4[i] : y4[i + 2];
        y2[i] = keep + xor_lane(send, 4);
    }
    const bool b = (lane >> 1) & 1;
    const double keep = b ? y2[1] : y2[0], send = b ? y2[0] : y2[1];
    const double y = keep + xor_lane(send, 2);
    return y + xor_lane(y, 1);
}

// Sums of P (a power of two <= 32) values over the 64 lanes by recursive halving, the
// largest lane strides first.  Returns the total of value (lane >> (6 - log2 P)) in
// every lane.
template <int P>
__device__ __forceinline__ double wave_sum_pow2(const double (&x)[P]) {
    static_assert(P >= 1 && P <= 32 && (P & (P - 1)) == 0, "P: power of two <= 32");
    const int lane = threadIdx.x & 63;
    if constexpr (P == 32) {
        return wave_sum32(x);
    } else {
        double y[P];
#pragma unroll
        for (int i = 0; i < P; ++i) y[i] = x[i];
        int n = P, m = 32;
        // halving steps: stride m keeps the half of the values selected by lane bit m
#pragma unroll
        for (; n > 1; n >>= 1, m >>= 1) {
#pragma unroll
            for (int i = 0; i < n / 2; ++i) {
                if (m == 32) {
                    y[i] = swap_add32(y[i], y[i + n / 2]);
                } else if (m == 16) {
                    y[i] = swap_add16(y[i], y[i + n / 2]);
                } else {
                    const bool b = (lane & m) != 0;
                    const double keep = b ? y[i + n / 2] : y[i], send = b ? y[i] : y[i + n / 2];
                    y[i] = keep + xor_lane(send, m);
                }
            }
        }
        double r = y[0];
#pragma unroll
        for (; m >= 1; m >>= 1) r += xor_lane(r, m);
        return r;
    }
}

// One compare-exchange stage (block KK, distance JD) of an ascending bitonic network
// over distinct 64-bit keys (identical padding keys are interchangeable); entry
// e = tid*PER + s sits in k[s] of thread tid.  Partners in the same thread swap in
// registers, in the same wave through lane exchanges, in another wave through LDS
// (s_key: NT*PER entries; XW: partner distance in entries from which that is needed).
template <int PER, int KK, int JD, int XW>
__device__ __forceinline__ void bitonic_stage(unsigned long long (&k)[PER], int tid, unsigned long long* s_key) {
    if constexpr (JD < PER) {
#pragma unroll
        for (int s = 0; s < PER; ++s) {
            if ((s & JD) == 0) {
                const int t = s | JD;
                const bool up = ((tid * PER + s) & KK) == 0;
                const bool sw = (k[t] < k[s]) != !up;
                const unsigned long long ks = k[s], kt = k[t];
                k[s] = sw ? kt : ks;
                k[t] = sw ? ks : kt;
            }
        }
    } else if constexpr (JD < XW) {
#pragma unroll
        for (int s = 0; s < PER; ++s) {
            const int e = tid * PER + s;
            const unsigned long long pk = xor_lane(k[s], JD / PER);
            const bool take = (pk < k[s]) != (((e & JD) == 0) != ((e & KK) == 0));
            k[s] = take ? pk : k[s];
        }
    } else {
        __syncthreads();
#pragma unroll
        for (int s = 0; s < PER; ++s) s_key[tid * PER + s] = k[s];
        __syncthreads();
#pragma unroll
        for (int s = 0; s < PER; ++s) {
            const int e = tid * PER + s;
            const unsigned long long pk = s_key[e ^ JD];
            const bool take = (pk < k[s]) != (((e & JD) == 0) != ((e & KK) == 0));
            k[s] = take ? pk : k[s];
        }
    }
}
// the whole network over N entries, stage by stage at compile time
template <int PER, int N, int XW, int KK = 2, int JD = 1>
__device__ __forceinline__ void bitonic_net(unsigned long long (&k)[PER], int tid, unsigned long long* s_key) {
    bitonic_stage<PER, KK, JD, XW>(k, tid, s_key);
    if constexpr (JD > 1) bitonic_net<PER, N, XW, KK, JD / 2>(k, tid, s_key);
    else if constexpr (KK < N) bitonic_net<PER, N, XW, KK * 2, KK>(k, tid, s_key);
}
// ascending register sort of the 64*PER keys of one wave
template <int PER>
__device__ __forceinline__ void wave_sort_keys(unsigned long long (&k)[PER]) {
    bitonic_net<PER, 64 * PER, 64 * PER>(k, threadIdx.x & 63, nullptr);
}

// The same network over 32-bit keys, registers and lane exchanges only (64*PER keys of one
// wave): an in-register compare-exchange is a min and a max, a cross-lane one the
// partner's key and a min or max -- about half the instructions of the 64-bit network.
template <int PER, int KK, int JD>
__device__ __forceinline__ void bitonic_stage_u32(unsigned (&k)[PER], int lane) {
    if constexpr (JD < PER) {
#pragma unroll
        for (int s = 0; s < PER; ++s) {
            if ((s & JD) == 0) {
                const int t = s | JD;
                const bool up = ((lane * PER + s) & KK) == 0;
                const unsigned lo = min(k[s], k[t]), hi = max(k[s], k[t]);
                k[s] = up ? lo : hi;
                k[t] = up ? hi : lo;
            }
        }
    } else {
#pragma unroll
        for (int s = 0; s < PER; ++s) {
            const int e = lane * PER + s;
            const unsigned pk = xor_lane(k[s], JD / PER);
            k[s] = (((e & JD) == 0) == ((e & KK) == 0)) ? min(pk, k[s]) : max(pk, k[s]);
        }
    }
}
template <int PER, int N, int KK = 2, int JD = 1>
__device__ __forceinline__ void bitonic_net_u32(unsigned (&k)[PER], int lane) {
    bitonic_stage_u32<PER, KK, JD>(k, lane);
    if constexpr (JD > 1) bitonic_net_u32<PER, N, KK, JD / 2>(k, lane);
    else if constexpr (KK < N) bitonic_net_u32<PER, N, KK * 2, KK>(k, lane);
}
// ascending register sort of the 64*PER 32-bit keys of one wave
template <int PER>
__device__ __forceinline__ void wave_sort_u32(unsigned (&k)[PER]) {
    bitonic_net_u32<PER, 64 * PER>(k, threadIdx.x & 63);
}

// Blocks are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md, Workgroup
// dispatch): relabel them so that each XCD runs one contiguous range of the grid and its
// L2 keeps the data neighbouring blocks share (bijective for any grid size).
// Finer variant: runs of S consecutive logical blocks share an XCD and the runs are dealt
// round-robin over the 8 XCDs (locality within a run, balance across runs).  Bijective
// when nb is a multiple of 8 * S; otherwise the blocks past the last whole round keep
// their own index.
__device__ __forceinline__ int xcd_block_runs(int b, int nb, int S) {
    const int whole = nb / (8 * S) * (8 * S);
    if (b >= whole) return b;
    const int x = b & 7, i = b >> 3;
    return ((i / S) * 8 + x) * S + (i % S);
}
__device__ __forceinline__ int xcd_block(int b, int nb) {
    const int q = nb >> 3, r = nb & 7, x = b & 7, i = b >> 3;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

}  // namespace se3icp
