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
    case 1: return (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0xB1, 0xF, 0xF, false);  // quad_perm [1,0,3,2]
    case 2: return (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x4E, 0xF, 0xF, false);  // quad_perm [2,3,0,1]
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

}  // namespace se3icp
