// knn_util.hpp — device helpers shared by the setup's kNN kernels (k_knn.hip, k_lrf8.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>

#include "wave.hpp"

namespace se3icp {
namespace knn {

__device__ __forceinline__ double l2_3(double ax, double ay, double az, double bx, double by, double bz) {
#pragma clang fp contract(off)
    const double d0 = ax - bx, d1 = ay - by, d2 = az - bz;
    return (d0 * d0 + d1 * d1) + d2 * d2;
}

// (d, idx) lexicographic order.  Written with bitwise operators: a short-circuit || / &&
// on per-lane values becomes divergent control flow (exec-mask branches) on the SIMD.
__device__ __forceinline__ bool key_less(double da, int ia, double db, int ib) {
    return (bool)((int)(da < db) | ((int)(da == db) & (int)(ia < ib)));
}
__device__ __forceinline__ bool key_le(double da, int ia, double db, int ib) {
    return (bool)((int)(da < db) | ((int)(da == db) & (int)(ia <= ib)));
}

// Set bits of a wave-uniform 64-bit mask in outward order from position p (p may lie
// outside [0, 64)): p, p+1, p-1, p+2, p-2, ... (nearest-first by a wave minimum per step
// and plain ascending order were measured slower).
// Neighbouring leaves in tree order are neighbours in space, so the bound tightens early.
struct OutwardBits {
    unsigned long long up, dn;
    bool flip = false;
    __device__ OutwardBits(unsigned long long m, int p) {
        if (p < 0) { up = m; dn = 0ull; }
        else if (p >= 64) { up = 0ull; dn = m; }
        else { dn = m & ((1ull << p) - 1ull); up = m & ~((1ull << p) - 1ull); }
    }
    __device__ int next() {
        const bool use_up = up != 0ull && (dn == 0ull || !flip);
        flip = !flip;
        if (use_up) { const int t = __builtin_ctzll(up); up &= up - 1ull; return t; }
        if (dn != 0ull) { const int t = 63 - __builtin_clzll(dn); dn &= ~(1ull << t); return t; }
        return -1;
    }
};

__device__ __forceinline__ double wsum(double x) { return wave_sum(x); }

// bits of the f32 value >= d (d >= 0): the f32 keys preserve <= of the f64 distances
__device__ __forceinline__ unsigned f32_up_bits(double d) {
    float f = (float)d;
    if ((double)f < d) f = __uint_as_float(__float_as_uint(f) + 1u);
    return __float_as_uint(f);
}

// squared distance from q to a 3-D box (f32; the boxes are inflated to bound the f64 points)
__device__ __forceinline__ float box_lb3(const float* lo, const float* hi, float qx, float qy, float qz) {
    const float dx = fmaxf(fmaxf(lo[0] - qx, qx - hi[0]), 0.f);
    const float dy = fmaxf(fmaxf(lo[1] - qy, qy - hi[1]), 0.f);
    const float dz = fmaxf(fmaxf(lo[2] - qz, qz - hi[2]), 0.f);
    return dx * dx + dy * dy + dz * dz;
}

// Per-query state parked in LDS between the kNN pass and the batched eigen-solves
// (slots of s_park[wave][query]).
// PK_SUM: the 21 neighbour sums of a query (see the sums pass), later its 6 TOLDI axis sums.
// PK_ZN: the TOLDI z axis (smallest-eigenvalue eigenvector) from the batched solve.
enum ParkSlot { PK_SUM = 0, PK_R = 21, PK_KK = 22, PK_GP = 23, PK_FLAGS = 24, PK_K = 25, PK_NTOP = 26, PK_ZN = 27, PK_N = 30 };
constexpr int kSums = 21;


}  // namespace knn
}  // namespace se3icp
