// k_gen.hip — the synthetic registration problems of the reference's benchmark
// (examples/benchmark_synthetic.cpp:91-160), generated on the GPU for batched runs:
//   source_c = RandomDownSample(base, ratio)       + N(0, noise_var I)   (B_SYN:99, :151)
//              (one subset for every case, its noise per case)
//   target_c = RandomDownSample(T_c base, ratio)   + N(0, noise_var I)   (B_SYN:149-153)
// with add_noise_to_point_cloud (B_SYN:13-56: diagonal covariance noise_var, i.e. standard
// deviation sqrt(noise_var) per axis) and Open3D RandomDownSample (a random subset of
// exactly (int)(ratio * n) points, in random order).  Source and target subsets are drawn
// independently.  The reference's own streams (mt19937, libstdc++ distributions, Open3D's
// shuffle), number for number, are the host generator gen_ref.cpp.
//
// One thread per output point.  The random subset of case c / side s is the image of
// 0..k-1 under a keyed bijection of [0, n): a 4-round Feistel network on the next even
// power of two >= n, cycle-walked back into [0, n) (every output index distinct, no sort
// or shared state).  The noise is Box-Muller on Philox4x32-10 counters (seed, case,
// side, point).  Counter-based streams replace the reference's mt19937 so that a GPU batch
// of any size is made in one pass: the protocol and its distributions are the same, the
// individual samples are not (tests/test_generators.py).
//
// se3icp_synthetic_reference_device is the reference-exact batch: the host draws the
// driver's own streams (refrand.hpp draw_reference: Open3D's shuffle, mt19937 T, the
// static normal_distribution noise) and k_apply_reference gathers, transforms and adds the
// noise with se3icp_synthetic_reference's arithmetic (Transform without FMA, p + sd * z), so
// the device clouds equal the host's bit for bit (tests/test_generators.py).
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <cmath>
#include <cstring>

#include "refrand.hpp"
#include "se3icp.h"

namespace se3icp {

namespace {

struct Philox {
    uint32_t v[4];
};

__device__ __forceinline__ Philox philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0,
                                                uint32_t k1) {
    constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
        const uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0;
        c1 = lo1;
        c2 = n2;
        c3 = lo0;
        k0 += W0;
        k1 += W1;
    }
    return Philox{{c0, c1, c2, c3}};
}

__device__ __forceinline__ uint32_t mix32(uint32_t x) {  // murmur3 finalizer
    x ^= x >> 16;
    x *= 0x85EBCA6Bu;
    x ^= x >> 13;
    x *= 0xC2B2AE35u;
    x ^= x >> 16;
    return x;
}

// keyed bijection of [0, 2^(2h)) (balanced Feistel, 4 rounds), cycle-walked into [0, n)
__device__ __forceinline__ uint32_t permute_index(uint32_t j, uint32_t n, int h, uint32_t key) {
    const uint32_t mask = (1u << h) - 1u;
    uint32_t x = j;
    do {
        uint32_t L = x >> h, R = x & mask;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const uint32_t F = mix32(R ^ (key + 0x9E3779B9u * (uint32_t)(r + 1))) & mask;
            const uint32_t nL = R;
            R = L ^ F;
            L = nL;
        }
        x = (L << h) | R;
    } while (x >= n);
    return x;
}

__device__ __forceinline__ double unit_open(uint32_t u) {  // (0, 1]
    return ((double)u + 1.0) * (1.0 / 4294967296.0);
}

__global__ __launch_bounds__(256) void k_synthetic(const double* __restrict__ base, uint32_t n, uint32_t k,
                                                   int n_cases, const double* __restrict__ T, double sd, int h,
                                                   uint32_t seed_lo, uint32_t seed_hi, double* __restrict__ src,
                                                   double* __restrict__ tgt) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per_side = (int64_t)n_cases * k;
    if (t >= 2 * per_side) return;
    const int side = (int)(t / per_side);  // 0 source, 1 target
    const int64_t r = t - side * per_side;
    const uint32_t c = (uint32_t)(r / k), j = (uint32_t)(r - (int64_t)c * k);
    // one source subset shared by every case (the driver downsamples the source once and
    // copies it per case, B_SYN:99, 146); an independent target subset per case (B_SYN:148)
    const uint32_t key = mix32(seed_lo ^ mix32(seed_hi ^ mix32(side == 0 ? 1u : 2u * c + 2u)));
    const uint32_t idx = permute_index(j, n, h, key);
    double p[3] = {base[3 * (size_t)idx], base[3 * (size_t)idx + 1], base[3 * (size_t)idx + 2]};
    if (side == 1) {  // target_final_notDS->Transform(T) (B_SYN:149)
        const double* M = T + 16 * (size_t)c;
        double q[3];
#pragma unroll
        for (int a = 0; a < 3; ++a) q[a] = M[4 * a] * p[0] + M[4 * a + 1] * p[1] + M[4 * a + 2] * p[2] + M[4 * a + 3];
        p[0] = q[0]; p[1] = q[1]; p[2] = q[2];
    }
    // three N(0, sd^2) samples: Box-Muller on one Philox block
    const Philox g = philox4x32_10(j, c, (uint32_t)side, 0x5E3u, seed_lo, seed_hi);
    const double r0 = sqrt(-2.0 * log(unit_open(g.v[0]))), a0 = 6.283185307179586 * unit_open(g.v[1]);
    const double r1 = sqrt(-2.0 * log(unit_open(g.v[2]))), a1 = 6.283185307179586 * unit_open(g.v[3]);
    double* out = (side == 0 ? src : tgt) + 3 * ((size_t)c * k + j);
    out[0] = p[0] + sd * r0 * cos(a0);
    out[1] = p[1] + sd * r0 * sin(a0);
    out[2] = p[2] + sd * r1 * cos(a1);
}

// one thread per output point: out = (T_c * cloud[idx] for a target) + sd * z, no FMA
// (refrand.hpp transform_point; add_noise_to_point_cloud, B_SYN:13-56)
__global__ __launch_bounds__(256) void k_apply_reference(const double* __restrict__ cloud,
                                                         const int32_t* __restrict__ src_idx,
                                                         const int32_t* __restrict__ tgt_idx,
                                                         const double* __restrict__ T, const double* __restrict__ z,
                                                         int64_t k, int n_cases, double sd, double* __restrict__ src,
                                                         double* __restrict__ tgt) {
#pragma clang fp contract(off)
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t per_side = (int64_t)n_cases * k;
    if (t >= 2 * per_side) return;
    const int side = (int)(t / per_side);
    const int64_t r = t - side * per_side;
    const int64_t c = r / k, i = r - c * k;
    const double* zz = z + ((size_t)c * 6 * k + (size_t)side * 3 * k + 3 * (size_t)i);
    double p[3];
    if (side == 0) {
        const double* a = cloud + 3 * (size_t)src_idx[i];
        p[0] = a[0]; p[1] = a[1]; p[2] = a[2];
    } else {
        const double* a = cloud + 3 * (size_t)tgt_idx[r];
        const double* M = T + 16 * (size_t)c;
#pragma unroll
        for (int e = 0; e < 3; ++e) p[e] = ((M[4 * e] * a[0] + M[4 * e + 1] * a[1]) + M[4 * e + 2] * a[2]) + M[4 * e + 3] * 1.0;
    }
    double* out = (side == 0 ? src : tgt) + 3 * (size_t)r;
#pragma unroll
    for (int e = 0; e < 3; ++e) out[e] = p[e] + sd * zz[e];
}

struct DevMem {
    void* p = nullptr;
    ~DevMem() {
        if (p) (void)hipFree(p);
    }
};

}  // namespace

}  // namespace se3icp

extern "C" int64_t se3icp_synthetic_pairs(int device, const double* base, int64_t n, int32_t n_cases,
                                          const double* T, double ratio, double noise_var, uint64_t seed,
                                          double* src_out, double* tgt_out, int outputs_on_device) {
    using namespace se3icp;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return SE3ICP_ERR_NO_DEVICE;
    if (!base || !T || !src_out || !tgt_out || n_cases <= 0 || !(ratio > 0.0) || ratio > 1.0 || noise_var < 0.0)
        return SE3ICP_ERR_INVALID_ARG;
    if (n <= 0) return SE3ICP_ERR_EMPTY_CLOUD;
    if (n >= (int64_t)1 << 30) return SE3ICP_ERR_INVALID_ARG;
    const int64_t k = (int64_t)(ratio * (double)n);  // Open3D RandomDownSample: (int)(ratio * n)
    if (k <= 0) return 0;
    if (hipSetDevice(device) != hipSuccess) return SE3ICP_ERR_HIP;
    int bits = 0;
    while (((int64_t)1 << bits) < n) ++bits;
    bits += bits & 1;
    const int h = bits / 2 > 0 ? bits / 2 : 1;
    const size_t out_bytes = sizeof(double) * 3 * (size_t)n_cases * (size_t)k;
    DevMem d_base, d_T, d_src, d_tgt;
    if (hipMalloc(&d_base.p, sizeof(double) * 3 * (size_t)n) != hipSuccess ||
        hipMalloc(&d_T.p, sizeof(double) * 16 * (size_t)n_cases) != hipSuccess)
        return SE3ICP_ERR_OUT_OF_MEMORY;
    double* so = src_out;
    double* to = tgt_out;
    if (!outputs_on_device) {
        if (hipMalloc(&d_src.p, out_bytes) != hipSuccess || hipMalloc(&d_tgt.p, out_bytes) != hipSuccess)
            return SE3ICP_ERR_OUT_OF_MEMORY;
        so = (double*)d_src.p;
        to = (double*)d_tgt.p;
    }
    if (hipMemcpy(d_base.p, base, sizeof(double) * 3 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_T.p, T, sizeof(double) * 16 * (size_t)n_cases, hipMemcpyHostToDevice) != hipSuccess)
        return SE3ICP_ERR_HIP;
    const int64_t total = 2 * (int64_t)n_cases * k;
    hipLaunchKernelGGL(k_synthetic, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, 0, (const double*)d_base.p,
                       (uint32_t)n, (uint32_t)k, (int)n_cases, (const double*)d_T.p, sqrt(noise_var), h,
                       (uint32_t)seed, (uint32_t)(seed >> 32), so, to);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return SE3ICP_ERR_HIP;
    if (!outputs_on_device) {
        if (hipMemcpy(src_out, so, out_bytes, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(tgt_out, to, out_bytes, hipMemcpyDeviceToHost) != hipSuccess)
            return SE3ICP_ERR_HIP;
    }
    return k;
}

extern "C" int64_t se3icp_synthetic_reference_device(int device, const double* cloud, int64_t n, int32_t n_cases,
                                                     double ratio, double noise_var, double t_range, double r_range,
                                                     int32_t flags, double* src_out, double* tgt_out, double* T_out,
                                                     int outputs_on_device) {
    using namespace se3icp;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return SE3ICP_ERR_NO_DEVICE;
    if (!cloud || !src_out || !tgt_out || n_cases <= 0 || !(ratio >= 0.0 && ratio <= 1.0) || !(noise_var >= 0.0))
        return SE3ICP_ERR_INVALID_ARG;
    if (n <= 0) return SE3ICP_ERR_EMPTY_CLOUD;
    if (n >= (int64_t)1 << 30) return SE3ICP_ERR_INVALID_ARG;
    const refrand::ReferenceDraws D =
        refrand::draw_reference(n, n_cases, ratio, t_range, r_range, (flags & SE3ICP_GEN_ARGS_LTR) != 0, true);
    const int64_t k = D.k;
    if (T_out) std::memcpy(T_out, D.T.data(), sizeof(double) * 16 * (size_t)n_cases);
    if (k <= 0) return 0;
    if (hipSetDevice(device) != hipSuccess) return SE3ICP_ERR_HIP;
    const size_t out_bytes = sizeof(double) * 3 * (size_t)n_cases * (size_t)k;
    DevMem d_cloud, d_si, d_ti, d_T, d_z, d_src, d_tgt;
    if (hipMalloc(&d_cloud.p, sizeof(double) * 3 * (size_t)n) != hipSuccess ||
        hipMalloc(&d_si.p, sizeof(int32_t) * D.src_idx.size()) != hipSuccess ||
        hipMalloc(&d_ti.p, sizeof(int32_t) * D.tgt_idx.size()) != hipSuccess ||
        hipMalloc(&d_T.p, sizeof(double) * D.T.size()) != hipSuccess ||
        hipMalloc(&d_z.p, sizeof(double) * D.z.size()) != hipSuccess)
        return SE3ICP_ERR_OUT_OF_MEMORY;
    double* so = src_out;
    double* to = tgt_out;
    if (!outputs_on_device) {
        if (hipMalloc(&d_src.p, out_bytes) != hipSuccess || hipMalloc(&d_tgt.p, out_bytes) != hipSuccess)
            return SE3ICP_ERR_OUT_OF_MEMORY;
        so = (double*)d_src.p;
        to = (double*)d_tgt.p;
    }
    if (hipMemcpy(d_cloud.p, cloud, sizeof(double) * 3 * (size_t)n, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_si.p, D.src_idx.data(), sizeof(int32_t) * D.src_idx.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_ti.p, D.tgt_idx.data(), sizeof(int32_t) * D.tgt_idx.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_T.p, D.T.data(), sizeof(double) * D.T.size(), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(d_z.p, D.z.data(), sizeof(double) * D.z.size(), hipMemcpyHostToDevice) != hipSuccess)
        return SE3ICP_ERR_HIP;
    const int64_t total = 2 * (int64_t)n_cases * k;
    hipLaunchKernelGGL(k_apply_reference, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, 0,
                       (const double*)d_cloud.p, (const int32_t*)d_si.p, (const int32_t*)d_ti.p, (const double*)d_T.p,
                       (const double*)d_z.p, k, (int)n_cases, std::sqrt(noise_var), so, to);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) return SE3ICP_ERR_HIP;
    if (!outputs_on_device) {
        if (hipMemcpy(src_out, so, out_bytes, hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(tgt_out, to, out_bytes, hipMemcpyDeviceToHost) != hipSuccess)
            return SE3ICP_ERR_HIP;
    }
    return k;
}
