// k_setup.hip — one-time per-pair setup kernels (gfx950).
//
//   ingest     AoS f64 input -> SoA xyz64, per-chunk sum/min/max, lounge confidences
//   radius     per-chunk max |p - c|                  (ISR.cpp:112-119, 571-573)
//   normalize  p' = (p + (-c)) * s in place, f32 copy, per-chunk bbox and |p'| max
//                                                      (ISR.cpp:576-582)
//   frames     TOLDI LRF -> SE(3) 12-vector (ISR.cpp:241-316), alpha/beta weights
//              (ISR.cpp:597-607), EstimateNormals (ISR.cpp:643), GICP covariance
//              (ISR.cpp:33-52), all fused per point.
// All reductions write fixed per-chunk partials combined in a fixed order (on the device
// for the registration path: k_pair_centers / k_pair_scales), so results are
// deterministic run to run.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>

#include "devmath.hpp"
#include "view.hpp"

namespace se3icp {

namespace {

template <typename T, class Op>
__device__ __forceinline__ T wave_reduce(T x, Op op) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) x = op(x, __shfl_xor(x, o, 64));
    return x;
}

// block (256 threads) reduction of NV doubles with op; result valid in thread 0
template <int NV, class Op>
__device__ __forceinline__ void block_reduce(double (&v)[NV], Op op) {
    __shared__ double red[4][NV];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = wave_reduce(v[i], op);
    if (lane == 0)
#pragma unroll
        for (int i = 0; i < NV; ++i) red[wid][i] = v[i];
    __syncthreads();
    if (threadIdx.x == 0)
#pragma unroll
        for (int i = 0; i < NV; ++i) v[i] = op(op(red[0][i], red[1][i]), op(red[2][i], red[3][i]));
}

struct OpAdd { __device__ double operator()(double a, double b) const { return a + b; } };
struct OpMin { __device__ double operator()(double a, double b) const { return fmin(a, b); } };
struct OpMax { __device__ double operator()(double a, double b) const { return fmax(a, b); } };

// ISR.cpp:16-30 lounge_point_confidence (min_depth, not squared, in the numerator)
__device__ __forceinline__ double lounge_conf(double depth) {
    const double p1 = 0.002203, p2 = -0.001028, p3 = 0.0005351, min_depth = 0.4;
    const double error = p1 * depth * depth + p2 * depth + p3;
    return (p1 * min_depth + p2 * min_depth + p3) / error;
}

// ------------------------------------------------------------------ ingest
__global__ __launch_bounds__(256) void k_ingest(View v, const ChunkWork* chunks, double* partial) {
    const ChunkWork cw = chunks[blockIdx.x];
    const CloudDev cl = v.clouds[cw.cloud];
    const CloudSetup st = v.setup[cw.cloud];
    const double* in = v.in_ptr[cw.cloud];
    double acc[9] = {0, 0, 0, DBL_MAX, DBL_MAX, DBL_MAX, -DBL_MAX, -DBL_MAX, -DBL_MAX};
    const int end = min(cw.p0 + kChunk, cl.n);
    for (int li = cw.p0 + threadIdx.x; li < end; li += blockDim.x) {
        const double x = in[3 * (size_t)li], y = in[3 * (size_t)li + 1], z = in[3 * (size_t)li + 2];
        const int g = cl.off + li;
        v.xyz64[g] = x;
        v.xyz64[v.ld + g] = y;
        v.xyz64[2 * v.ld + g] = z;
        v.cloud_of[g] = cw.cloud;
        if (st.want_conf) v.conf64[g] = lounge_conf(z);
        acc[0] += x; acc[1] += y; acc[2] += z;
        acc[3] = fmin(acc[3], x); acc[4] = fmin(acc[4], y); acc[5] = fmin(acc[5], z);
        acc[6] = fmax(acc[6], x); acc[7] = fmax(acc[7], y); acc[8] = fmax(acc[8], z);
    }
    double s3[3] = {acc[0], acc[1], acc[2]};
    double mn[3] = {acc[3], acc[4], acc[5]};
    double mx[3] = {acc[6], acc[7], acc[8]};
    block_reduce<3>(s3, OpAdd());
    __syncthreads();
    block_reduce<3>(mn, OpMin());
    __syncthreads();
    block_reduce<3>(mx, OpMax());
    if (threadIdx.x == 0) {
        double* o = partial + (size_t)blockIdx.x * 9;
        o[0] = s3[0]; o[1] = s3[1]; o[2] = s3[2];
        o[3] = mn[0]; o[4] = mn[1]; o[5] = mn[2];
        o[6] = mx[0]; o[7] = mx[1]; o[8] = mx[2];
    }
}

// ------------------------------------------------------------------ radius
__global__ __launch_bounds__(256) void k_radius(View v, const ChunkWork* chunks, const double* centers, double* partial) {
    const ChunkWork cw = chunks[blockIdx.x];
    const CloudDev cl = v.clouds[cw.cloud];
    const double cx = centers[3 * cw.cloud], cy = centers[3 * cw.cloud + 1], cz = centers[3 * cw.cloud + 2];
    double m[1] = {-1.0};
    const int end = min(cw.p0 + kChunk, cl.n);
    for (int li = cw.p0 + threadIdx.x; li < end; li += blockDim.x) {
        const int g = cl.off + li;
        const double dx = v.xyz64[g] - cx, dy = v.xyz64[v.ld + g] - cy, dz = v.xyz64[2 * v.ld + g] - cz;
        m[0] = fmax(m[0], sqrt(dx * dx + dy * dy + dz * dz));
    }
    block_reduce<1>(m, OpMax());
    if (threadIdx.x == 0) partial[blockIdx.x] = m[0];
}

// ------------------------------------------------------------------ normalize
// p' = (p + (-c)) * s   (Translate(-c) then Scale(s, 0); ISR.cpp:576-582)
__global__ __launch_bounds__(256) void k_normalize(View v, const ChunkWork* chunks, double* partial) {
    const ChunkWork cw = chunks[blockIdx.x];
    const CloudDev cl = v.clouds[cw.cloud];
    const CloudSetup st = v.setup[cw.cloud];
    const double ncx = -st.norm_center[0], ncy = -st.norm_center[1], ncz = -st.norm_center[2];
    const double s = st.norm_scale;
    double mn[3] = {DBL_MAX, DBL_MAX, DBL_MAX}, mx[3] = {-DBL_MAX, -DBL_MAX, -DBL_MAX}, r3[1] = {0.0};
    const int end = min(cw.p0 + kChunk, cl.n);
    for (int li = cw.p0 + threadIdx.x; li < end; li += blockDim.x) {
        const int g = cl.off + li;
        const double x = (v.xyz64[g] + ncx) * s;
        const double y = (v.xyz64[v.ld + g] + ncy) * s;
        const double z = (v.xyz64[2 * v.ld + g] + ncz) * s;
        v.xyz64[g] = x;
        v.xyz64[v.ld + g] = y;
        v.xyz64[2 * v.ld + g] = z;
        const double fx = x - st.f32_center[0], fy = y - st.f32_center[1], fz = z - st.f32_center[2];
        v.xyz32[g] = (float)fx;
        v.xyz32[v.ld + g] = (float)fy;
        v.xyz32[2 * v.ld + g] = (float)fz;
        mn[0] = fmin(mn[0], x); mn[1] = fmin(mn[1], y); mn[2] = fmin(mn[2], z);
        mx[0] = fmax(mx[0], x); mx[1] = fmax(mx[1], y); mx[2] = fmax(mx[2], z);
        r3[0] = fmax(r3[0], sqrt(fx * fx + fy * fy + fz * fz));
    }
    block_reduce<3>(mn, OpMin());
    __syncthreads();
    block_reduce<3>(mx, OpMax());
    __syncthreads();
    block_reduce<1>(r3, OpMax());
    if (threadIdx.x == 0) {
        double* o = partial + (size_t)blockIdx.x * 7;
        o[0] = mn[0]; o[1] = mn[1]; o[2] = mn[2];
        o[3] = mx[0]; o[4] = mx[1]; o[5] = mx[2];
        o[6] = r3[0];
    }
}

// ------------------------------------------------------------------ normalization parameters
// The combination of the chunk partials, on the device so the setup never waits for the
// host: one wavefront per cloud / pair, lane l folds chunks l, l+64, ... in order, then a
// fixed butterfly combines the lanes (deterministic run to run).
// GetCenter (arithmetic mean) of every cloud, ISR.cpp:568-570.
__global__ __launch_bounds__(64) void k_pair_centers(View v, const ChunkWork* chunks, int nch, const double* partial,
                                                     double* centers) {
    const int c = blockIdx.x, lane = threadIdx.x;
    double sum[3] = {0.0, 0.0, 0.0};
    for (int k = lane; k < nch; k += 64)
        if (chunks[k].cloud == c)
            for (int a = 0; a < 3; ++a) sum[a] += partial[9 * (size_t)k + a];
    for (int a = 0; a < 3; ++a) sum[a] = wave_reduce(sum[a], OpAdd());
    const int n = v.clouds[c].n;
    if (lane < 3) centers[3 * c + lane] = n > 0 ? sum[lane] / (double)n : 0.0;
}

// s = scale_pre / max(r_src, r_tgt) (ISR.cpp:571-574) and the clouds' CloudSetup
// normalization fields (ISR.cpp:576-582).
__global__ __launch_bounds__(64) void k_pair_scales(View v, const ChunkWork* chunks, int nch, const double* partial,
                                                    const double* centers, double scale_pre, double* scales) {
    const int p = blockIdx.x, lane = threadIdx.x;
    double rad[2] = {-1.0, -1.0};
    for (int k = lane; k < nch; k += 64) {
        const int c = chunks[k].cloud;
        if ((c >> 1) == p) rad[c & 1] = fmax(rad[c & 1], partial[k]);
    }
    rad[0] = wave_reduce(rad[0], OpMax());
    rad[1] = wave_reduce(rad[1], OpMax());
    const double rmax = fmax(rad[0], rad[1]);
    const double sf = scale_pre * (1.0 / rmax);
    if (lane < 2) {
        CloudSetup& st = v.setup[2 * p + lane];
        for (int a = 0; a < 3; ++a) {
            st.norm_center[a] = centers[3 * (2 * p + lane) + a];
            st.f32_center[a] = 0.0;
        }
        st.norm_scale = sf;
    }
    if (lane == 0) scales[p] = sf;
}

// Norm bounds of the targets' search vectors (f32 error certificate, k_nn.hip) from the
// root boxes of their kd-trees: PairDev.tgt_norm3 / tgt_norm12, and PairState.sf.
__device__ float root_norm(const float* lo, const float* hi, int D) {
    double n2 = 0;
    for (int d = 0; d < D; ++d) {
        const double m = fmax(fabs((double)lo[d]), fabs((double)hi[d]));
        n2 += m * m;
    }
    return (float)(sqrt(n2) * (1.0 + 1e-6));
}
__global__ void k_pair_norms(View v, int nnodes3, int nnodes12, const double* scales, double* state_sf,
                             int state_stride) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= v.npairs) return;
    const int c = 2 * p + 1;
    PairDev& P = v.pairs[p];
    P.tgt_norm3 = root_norm(v.t3.lo + (size_t)c * nnodes3 * 3, v.t3.hi + (size_t)c * nnodes3 * 3, 3);
    P.tgt_norm12 = nnodes12 > 0 ? root_norm(v.t12.lo + (size_t)c * nnodes12 * 12, v.t12.hi + (size_t)c * nnodes12 * 12, 12)
                                : 0.f;
    if (scales) state_sf[(size_t)p * state_stride] = scales[p];
}

}  // namespace

// ------------------------------------------------------------------ launchers
void launch_pair_centers(const View& v, const ChunkWork* chunks, int nchunks, const double* partial, double* centers,
                         hipStream_t s) {
    hipLaunchKernelGGL(k_pair_centers, dim3(v.nclouds), dim3(64), 0, s, v, chunks, nchunks, partial, centers);
}
void launch_pair_scales(const View& v, const ChunkWork* chunks, int nchunks, const double* partial,
                        const double* centers, double scale_pre, double* scales, hipStream_t s) {
    hipLaunchKernelGGL(k_pair_scales, dim3(v.nclouds / 2), dim3(64), 0, s, v, chunks, nchunks, partial, centers,
                       scale_pre, scales);
}
void launch_pair_norms(const View& v, int nnodes3, int nnodes12, const double* scales, double* state_sf,
                       int state_stride, hipStream_t s) {
    hipLaunchKernelGGL(k_pair_norms, dim3((v.npairs + 63) / 64), dim3(64), 0, s, v, nnodes3, nnodes12, scales,
                       state_sf, state_stride);
}
void launch_ingest(const View& v, const ChunkWork* chunks, int nchunks, double* partial, hipStream_t s) {
    if (nchunks > 0) hipLaunchKernelGGL(k_ingest, dim3(nchunks), dim3(256), 0, s, v, chunks, partial);
}
void launch_radius(const View& v, const ChunkWork* chunks, int nchunks, const double* centers, double* partial,
                   hipStream_t s) {
    if (nchunks > 0) hipLaunchKernelGGL(k_radius, dim3(nchunks), dim3(256), 0, s, v, chunks, centers, partial);
}
void launch_normalize(const View& v, const ChunkWork* chunks, int nchunks, double* partial, hipStream_t s) {
    if (nchunks > 0) hipLaunchKernelGGL(k_normalize, dim3(nchunks), dim3(256), 0, s, v, chunks, partial);
}

}  // namespace se3icp
