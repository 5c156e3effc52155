// k_setup.hip — one-time per-pair setup kernels (gfx950).
//
//   ingest     AoS f64 input -> SoA xyz64, per-chunk sum/min/max, lounge confidences
//   radius     per-chunk max |p - c|                  (ISR.cpp:112-119, 571-573)
//   normalize  p' = (p + (-c)) * s in place, f32 copy, per-chunk bbox and |p'| max
//                                                      (ISR.cpp:576-582)
//   grid_*     uniform grid (counting sort by cell) over every cloud of the batch
//   knn        exact k nearest neighbours, one wavefront per query point
//                                                      (KDTreeFlann::SearchKNN, ISR.cpp:253)
//   frames     TOLDI LRF -> SE(3) 12-vector (ISR.cpp:241-316), alpha/beta weights
//              (ISR.cpp:597-607), EstimateNormals (ISR.cpp:643), GICP covariance
//              (ISR.cpp:33-52), all fused per point.
// All reductions write fixed per-chunk partials that the host combines in order,
// so results are deterministic run to run.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cfloat>
#include <climits>

#include "devmath.hpp"
#include "view.hpp"

namespace se3icp {

namespace {

__device__ __forceinline__ int find_cloud(const CloudDev* clouds, int nclouds, int g) {
    int lo = 0, hi = nclouds - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (clouds[mid].off <= g) lo = mid; else hi = mid - 1;
    }
    return lo;
}

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

// ------------------------------------------------------------------ uniform grid
__device__ __forceinline__ int cell_coord(double x, double org, double inv_h, int dim) {
    int c = (int)floor((x - org) * inv_h);
    return min(max(c, 0), dim - 1);
}

__global__ __launch_bounds__(256) void k_grid_count(View v) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= v.npts) return;
    const int c = v.cloud_of[g];
    const CloudDev cl = v.clouds[c];
    if (cl.ncells == 0) return;
    const int ix = cell_coord(v.xyz64[g], cl.org[0], cl.inv_h, cl.dims[0]);
    const int iy = cell_coord(v.xyz64[v.ld + g], cl.org[1], cl.inv_h, cl.dims[1]);
    const int iz = cell_coord(v.xyz64[2 * v.ld + g], cl.org[2], cl.inv_h, cl.dims[2]);
    const int cell = cl.cell_off + (iz * cl.dims[1] + iy) * cl.dims[0] + ix;
    v.slot[g] = atomicAdd(&v.cell_cnt[cell], 1);
}

__global__ __launch_bounds__(256) void k_grid_scatter(View v) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= v.npts) return;
    const int c = v.cloud_of[g];
    const CloudDev cl = v.clouds[c];
    if (cl.ncells == 0) return;
    const double x = v.xyz64[g], y = v.xyz64[v.ld + g], z = v.xyz64[2 * v.ld + g];
    const int ix = cell_coord(x, cl.org[0], cl.inv_h, cl.dims[0]);
    const int iy = cell_coord(y, cl.org[1], cl.inv_h, cl.dims[1]);
    const int iz = cell_coord(z, cl.org[2], cl.inv_h, cl.dims[2]);
    const int cell = cl.cell_off + (iz * cl.dims[1] + iy) * cl.dims[0] + ix;
    const int pos = v.cell_start[cell] + v.slot[g];
    v.sidx[pos] = g - cl.off;
    v.sxyz[pos] = x;
    v.sxyz[v.ld + pos] = y;
    v.sxyz[2 * v.ld + pos] = z;
}

// ------------------------------------------------------------------ kNN
// nanoflann L2 order for 3 dims: ((d0^2 + d1^2) + d2^2), no FMA contraction.
__device__ __forceinline__ double l2_3(double ax, double ay, double az, double bx, double by, double bz) {
#pragma clang fp contract(off)
    const double d0 = ax - bx, d1 = ay - by, d2 = az - bz;
    return (d0 * d0 + d1 * d1) + d2 * d2;
}

__device__ __forceinline__ bool key_less(double da, int ia, double db, int ib) {
    return da < db || (da == db && ia < ib);
}

constexpr int kKnnWaves = 4;
constexpr int kKnnBuf = 256;  // top list (<= 128) + staging

// Sort the wave's 256-entry (d2, idx) buffer ascending: register bitonic network,
// 4 keys per lane, cross-lane stages through ds_bpermute (__shfl).
__device__ __forceinline__ void wave_bitonic256(double* bd, int* bi, int lane, int cnt) {
    double kd[4];
    int ki[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int e = lane * 4 + s;
        kd[s] = e < cnt ? bd[e] : DBL_MAX;
        ki[s] = e < cnt ? bi[e] : INT_MAX;
    }
#pragma unroll
    for (int k = 2; k <= 256; k <<= 1) {
#pragma unroll
        for (int jd = k >> 1; jd > 0; jd >>= 1) {
            if (jd >= 4) {
                const int pl = lane ^ (jd >> 2);
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    const int e = lane * 4 + s;
                    const double pd = __shfl(kd[s], pl, 64);
                    const int pi = __shfl(ki[s], pl, 64);
                    const bool up = (e & k) == 0;
                    const bool lower = (e & jd) == 0;
                    const bool pless = key_less(pd, pi, kd[s], ki[s]);
                    const bool mless = key_less(kd[s], ki[s], pd, pi);
                    const bool take = (lower == up) ? pless : mless;
                    if (take) { kd[s] = pd; ki[s] = pi; }
                }
            } else {
#pragma unroll
                for (int s = 0; s < 4; ++s) {
                    if ((s & jd) == 0) {
                        const int t = s | jd;
                        const int e = lane * 4 + s;
                        const bool up = (e & k) == 0;
                        const bool sw = up ? key_less(kd[t], ki[t], kd[s], ki[s]) : key_less(kd[s], ki[s], kd[t], ki[t]);
                        if (sw) {
                            const double td = kd[s]; kd[s] = kd[t]; kd[t] = td;
                            const int ti = ki[s]; ki[s] = ki[t]; ki[t] = ti;
                        }
                    }
                }
            }
        }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        bd[lane * 4 + s] = kd[s];
        bi[lane * 4 + s] = ki[s];
    }
}

// One wavefront per query point: visit grid cells in growing cubes around the
// query cell, keep the k smallest (d2, idx) keys, stop once the k-th distance is
// below the distance to every unvisited cell.  Exact (ties -> lowest index).
__global__ __launch_bounds__(256) void k_knn(View v) {
    __shared__ double s_d[kKnnWaves][kKnnBuf];
    __shared__ int s_i[kKnnWaves][kKnnBuf];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    const int g = blockIdx.x * kKnnWaves + wid;
    if (g >= v.npts) return;
    const int c = v.cloud_of[g];
    const CloudDev cl = v.clouds[c];
    const int K = v.setup[c].k_knn;
    if (K == 0 || cl.ncells == 0) return;
    double* bd = s_d[wid];
    int* bi = s_i[wid];
    const double qx = v.xyz64[g], qy = v.xyz64[v.ld + g], qz = v.xyz64[2 * v.ld + g];
    const int dx = cl.dims[0], dy = cl.dims[1], dz = cl.dims[2];
    const int ix = cell_coord(qx, cl.org[0], cl.inv_h, dx);
    const int iy = cell_coord(qy, cl.org[1], cl.inv_h, dy);
    const int iz = cell_coord(qz, cl.org[2], cl.inv_h, dz);
    const int Kw = min(K, cl.n);
    const int* cs = v.cell_start;
    int nTop = 0, nStg = 0;
    double thr = DBL_MAX;
    int thr_i = INT_MAX;
    const int rmax = max(dx, max(dy, dz));
    for (int r = 1; r <= rmax; ++r) {
        const int x0 = max(ix - r, 0), x1 = min(ix + r, dx - 1);
        const int y0 = max(iy - r, 0), y1 = min(iy + r, dy - 1);
        const int z0 = max(iz - r, 0), z1 = min(iz + r, dz - 1);
        const int ny = y1 - y0 + 1, nrows = ny * (z1 - z0 + 1);
        for (int rb = 0; rb < nrows; rb += 64) {
            const int row = rb + lane;
            int sa = 0, la = 0, sb = 0, lb = 0;
            if (row < nrows) {
                const int y = y0 + row % ny, z = z0 + row / ny;
                const int base = cl.cell_off + (z * dy + y) * dx;
                const bool inner = (r > 1) && abs(y - iy) < r && abs(z - iz) < r;
                if (!inner) {
                    sa = cs[base + x0];
                    la = cs[base + x1 + 1] - sa;
                } else {
                    if (ix - r >= 0) { sa = cs[base + ix - r]; la = cs[base + ix - r + 1] - sa; }
                    if (ix + r < dx) { sb = cs[base + ix + r]; lb = cs[base + ix + r + 1] - sb; }
                }
            }
            // wave inclusive scan of per-lane candidate counts
            const int tl = la + lb;
            int incl = tl;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const int t = __shfl_up(incl, o, 64);
                if (lane >= o) incl += t;
            }
            const int excl = incl - tl;
            const int total = __shfl(incl, 63, 64);
            for (int cb = 0; cb < total; cb += 64) {
                const int ci = cb + lane;
                // owner lane: number of lanes whose inclusive count is <= ci
                int pos = 0;
#pragma unroll
                for (int b = 32; b >= 1; b >>= 1) {
                    const int cand = pos + b;
                    const int iv = __shfl(incl, min(cand, 64) - 1, 64);
                    if (cand <= 64 && iv <= ci) pos = cand;
                }
                const int o = min(pos, 63);
                const int o_sa = __shfl(sa, o, 64), o_la = __shfl(la, o, 64);
                const int o_sb = __shfl(sb, o, 64), o_ex = __shfl(excl, o, 64);
                bool acc = false;
                double d = DBL_MAX;
                int li = INT_MAX;
                if (ci < total) {
                    const int off = ci - o_ex;
                    const int sp = off < o_la ? o_sa + off : o_sb + (off - o_la);
                    li = v.sidx[sp];
                    d = l2_3(qx, qy, qz, v.sxyz[sp], v.sxyz[v.ld + sp], v.sxyz[2 * v.ld + sp]);
                    acc = (nTop < Kw) || key_less(d, li, thr, thr_i);
                }
                const unsigned long long m = __ballot(acc);
                if (acc) {
                    const int at = nTop + nStg + __popcll(m & ((1ull << lane) - 1ull));
                    bd[at] = d;
                    bi[at] = li;
                }
                nStg += __popcll(m);
                if (nTop + nStg > kKnnBuf - 64) {
                    __builtin_amdgcn_wave_barrier();
                    wave_bitonic256(bd, bi, lane, nTop + nStg);
                    __builtin_amdgcn_wave_barrier();
                    nTop = min(Kw, nTop + nStg);
                    nStg = 0;
                    if (nTop == Kw) { thr = bd[Kw - 1]; thr_i = bi[Kw - 1]; }
                }
            }
        }
        if (nStg > 0) {
            __builtin_amdgcn_wave_barrier();
            wave_bitonic256(bd, bi, lane, nTop + nStg);
            __builtin_amdgcn_wave_barrier();
            nTop = min(Kw, nTop + nStg);
            nStg = 0;
            if (nTop == Kw) { thr = bd[Kw - 1]; thr_i = bi[Kw - 1]; }
        }
        const bool covered = x0 == 0 && y0 == 0 && z0 == 0 && x1 == dx - 1 && y1 == dy - 1 && z1 == dz - 1;
        if (covered) break;
        if (nTop == Kw) {
            const double h = cl.h;
            double m = DBL_MAX;
            if (x0 > 0) m = fmin(m, qx - (cl.org[0] + x0 * h));
            if (x1 < dx - 1) m = fmin(m, (cl.org[0] + (x1 + 1) * h) - qx);
            if (y0 > 0) m = fmin(m, qy - (cl.org[1] + y0 * h));
            if (y1 < dy - 1) m = fmin(m, (cl.org[1] + (y1 + 1) * h) - qy);
            if (z0 > 0) m = fmin(m, qz - (cl.org[2] + z0 * h));
            if (z1 < dz - 1) m = fmin(m, (cl.org[2] + (z1 + 1) * h) - qz);
            m -= 1e-9 * h;
            if (m > 0 && thr < m * m) break;
        }
    }
    int* out = v.knn + (size_t)g * v.kmax;
    for (int j = lane; j < K; j += 64) out[j] = j < nTop ? bi[j] : -1;
}

// ------------------------------------------------------------------ frames
__device__ __forceinline__ void atomic_max_nonneg(uint32_t* p, float x) {
    atomicMax(p, __float_as_uint(x));
}

__global__ __launch_bounds__(256) void k_frames(View v) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= v.npts) return;
    const int c = v.cloud_of[g];
    const CloudSetup st = v.setup[c];
    if (st.k_lrf == 0 && st.k_nrm == 0) return;
    const CloudDev cl = v.clouds[c];
    const int* nb = v.knn + (size_t)g * v.kmax;
    const double* X = v.xyz64 + cl.off;
    const double* Y = v.xyz64 + v.ld + cl.off;
    const double* Z = v.xyz64 + 2 * (size_t)v.ld + cl.off;
    const d3 p{v.xyz64[g], v.xyz64[v.ld + g], v.xyz64[2 * v.ld + g]};
    if (st.k_lrf > 0) {
        // computeSingleTOLDISE3Frame, ISR.cpp:241-316
        const int kk = min(st.k_lrf, cl.n);
        const int far = nb[kk - 1];
        const double computed_radius = sqrt(dot3(p - mk3(X[far], Y[far], Z[far]), p - mk3(X[far], Y[far], Z[far])));
        const int rz = kk / 3;
        d3 cen{0, 0, 0};
        for (int i = 1; i < rz; ++i) { const int j = nb[i]; cen = cen + mk3(X[j], Y[j], Z[j]); }
        cen = d3{cen.x / (double)rz, cen.y / (double)rz, cen.z / (double)rz};
        double c00 = 0, c01 = 0, c02 = 0, c11 = 0, c12 = 0, c22 = 0;
        for (int i = 1; i < rz + 1; ++i) {
            const int j = nb[i];
            const d3 q = mk3(X[j], Y[j], Z[j]) - cen;
            c00 += q.x * q.x; c01 += q.x * q.y; c02 += q.x * q.z;
            c11 += q.y * q.y; c12 += q.y * q.z; c22 += q.z * q.z;
        }
        d3 n = jacobi_smallest_evec(c00, c01, c02, c11, c12, c22);
        d3 acc{0, 0, 0}, accs{0, 0, 0};
        for (int i = 1; i < kk; ++i) {
            const int j = nb[i];
            const d3 a = mk3(X[j], Y[j], Z[j]) - p;
            acc = acc + a;
            const double an = dot3(n, a);
            const double r = computed_radius - sqrt(dot3(a, a));
            accs = accs + ((r * r) * (an * an)) * a;
        }
        if (dot3(n, acc) < 0.0) n = d3{-n.x, -n.y, -n.z};
        const d3 zax = n;
        d3 xax = accs - dot3(accs, zax) * zax;
        xax = (1.0 / sqrt(dot3(xax, xax))) * xax;
        const d3 yax = cross3(zax, xax);
        const double al = st.alpha, be = st.beta;
        double f[12] = {al * xax.x, al * xax.y, al * xax.z, al * yax.x, al * yax.y, al * yax.z,
                        al * zax.x, al * zax.y, al * zax.z, be * p.x, be * p.y, be * p.z};
#pragma unroll
        for (int r = 0; r < 12; ++r) v.fr64[(size_t)r * v.ld + g] = f[r];
        if (st.is_target) {
            if (st.cf_target) { f[9] = p.x; f[10] = p.y; f[11] = p.z; }
            double n2 = 0;
#pragma unroll
            for (int r = 0; r < 12; ++r) {
                v.fr32[(size_t)r * v.ld + g] = (float)f[r];
                n2 += f[r] * f[r];
            }
            atomic_max_nonneg(&v.norm12_bits[c], (float)(sqrt(n2) * (1.0 + 1e-6)));
        }
    }
    if (st.k_nrm > 0) {
        // EstimatePerPointCovariances -> ComputeCovariance (cumulants, incl. self) -> FastEigen3x3
        const int kn = min(st.k_nrm, cl.n);
        double c00 = 1, c01 = 0, c02 = 0, c11 = 1, c12 = 0, c22 = 1;
        if (kn >= 3) {
            double cu[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            for (int i = 0; i < kn; ++i) {
                const int j = nb[i];
                const double x = X[j], y = Y[j], z = Z[j];
                cu[0] += x; cu[1] += y; cu[2] += z;
                cu[3] += x * x; cu[4] += x * y; cu[5] += x * z;
                cu[6] += y * y; cu[7] += y * z; cu[8] += z * z;
            }
#pragma unroll
            for (int i = 0; i < 9; ++i) cu[i] /= (double)kn;
            c00 = cu[3] - cu[0] * cu[0];
            c11 = cu[6] - cu[1] * cu[1];
            c22 = cu[8] - cu[2] * cu[2];
            c01 = cu[4] - cu[0] * cu[1];
            c02 = cu[5] - cu[0] * cu[2];
            c12 = cu[7] - cu[1] * cu[2];
        }
        d3 n = fast_eigen3x3(c00, c01, c02, c11, c12, c22);
        if (sqrt(dot3(n, n)) == 0.0) n = d3{0, 0, 1};
        v.nrm64[g] = n.x;
        v.nrm64[v.ld + g] = n.y;
        v.nrm64[2 * (size_t)v.ld + g] = n.z;
        if (st.want_cov) {
            double cv[6];
            gicp_cov_from_normal(n, 1e-3, cv);
#pragma unroll
            for (int r = 0; r < 6; ++r) v.cov64[(size_t)r * v.ld + g] = cv[r];
        }
    }
    if (st.is_target) {
        const double fx = p.x - st.f32_center[0], fy = p.y - st.f32_center[1], fz = p.z - st.f32_center[2];
        atomic_max_nonneg(&v.norm3_bits[c], (float)(sqrt(fx * fx + fy * fy + fz * fz) * (1.0 + 1e-6)));
    }
}

}  // namespace

// ------------------------------------------------------------------ launchers
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
void launch_grid_count(const View& v, hipStream_t s) {
    hipLaunchKernelGGL(k_grid_count, dim3((v.npts + 255) / 256), dim3(256), 0, s, v);
}
int launch_grid_scan(const View& v, int32_t ncells_total, void* temp, size_t* temp_bytes, hipStream_t s) {
    hipError_t e = hipcub::DeviceScan::ExclusiveSum(temp, *temp_bytes, v.cell_cnt, v.cell_start, ncells_total + 1, s);
    return e == hipSuccess ? 0 : -1;
}
void launch_grid_scatter(const View& v, hipStream_t s) {
    hipLaunchKernelGGL(k_grid_scatter, dim3((v.npts + 255) / 256), dim3(256), 0, s, v);
}
void launch_knn(const View& v, hipStream_t s) {
    hipLaunchKernelGGL(k_knn, dim3((v.npts + kKnnWaves - 1) / kKnnWaves), dim3(64 * kKnnWaves), 0, s, v);
}
void launch_frames(const View& v, hipStream_t s) {
    hipLaunchKernelGGL(k_frames, dim3((v.npts + 255) / 256), dim3(256), 0, s, v);
}

}  // namespace se3icp
