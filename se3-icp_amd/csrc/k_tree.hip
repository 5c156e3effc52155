// k_tree.hip — balanced kd-trees over every cloud of a batch, built on the GPU.
//
// The reference searches nanoflann kd-trees (3-D for TOLDI/normals/R3 NN, 12-D for the
// SE(3) NN, ISR.cpp:586-587, 626).  Here one implicit, balanced tree per cloud is built
// level-synchronously for all clouds at once:
//   level l: every node i covers tree positions [n*i/2^l, n*(i+1)/2^l) of its cloud;
//   its widest dimension is estimated from the bounding box of every kSplitSample-th
//   point (wave-segmented reduction + one atomic per segment), and ONE global radix
//   sort of (cloud, node, coordinate) keys re-orders every node's range so that its
//   lower half forms the left child (a median split).  After L levels the leaves hold
//   <= 64 points: one wavefront.  The exact boxes are then computed bottom-up: a
//   wave per leaf over the tree-ordered vectors, then unions of the children.
// Outputs per cloud: perm (tree position -> point), pos (inverse), the vectors in tree
// order (coalesced leaf loads) and f32 AABBs of all 2^(L+1)-1 nodes (heap order),
// inflated by a few ulps so the f32 boxes bound the f64 points they stand for.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include "tree.hpp"
#include "wave.hpp"

namespace se3icp {

namespace {

__device__ __forceinline__ uint32_t ord_bits(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord_float(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

__global__ __launch_bounds__(256) void k_tree_init(TreeView t) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < t.npts) {
        const CloudDev cl = t.clouds[t.cloud_of[g]];
        t.perm[g] = g - cl.off;
    }
    const size_t nb = (size_t)t.nclouds * t.nnodes * t.D;
    for (size_t i = g; i < nb; i += (size_t)gridDim.x * blockDim.x) {
        t.blo[i] = 0xffffffffu;
        t.bhi[i] = 0u;
    }
}

// Bounding boxes of the nodes of one level: each wave reduces its contiguous runs of
// equal (cloud, node) with a segmented shuffle reduction; run heads issue the atomics.
constexpr int kSplitSample = 8;  // every 8th tree position decides a node's split dimension

template <int D>
__global__ __launch_bounds__(256) void k_tree_bbox(TreeView t, int level) {
    const int g = (blockIdx.x * blockDim.x + threadIdx.x) * kSplitSample;
    const int lane = threadIdx.x & 63;
    const bool valid = g < t.npts;
    int c = -1, node = -1;
    uint32_t lo[D], hi[D];
    if (valid) {
        c = t.cloud_of[g];
        const CloudDev cl = t.clouds[c];
        const int x = g - cl.off;
        node = tree_node_of(x, cl.n, level);
        const int pt = cl.off + t.perm[g];
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const uint32_t u = ord_bits(t.vec[tree_in_ix(t, d, pt)]);
            lo[d] = u;
            hi[d] = u;
        }
    } else {
#pragma unroll
        for (int d = 0; d < D; ++d) { lo[d] = 0xffffffffu; hi[d] = 0u; }
    }
    const long long key = valid ? ((long long)c << 32) | (unsigned)node : -1;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const long long ok = __shfl_down(key, o, 64);
        const bool same = (lane + o < 64) && ok == key;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            const uint32_t ol = __shfl_down(lo[d], o, 64);
            const uint32_t oh = __shfl_down(hi[d], o, 64);
            if (same) { lo[d] = min(lo[d], ol); hi[d] = max(hi[d], oh); }
        }
    }
    const long long prev = __shfl_up(key, 1, 64);
    const bool head = valid && (lane == 0 || prev != key);
    if (head) {
        const size_t base = ((size_t)c * t.nnodes + tree_heap(level, node)) * D;
#pragma unroll
        for (int d = 0; d < D; ++d) {
            atomicMin(&t.blo[base + d], lo[d]);
            atomicMax(&t.bhi[base + d], hi[d]);
        }
    }
}

// widest dimension of every node of the level, then the sort keys:
//   key = (cloud << L | node << (L - level)) << 32 | orderable(coordinate along that dim)
__global__ __launch_bounds__(256) void k_tree_keys(TreeView t, int level, unsigned long long* keys, int32_t* vals) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= t.npts) return;
    const int c = t.cloud_of[g];
    const CloudDev cl = t.clouds[c];
    const int node = tree_node_of(g - cl.off, cl.n, level);
    const size_t base = ((size_t)c * t.nnodes + tree_heap(level, node)) * t.D;
    int best = 0;
    float ext = -1.f;
    for (int d = 0; d < t.D; ++d) {
        const float e = ord_float(t.bhi[base + d]) - ord_float(t.blo[base + d]);
        if (e > ext) { ext = e; best = d; }
    }
    const int p = t.perm[g];
    const uint32_t u = ord_bits(t.vec[tree_in_ix(t, best, cl.off + p)]);
    const unsigned long long hiw = ((unsigned long long)c << t.L) | ((unsigned long long)node << (t.L - level));
    keys[g] = (hiw << 32) | u;
    vals[g] = p;
}

// 32-bit variant: key = ((cloud << level) | node) << qbits | q, with q the coordinate
// quantised to qbits over the node's (sampled) extent.  Any partition at the median
// position yields a valid tree -- the boxes are computed exactly afterwards -- so ties
// from the quantisation only cost split quality, and the sort needs 3-4 digit passes
// of 4-byte keys instead of 5-6 of 8-byte keys.
__global__ __launch_bounds__(256) void k_tree_keys32(TreeView t, int level, int qbits, uint32_t* keys, int32_t* vals) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= t.npts) return;
    const int c = t.cloud_of[g];
    const CloudDev cl = t.clouds[c];
    const int node = tree_node_of(g - cl.off, cl.n, level);
    const size_t base = ((size_t)c * t.nnodes + tree_heap(level, node)) * t.D;
    int best = 0;
    float ext = -1.f, lo = 0.f;
    for (int d = 0; d < t.D; ++d) {
        const float l = ord_float(t.blo[base + d]);
        const float e = ord_float(t.bhi[base + d]) - l;
        if (e > ext) { ext = e; best = d; lo = l; }
    }
    const int p = t.perm[g];
    const float x = t.vec[tree_in_ix(t, best, cl.off + p)];
    const float qmax = (float)((1u << qbits) - 1u);
    float qf = (ext > 0.f && ext < INFINITY) ? (x - lo) * (qmax / ext) : 0.f;
    qf = fminf(fmaxf(qf, 0.f), qmax);  // NaN -> 0
    const uint32_t q = (uint32_t)qf;
    keys[g] = ((((uint32_t)c << level) | (uint32_t)node) << qbits) | q;
    vals[g] = p;
}

// The levels below G in one workgroup per level-G node (<= kLocalMax points): the node's
// permutation stays in LDS and every level is a bitonic sort of (sub-node, coordinate
// along the sub-node's widest dimension) keys -- the same median splits as the global
// levels, without a device-wide radix sort per level.
#ifndef SE3ICP_LOCAL_MAX
#define SE3ICP_LOCAL_MAX 4096
#endif
constexpr int kLocalMax = SE3ICP_LOCAL_MAX;  // power of two
constexpr int kLocalBits = __builtin_ctz(kLocalMax);  // element field of the block sort keys
constexpr int kWaveSortPer = 8;  // sub-nodes of <= 512 points: register sort by one wave
#ifndef SE3ICP_TREE_SPLIT
#define SE3ICP_TREE_SPLIT 1
#endif
#ifndef SE3ICP_TREE_STRIDE
#define SE3ICP_TREE_STRIDE 16
#endif
constexpr int kLocalThreads = 512;

template <int D>
__global__ __launch_bounds__(kLocalThreads) void k_tree_local(TreeView t, int G) {
    __shared__ unsigned long long s_key[kLocalMax];
    __shared__ int32_t s_val[kLocalMax];
    __shared__ int s_best[128];
    const int nG = 1 << G;
    const int c = blockIdx.x / nG, i = blockIdx.x % nG;
    const CloudDev cl = t.clouds[c];
    const int n = cl.n;
    const int A = tree_first(n, G, i), m = tree_first(n, G, i + 1) - A;
    const int tid = threadIdx.x;
    if (m <= 1) return;
    for (int e = tid; e < kLocalMax; e += kLocalThreads) s_val[e] = e < m ? t.perm[cl.off + A + e] : -1;
    for (int l = G; l < t.L; ++l) {
        const int r = l - G;
        const int nsub = 1 << r;  // sub-nodes of this level under the WG's node (<= 128: see the host)
        // split dimension of each sub-node: widest extent of the box of every
        // kSplitSample-th point (the sample of the global levels), a wave per sub-node
        {
            const int lane = tid & 63, wv = tid >> 6;
            for (int k = wv; k < nsub; k += kLocalThreads / 64) {
                const int a0 = tree_first(n, l, (i << r) + k) - A, a1 = tree_first(n, l, (i << r) + k + 1) - A;
                // every 16th point: denser samples measured slower overall (strides 1, 4, 8,
                // 16, 32, 64 tried) -- the 12-D gathers cost build time and did not buy
                // better trees
                const int stride = SE3ICP_TREE_STRIDE;
#if SE3ICP_TREE_SPLIT == 1
                // widest spread: the dimension of largest sample variance
                float s1[D], s2[D];
#pragma unroll
                for (int d = 0; d < D; ++d) { s1[d] = 0.f; s2[d] = 0.f; }
                int cnt = 0;
                for (int e = a0 + lane * stride; e < a1; e += 64 * stride) {
                    const int p = s_val[e];
                    ++cnt;
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        const float x = t.vec[tree_in_ix(t, d, cl.off + p)];
                        s1[d] += x;
                        s2[d] = fmaf(x, x, s2[d]);
                    }
                }
                for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
                const float inv = cnt > 0 ? 1.f / (float)cnt : 0.f;
                int best = 0;
                float ext = -1.f;
#pragma unroll 1  // (a full unroll here crashes amdgcn instruction selection in ROCm 7.2)
                for (int d = 0; d < D; ++d) {
                    float a = s1[d], b = s2[d];
#pragma unroll
                    for (int o = 32; o >= 1; o >>= 1) {
                        a += __shfl_xor(a, o, 64);
                        b += __shfl_xor(b, o, 64);
                    }
                    const float mu = a * inv;
                    const float e = b * inv - mu * mu;
                    if (e > ext) { ext = e; best = d; }
                }
#else
                float lo[D], hi[D];
#pragma unroll
                for (int d = 0; d < D; ++d) { lo[d] = INFINITY; hi[d] = -INFINITY; }
                for (int e = a0 + lane * stride; e < a1; e += 64 * stride) {
                    const int p = s_val[e];
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        const float x = t.vec[tree_in_ix(t, d, cl.off + p)];
                        lo[d] = fminf(lo[d], x);
                        hi[d] = fmaxf(hi[d], x);
                    }
                }
                int best = 0;
                float ext = -1.f;
#pragma unroll 1  // (a full unroll here crashes amdgcn instruction selection in ROCm 7.2)
                for (int d = 0; d < D; ++d) {
                    float l0 = lo[d], h0 = hi[d];
#pragma unroll
                    for (int o = 32; o >= 1; o >>= 1) {
                        l0 = fminf(l0, __shfl_xor(l0, o, 64));
                        h0 = fmaxf(h0, __shfl_xor(h0, o, 64));
                    }
                    const float e = h0 - l0;
                    if (e > ext) { ext = e; best = d; }
                }
#endif
                if (lane == 0) s_best[k] = best;
            }
        }
        __syncthreads();
        const int max_sub = (m + nsub - 1) / nsub + 1;  // sub-node sizes differ by <= 1
        if (max_sub <= 64 * kWaveSortPer) {
            // small sub-nodes: one wave sorts each in registers, (coordinate, point) keys
            const int lane = tid & 63, wv = tid >> 6;
            for (int k = wv; k < nsub; k += kLocalThreads / 64) {
                const int a0 = tree_first(n, l, (i << r) + k) - A, a1 = tree_first(n, l, (i << r) + k + 1) - A;
                const int bd = s_best[k];
                unsigned long long key[kWaveSortPer];
#pragma unroll
                for (int u = 0; u < kWaveSortPer; ++u) {
                    const int e = a0 + lane * kWaveSortPer + u;
                    key[u] = ~0ull;
                    if (e < a1) {
                        const int p = s_val[e];
                        key[u] = ((unsigned long long)ord_bits(t.vec[tree_in_ix(t, bd, cl.off + p)]) << 32) | (unsigned)p;
                    }
                }
                wave_sort_keys<kWaveSortPer>(key);
#pragma unroll
                for (int u = 0; u < kWaveSortPer; ++u) {
                    const int e = a0 + lane * kWaveSortPer + u;
                    if (e < a1) s_val[e] = (int32_t)(unsigned)key[u];
                }
            }
            __syncthreads();
            continue;
        }
        // large sub-nodes: block-wide bitonic sort of (sub-node, coordinate, element) keys
        // (7 + 32 + log2(kLocalMax) bits), kLocalMax / 512 per thread in registers; only the stages with partners
        // in another wave go through LDS
        {
            constexpr int PER = kLocalMax / kLocalThreads;
            unsigned long long k[PER];
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int e = tid * PER + u;
                k[u] = ~0ull;
                if (e < m) {
                    const int sub = tree_node_of(A + e, n, l) - (i << r);
                    const uint32_t c = ord_bits(t.vec[tree_in_ix(t, s_best[sub], cl.off + s_val[e])]);
                    k[u] = ((unsigned long long)(unsigned)sub << (32 + kLocalBits)) | ((unsigned long long)c << kLocalBits) |
                           (unsigned)e;
                }
            }
            bitonic_net<PER, kLocalMax, 64 * PER>(k, tid, s_key);
            __syncthreads();
#pragma unroll
            for (int u = 0; u < PER; ++u) s_key[tid * PER + u] = k[u];
            __syncthreads();
            // gather the permutation through the element field
            int nv[PER];
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int e = tid * PER + u;
                nv[u] = e < m ? s_val[(int)(s_key[e] & (unsigned long long)(kLocalMax - 1))] : 0;
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int e = tid * PER + u;
                if (e < m) s_val[e] = nv[u];
            }
            __syncthreads();
        }
    }
    for (int e = tid; e < m; e += kLocalThreads) t.perm[cl.off + A + e] = s_val[e];
}

__global__ __launch_bounds__(256) void k_tree_finish(TreeView t) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < t.npts) {
        const CloudDev cl = t.clouds[t.cloud_of[g]];
        const int p = t.perm[g];
        const int src = cl.off + p;
        t.pos[src] = g - cl.off;
        const bool want64 = (t.tvec64 != nullptr) & !((t.vec64_sources_only != 0) & ((t.cloud_of[g] & 1) != 0));
        if (t.D == 12) {  // one 48-B and one 96-B row per point (16-B loads)
            const float4* r32 = reinterpret_cast<const float4*>(t.vec + (size_t)src * 12);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const float4 x = r32[k];
                t.tvec[(size_t)(4 * k) * t.ld + g] = x.x;
                t.tvec[(size_t)(4 * k + 1) * t.ld + g] = x.y;
                t.tvec[(size_t)(4 * k + 2) * t.ld + g] = x.z;
                t.tvec[(size_t)(4 * k + 3) * t.ld + g] = x.w;
            }
            if (want64) {
                const double2* r64 = reinterpret_cast<const double2*>(t.vec64 + (size_t)src * 12);
#pragma unroll
                for (int k = 0; k < 6; ++k) {
                    const double2 x = r64[k];
                    t.tvec64[(size_t)(2 * k) * t.ld + g] = x.x;
                    t.tvec64[(size_t)(2 * k + 1) * t.ld + g] = x.y;
                }
            }
        } else {
            for (int d = 0; d < t.D; ++d) t.tvec[(size_t)d * t.ld + g] = t.vec[(size_t)d * t.ld + src];
            if (want64)
                for (int d = 0; d < t.D; ++d) t.tvec64[(size_t)d * t.ld + g] = t.vec64[(size_t)d * t.ld + src];
        }
    }
}

// exact f32 box of every leaf from the tree-ordered vectors (one wave per leaf),
// inflated so that it bounds the f64 values the f32 vectors were rounded from
template <int D>
__global__ __launch_bounds__(256) void k_tree_leafbox(TreeView t) {
    const int lane = threadIdx.x & 63;
    const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int nleaf = 1 << t.L;
    if (w >= t.nclouds * nleaf) return;
    const int c = w / nleaf, i = w % nleaf;
    const CloudDev cl = t.clouds[c];
    const int a = tree_first(cl.n, t.L, i), b = tree_first(cl.n, t.L, i + 1);
    const bool valid = lane < b - a;
    const size_t base = ((size_t)c * t.nnodes + tree_heap(t.L, i)) * D;
#pragma unroll
    for (int d = 0; d < D; ++d) {
        float lo = INFINITY, hi = -INFINITY;
        if (valid) lo = hi = t.tvec[(size_t)d * t.ld + cl.off + a + lane];
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            lo = fminf(lo, __shfl_xor(lo, o, 64));
            hi = fmaxf(hi, __shfl_xor(hi, o, 64));
        }
        if (lane == 0) {
            if (lo <= hi) {
                lo = lo - (fabsf(lo) * 4.8e-7f + 1e-30f);
                hi = hi + (fabsf(hi) * 4.8e-7f + 1e-30f);
            }
            t.lo[base + d] = lo;  // empty leaf: [inf, -inf], a box no query reaches
            t.hi[base + d] = hi;
        }
    }
}

// internal boxes = unions of the children, level by level (one block per cloud)
__global__ __launch_bounds__(1024) void k_tree_up(TreeView t) {
    const int c = blockIdx.x;
    for (int l = t.L - 1; l >= 0; --l) {
        const int items = (1 << l) * t.D;
        for (int it = threadIdx.x; it < items; it += blockDim.x) {
            const int i = it / t.D, d = it % t.D;
            const int h = tree_heap(l, i);
            const size_t o = (size_t)c * t.nnodes * t.D;
            const size_t cl = o + (size_t)(2 * h + 1) * t.D + d, cr = o + (size_t)(2 * h + 2) * t.D + d;
            t.lo[o + (size_t)h * t.D + d] = fminf(t.lo[cl], t.lo[cr]);
            t.hi[o + (size_t)h * t.D + d] = fmaxf(t.hi[cl], t.hi[cr]);
        }
        __syncthreads();
    }
}

}  // namespace

int build_trees(TreeView t, void* sort_tmp, size_t sort_tmp_bytes, unsigned long long* keys0,
                unsigned long long* keys1, int32_t* vals1, hipStream_t s) {
    const int nb = (t.npts + 255) / 256;
    const int nbs = (t.npts + 256 * kSplitSample - 1) / (256 * kSplitSample);
    const int gfill = std::max(nb, 64);
    auto bbox = (t.D == 12) ? k_tree_bbox<12> : k_tree_bbox<3>;
    hipLaunchKernelGGL(k_tree_init, dim3(gfill), dim3(256), 0, s, t);
    int cbits = 0;
    while ((1 << cbits) < t.nclouds) ++cbits;
    const int end_bit = 32 + t.L + cbits;
    // global levels until every node fits one workgroup's LDS sort (and <= 128 sub-nodes below)
    int max_n = 0;
    for (int c = 0; c < t.nclouds; ++c) max_n = std::max(max_n, t.host_n ? t.host_n[c] : 0);
    int G = 0;
    while (G < t.L && (((long long)max_n + (1ll << G) - 1) >> G) > kLocalMax) ++G;
    if (t.L - 1 - G > 7) G = t.L - 8;
    if (!t.host_n) G = t.L;
    for (int l = 0; l < G; ++l) {
        hipLaunchKernelGGL(bbox, dim3(nbs), dim3(256), 0, s, t, l);
        // 24-bit keys (3 passes) while >= 8 quantisation bits remain, then 32-bit keys,
        // then the exact 64-bit keys (very large batches only)
        const int q24 = 24 - cbits - l, q32 = 32 - cbits - l;
        size_t bytes = sort_tmp_bytes;
        if (q24 >= 8 || q32 >= 8) {
            const int qb = q24 >= 8 ? q24 : q32;
            const int eb = q24 >= 8 ? 24 : 32;
            uint32_t* k0 = reinterpret_cast<uint32_t*>(keys0);
            uint32_t* k1 = reinterpret_cast<uint32_t*>(keys1);
            hipLaunchKernelGGL(k_tree_keys32, dim3(nb), dim3(256), 0, s, t, l, qb, k0, vals1);
            if (hipcub::DeviceRadixSort::SortPairs(sort_tmp, bytes, k0, k1, vals1, t.perm, t.npts, 0, eb, s) !=
                hipSuccess)
                return -1;
        } else {
            hipLaunchKernelGGL(k_tree_keys, dim3(nb), dim3(256), 0, s, t, l, keys0, vals1);
            if (hipcub::DeviceRadixSort::SortPairs(sort_tmp, bytes, keys0, keys1, vals1, t.perm, t.npts, 0, end_bit,
                                                   s) != hipSuccess)
                return -1;
        }
    }
    if (G < t.L)
        hipLaunchKernelGGL(t.D == 12 ? k_tree_local<12> : k_tree_local<3>, dim3(t.nclouds << G), dim3(kLocalThreads), 0,
                           s, t, G);
    hipLaunchKernelGGL(k_tree_finish, dim3(nb), dim3(256), 0, s, t);
    const int nleaves = t.nclouds << t.L;
    hipLaunchKernelGGL(t.D == 12 ? k_tree_leafbox<12> : k_tree_leafbox<3>, dim3((nleaves + 3) / 4), dim3(256), 0, s, t);
    hipLaunchKernelGGL(k_tree_up, dim3(t.nclouds), dim3(1024), 0, s, t);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t tree_sort_temp_bytes(int npts, int end_bit) {
    size_t b64 = 0, b32 = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, b64, (unsigned long long*)nullptr, (unsigned long long*)nullptr,
                                             (int32_t*)nullptr, (int32_t*)nullptr, npts, 0, end_bit, (hipStream_t)0);
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, b32, (uint32_t*)nullptr, (uint32_t*)nullptr, (int32_t*)nullptr,
                                             (int32_t*)nullptr, npts, 0, 32, (hipStream_t)0);
    return std::max(b64, b32);
}

}  // namespace se3icp
