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
            const uint32_t u = ord_bits(t.vec[(size_t)d * t.ld + pt]);
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
    const uint32_t u = ord_bits(t.vec[(size_t)best * t.ld + cl.off + p]);
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
    const float x = t.vec[(size_t)best * t.ld + cl.off + p];
    const float qmax = (float)((1u << qbits) - 1u);
    float qf = (ext > 0.f && ext < INFINITY) ? (x - lo) * (qmax / ext) : 0.f;
    qf = fminf(fmaxf(qf, 0.f), qmax);  // NaN -> 0
    const uint32_t q = (uint32_t)qf;
    keys[g] = ((((uint32_t)c << level) | (uint32_t)node) << qbits) | q;
    vals[g] = p;
}

__global__ __launch_bounds__(256) void k_tree_finish(TreeView t) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < t.npts) {
        const CloudDev cl = t.clouds[t.cloud_of[g]];
        const int p = t.perm[g];
        t.pos[cl.off + p] = g - cl.off;
        for (int d = 0; d < t.D; ++d) t.tvec[(size_t)d * t.ld + g] = t.vec[(size_t)d * t.ld + cl.off + p];
        if (t.tvec64)
            for (int d = 0; d < t.D; ++d) t.tvec64[(size_t)d * t.ld + g] = t.vec64[(size_t)d * t.ld + cl.off + p];
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
    for (int l = 0; l < t.L; ++l) {
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
