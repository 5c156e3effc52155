// k_tree.hip — balanced kd-trees over every cloud of a batch, built on the GPU.
//
// The reference searches nanoflann kd-trees (3-D for TOLDI/normals/R3 NN, 12-D for the
// SE(3) NN, ISR.cpp:586-587, 626).  Here one implicit, balanced tree per cloud is built
// level-synchronously for all clouds at once (build_trees at the end of this file):
//   level l: every node i covers tree positions [n*i/2^l, n*(i+1)/2^l) of its cloud and is
//   split by a stable median partition (ties keep tree order) of a coordinate quantised to
//   a 22-bit key -- no device-wide sort.
//   * global levels while the nodes hold more than kLocalMax (4096) points: the first ones,
//     while there are fewer than kTreeWgMin nodes (12-D: 2 kTreeWgMin), by the multi-pass k_part_* sequence
//     (sampled box -> split dimension, block histograms of the top 11 key bits, the median
//     bin, its low 11 bits, segmented counts, one carry scan, scatter); the rest by one
//     k_tree_level launch per level (a workgroup per node);
//   * below that, k_tree_local: one workgroup per node holds its permutation in LDS, splits
//     every sub-node at the median of its largest-sample-variance coordinate, and writes
//     the final permutation, its inverse, the tree-ordered vectors and the boxes of its
//     leaves and inner nodes; k_tree_up unions the boxes above.
//   At C4 (16 clouds of ~120k points): 17 launches for the 3-D tree, 25 for the 12-D one.
//   Leaves hold <= 64 points.
// Outputs per cloud: perm (tree position -> point), pos (inverse), the vectors in tree
// order (coalesced leaf loads) and f32 AABBs of all 2^(L+1)-1 nodes (heap order),
// inflated by a few ulps so the f32 boxes bound the f64 points they stand for.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <type_traits>

#include "tree.hpp"
#include "wave.hpp"

namespace se3icp {

namespace {

#ifdef SE3ICP_PROF
// k_tree_local phase ends over all workgroups (100 MHz clock): [D == 12][0] start (min),
// [1..4] the latest end of load / levels / final / boxes
__device__ unsigned long long g_tree_prof[2][5] = {{~0ull, 0, 0, 0, 0}, {~0ull, 0, 0, 0, 0}};
// k_tree_local per level below G: summed workgroup time of levels 0..7, [8] workgroups
__device__ unsigned long long g_tree_lev[2][9];
#endif

__device__ __forceinline__ uint32_t ord_bits(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord_float(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

// identity permutations; the 12-D input rows copied into columns (t.vecT); the sampled-box
// scratch of the first `box_nodes` heap nodes of every cloud (the levels k_tree_bbox serves)
// cleared
__global__ __launch_bounds__(256) void k_tree_init(TreeView t, int32_t* perm2, int box_nodes) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g < t.npts) {
        const CloudDev cl = t.clouds[t.cloud_of[g]];
        t.perm[g] = g - cl.off;
        perm2[g] = g - cl.off;  // (both buffers hold valid point indices at all times)
        if (t.D == 12) {
            const float4* r = reinterpret_cast<const float4*>(t.vec + (size_t)g * 12);
#pragma unroll
            for (int k = 0; k < 3; ++k) {
                const float4 x = r[k];
                t.vecT[(size_t)(4 * k) * t.ld + g] = x.x;
                t.vecT[(size_t)(4 * k + 1) * t.ld + g] = x.y;
                t.vecT[(size_t)(4 * k + 2) * t.ld + g] = x.z;
                t.vecT[(size_t)(4 * k + 3) * t.ld + g] = x.w;
            }
        }
    }
    const int per = box_nodes * t.D;
    const size_t nb = (size_t)t.nclouds * per;
    for (size_t i = g; i < nb; i += (size_t)gridDim.x * blockDim.x) {
        const size_t at = (i / per) * ((size_t)t.nnodes * t.D) + i % per;
        t.blo[at] = 0xffffffffu;
        t.bhi[at] = 0u;
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
    // a wave whose samples all fall in one node (the common case: nodes of the global
    // levels span thousands of positions) reduces with DPP / permlane butterflies; a wave
    // spanning several nodes, by a segmented shuffle reduction
    const long long key0 = ((long long)__builtin_amdgcn_readfirstlane((int)(key >> 32)) << 32) |
                           (unsigned)__builtin_amdgcn_readfirstlane((int)key);
    const bool uniform = __ballot(key == key0) == ~0ull;
    bool head;
    if (uniform) {
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                lo[d] = min(lo[d], xor_lane(lo[d], o));
                hi[d] = max(hi[d], xor_lane(hi[d], o));
            }
        }
        head = (int)valid & (int)(lane == 0);
    } else {
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
        head = valid && (lane == 0 || prev != key);
    }
    // the block's waves combine in LDS first (the block's samples span at most a few nodes):
    // one global atomic per node, dimension and block instead of one per wave
    __shared__ uint32_t s_lo[4][D], s_hi[4][D];
    __shared__ long long s_key0;
    if (threadIdx.x < 4 * D) {
        s_lo[threadIdx.x / D][threadIdx.x % D] = 0xffffffffu;
        s_hi[threadIdx.x / D][threadIdx.x % D] = 0u;
    }
    if (threadIdx.x == 0) s_key0 = key;  // (the block's first sample: the smallest key)
    __syncthreads();
    const long long k0 = s_key0;
    const int slot = (k0 >= 0 && valid && (key >> 32) == (k0 >> 32)) ? node - (int)(unsigned)k0 : 4;
    if (head) {
        if ((unsigned)slot < 4u) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                atomicMin(&s_lo[slot][d], lo[d]);
                atomicMax(&s_hi[slot][d], hi[d]);
            }
        } else {
            const size_t base = ((size_t)c * t.nnodes + tree_heap(level, node)) * D;
#pragma unroll
            for (int d = 0; d < D; ++d) {
                atomicMin(&t.blo[base + d], lo[d]);
                atomicMax(&t.bhi[base + d], hi[d]);
            }
        }
    }
    __syncthreads();
    if ((int)(threadIdx.x < 4 * D) & (int)(k0 >= 0)) {
        const int sl = threadIdx.x / D, d = threadIdx.x % D;
        if (s_lo[sl][d] <= s_hi[sl][d]) {
            const int c0 = (int)(k0 >> 32), n0 = (int)(unsigned)k0 + sl;
            const size_t base = ((size_t)c0 * t.nnodes + tree_heap(level, n0)) * D;
            atomicMin(&t.blo[base + d], s_lo[sl][d]);
            atomicMax(&t.bhi[base + d], s_hi[sl][d]);
        }
    }
}

// ---- global levels: a stable median partition of every node of the level, all clouds at
// once, in five passes over the level's points (no device-wide sort).
//   hist    the coordinate along the node's widest (sampled) dimension, quantised to
//           kPartBins bins of the node's extent -> per-block histograms in LDS (q kept per point)
//   select  per node: its histogram from its blocks', the bin holding the median position, and how many of its points
//           go left (the rest of that bin goes right; any partition at the median
//           position is a valid tree: the boxes are computed exactly afterwards)
//   hist2 / select2  the same inside the median bin with the key's fine bits (a 22-bit split)
//   count   per block of kPartElems consecutive tree positions: the (left, tie) counts of
//           the points after the block's last node start (segmented carries)
//   scan    the carries across blocks (one workgroup)
//   scatter each point's rank among its node's points of the same class -> its new position
// Ties keep their tree order, so the build is deterministic.
constexpr int kPartBits = 11, kPartBins = 1 << kPartBits;  // bins per pass; keys of 2 * kPartBits bits
// (split dimension: the widest sampled extent; the largest sample variance, as the LDS
// levels use, measured +9 % SE(3) NN time at the global levels)
constexpr int kPartThreads = 256, kPartPer = 4, kPartElems = kPartThreads * kPartPer;
constexpr int kSelThreads = 1024, kSelPer = kPartBins / kSelThreads;
constexpr int kHistPer = 8, kHistElems = kPartThreads * kHistPer;  // tree positions per histogram block

struct PartSel {
    int32_t bin;   // the median bin
    int32_t tie_left;  // its points that go left (in tree order)
    int32_t tie_n;     // its points
    int32_t pad;
};

// split of a node: its widest dimension and the quantisation of that coordinate
struct PartDim {
    int32_t best;
    float lo, scale;  // key = (x - lo) * scale, clamped to [0, 2^(2 kPartBits) - 1]
    int32_t pad;
};
constexpr float kKeyMax = (float)((1 << (2 * kPartBits)) - 1);

// widest dimension of a box given as orderable bits (blo/bhi)
__device__ __forceinline__ PartDim part_dim_of(const uint32_t* blo, const uint32_t* bhi, int D) {
    int best = 0;
    float ext = -1.f, lo = 0.f;
    for (int d = 0; d < D; ++d) {
        const float l = ord_float(blo[d]);
        const float e = ord_float(bhi[d]) - l;
        if (e > ext) { ext = e; best = d; lo = l; }
    }
    PartDim r;
    r.best = best;
    r.lo = lo;
    r.scale = (ext > 0.f && ext < INFINITY) ? kKeyMax / ext : 0.f;
    r.pad = 0;
    return r;
}

// every node's split from its sampled box (k_tree_bbox); once per node, not per point
__global__ __launch_bounds__(64) void k_part_dims(TreeView t, int level, PartDim* dims) {
    const int id = blockIdx.x * 64 + threadIdx.x;
    if (id >= (t.nclouds << level)) return;
    const int c = id >> level, node = id & ((1 << level) - 1);
    const size_t base = ((size_t)c * t.nnodes + tree_heap(level, node)) * t.D;
    dims[id] = part_dim_of(t.blo + base, t.bhi + base, t.D);
}

// node ids (cloud << level | node) grow with the tree position
__device__ __forceinline__ int part_node_id(int c, int level, int node) { return (c << level) + node; }
__device__ __forceinline__ int part_node_id_at(const TreeView& t, int level, int g) {
    const int c = t.cloud_of[g];
    const CloudDev cl = t.clouds[c];
    return part_node_id(c, level, tree_node_of(g - cl.off, cl.n, level));
}

// Per block of kHistElems tree positions: the histograms of the (at most) two nodes the
// block starts in, in LDS, written out whole (dense[block][2][bins]); points of further
// nodes (small clouds) go to the per-node overflow histograms by global atomics.
__global__ __launch_bounds__(kPartThreads) void k_part_hist(TreeView t, int level, const PartDim* dims, uint32_t* q_out,
                                                           uint32_t* overflow) {
    __shared__ uint32_t s_h[2 * kPartBins];
    const int tid = threadIdx.x;
    for (int i = tid; i < 2 * kPartBins; i += kPartThreads) s_h[i] = 0u;
    const int g0 = blockIdx.x * kHistElems;
    const int id0 = part_node_id_at(t, level, g0);
    __syncthreads();
#pragma unroll 4
    for (int u = 0; u < kHistPer; ++u) {
        const int g = g0 + u * kPartThreads + tid;
        if (g < t.npts) {
            const int c = t.cloud_of[g];
            const CloudDev cl = t.clouds[c];
            const int node = tree_node_of(g - cl.off, cl.n, level);
            const int id = part_node_id(c, level, node), slot = id - id0;
            const PartDim pd = dims[id];
            const float x = tree_in_col(t, pd.best, cl.off + t.perm[g]);
            float qf = (x - pd.lo) * pd.scale;
            qf = fminf(fmaxf(qf, 0.f), kKeyMax);  // NaN -> 0
            const uint32_t key = (uint32_t)qf;
            q_out[g] = key;
            const uint32_t q = key >> kPartBits;  // coarse bin
            if (slot < 2) atomicAdd(&s_h[slot * kPartBins + q], 1u);
            else atomicAdd(&overflow[(size_t)id * kPartBins + q], 1u);
        }
    }
    __syncthreads();
    // the block's two node histograms added into the per-node histograms (its non-zero bins;
    // integer adds: the order does not matter), so k_part_select reads one histogram per node
    for (int i = tid; i < 2 * kPartBins; i += kPartThreads) {
        const uint32_t x = s_h[i];
        if (x) atomicAdd(&overflow[(size_t)(id0 + i / kPartBins) * kPartBins + (i & (kPartBins - 1))], x);
    }
}

// one workgroup per node of the level: its histogram (summed by k_part_hist's atomics),
// the median bin; the overflow histogram is cleared for the next level
__global__ __launch_bounds__(kSelThreads) void k_part_select(TreeView t, int level, uint32_t* overflow, PartSel* sel) {
    __shared__ uint32_t s_sum[kSelThreads];
    const int nl = 1 << level;
    const int id = blockIdx.x;
    const int c = id >> level, node = id & (nl - 1);
    const CloudDev cl = t.clouds[c];
    const int a = tree_first(cl.n, level, node);
    const int mL = tree_first(cl.n, level + 1, 2 * node + 1) - a;
    const int tid = threadIdx.x;
    uint32_t v[kSelPer];
    uint32_t* ov = overflow + (size_t)id * kPartBins;
#pragma unroll
    for (int k = 0; k < kSelPer; ++k) {
        v[k] = ov[tid * kSelPer + k];
        ov[tid * kSelPer + k] = 0u;
    }
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < kSelPer; ++k) tot += v[k];
    s_sum[tid] = tot;
    __syncthreads();
    for (int o = 1; o < kSelThreads; o <<= 1) {  // inclusive scan of the threads' totals
        const uint32_t add = tid >= o ? s_sum[tid - o] : 0u;
        __syncthreads();
        s_sum[tid] += add;
        __syncthreads();
    }
    uint32_t cum = tid > 0 ? s_sum[tid - 1] : 0u;  // points in the bins before this thread's
    // the first bin whose inclusive count reaches mL (bin 0 when mL = 0: everything goes right)
#pragma unroll
    for (int k = 0; k < kSelPer; ++k) {
        const uint32_t nxt = cum + v[k];
        if (((int)(cum < (uint32_t)mL) & (int)(nxt >= (uint32_t)mL)) | ((int)(mL == 0) & (int)(tid == 0) & (int)(k == 0))) {
            PartSel r;
            r.bin = tid * kSelPer + k;
            r.tie_left = mL - (int)cum;
            r.tie_n = (int)v[k];
            r.pad = 0;
            sel[id] = r;
        }
        cum = nxt;
    }
}

// second pass inside the median bin: the fine bits of its points' keys
__global__ __launch_bounds__(256) void k_part_hist2(TreeView t, int level, const uint32_t* key, const PartSel* sel,
                                                   uint32_t* fine) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= t.npts) return;
    const int id = part_node_id_at(t, level, g);
    const uint32_t k = key[g];
    if ((int)(k >> kPartBits) == sel[id].bin) atomicAdd(&fine[(size_t)id * kPartBins + (k & (kPartBins - 1))], 1u);
}

// the fine bin holding the median position; sel becomes the full-key threshold
__global__ __launch_bounds__(256) void k_part_select2(uint32_t* fine, PartSel* sel) {
    __shared__ uint32_t s_sum[256];
    constexpr int kPer = kPartBins / 256;
    const int id = blockIdx.x, tid = threadIdx.x;
    const PartSel r = sel[id];
    const int want = r.tie_left;  // points of the coarse bin that go left
    uint32_t* h = fine + (size_t)id * kPartBins;
    uint32_t v[kPer];
    uint32_t tot = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        v[k] = h[tid * kPer + k];
        h[tid * kPer + k] = 0u;
        tot += v[k];
    }
    s_sum[tid] = tot;
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {
        const uint32_t add = tid >= o ? s_sum[tid - o] : 0u;
        __syncthreads();
        s_sum[tid] += add;
        __syncthreads();
    }
    uint32_t cum = tid > 0 ? s_sum[tid - 1] : 0u;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const uint32_t nxt = cum + v[k];
        if (((int)(cum < (uint32_t)want) & (int)(nxt >= (uint32_t)want)) | ((int)(want == 0) & (int)(tid == 0) & (int)(k == 0))) {
            PartSel o;
            o.bin = (r.bin << kPartBits) | (tid * kPer + k);
            o.tie_left = want - (int)cum;
            o.tie_n = (int)v[k];
            o.pad = 0;
            sel[id] = o;
        }
        cum = nxt;
    }
}

// (flag, packed counts) segmented sums: flag = a node starts in the span; counts = points
// of class left (low 32 bits) and tie (high 32 bits) since the span's last node start
struct SegCnt {
    unsigned long long v;
    int f;
};
__device__ __forceinline__ SegCnt seg_add(SegCnt a, SegCnt b) { return SegCnt{b.f ? b.v : a.v + b.v, a.f | b.f}; }

__device__ __forceinline__ SegCnt part_class(const TreeView& t, int level, const uint32_t* q, const PartSel* sel, int g,
                                             int* cls, int* node_out, int* c_out) {
    const int c = t.cloud_of[g];
    const CloudDev cl = t.clouds[c];
    const int x = g - cl.off;
    const int node = tree_node_of(x, cl.n, level);
    const PartSel r = sel[part_node_id(c, level, node)];
    const int qq = (int)q[g];  // (full key against the full-key threshold)
    const int k = qq < r.bin ? 0 : (qq == r.bin ? 1 : 2);
    *cls = k;
    *node_out = node;
    *c_out = c;
    return SegCnt{k == 0 ? 1ull : (k == 1 ? (1ull << 32) : 0ull), x == tree_first(cl.n, level, node) ? 1 : 0};
}

// block-wide segmented scan of one SegCnt per thread (256 threads): the inclusive value
// and the exclusive one (what precedes the thread in the block)
__device__ __forceinline__ SegCnt block_seg_scan(SegCnt x, SegCnt* s_wave, SegCnt* excl) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        SegCnt y;
        y.v = __shfl_up(x.v, o, 64);
        y.f = __shfl_up(x.f, o, 64);
        if (lane >= o) x = seg_add(y, x);
    }
    SegCnt ex;
    ex.v = __shfl_up(x.v, 1, 64);
    ex.f = __shfl_up(x.f, 1, 64);
    if (lane == 0) ex = SegCnt{0ull, 0};
    if (lane == 63) s_wave[wv] = x;
    __syncthreads();
    SegCnt pre{0ull, 0};
    for (int w = 0; w < wv; ++w) pre = seg_add(pre, s_wave[w]);
    __syncthreads();
    *excl = seg_add(pre, ex);
    return seg_add(pre, x);
}

__global__ __launch_bounds__(kPartThreads) void k_part_count(TreeView t, int level, const uint32_t* q, const PartSel* sel,
                                                            SegCnt* tails) {
    __shared__ SegCnt s_wave[kPartThreads / 64];
    const int g0 = blockIdx.x * kPartElems + threadIdx.x * kPartPer;
    SegCnt acc{0ull, 0};
#pragma unroll
    for (int u = 0; u < kPartPer; ++u) {
        const int g = g0 + u;
        if (g < t.npts) {
            int k, node, c;
            acc = seg_add(acc, part_class(t, level, q, sel, g, &k, &node, &c));
        }
    }
    SegCnt ex;
    const SegCnt inc = block_seg_scan(acc, s_wave, &ex);
    if (threadIdx.x == kPartThreads - 1) tails[blockIdx.x] = inc;
}

// exclusive segmented scan of the blocks' tails: carry[k] = the counts entering block k
__global__ __launch_bounds__(1024) void k_part_scan(const SegCnt* tails, int nblk, SegCnt* carry) {
    __shared__ SegCnt s_t[1024];
    const int tid = threadIdx.x;
    const int per = (nblk + 1023) / 1024;
    const int k0 = tid * per, k1 = min(nblk, k0 + per);
    SegCnt acc{0ull, 0};
    for (int k = k0; k < k1; ++k) acc = seg_add(acc, tails[k]);
    s_t[tid] = acc;
    __syncthreads();
    for (int o = 1; o < 1024; o <<= 1) {
        const SegCnt y = tid >= o ? s_t[tid - o] : SegCnt{0ull, 0};
        __syncthreads();
        if (tid >= o) s_t[tid] = seg_add(y, s_t[tid]);
        __syncthreads();
    }
    SegCnt run = tid > 0 ? s_t[tid - 1] : SegCnt{0ull, 0};
    for (int k = k0; k < k1; ++k) {
        carry[k] = run;
        run = seg_add(run, tails[k]);
    }
}

__global__ __launch_bounds__(kPartThreads) void k_part_scatter(TreeView t, int level, const uint32_t* q, const PartSel* sel,
                                                              const SegCnt* carry, int32_t* perm_out) {
    __shared__ SegCnt s_wave[kPartThreads / 64];
    const int g0 = blockIdx.x * kPartElems + threadIdx.x * kPartPer;
    SegCnt self[kPartPer];
    int cls[kPartPer], nodes[kPartPer], cs[kPartPer];
    SegCnt acc{0ull, 0};
#pragma unroll
    for (int u = 0; u < kPartPer; ++u) {
        const int g = g0 + u;
        self[u] = SegCnt{0ull, 0};
        cls[u] = 2;
        nodes[u] = 0;
        cs[u] = 0;
        if (g < t.npts) self[u] = part_class(t, level, q, sel, g, &cls[u], &nodes[u], &cs[u]);
        acc = seg_add(acc, self[u]);
    }
    SegCnt ex;
    (void)block_seg_scan(acc, s_wave, &ex);
    // the counts of this thread's node before its first point: the block's carry, then the
    // threads before it in the block
    SegCnt run = seg_add(carry[blockIdx.x], ex);
#pragma unroll
    for (int u = 0; u < kPartPer; ++u) {
        const int g = g0 + u;
        if (self[u].f) run = SegCnt{0ull, 0};
        if (g < t.npts) {
            const CloudDev cl = t.clouds[cs[u]];
            const int a = tree_first(cl.n, level, nodes[u]);
            const int mL = tree_first(cl.n, level + 1, 2 * nodes[u] + 1) - a;
            const PartSel r = sel[part_node_id(cs[u], level, nodes[u])];
            const int r0 = (int)(unsigned)run.v, r1 = (int)(unsigned)(run.v >> 32);
            const int x = g - cl.off;
            int dst;
            if (cls[u] == 0) dst = a + r0;
            else if (cls[u] == 1) dst = r1 < r.tie_left ? a + (mL - r.tie_left) + r1 : a + mL + (r1 - r.tie_left);
            else dst = a + mL + (r.tie_n - r.tie_left) + ((x - a) - r0 - r1);
            if ((unsigned)dst < (unsigned)cl.n) perm_out[cl.off + dst] = t.perm[g];  // (always, by construction)
        }
        run = seg_add(run, SegCnt{self[u].v, 0});
    }
}

// ---- global levels, one launch per level: a workgroup per node of the level computes
// the same split as the passes above (the sampled box of every kSplitSample-th global tree
// position, the 22-bit key over its widest extent, the median by two 11-bit histograms,
// the stable left / tie / right partition), with LDS histograms and one block scan instead
// of device-wide passes.  A node's points are read as wave-contiguous 64-position chunks.
// levels with at least this many nodes (over all clouds) use k_tree_level (32 / 64 / 128
// within noise of each other at C4; 32 leaves only the root level to the nine-launch
// multi-pass path: 16 tree launches per tree; 16 was slower -- a 120k-point root in one
// workgroup; one launch with a grid barrier per node for the top levels measured slower
// too: ~17 us per cross-XCD node barrier)
constexpr int kTreeWgMin = 32;
constexpr int kLevThreads = 1024, kLevWaves = kLevThreads / 64;
constexpr int kLevU = 16;  // loads in flight per thread in the passes over a node

// block-wide exclusive scan of one u32 per thread (kLevThreads): returns the exclusive
// prefix, *total the block's sum (two barriers)
__device__ __forceinline__ uint32_t lev_scan(uint32_t x, uint32_t* s_w, uint32_t* total) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o, 64);
        if (lane >= o) inc += y;
    }
    if (lane == 63) s_w[wv] = inc;
    __syncthreads();
    uint32_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < kLevWaves; ++w) {
        const uint32_t v = s_w[w];
        pre += w < wv ? v : 0u;
        tot += v;
    }
    __syncthreads();
    *total = tot;
    return pre + inc - x;
}

// the bin (2 per thread) where the cumulative count reaches `want` (bin 0 when want = 0),
// as k_part_select / k_part_select2 choose it; the thread that owns it writes
// (bin, want - count before it, its count).  The thread's bins are cleared for the next pass.
__device__ __forceinline__ void lev_select(uint32_t* s_h, uint32_t* s_w, int* s_sel, int want, int shift_prev) {
    const int tid = threadIdx.x;
    const uint32_t v0 = s_h[2 * tid], v1 = s_h[2 * tid + 1];
    uint32_t tot;
    const uint32_t cum = lev_scan(v0 + v1, s_w, &tot);
    s_h[2 * tid] = 0u;
    s_h[2 * tid + 1] = 0u;
    const uint32_t w = (uint32_t)want;
    const uint32_t c1 = cum + v0;
    const int pick = ((int)(cum < w) & (int)(c1 >= w)) | ((int)(want == 0) & (int)(tid == 0)) ? 0
                     : ((int)(c1 < w) & (int)(c1 + v1 >= w)) ? 1 : -1;
    if (pick >= 0) {
        const int bin = 2 * tid + pick;
        s_sel[0] = shift_prev >= 0 ? (shift_prev << kPartBits) | bin : bin;
        s_sel[1] = want - (int)(pick ? c1 : cum);
        s_sel[2] = (int)(pick ? v1 : v0);
    }
}

template <int D>
__global__ __launch_bounds__(kLevThreads) void k_tree_level(TreeView t, int level, const int32_t* __restrict__ perm_in,
                                                            int32_t* __restrict__ perm_out, uint32_t* __restrict__ qbuf) {
    __shared__ uint32_t s_h[kPartBins];
    __shared__ uint32_t s_lo[D], s_hi[D];
    __shared__ uint32_t s_w[kLevWaves];
    __shared__ int s_sel[3];
    __shared__ uint32_t s_cnt[kLevWaves][2];
    const int c = blockIdx.x >> level, node = blockIdx.x & ((1 << level) - 1);
    const CloudDev cl = t.clouds[c];
    const int n = cl.n;
    const int a = tree_first(n, level, node), m = tree_first(n, level, node + 1) - a;
    const int mL = tree_first(n, level + 1, 2 * node + 1) - a;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (m <= 0) return;  // (block-uniform)
#ifdef SE3ICP_PROF
    unsigned long long tp[6];
    tp[0] = __builtin_amdgcn_s_memtime();
#define LEV_T(i) tp[i] = __builtin_amdgcn_s_memtime()
#else
#define LEV_T(i)
#endif
    const int base = cl.off + a;  // global tree position of the node's first point
    for (int i = tid; i < kPartBins; i += kLevThreads) s_h[i] = 0u;
    if (tid < D) {
        s_lo[tid] = 0xffffffffu;
        s_hi[tid] = 0u;
    }
    // 1. the box of the samples: global tree positions that are multiples of kSplitSample
    {
        uint32_t lo[D], hi[D];
#pragma unroll
        for (int d = 0; d < D; ++d) { lo[d] = 0xffffffffu; hi[d] = 0u; }
        const int e0 = (kSplitSample - base % kSplitSample) % kSplitSample;
        constexpr int U1 = D == 12 ? 4 : 8;  // samples in flight per thread
#pragma clang loop unroll(disable) vectorize(disable)
        for (int e1 = e0 + tid * kSplitSample; e1 < m; e1 += U1 * kLevThreads * kSplitSample) {
            int pp[U1];
#pragma unroll
            for (int u = 0; u < U1; ++u) {
                const int e = e1 + u * kLevThreads * kSplitSample;
                pp[u] = e < m ? cl.off + perm_in[base + e] : -1;
            }
            float x[U1][D];
#pragma unroll
            for (int u = 0; u < U1; ++u)
#pragma unroll
                for (int d = 0; d < D; ++d) x[u][d] = t.vec[tree_in_ix(t, d, pp[u] < 0 ? cl.off : pp[u])];
#pragma unroll
            for (int u = 0; u < U1; ++u)
                if (pp[u] >= 0) {
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        const uint32_t o = ord_bits(x[u][d]);
                        lo[d] = min(lo[d], o);
                        hi[d] = max(hi[d], o);
                    }
                }
        }
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                lo[d] = min(lo[d], xor_lane(lo[d], o));
                hi[d] = max(hi[d], xor_lane(hi[d], o));
            }
        }
        __syncthreads();  // (s_lo / s_hi initialised)
        if (lane == 0) {
#pragma unroll
            for (int d = 0; d < D; ++d) {
                atomicMin(&s_lo[d], lo[d]);
                atomicMax(&s_hi[d], hi[d]);
            }
        }
        __syncthreads();
    }
    LEV_T(1);
    const PartDim pd = part_dim_of(s_lo, s_hi, D);
    // 2. keys (kept in qbuf) and the coarse histogram; kLevU independent loads in flight
    // per thread (the node is read by latency-bound chains otherwise)
#pragma unroll 1
    for (int e0 = tid; e0 < m; e0 += kLevU * kLevThreads) {
        int pp[kLevU];
        float x[kLevU];
#pragma unroll
        for (int u = 0; u < kLevU; ++u) {
            const int e = e0 + u * kLevThreads;
            pp[u] = e < m ? perm_in[base + e] : 0;
        }
#pragma unroll
        for (int u = 0; u < kLevU; ++u) x[u] = tree_in_col(t, pd.best, cl.off + pp[u]);
#pragma unroll
        for (int u = 0; u < kLevU; ++u) {
            const int e = e0 + u * kLevThreads;
            float qf = (x[u] - pd.lo) * pd.scale;
            qf = fminf(fmaxf(qf, 0.f), kKeyMax);  // NaN -> 0
            const uint32_t key = (uint32_t)qf;
            if (e < m) {
                qbuf[base + e] = key;
                atomicAdd(&s_h[key >> kPartBits], 1u);
            }
        }
    }
    __syncthreads();
    LEV_T(2);
    lev_select(s_h, s_w, s_sel, mL, -1);
    __syncthreads();
    // 3. the fine histogram inside the median bin (each thread re-reads its own keys)
    const int bin = s_sel[0];
#pragma unroll 1
    for (int e0 = tid; e0 < m; e0 += kLevU * kLevThreads) {
        uint32_t k[kLevU];
#pragma unroll
        for (int u = 0; u < kLevU; ++u) {
            const int e = e0 + u * kLevThreads;
            k[u] = e < m ? qbuf[base + e] : 0xffffffffu;
        }
#pragma unroll
        for (int u = 0; u < kLevU; ++u)
            if ((int)(k[u] >> kPartBits) == bin) atomicAdd(&s_h[k[u] & (kPartBins - 1)], 1u);
    }
    __syncthreads();
    LEV_T(3);
    lev_select(s_h, s_w, s_sel, s_sel[1], bin);
    __syncthreads();
    LEV_T(4);
    const int T = s_sel[0], tl = s_sel[1], tn = s_sel[2];
    // 4. stable partition: wave w owns the 64-position chunks [w S, (w + 1) S) of the node;
    // its (left, tie) counts, their prefix over the waves, then every point's rank by ballots
    const int S = ((m + kLevWaves * 64 - 1) / (kLevWaves * 64)) * 64;
    const int s0 = wv * S, s1 = min(m, s0 + S);
    uint32_t nl = 0, nt = 0;
#pragma unroll 1
    for (int e0 = s0; e0 < s1; e0 += kLevU * 64) {
        int q[kLevU];
#pragma unroll
        for (int u = 0; u < kLevU; ++u) {
            const int e = e0 + u * 64 + lane;
            q[u] = e < s1 ? (int)qbuf[base + e] : 0x7fffffff;
        }
#pragma unroll
        for (int u = 0; u < kLevU; ++u) {
            nl += __popcll(__ballot(q[u] < T));
            nt += __popcll(__ballot(q[u] == T));
        }
    }
    if (lane == 0) { s_cnt[wv][0] = nl; s_cnt[wv][1] = nt; }
    __syncthreads();
    uint32_t r0 = 0, r1 = 0;
#pragma unroll 1
    for (int w = 0; w < wv; ++w) { r0 += s_cnt[w][0]; r1 += s_cnt[w][1]; }
#pragma unroll 1
    for (int e0 = s0; e0 < s1; e0 += kLevU * 64) {
        int q[kLevU], pp[kLevU];
#pragma unroll
        for (int u = 0; u < kLevU; ++u) {
            const int e = e0 + u * 64 + lane;
            q[u] = e < s1 ? (int)qbuf[base + e] : 0x7fffffff;
            pp[u] = e < s1 ? perm_in[base + e] : 0;
        }
#pragma unroll
        for (int u = 0; u < kLevU; ++u) {
            const int e = e0 + u * 64 + lane;
            const unsigned long long bl = __ballot(q[u] < T), bt = __ballot(q[u] == T);
            const int rl = (int)r0 + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bl >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bl, 0u));
            const int rt = (int)r1 + (int)__builtin_amdgcn_mbcnt_hi((unsigned)(bt >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)bt, 0u));
            int dst;
            if (q[u] < T) dst = rl;
            else if (q[u] == T) dst = rt < tl ? (mL - tl) + rt : mL + (rt - tl);
            else dst = mL + (tn - tl) + (e - rl - rt);
            if ((int)(e < s1) & (int)((unsigned)dst < (unsigned)m)) perm_out[base + dst] = pp[u];  // (always, by construction)
            r0 += (uint32_t)__popcll(bl);
            r1 += (uint32_t)__popcll(bt);
        }
    }
#ifdef SE3ICP_PROF
    LEV_T(5);
    if ((int)(tid == 0) & (int)(blockIdx.x == 0))
        printf("[tree] D=%d level %d m=%d: box %llu keys %llu fine %llu select %llu partition %llu cycles\n", D, level, m,
               tp[1] - tp[0], tp[2] - tp[1], tp[3] - tp[2], tp[4] - tp[3], tp[5] - tp[4]);
#endif
#undef LEV_T
}

// The levels below G in one workgroup per level-G node (<= kLocalMax points): the node's
// permutation stays in LDS and every level splits its sub-nodes at the median of the
// coordinate of largest sample variance (a register sort by one wave for sub-nodes of
// <= 512 points, a stable LDS partition above).  The node's vectors are first copied into
// t.scr at their level-G positions, one column per dimension, so the levels read a few
// L2-resident columns instead of gathering rows of the input.  The workgroup then finishes its subtree
// in place of k_tree_finish / k_tree_leafbox / k_tree_up: the final permutation and its
// inverse, the tree-ordered f32 (and f64) vectors, and the boxes of every leaf and inner
// node below level G.  s_val holds level-G positions e (s_p[e]: the point).
#ifndef SE3ICP_TREE_LDS_SAMPLE
#define SE3ICP_TREE_LDS_SAMPLE 1
#endif
#ifndef SE3ICP_TREE_EMPTY_FALLBACK
#define SE3ICP_TREE_EMPTY_FALLBACK 1
#endif
#ifndef SE3ICP_TREE_SRC_ORDER_ONLY
#define SE3ICP_TREE_SRC_ORDER_ONLY 1
#endif
constexpr int kLocalMax = 4096;  // power of two
constexpr int kWaveSortPer = 8;  // sub-nodes of <= 512 points: register sort by one wave
constexpr int kLocalThreads = 512;
static_assert(kLocalMax <= 4096, "wave-sort keys carry the position in 12 bits");

template <int D>
// (4 waves per SIMD: two workgroups per CU, <= 128 VGPRs)
__global__ __launch_bounds__(kLocalThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_tree_local(TreeView t, int G) {
    __shared__ unsigned long long s_key[kLocalMax];  // (histograms, then one column of the node)
    __shared__ int32_t s_val[kLocalMax];
    __shared__ int32_t s_p[kLocalMax];
    __shared__ int s_best[128];
    __shared__ float s_mu[128], s_sd[128];  // the split coordinate's sample mean and sd (variance splits)
    // the split-dimension sample: the vectors of the level-G positions 16 j, kept in LDS for
    // every level (round 4 gathered every 16th point of each sub-node from the node's 12
    // columns at every level: scattered 4-B reads that fetched ~40 B of 128-B lines per
    // point and level, a third of the kernel's traffic), and their current positions
    constexpr int kSmp = kLocalMax / 16;
    __shared__ float s_smp[D][kSmp];
    __shared__ int32_t s_spos[kSmp];
    const int nG = 1 << G;
    const int c = blockIdx.x / nG, i = blockIdx.x % nG;
    const CloudDev cl = t.clouds[c];
    const int n = cl.n;
    const int A = tree_first(n, G, i), m = tree_first(n, G, i + 1) - A;
    const int tid = threadIdx.x;
    const size_t ld = t.ld;
    // the node's vectors at the level-G positions, one column per dimension (col0[d * m + e]):
    // a level gathers one coordinate of every point, 4 B from a 16-KB column instead of a
    // 64-B sector of a 48-B row (round 3: 1.7 GB of HBM traffic per 12-D launch)
    float* col0 = t.scr + (size_t)(cl.off + A) * D;
#ifdef SE3ICP_PROF
    unsigned long long tq[5];
    tq[0] = __builtin_amdgcn_s_memrealtime();
#endif
    // the node's points and their vectors at the level-G positions: every permutation entry
    // of the thread first, then the rows in batches of LB with all their loads issued before
    // the column stores (a load after a store to another global array is not hoisted above
    // it, so one point at a time was two dependent round trips per point)
    {
        constexpr int LP = kLocalMax / kLocalThreads;
        constexpr int LB = D == 12 ? 4 : LP;
        static_assert(LP % LB == 0, "whole batches");
        int pl[LP];
#pragma unroll
        for (int u = 0; u < LP; ++u) {
            const int e = tid + u * kLocalThreads;
            pl[u] = e < m ? t.perm[cl.off + A + e] : -1;
        }
#pragma unroll
        for (int u = 0; u < LP; ++u) {
            const int e = tid + u * kLocalThreads;
            s_val[e] = e;
            s_p[e] = pl[u];
        }
#pragma unroll
        for (int u0 = 0; u0 < LP; u0 += LB) {
            float x[LB][D];
#pragma unroll
            for (int u = 0; u < LB; ++u) {
                const int p = pl[u0 + u] >= 0 ? pl[u0 + u] : 0;
                if constexpr (D == 12) {
                    const float4* r = reinterpret_cast<const float4*>(t.vec + (size_t)(cl.off + p) * 12);
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        const float4 q = r[k];
                        x[u][4 * k] = q.x; x[u][4 * k + 1] = q.y; x[u][4 * k + 2] = q.z; x[u][4 * k + 3] = q.w;
                    }
                } else {
#pragma unroll
                    for (int d = 0; d < D; ++d) x[u][d] = t.vec[(size_t)d * ld + cl.off + p];
                }
            }
#pragma unroll
            for (int u = 0; u < LB; ++u) {
                const int e = tid + (u0 + u) * kLocalThreads;
                if (pl[u0 + u] >= 0) {
#pragma unroll
                    for (int d = 0; d < D; ++d) col0[d * m + e] = x[u][d];
                    if ((e & 15) == 0) {
#pragma unroll
                        for (int d = 0; d < D; ++d) s_smp[d][e >> 4] = x[u][d];
                    }
                }
            }
        }
    }
    __syncthreads();  // (global writes of the workgroup, read back by other threads of it)
#ifdef SE3ICP_PROF
    tq[1] = __builtin_amdgcn_s_memrealtime();
#endif
#ifdef SE3ICP_PROF
    unsigned long long t_lev = tq[1];
#endif
    for (int l = G; l < t.L; ++l) {
        const int r = l - G;
#ifdef SE3ICP_PROF
        if ((int)(r > 0) & (int)(tid == 0) & (int)(r <= 8)) {
            const unsigned long long now = __builtin_amdgcn_s_memrealtime();
            atomicAdd(&g_tree_lev[D == 12][r - 1], now - t_lev);
            t_lev = now;
        }
#endif
        const int nsub = 1 << r;  // sub-nodes of this level under the WG's node (<= 128: see the host)
        // the sample's current positions (the sub-node of each sample point)
        const int nsmp = (m + 15) >> 4;
        for (int e = tid; e < m; e += kLocalThreads) {
            const int q = s_val[e];
            if ((q & 15) == 0) s_spos[q >> 4] = e;
        }
        __syncthreads();
        // split dimension of each sub-node: the dimension of largest variance over the
        // sample points it holds (1 in 16: denser samples measured slower overall -- strides
        // 1, 4, 8, 16, 32, 64 tried in round 2), a wave per sub-node, LDS reads only
        {
            const int lane = tid & 63, wv = tid >> 6;
            for (int k = wv; k < nsub; k += kLocalThreads / 64) {
                const int a0 = tree_first(n, l, (i << r) + k) - A, a1 = tree_first(n, l, (i << r) + k + 1) - A;
                // widest spread: the dimension of largest sample variance
                float s1[D], s2[D];
#pragma unroll
                for (int d = 0; d < D; ++d) { s1[d] = 0.f; s2[d] = 0.f; }
                int cnt = 0;
#if SE3ICP_TREE_LDS_SAMPLE
                for (int j = lane; j < nsmp; j += 64) {
                    const int e = s_spos[j];
                    if ((int)(e < a0) | (int)(e >= a1)) continue;
                    ++cnt;
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        const float x = s_smp[d][j];
                        s1[d] += x;
                        s2[d] = fmaf(x, x, s2[d]);
                    }
                }
#else
                for (int e = a0 + lane * 16; e < a1; e += 64 * 16) {  // (round 4: every 16th point from the columns)
                    const int p = s_val[e];
                    ++cnt;
#pragma unroll
                    for (int d = 0; d < D; ++d) {
                        const float x = col0[d * m + p];
                        s1[d] += x;
                        s2[d] = fmaf(x, x, s2[d]);
                    }
                }
#endif
                for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
#if SE3ICP_TREE_LDS_SAMPLE && SE3ICP_TREE_EMPTY_FALLBACK
                if (cnt == 0) {
                    // (wave-uniform) a sub-node holding none of the fixed sample points -- deep
                    // levels, small nodes: its own points from the columns, every one of them
                    // (round 5 split such a sub-node on dimension 0 with mean = sd = 0, i.e. by
                    // index)
                    for (int e = a0 + lane; e < a1; e += 64) {
                        const int p = s_val[e];
                        ++cnt;
#pragma unroll
                        for (int d = 0; d < D; ++d) {
                            const float x = col0[d * m + p];
                            s1[d] += x;
                            s2[d] = fmaf(x, x, s2[d]);
                        }
                    }
                    for (int o = 32; o >= 1; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
                }
#endif
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
                    if (e > ext) { ext = e; best = d; if (lane == 0) { s_mu[k] = mu; s_sd[k] = sqrtf(fmaxf(e, 0.f)); } }
                }
                if (lane == 0) s_best[k] = best;
            }
        }
        __syncthreads();
        const int max_sub = (m + nsub - 1) / nsub + 1;  // sub-node sizes differ by <= 1
        if (max_sub <= 64 * kWaveSortPer) {
            // small sub-nodes: one wave sorts each in registers, in a network of the sub-node's
            // size (128, 256 or 512 keys) over 32-bit keys: the split coordinate quantised to
            // 20 bits over the sub-node's sample mean +- 8 sd | the level-G position (12 bits,
            // which also orders ties).  Any order gives a valid balanced tree (the searches
            // are exact over the node boxes); this one keeps the split at the median.
            const int lane = tid & 63, wv = tid >> 6;
            auto wave_level = [&](auto per_tag) {
                constexpr int PER = decltype(per_tag)::value;
                for (int k = wv; k < nsub; k += kLocalThreads / 64) {
                    const int a0 = tree_first(n, l, (i << r) + k) - A, a1 = tree_first(n, l, (i << r) + k + 1) - A;
                    const int bd = s_best[k];
                    const float sd = s_sd[k], qlo = s_mu[k] - 8.f * sd;
                    const float qs = sd > 0.f ? 1048575.f / (16.f * sd) : 0.f;
                    unsigned key[PER];
#pragma unroll
                    for (int u = 0; u < PER; ++u) {
                        const int e = a0 + lane * PER + u;
                        key[u] = ~0u;
                        if (e < a1) {
                            const int p = s_val[e];
                            const float qf = fminf(fmaxf((col0[bd * m + p] - qlo) * qs, 0.f), 1048575.f);  // NaN -> 0
                            key[u] = ((unsigned)qf << 12) | (unsigned)p;
                        }
                    }
                    wave_sort_u32<PER>(key);
#pragma unroll
                    for (int u = 0; u < PER; ++u) {
                        const int e = a0 + lane * PER + u;
                        if (e < a1) s_val[e] = (int32_t)(key[u] & 0xfffu);
                    }
                }
            };
            if (max_sub <= 128) wave_level(std::integral_constant<int, 2>{});
            else if (max_sub <= 256) wave_level(std::integral_constant<int, 4>{});
            else wave_level(std::integral_constant<int, kWaveSortPer>{});
            __syncthreads();
            continue;
        }
        // large sub-nodes (<= 4 of them): a stable median partition in LDS, as the global
        // levels do -- the split coordinate quantised to 22 bits over the sub-node's sample
        // mean +- 8 sd, the median bin by two 11-bit histogram passes, then each point's
        // rank among its sub-node's points of the same class (left / tie / right) by a
        // block scan; ties keep their order.  Thread t owns the points t*8 .. t*8+7.
        {
            constexpr int PER = kLocalMax / kLocalThreads;
            constexpr int kB = 2048;  // bins per pass
            uint32_t* s_h = reinterpret_cast<uint32_t*>(s_key);  // nsub x kB histogram words
            __shared__ int s_sel[4][4];  // per sub-node: bin / threshold, tie_left, tie_n, cum
            __shared__ uint32_t s_scan[kLocalThreads / 64][8];
            for (int x = tid; x < nsub * kB; x += kLocalThreads) s_h[x] = 0u;
            uint32_t q[PER];
            int sb[PER];
            int32_t val[PER];
            __syncthreads();
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int e = tid * PER + u;
                q[u] = 0u;
                sb[u] = 0;
                val[u] = -1;
                if (e < m) {
                    const int sub = tree_node_of(A + e, n, l) - (i << r);
                    const int p = s_val[e];
                    const float sd = s_sd[sub];
                    const float x = col0[s_best[sub] * m + p];
                    float qf = sd > 0.f ? (x - (s_mu[sub] - 8.f * sd)) * (4194303.f / (16.f * sd)) : 0.f;
                    qf = fminf(fmaxf(qf, 0.f), 4194303.f);  // NaN -> 0
                    q[u] = (uint32_t)qf;
                    sb[u] = sub;
                    val[u] = p;
                    atomicAdd(&s_h[sub * kB + (q[u] >> 11)], 1u);
                }
            }
            __syncthreads();
            const int lane = tid & 63, wv = tid >> 6;
            // a wave per sub-node: the bin where the count reaches the left child's size
            auto find_bin = [&](int k, int want, int pass) {
                const uint32_t* hk = s_h + k * kB + lane * (kB / 64);
                uint32_t tot = 0;
                for (int j = 0; j < kB / 64; ++j) tot += hk[j];
                uint32_t inc = tot;  // inclusive wave scan of the lanes' totals
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_up(inc, o, 64);
                    if (lane >= o) inc += y;
                }
                uint32_t cum = inc - tot;
                if ((int)(cum >= (uint32_t)want || inc < (uint32_t)want) & (int)!(want == 0 && lane == 0)) return;
                for (int j = 0; j < kB / 64; ++j) {
                    const uint32_t vj = hk[j], nxt = cum + vj;
                    const int bin = lane * (kB / 64) + j;
                    if (((int)(cum < (uint32_t)want) & (int)(nxt >= (uint32_t)want)) | ((int)(want == 0) & (int)(bin == 0))) {
                        if (pass == 0) {
                            s_sel[k][0] = bin;
                        } else {
                            s_sel[k][0] = (s_sel[k][0] << 11) | bin;
                            s_sel[k][2] = (int)vj;
                        }
                        s_sel[k][1] = want - (int)cum;
                        break;
                    }
                    cum = nxt;
                }
            };
            if (wv < nsub) {
                const int a0 = tree_first(n, l, (i << r) + wv) - A;
                const int mL = tree_first(n, l + 1, 2 * ((i << r) + wv) + 1) - A - a0;
                find_bin(wv, mL, 0);
            }
            __syncthreads();
            for (int x = tid; x < nsub * kB; x += kLocalThreads) s_h[x] = 0u;
            __syncthreads();
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int e = tid * PER + u;
                if ((int)(e < m) & (int)((int)(q[u] >> 11) == s_sel[sb[u]][0])) atomicAdd(&s_h[sb[u] * kB + (q[u] & 2047u)], 1u);
            }
            __syncthreads();
            if (wv < nsub) find_bin(wv, s_sel[wv][1], 1);
            __syncthreads();
            // class counts per sub-node (16-bit left | 16-bit tie), thread-exclusive block scan
            uint32_t cnt[4] = {0u, 0u, 0u, 0u};
            int cls[PER];
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int e = tid * PER + u;
                cls[u] = 2;
                if (e < m) {
                    const int T = s_sel[sb[u]][0];
                    cls[u] = (int)q[u] < T ? 0 : ((int)q[u] == T ? 1 : 2);
                }
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    cnt[k] += (sb[u] == k && e < m) ? (cls[u] == 0 ? 1u : (cls[u] == 1 ? 65536u : 0u)) : 0u;
            }
            uint32_t pre[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                uint32_t inc = cnt[k];
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = __shfl_up(inc, o, 64);
                    if (lane >= o) inc += y;
                }
                if (lane == 63) s_scan[wv][k] = inc;
                pre[k] = inc - cnt[k];
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < 4; ++k)
                for (int w = 0; w < wv; ++w) pre[k] += s_scan[w][k];
            int dst[PER];
#pragma unroll
            for (int u = 0; u < PER; ++u) {
                const int e = tid * PER + u;
                dst[u] = -1;
                if (e < m) {
                    const int k = sb[u];
                    const uint32_t run = k == 0 ? pre[0] : (k == 1 ? pre[1] : (k == 2 ? pre[2] : pre[3]));
                    const int r0 = (int)(run & 0xffffu), r1 = (int)(run >> 16);
                    const int a0 = tree_first(n, l, (i << r) + k) - A;
                    const int mL = tree_first(n, l + 1, 2 * ((i << r) + k) + 1) - A - a0;
                    const int tl = s_sel[k][1], tn = s_sel[k][2];
                    if (cls[u] == 0) dst[u] = a0 + r0;
                    else if (cls[u] == 1) dst[u] = r1 < tl ? a0 + (mL - tl) + r1 : a0 + mL + (r1 - tl);
                    else dst[u] = a0 + mL + (tn - tl) + ((e - a0) - r0 - r1);
                    const uint32_t add = cls[u] == 0 ? 1u : (cls[u] == 1 ? 65536u : 0u);
                    if (k == 0) pre[0] += add; else if (k == 1) pre[1] += add; else if (k == 2) pre[2] += add; else pre[3] += add;
                }
            }
            __syncthreads();
#pragma unroll
            for (int u = 0; u < PER; ++u)
                if ((unsigned)dst[u] < (unsigned)m) s_val[dst[u]] = val[u];
            __syncthreads();
        }
    }
#ifdef SE3ICP_PROF
    tq[2] = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
        const int last = t.L - G - 1;
        if (last >= 0 && last < 8) atomicAdd(&g_tree_lev[D == 12][last], tq[2] - t_lev);
        atomicAdd(&g_tree_lev[D == 12][8], 1ull);
    }
#endif
    // the final order, a wave per leaf (<= 64 consecutive tree positions): permutation,
    // inverse, f32 and f64 vectors (the layouts k_tree_finish writes) and the leaf's box
    // (inflated as k_tree_leafbox does)
    const bool want64 = (t.tvec64 != nullptr) & !((t.vec64_sources_only != 0) & ((c & 1) != 0));
    // a source cloud of the loop's 12-D trees (even ids): the searches walk the TARGET trees
    // only, so a source tree is its order (perm: the queries' chunks) and its f64 translation
    // rows -- no inverse, no f32 rows, no boxes, and no gather of its 48-B input rows
    const bool order_only = SE3ICP_TREE_SRC_ORDER_ONLY && (D == 12) && (t.vec64_sources_only != 0) && ((c & 1) == 0);
    const int R = t.L - G;  // levels of the subtree below its root
    const int lane = tid & 63, wv = tid >> 6;
    const size_t bbase = (size_t)c * t.nnodes * D;
    // FB leaves per wave at a time: their row loads are issued together, then each leaf's
    // stores and box (one leaf at a time was two dependent round trips per leaf)
    constexpr int FB = D == 12 ? 2 : 4;
    constexpr int NWV = kLocalThreads / 64;
    for (int j0 = wv; j0 < (1 << R); j0 += FB * NWV) {
        float v[FB][D];  // (the input vectors of the point: a 48-B row / three columns)
        double w64[FB][3];
        int xq[FB], pq[FB];
        bool inq[FB];
#pragma unroll
        for (int b = 0; b < FB; ++b) {
            const int j = j0 + b * NWV;
            const int leaf = (i << R) + j;
            const bool live = j < (1 << R);
            const int a0 = live ? tree_first(n, t.L, leaf) : A, a1 = live ? tree_first(n, t.L, leaf + 1) : A;
            inq[b] = lane < a1 - a0;
            xq[b] = a0 - A + (inq[b] ? lane : 0);
            // lanes outside the leaf load nothing: for an empty node (m == 0) or a trailing
            // empty leaf s_val / s_p hold no point of this cloud, and cl.off + s_p[..] could
            // lie before the buffer
            pq[b] = inq[b] ? s_p[s_val[xq[b]]] : 0;
            const int src = cl.off + pq[b];
#pragma unroll
            for (int d = 0; d < D; ++d) v[b][d] = 0.0f;
            if ((int)inq[b] & (int)!order_only) {
                if constexpr (D == 12) {
                    const float4* r = reinterpret_cast<const float4*>(t.vec + (size_t)src * 12);
#pragma unroll
                    for (int k = 0; k < 3; ++k) {
                        const float4 q = r[k];
                        v[b][4 * k] = q.x; v[b][4 * k + 1] = q.y; v[b][4 * k + 2] = q.z; v[b][4 * k + 3] = q.w;
                    }
                } else {
#pragma unroll
                    for (int d = 0; d < D; ++d) v[b][d] = t.vec[(size_t)d * ld + src];
                }
            }
            w64[b][0] = w64[b][1] = w64[b][2] = 0.0;
            if ((int)want64 & (int)inq[b]) {
                if constexpr (D == 12) {  // the translation rows only (the loop reads the frames by point)
                    // (byte offset 96*src + 72 is 8 mod 16: three 8-B loads, no double2)
                    const double* r64 = t.vec64 + (size_t)src * 12 + 9;
                    w64[b][0] = r64[0]; w64[b][1] = r64[1]; w64[b][2] = r64[2];
                } else {
#pragma unroll
                    for (int d = 0; d < D; ++d) w64[b][d] = t.vec64[(size_t)d * ld + src];
                }
            }
        }
#pragma unroll
        for (int b = 0; b < FB; ++b) {
            const int j = j0 + b * NWV;
            if (j >= (1 << R)) break;  // (wave-uniform)
            const int leaf = (i << R) + j;
            const bool in = inq[b];
            const int x = xq[b], p = pq[b];
            const int g = cl.off + A + x, src = cl.off + p;
            if (in) {
                t.perm[g] = p;
                if (order_only) {  // (pos is read for target clouds only: the previous match's slot)
                } else if constexpr (D == 12) {
                    t.pos[src] = A + x;
                    float4* o = reinterpret_cast<float4*>(t.tvec + (size_t)g * 12);
#pragma unroll
                    for (int k = 0; k < 3; ++k) o[k] = make_float4(v[b][4 * k], v[b][4 * k + 1], v[b][4 * k + 2], v[b][4 * k + 3]);
                } else {
                    t.pos[src] = A + x;
#pragma unroll
                    for (int d = 0; d < D; ++d) t.tvec[(size_t)d * ld + g] = v[b][d];
                }
                if (want64) {
#pragma unroll
                    for (int d = 0; d < 3; ++d) t.tvec64[(size_t)d * ld + g] = w64[b][d];
                    if constexpr (D == 3) {
                        if (t.tpt64) t.tpt64[g] = make_double4(w64[b][0], w64[b][1], w64[b][2], 0.0);
                    }
                }
            }
            if (order_only) continue;  // (wave-uniform)
            const size_t hb = bbase + (size_t)tree_heap(t.L, leaf) * D;
#pragma unroll
            for (int d = 0; d < D; ++d) {
                float lo = in ? v[b][d] : INFINITY, hi = in ? v[b][d] : -INFINITY;
#pragma unroll
                for (int o = 32; o >= 1; o >>= 1) {  // (DPP / swizzle / permlane exchanges)
                    lo = fminf(lo, xor_lane(lo, o));
                    hi = fmaxf(hi, xor_lane(hi, o));
                }
                if (lo <= hi) {
                    lo = lo - (fabsf(lo) * 4.8e-7f + 1e-30f);
                    hi = hi + (fabsf(hi) * 4.8e-7f + 1e-30f);
                }
                if (lane == d) {  // empty leaf: [inf, -inf], a box no query reaches
                    t.lo[hb + d] = lo;
                    t.hi[hb + d] = hi;
                }
            }
        }
    }
#ifdef SE3ICP_PROF
    tq[3] = __builtin_amdgcn_s_memrealtime();
#endif
    __syncthreads();
    for (int rr = order_only ? -1 : R - 1; rr >= 0; --rr) {
        for (int it = tid; it < (D << rr); it += kLocalThreads) {
            const int j = it / D, d = it % D;
            const size_t h = (size_t)tree_heap(G + rr, (i << rr) + j);
            const size_t cl_ = bbase + (2 * h + 1) * D + d, cr_ = bbase + (2 * h + 2) * D + d;
            t.lo[bbase + h * D + d] = fminf(t.lo[cl_], t.lo[cr_]);
            t.hi[bbase + h * D + d] = fmaxf(t.hi[cl_], t.hi[cr_]);
        }
        __syncthreads();
    }
#ifdef SE3ICP_PROF
    tq[4] = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) {
        atomicMin(&g_tree_prof[D == 12][0], tq[0]);
        for (int k = 1; k < 5; ++k) atomicMax(&g_tree_prof[D == 12][k], tq[k]);
    }
#endif
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
            float4* o = reinterpret_cast<float4*>(t.tvec + (size_t)g * 12);
#pragma unroll
            for (int k = 0; k < 3; ++k) o[k] = r32[k];
            if (want64) {  // the translation rows only
                const double* r64 = t.vec64 + (size_t)src * 12 + 9;
                for (int k = 0; k < 3; ++k) t.tvec64[(size_t)k * t.ld + g] = r64[k];
            }
        } else {
            for (int d = 0; d < t.D; ++d) t.tvec[(size_t)d * t.ld + g] = t.vec[(size_t)d * t.ld + src];
            if (want64) {
                double x[3] = {0.0, 0.0, 0.0};
                for (int d = 0; d < t.D; ++d) t.tvec64[(size_t)d * t.ld + g] = x[d < 3 ? d : 0] = t.vec64[(size_t)d * t.ld + src];
                if (t.tpt64) t.tpt64[g] = make_double4(x[0], x[1], x[2], 0.0);
            }
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
        if (valid) lo = hi = t.tvec[tree_tv_ix<D>(t.ld, cl.off + a + lane, d)];
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

// internal boxes of the levels above `top` = unions of the children, level by level (one
// block per cloud)
__global__ __launch_bounds__(1024) void k_tree_up(TreeView t, int top) {
    const int c = blockIdx.x;
    // (a loop source cloud's 12-D tree has no boxes: see k_tree_local's order_only)
    if (SE3ICP_TREE_SRC_ORDER_ONLY && (t.D == 12) && (t.vec64_sources_only != 0) && ((c & 1) == 0)) return;
    for (int l = top - 1; l >= 0; --l) {
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

int tree_global_levels(int max_n, int L) {
    int G = 0;  // global levels until every node fits one workgroup's LDS sort (and <= 128 sub-nodes below)
    while (G < L && (((long long)max_n + (1ll << G) - 1) >> G) > kLocalMax) ++G;
    if (L - 1 - G > 7) G = L - 8;
    return G;
}

namespace {
struct PartScratch {
    uint32_t* overflow;  // per node of the multi-pass levels: histogram (coarse, then fine)
    PartSel* sel;
    PartDim* dims;
    SegCnt* tails;
    SegCnt* carry;
    size_t overflow_words;
};
size_t part_layout(int npts, int nclouds, int G, char* base, PartScratch* ps) {
    const size_t nodes = G > 0 ? (size_t)nclouds << (G - 1) : 0;
    const size_t nblk = ((size_t)npts + kPartElems - 1) / kPartElems;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t at = off;
        off += (bytes + 255) & ~(size_t)255;
        return base ? base + at : nullptr;
    };
    char* ov = take(nodes * kPartBins * sizeof(uint32_t));
    char* sl = take(nodes * sizeof(PartSel));
    char* d0 = take(nodes * sizeof(PartDim));
    char* tl = take(nblk * sizeof(SegCnt));
    char* cr = take(nblk * sizeof(SegCnt));
    if (ps) {
        ps->overflow = (uint32_t*)ov;
        ps->sel = (PartSel*)sl;
        ps->dims = (PartDim*)d0;
        ps->tails = (SegCnt*)tl;
        ps->carry = (SegCnt*)cr;
        ps->overflow_words = nodes * kPartBins;
    }
    return off;
}

__global__ __launch_bounds__(256) void k_clear_words(uint32_t* p, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) p[i] = 0u;
}
}  // namespace

int build_trees(TreeView t, void* tmp, size_t tmp_bytes, uint32_t* qbuf, int32_t* perm_alt, hipStream_t s) {
    const int nb = (t.npts + 255) / 256;
    const int nbs = (t.npts + 256 * kSplitSample - 1) / (256 * kSplitSample);
    const int gfill = std::max(nb, 64);
    auto bbox = (t.D == 12) ? k_tree_bbox<12> : k_tree_bbox<3>;
    int max_n = 0;
    for (int c = 0; c < t.nclouds; ++c) max_n = std::max(max_n, t.host_n[c]);
    const int G = tree_global_levels(max_n, t.L);
    PartScratch ps;
    if (part_layout(t.npts, t.nclouds, G, (char*)tmp, &ps) > tmp_bytes) return -1;
    // the level scatters alternate between the two permutation buffers: start in the one
    // that makes the last global level land in t.perm
    int32_t* const final_perm = t.perm;
    TreeView tc = t;
    tc.perm = (G % 2 == 0) ? final_perm : perm_alt;
    int32_t* other = (G % 2 == 0) ? perm_alt : final_perm;
    int H = 0;  // levels of the multi-pass path (k_tree_bbox / k_part_*)
    // (12-D: a level of 32 nodes through the multi-pass sequence too -- one 1024-thread
    // workgroup per 60k-point node left 7/8 of the CUs idle for 120 us; 3-D breaks even)
    const int wg_min = t.D == 12 ? 2 * kTreeWgMin : kTreeWgMin;
    while (H < G && (t.nclouds << H) < wg_min) ++H;
    hipLaunchKernelGGL(k_tree_init, dim3(gfill), dim3(256), 0, s, tc, other, (1 << H) - 1);
    if (ps.overflow_words) hipLaunchKernelGGL(k_clear_words, dim3(256), dim3(256), 0, s, ps.overflow, ps.overflow_words);
    const int nblk = (t.npts + kPartElems - 1) / kPartElems;
    const int nhist = (t.npts + kHistElems - 1) / kHistElems;
    for (int l = 0; l < G; ++l) {
        if (l >= H) {
            // enough nodes to fill the GPU with a workgroup each: one launch for the level
            hipLaunchKernelGGL(t.D == 12 ? k_tree_level<12> : k_tree_level<3>, dim3(t.nclouds << l), dim3(kLevThreads), 0,
                               s, tc, l, (const int32_t*)tc.perm, other, qbuf);
            std::swap(tc.perm, other);
            continue;
        }
        PartDim* dims = ps.dims;
        // (the split dimension from every kSplitSample-th point's box: estimating the
        // children's boxes from the parent's cut was measured to give slower searches)
        hipLaunchKernelGGL(bbox, dim3(nbs), dim3(256), 0, s, tc, l);
        hipLaunchKernelGGL(k_part_dims, dim3(((t.nclouds << l) + 63) / 64), dim3(64), 0, s, tc, l, dims);
        hipLaunchKernelGGL(k_part_hist, dim3(nhist), dim3(kPartThreads), 0, s, tc, l, dims, qbuf, ps.overflow);
        hipLaunchKernelGGL(k_part_select, dim3(t.nclouds << l), dim3(kSelThreads), 0, s, tc, l, ps.overflow, ps.sel);
        hipLaunchKernelGGL(k_part_hist2, dim3(nb), dim3(256), 0, s, tc, l, (const uint32_t*)qbuf, (const PartSel*)ps.sel,
                           ps.overflow);
        hipLaunchKernelGGL(k_part_select2, dim3(t.nclouds << l), dim3(256), 0, s, ps.overflow, ps.sel);
        hipLaunchKernelGGL(k_part_count, dim3(nblk), dim3(kPartThreads), 0, s, tc, l, (const uint32_t*)qbuf,
                           (const PartSel*)ps.sel, ps.tails);
        hipLaunchKernelGGL(k_part_scan, dim3(1), dim3(1024), 0, s, (const SegCnt*)ps.tails, nblk, ps.carry);
        hipLaunchKernelGGL(k_part_scatter, dim3(nblk), dim3(kPartThreads), 0, s, tc, l, (const uint32_t*)qbuf,
                           (const PartSel*)ps.sel, (const SegCnt*)ps.carry, other);
        std::swap(tc.perm, other);
    }
    t.perm = final_perm;
    if (G < t.L) {
        // the levels below G, the tree-ordered vectors and the boxes below G per level-G node
        hipLaunchKernelGGL(t.D == 12 ? k_tree_local<12> : k_tree_local<3>, dim3(t.nclouds << G), dim3(kLocalThreads), 0,
                           s, t, G);
        hipLaunchKernelGGL(k_tree_up, dim3(t.nclouds), dim3(1024), 0, s, t, G);
    } else {
        hipLaunchKernelGGL(k_tree_finish, dim3(nb), dim3(256), 0, s, t);
        const int nleaves = t.nclouds << t.L;
        hipLaunchKernelGGL(t.D == 12 ? k_tree_leafbox<12> : k_tree_leafbox<3>, dim3((nleaves + 3) / 4), dim3(256), 0, s, t);
        hipLaunchKernelGGL(k_tree_up, dim3(t.nclouds), dim3(1024), 0, s, t, t.L);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

void tree_prof_report() {
#ifdef SE3ICP_PROF
    unsigned long long h[2][5];
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(g_tree_prof), sizeof(h)) != hipSuccess) return;
    for (int k = 0; k < 2; ++k)
        if (h[k][0] && h[k][0] != ~0ull)
            std::fprintf(stderr, "[prof] k_tree_local<%d>: latest phase ends load %.1f levels %.1f final %.1f boxes %.1f us\n",
                         k ? 12 : 3, (h[k][1] - h[k][0]) / 100.0, (h[k][2] - h[k][0]) / 100.0, (h[k][3] - h[k][0]) / 100.0,
                         (h[k][4] - h[k][0]) / 100.0);
    unsigned long long z[2][5];
    for (int k = 0; k < 2; ++k) { z[k][0] = ~0ull; for (int j = 1; j < 5; ++j) z[k][j] = 0; }
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tree_prof), z, sizeof(z));
    unsigned long long lv[2][9];
    if (hipMemcpyFromSymbol(lv, HIP_SYMBOL(g_tree_lev), sizeof(lv)) == hipSuccess) {
        for (int k = 0; k < 2; ++k) {
            if (!lv[k][8]) continue;
            std::fprintf(stderr, "[prof] k_tree_local<%d> per workgroup and level below G (us):", k ? 12 : 3);
            for (int j = 0; j < 8; ++j)
                if (lv[k][j]) std::fprintf(stderr, " %.1f", lv[k][j] / 100.0 / lv[k][8]);
            std::fprintf(stderr, "\n");
        }
        const unsigned long long zl[2][9] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tree_lev), zl, sizeof(zl));
    }
#endif
}

size_t tree_build_temp_bytes(int npts, int nclouds, int max_n, int L) {
    return part_layout(npts, nclouds, tree_global_levels(max_n, L), nullptr, nullptr);
}

}  // namespace se3icp
