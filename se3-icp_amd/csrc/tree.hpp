// tree.hpp — implicit balanced kd-trees (k_tree.hip) and their query helpers.
//
// Tree of a cloud with n points and depth L: node i of level l covers the tree
// positions [n*i/2^l, n*(i+1)/2^l); heap index 2^l - 1 + i; leaves are level L.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "common.hpp"

namespace se3icp {

constexpr int kLeafMax = 64;  // points per leaf (one wavefront)

struct TreeView {
    int32_t D;        // 3 or 12
    int32_t L;        // depth (leaves at level L)
    int32_t nnodes;   // 2^(L+1) nodes reserved per cloud (heap order)
    int32_t nclouds;
    int32_t npts;
    int32_t ld;
    const CloudDev* clouds;
    const int32_t* cloud_of;
    const float* vec;  // input vectors, original order: 12-D [ld][12] rows, 3-D [3][ld] columns
    // the input as [D][ld] columns (3-D: vec itself; 12-D: a copy k_tree_init writes), for the
    // passes that gather ONE coordinate per point (a 4-B column entry, not a 48-B row's sector)
    float* vecT;
    int32_t* perm;     // [ld] tree position (global slot) -> local point index
    int32_t* pos;      // [ld] point (global slot) -> local tree position
    float* tvec;       // vectors in tree order: 3-D [3][ld] columns, 12-D [ld][12] rows (tree_tv_ix)
    const double* vec64;  // optional f64 vectors (original order, the layout of vec) ...
    double* tvec64;       // ... copied into tree order (coalesced leaf / query-chunk loads): [3][ld], the
                          // points (3-D) or the translation rows (12-D: the loop reads whole frames by point)
    double4* tpt64;       // 3-D: the tree-ordered f64 points as (x, y, z, 0) records (one line per gather)
    int32_t vec64_sources_only;  // copy the f64 vectors of even (source) clouds only
    uint32_t* blo;     // [nclouds][nnodes][D] build scratch (orderable bits)
    uint32_t* bhi;
    float* scr;        // [D][ld] build scratch (k_tree_local: the vectors at the level-G positions)
    float* lo;         // [nclouds][nnodes][D] node boxes
    float* hi;
    const int32_t* host_n;  // host copy of the clouds' point counts (level split of the build)
};

__host__ __device__ __forceinline__ int tree_first(int n, int level, int i) {
    return (int)(((long long)n * i) >> level);
}
// node of level `level` containing local tree position x
__host__ __device__ __forceinline__ int tree_node_of(int x, int n, int level) {
    const long long v = ((long long)(x + 1) << level) + n - 1;
    return (int)(v / n) - 1;
}
__host__ __device__ __forceinline__ int tree_heap(int level, int i) { return (1 << level) - 1 + i; }
// element d of the input vector at global slot p: the 12-D vectors (SE(3) frames) are
// rows (a gather by the permutation reads one or two cache lines, not twelve), the 3-D
// points columns
__device__ __forceinline__ size_t tree_in_ix(const TreeView& t, int d, int p) {
    return t.D == 12 ? (size_t)p * 12 + d : (size_t)d * t.ld + p;
}
// coordinate d of the input vector at global slot p, from the column copy
__device__ __forceinline__ float tree_in_col(const TreeView& t, int d, int p) { return t.vecT[(size_t)d * t.ld + p]; }

// element d of the tree-ordered vector at global tree slot x: the 12-D vectors are 48-B
// rows (a leaf's 64 targets are one contiguous 3-KB run: three 16-B loads per lane instead
// of twelve strided ones), the 3-D points columns
template <int D>
__host__ __device__ __forceinline__ size_t tree_tv_ix(size_t ld, int x, int d) {
    return D == 12 ? (size_t)x * 12 + d : (size_t)d * ld + x;
}

inline int tree_depth_for(int max_n) {
    int L = 0;
    while (((long long)max_n + (1ll << L) - 1) >> L > kLeafMax) ++L;
    return L;
}

// qbuf: [npts] u32 scratch, perm_alt: [npts] the second permutation buffer of the global levels
int build_trees(TreeView t, void* tmp, size_t tmp_bytes, uint32_t* qbuf, int32_t* perm_alt, hipStream_t s);
size_t tree_build_temp_bytes(int npts, int nclouds, int max_n, int L);
int tree_global_levels(int max_n, int L);
void tree_prof_report();  // (SE3ICP_PROF builds: k_tree_local's phase timeline, then reset)

}  // namespace se3icp
