// view.hpp — the device-pointer bundle every kernel receives by value, and the
// host-callable launchers of k_setup.hip / k_loop.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.hpp"

namespace se3icp {

// Per-cloud setup request + results of the setup stages.
struct CloudSetup {
    int32_t k_knn;      // length of the kNN list to compute (0: none)
    int32_t k_lrf;      // TOLDI k (0: no frames)
    int32_t k_nrm;      // EstimateNormals k (0: no normals)
    int32_t want_cov;   // GICP: covariances from the normals (computed where k_reduce uses them)
    int32_t want_conf;  // lounge confidences (run_se3_icp_with_cf)
    int32_t is_target;
    int32_t cf_target;  // 12-D search rows take translation from the points (ISR.cpp:834-836)
    int32_t _pad;
    double alpha, beta;
    double norm_center[3];  // p' = (p - norm_center) * norm_scale  (ISR.cpp:576-582)
    double norm_scale;
    double f32_center[3];   // xyz32 = float(p' - f32_center)
};

// Read-only view of the kd-trees of one dimension (tree.hpp) for the query kernels.
struct TreeRef {
    int32_t L;        // depth: leaves at level L
    int32_t GL;       // level whose nodes are the loop's query groups (<= 64 points)
    int32_t nnodes;   // heap slots per cloud
    const int32_t* perm;  // [ld] tree position (cloud.off + x) -> local point index
    const int32_t* pos;   // [ld] point (cloud.off + i) -> local tree position
    const float* tvec;    // vectors in tree order: 3-D [3][ld] columns, 12-D [ld][12] rows (tree_tv_ix)
    const double* tvec64; // [3][ld] f64 in tree order: the points (3-D), the frames' translation rows (12-D)
    const double4* tpt64; // [ld] the same, one (x, y, z, 0) record per point (3-D trees: the setup's gathers)
    const float* lo;      // [nclouds][nnodes][D]
    const float* hi;
};

// k_nn.hip certificate record of a query (View::cert), written by its last search:
//   d1: the match is at most d1 away (exact distance, conservatively rounded), l2: every
//   other target at least l2, iter: the iteration of that search (-1: none), j: the match
//   (target index), t: the match's anchor for the stored distance (ISR.cpp:465-468 / 411-413:
//   the target's translation row in the SE(3) phase, its point in the R3 phase), margin: the
//   search-radius expansion of a query searched in the current iteration (k_nn_prep)
struct alignas(16) NNCert {
    float d1, l2;
    int32_t iter, j;
    double t[3];
    float margin;
    int32_t _pad;
};
static_assert(sizeof(NNCert) == 48, "three 16-B words");

struct View {
    int32_t ld;        // SoA row stride (total points of the batch, padded to 64)
    int32_t npts;      // real points of the batch (per-point kernels stop here)
    int32_t nclouds;
    int32_t npairs;
    int32_t kmax;      // row stride of the knn table
    CloudDev* clouds;
    CloudSetup* setup;
    PairDev* pairs;
    int32_t* cloud_of;
    const double* const* in_ptr;  // per cloud: AoS xyz input (device)
    double* xyz64;
    float* xyz32;
    double* fr64;  // [ld][12] SE(3) 12-vectors of every point (rows: gathered by point)
    float* fr32;   // [ld][12] their f32 copies (the 12-D trees' input)
    double* nrm64;
    double* conf64;
    // [ld][8] geometry rows of the target points (x y z nx ny nz conf 0, normalized frame),
    // written once per batch by k_geo_rows: k_reduce gathers one 64-B row per kept
    // correspondence instead of seven 8-B words from seven SoA rows (one 128-B line each)
    double* tgeo;
    int32_t* knn;
    // per-cloud f32 error-bound norms (float bits, atomicMax)
    // loop
    int32_t* corr_idx;
    float* corr_dist;
    unsigned long long* stats;  // [4] NN work counters: se3 dist evals, se3 box tests, r3 dist evals, r3 box tests
    int32_t* flag_count;  // [3] (unused), single-query lists (SE(3), R3)
    uint64_t* trim_key;   // [npairs] cut key, then [npairs] k_trim window state
    unsigned long long* trim_cand;  // [npairs][kTrimList] k_trim window keys
    unsigned* trim_ctr;   // [npairs][4] k_trim counters (zero between launches)
    unsigned* trim_hist;  // [npairs][4096] top-12-bit key histogram (zero between launches)
    double* red_partial;  // [nwork * kRedVals]
    double* red_out;      // [npairs * kRedVals]
    const BlockWork* work;
    int32_t nwork;
    int32_t* pair_rechecked;  // [npairs]
    // kd-trees (k_tree.hip) over the f32 vectors: 3-D points (xyz32) and 12-D SE(3) elements (fr32)
    TreeRef t3, t12;
    // loop NN work (k_nn.hip): chunk c = node (c mod 2^CL) of level CL of pair (c >> CL)'s
    // source tree (<= kChunkQ positions); k_nn_prep compacts the chunk's queries that its
    // certificate cannot settle into qlist, k_nn_search sweeps them 64 per wavefront
    int32_t chunk_level;  // CL
    int32_t nchunks;      // npairs << CL
    int32_t* qlist;       // [nchunks * kChunkQ] global slots of the searched queries, tree order
    int32_t* qcount;      // [nchunks][16] lanes of each group (0: none)
    int32_t* sq_list;     // [ld] queries of sparse chunks (global source tree slots), one per wave:
                          // SE(3) phase from the front (count flag_count[1]), R3 from the back ([2])
    const double* hist;   // [kHist][npairs][12] pose T used at iteration k, row k % kHist
    // NN certificate of each source point from its last search, one 48-B record per slot of
    // the PHASE's source tree (12-D in the SE(3) phase, 3-D in the R3 phase: a certificate of
    // the other phase is void anyway), so k_nn_prep reads them in tree order, coalesced
    NNCert* cert;
    uint32_t* gcost;      // [nchunks * 16] duration of each group's last search wave, either phase (100 MHz ticks; 0: none)
    int32_t* cls;         // cost-ordered dispatch: [2 phases][8 XCDs][16 classes] counts, then the lists
};

// ---- k_setup.hip
// chunk table for setup reductions: entries (cloud, first local idx), 2048 points each
constexpr int kChunk = 2048;
struct ChunkWork { int32_t cloud; int32_t p0; };

void launch_ingest(const View& v, const ChunkWork* chunks, int nchunks, double* partial /*[nchunks*9]*/, hipStream_t s);
void launch_radius(const View& v, const ChunkWork* chunks, int nchunks, const double* centers /*[nclouds*3]*/,
                   double* partial /*[nchunks]*/, hipStream_t s);
void launch_normalize(const View& v, const ChunkWork* chunks, int nchunks, double* partial /*[nchunks*7]*/,
                      hipStream_t s);
// device-side normalization parameters of pairs (clouds 2p, 2p+1): centers [nclouds*3]
// from the ingest partials, scales [npairs] and the CloudSetup fields from the radius
// partials; then the targets' root-box norm bounds into PairDev (and scales into the
// PairState sf fields, stride in doubles) once the trees and the pair records exist
void launch_pair_centers(const View& v, const ChunkWork* chunks, int nchunks, const double* partial, double* centers,
                         hipStream_t s);
void launch_pair_scales(const View& v, const ChunkWork* chunks, int nchunks, const double* partial,
                        const double* centers, double scale_pre, double* scales, hipStream_t s);
void launch_pair_norms(const View& v, int nnodes3, int nnodes12, const double* scales, double* state_sf,
                       int state_stride, hipStream_t s);
// fused kNN + TOLDI frame + normals/GICP covariance (k_knn.hip); knn list only if v.knn
void launch_lrf(const View& v, int write_knn, hipStream_t s);
// the same for the listed tree slots qlist[0 .. *qcount) (device count; grid-strided)
// (qpw: queries per wave, 0 = the default)
void launch_lrf_list(const View& v, const int32_t* qlist, const int32_t* qcount, hipStream_t s, int qpw = 0);
// eight queries per wavefront (k_lrf8.hip); wave_base[c] = first wave of cloud c (waves
// aligned to each cloud); this launch runs waves w_lo .. w_hi-1; the queries it cannot
// resolve exactly from f32 keys are appended to fb_list (count fb_count, zeroed by the
// caller) for launch_lrf_list
void launch_lrf8(const View& v, const int32_t* wave_base, int w_lo, int w_hi, int32_t* fb_list, int32_t* fb_count,
                 hipStream_t s);
// neighbourhoods over kSmallK (k_knn_big.hip): one wavefront per query with a global-memory
// candidate buffer of `cap` entries per block; queries with Kw = min(k, n) <= k_min are
// skipped (the LDS kernels'); qlist = nullptr: every point
int knn_big_cap(int kw_max);
int knn_big_blocks(int cap, int nq);
void launch_knn_big(const View& v, int write_knn, int k_min, const int32_t* qlist, const int32_t* qcount, int nblocks,
                    double* scratch_d, int32_t* scratch_i, int cap, hipStream_t s);

// ---- k_loop.hip
// exact 1-NN of every active pair's source points: k_nn_prep settles the queries whose
// certificate still holds and lists the rest, k_nn_search sweeps those 64 per wavefront
// (and the queries of sparse chunks one per wavefront, in the same grid)
// through the target kd-tree (12-D in the SE(3) phase, 3-D in the R3 phase)
// publish: host slot that receives every pair's phase at the start of the launch (or null)
void launch_nn_prep(const View& v, int32_t* publish, hipStream_t s);
void nn_prof_report();  // (SE3ICP_PROF builds: k_nn_prep block phases, then reset)
void trim_prof_report();  // (SE3ICP_PROF builds: k_trim phases, then reset)
#ifdef SE3ICP_PROF
double nn_prep_span();        // span of the last k_nn_prep launch (us)
void nn_wave_report(int it);  // SE(3) group-wave durations since the last call
#endif
// the search of a phase (D = 12 or 3): one grid, single-query waves first, then the groups
void launch_nn(const View& v, int D, hipStream_t s);
// words of View::cls for nchunks chunks (counts + per-XCD class lists)
size_t nn_cls_words(int nchunks);
void launch_trim(const View& v, hipStream_t s);
// the target points' geometry rows (View::tgeo) from xyz64 / nrm64 / conf64
void launch_geo_rows(const View& v, hipStream_t s);
// reduce + (k_reduce_final) per-pair solve and loop state machine; next_phase[p] receives
// pair p's phase in the next iteration (PHASE_IDLE: finished)
struct PairState;
void launch_reduce(const View& v, const int32_t* pair_wb, const int32_t* pair_wn, PairState* state, double* hist,
                   int32_t* next_phase, hipStream_t s);

}  // namespace se3icp
