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
    int32_t want_cov;   // GICP covariances from normals
    int32_t want_conf;  // lounge confidences (run_se3_icp_with_cf)
    int32_t is_target;
    int32_t cf_target;  // 12-D search rows take translation from the points (ISR.cpp:834-836)
    int32_t _pad;
    double alpha, beta;
    double norm_center[3];  // p' = (p - norm_center) * norm_scale  (ISR.cpp:576-582)
    double norm_scale;
    double f32_center[3];   // xyz32 = float(p' - f32_center)
};

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
    double* fr64;
    float* fr32;
    double* nrm64;
    double* cov64;
    double* conf64;
    int32_t* knn;
    // uniform grid
    int32_t* cell_cnt;
    int32_t* cell_start;
    int32_t* slot;
    int32_t* sidx;
    double* sxyz;
    // per-cloud f32 error-bound norms (float bits, atomicMax)
    uint32_t* norm12_bits;
    uint32_t* norm3_bits;
    // loop
    int32_t* corr_idx;
    float* corr_dist;
    Cand* cand;        // [nsplit * ld]
    int32_t nsplit;
    int32_t* flag_list;
    int32_t* flag_count;  // [1]
    uint64_t* trim_key;   // [npairs]
    double* red_partial;  // [nwork * kRedVals]
    double* red_out;      // [npairs * kRedVals]
    const BlockWork* work;
    int32_t nwork;
    int32_t* pair_rechecked;  // [npairs]
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
void launch_grid_count(const View& v, hipStream_t s);
int launch_grid_scan(const View& v, int32_t ncells_total, void* temp, size_t* temp_bytes, hipStream_t s);
void launch_grid_scatter(const View& v, hipStream_t s);
void launch_knn(const View& v, hipStream_t s);
void launch_frames(const View& v, hipStream_t s);

// ---- k_loop.hip
void launch_sweep_se3(const View& v, hipStream_t s);
void launch_sweep_r3(const View& v, hipStream_t s);
void launch_finalize(const View& v, hipStream_t s);
void launch_recheck(const View& v, int nblocks, hipStream_t s);
void launch_trim(const View& v, hipStream_t s);
void launch_reduce(const View& v, const int32_t* pair_wb, const int32_t* pair_wn, hipStream_t s);

}  // namespace se3icp
