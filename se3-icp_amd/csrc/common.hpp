// common.hpp — data layout shared by the HIP kernels and the host engine.
//
// HBM layout (one batch = P independent pairs = 2P clouds, all concatenated):
//   cloud c occupies global point indices [CloudDev.off, CloudDev.off + n).
//   Every per-point array is SoA with row stride `ld` (= total points, padded):
//     xyz64[3][ld]   normalized coordinates (source_/target_ after ISR.cpp:576-582)
//     xyz32[3][ld]   f32 copy for the R3 sweep (centered, see k_setup.hip)
//     fr64 [12][ld]  alpha/beta-weighted TOLDI SE(3) element as a 12-vector in the
//                    reference's packing [R00 R10 R20 R01 R11 R21 R02 R12 R22 t0 t1 t2]
//                    (ISR.cpp:450-453, 613-624)
//     fr32 [12][ld]  f32 copy of target frames for the SE(3) sweep
//     nrm64[3][ld], conf64[ld] (GICP covariances are recomputed from nrm64 where used)
// Source clouds are never rewritten inside the loop: the current pose T of a pair
// is applied on the fly (query = T * M0), see DESIGN.md "Pose on the fly".
#pragma once
#include <stdint.h>

namespace se3icp {

constexpr int kSmallK = 128;      // neighbourhoods the LDS kNN kernels hold; larger ones: k_knn_big.hip
constexpr int kBlock = 256;       // threads per block of the streaming/sweep kernels
constexpr int kRedVals = 28;      // 21 JTJ upper + 6 JTr + 1 mse-sum (pt2pt reuses the slots)
constexpr int kStatCols = 17;     // columns of the device work-counter table (View::stats); 8..14: SE3ICP_PROF section cycles
// NN work: occupied (query, target) distance evaluations of the SE(3) / R3 searches (the
// lane-evaluation slots they issue are columns 0 and 2)
constexpr int kStatUseSe3 = 15, kStatUseR3 = 16;
constexpr int kHist = 256;        // pose history ring of the loop (View::hist), iterations
constexpr int kTrimList = 4096;   // k_trim: LDS key list / window capacity per pair
constexpr int kTrimBlocks = 32;   // k_trim_window: blocks per pair
constexpr int kChunkQ = 1024;     // source tree positions per NN work chunk (16 query groups)

enum Phase : int32_t { PHASE_IDLE = 0, PHASE_SE3 = 1, PHASE_R3 = 2 };
enum Estimator : int32_t { EST_PT2PT = 0, EST_PT2PL = 1, EST_GICP = 2 };

struct CloudDev {
    int32_t off;        // first global point index
    int32_t n;          // points
};

// Rewritten by the host every iteration (tiny H2D copy).
struct PairDev {
    double T[12];          // accumulated pose, rows 0..2 of the 4x4 (row-major 3x4)
    double f32_center[3];  // center subtracted from the f32 copies of this pair (R3 sweep)
    int32_t src, tgt;      // cloud ids
    int32_t phase;         // Phase
    int32_t est;           // Estimator
    int32_t cf;            // run_se3_icp_with_cf weighting / mse
    int32_t trim;          // 1 if ratio < 1 (threshold key valid)
    int32_t nkeep;         // floor(float(ratio) * float(ns))
    int32_t iter;          // 1-based iteration number (num_iterations_ after this iteration)
    float tgt_norm12;      // max |target 12-vector| (f32 sweep error bound)
    float tgt_norm3;       // max |centered target xyz| (f32 R3 error bound)
    int32_t phase_start;   // first iteration of the current phase (older NN certificates are void)
    int32_t _pad;
};

// k_reduce: threads per block, queries per thread (all of a thread's loads are issued
// before its first term; measured at C4: 2 per thread 146 VGPRs, 1,024-thread blocks: both
// slower than 256 x 1) and queries per block
constexpr int kRedThreads = 256;
constexpr int kRedPer = 1;
constexpr int kRedQ = kRedThreads * kRedPer;

// Static work table of k_reduce: one entry per kRedQ-query block of every pair.
struct BlockWork {
    int32_t pair;
    int32_t q0, q1;        // local query range [q0, q1) of the block
    int32_t s_off, t_off;  // global slots of the pair's source / target cloud
    int32_t _pad[3];
};

}  // namespace se3icp
