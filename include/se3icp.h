/*
 * se3icp.h — C-ABI of the MI355X-native SE(3)-ICP engine (libse3icp.so).
 *
 * Drop-in boundary for the reference's engine class
 *   class IterativeSE3Registration   include/iterative_SE3_registration.hpp:27-99
 * (kenahm/se3-icp).  Plain pointers and sizes only; no C++/torch types.
 *
 * Two surfaces:
 *   1. The object surface mirrors the reference class member for member
 *      (constructor, setSourceCloud/setTargetCloud, public config fields,
 *      run_icp / run_se3_icp / run_se3_icp_with_cf / run_se3_pure, and the
 *      result fields current_estimated_T_, num_iterations_,
 *      num_pure_se3_iterations_).  A binding for the reference would map each
 *      call 1:1.
 *   2. The batch surface registers many independent scan pairs in lockstep on
 *      one GPU (the loop the reference's benchmark drivers run serially,
 *      examples/benchmark_kitti.cpp:120-197), from host or device (HBM) buffers.
 *
 * Errors: functions return 0 on success and a negative se3icp_status otherwise;
 * se3icp_status_string() describes a code.  Point arrays are AoS xyz float64
 * (n*3 doubles), the layout of open3d::geometry::PointCloud::points_.
 * Matrices are 4x4 row-major float64.
 */
#ifndef SE3ICP_H
#define SE3ICP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SE3ICP_ABI_VERSION 4

typedef enum se3icp_status {
    SE3ICP_OK = 0,
    SE3ICP_ERR_INVALID_ARG = -1,
    SE3ICP_ERR_INVALID_METHOD = -2,   /* name not in the reference's whitelist */
    SE3ICP_ERR_EMPTY_CLOUD = -3,
    SE3ICP_ERR_K_TOO_LARGE = -4,      /* unused since ABI 3: number_of_nn_for_LRF is unbounded, as
                                         the reference's (ISR.hpp:80, ISR.cpp:253); k beyond what
                                         HBM holds fails with SE3ICP_ERR_OUT_OF_MEMORY */
    SE3ICP_ERR_NO_DEVICE = -5,        /* no HIP device / kernels not loadable: never a CPU fallback */
    SE3ICP_ERR_HIP = -6,              /* HIP runtime error */
    SE3ICP_ERR_NONFINITE = -7,        /* NaN/Inf in the resulting pose */
    SE3ICP_ERR_OUT_OF_MEMORY = -8
} se3icp_status;

/* Registration methods.  Names match examples/run_registration_method.cpp:19-24
 * ("pt2pt","pt2pl","gicp","se3_pt2pt","se3_pt2pl","se3_gicp") plus the two run
 * methods the CLI does not expose (run_se3_icp_with_cf, run_se3_pure). */
typedef enum se3icp_method {
    SE3ICP_PT2PT = 0,            /* run_icp("pt2pt")       ISR.cpp:473-552 */
    SE3ICP_PT2PL = 1,            /* run_icp("pt2pl")                        */
    SE3ICP_GICP = 2,             /* run_icp("gicp")                         */
    SE3ICP_SE3_PT2PT = 3,        /* run_se3_icp("pt2pt")   ISR.cpp:555-739 */
    SE3ICP_SE3_PT2PL = 4,        /* run_se3_icp("pt2pl")                    */
    SE3ICP_SE3_GICP = 5,         /* run_se3_icp("gicp")                     */
    SE3ICP_SE3_GICP_WITH_CF = 6, /* run_se3_icp_with_cf()  ISR.cpp:742-959 */
    SE3ICP_SE3_PURE_PT2PT = 7,   /* run_se3_pure("pt2pt")  ISR.cpp:962-1127 */
    SE3ICP_SE3_PURE_PT2PL = 8,
    SE3ICP_SE3_PURE_GICP = 9,
    SE3ICP_NUM_METHODS = 10
} se3icp_method;

/* Public config fields of IterativeSE3Registration (ISR.hpp:80-95); defaults are
 * the constructor's (ISR.cpp:334-348). */
typedef struct se3icp_params {
    int32_t max_num_iterations;     /* 150   max_num_iterations_       */
    int32_t max_num_se3_iterations; /* 20    max_num_se3_iterations_   */
    int32_t number_of_nn_for_LRF;   /* 30    number_of_nn_for_LRF_     */
    int32_t _reserved;
    double mse;                     /* 1e-5  mse_                      */
    double mse_switch_error;        /* 1e-3  mse_switch_error_         */
    double estimated_overlap;       /* 1.0   estimated_overlap_        */
    double alpha_rot;               /* 3.0   alpha_rot                 */
    double beta_transl;             /* 1.0   beta_transl               */
    double scale_preprocessing;     /* 3.0   scale_preprocessing       */
} se3icp_params;

/* Result of one registration (the reference's result members, ISR.hpp:85-98). */
typedef struct se3icp_result {
    double T[16];                     /* current_estimated_T_ (row-major)       */
    int32_t num_iterations;           /* num_iterations_                        */
    int32_t num_pure_se3_iterations;  /* num_pure_se3_iterations_ (-1 for run_icp, as the ctor) */
    int32_t status;                   /* se3icp_status of this pair             */
    int32_t num_rechecked;            /* NN queries re-resolved in f64 (diagnostic) */
    double scaling_factor;            /* 3 / max radius (1 for run_icp)         */
    double time_setup_ms;             /* normalization + TOLDI + normals (batch, GPU timeline) */
    double time_loop_ms;              /* ICP loop (batch, GPU timeline)                        */
    double time_se3_correspondence_search_ms; /* time_se3_correspondence_search_ */
    double time_before_pure_icp_ms;   /* time_before_pure_icp_: the whole run_se3_icp_with_cf
                                         (ISR.cpp:754, 957-958), GPU timeline; 0 for the other
                                         methods (the reference never sets it there).
                                         The times above are BATCH-WIDE: a batch of n_pairs > 1
                                         registers its pairs in lockstep, and every pair gets
                                         the batch's setup / loop / NN / total time, not a
                                         per-pair share (the reference times one registration;
                                         a batched caller divides by the batch size for a mean). */
} se3icp_result;

/* ------------------------------------------------------------- misc */
int se3icp_abi_version(void);
const char* se3icp_status_string(int status);
/* "se3_pt2pl" -> SE3ICP_SE3_PT2PL ...; also "se3_gicp_with_cf", "se3_pure_pt2pt" ...
 * Returns SE3ICP_ERR_INVALID_METHOD for any other string. */
int se3icp_method_from_name(const char* name);
const char* se3icp_method_name(int method);
void se3icp_default_params(se3icp_params* p);
/* Number of visible HIP devices (0 if none). */
int se3icp_device_count(void);

/* ------------------------------------------------------------- object surface
 * Mirrors IterativeSE3Registration (ISR.hpp:27-99). One object = one pair,
 * single use, like the reference (its run_* normalize member clouds in place). */
typedef struct se3icp_registration se3icp_registration;

se3icp_registration* se3icp_registration_new(void);           /* IterativeSE3Registration()   ISR.cpp:334 */
void se3icp_registration_free(se3icp_registration* r);
/* setSourceCloud(const PointCloud&) ISR.cpp:358-366 — APPENDS like the reference */
int se3icp_set_source_cloud(se3icp_registration* r, const double* xyz, int64_t n);
/* setTargetCloud(const PointCloud&) ISR.cpp:372-376 — appends */
int se3icp_set_target_cloud(se3icp_registration* r, const double* xyz, int64_t n);
/* the public config fields */
se3icp_params* se3icp_params_of(se3icp_registration* r);
/* run_icp(variant)  ISR.cpp:473 ;  variant in {"pt2pt","pt2pl","gicp"} */
int se3icp_run_icp(se3icp_registration* r, const char* variant);
/* run_se3_icp(variant)  ISR.cpp:555 */
int se3icp_run_se3_icp(se3icp_registration* r, const char* variant);
/* run_se3_icp_with_cf()  ISR.cpp:742 */
int se3icp_run_se3_icp_with_cf(se3icp_registration* r);
/* run_se3_pure(variant)  ISR.cpp:962 */
int se3icp_run_se3_pure(se3icp_registration* r, const char* variant);
/* result members */
int se3icp_get_result(const se3icp_registration* r, se3icp_result* out);

/* ------------------------------------------------------------- batch surface
 * Register n_pairs independent (source, target) pairs with one method and one
 * parameter set, on device `device` (HIP ordinal).  Host buffers.
 * Every entry taking `device` accepts `ordinal | slot << 8` (slot 0..15): slot s > 0 is a
 * further engine on the same GPU with its own stream and buffers, so independent batches
 * may be registered from several host threads at once (one engine serialises its calls). */
int se3icp_register_batch(int device, int32_t n_pairs, const double* const* src_xyz, const int64_t* n_src,
                          const double* const* tgt_xyz, const int64_t* n_tgt, int method,
                          const se3icp_params* params, se3icp_result* results);

/* Same, with all clouds already resident in HBM: d_src_xyz / d_tgt_xyz are
 * device pointers to the concatenation of every pair's AoS xyz; the host arrays
 * src_off/tgt_off (n_pairs+1 entries) give each pair's point range.
 * `hip_stream` is a hipStream_t (NULL = the engine's own stream); every kernel of the batch
 * runs on it, so work queued on `hip_stream` before the call is ordered before them. */
int se3icp_register_batch_device(int device, int32_t n_pairs, const double* d_src_xyz, const int64_t* src_off,
                                 const double* d_tgt_xyz, const int64_t* tgt_off, int method,
                                 const se3icp_params* params, se3icp_result* results, void* hip_stream);

/* Single pair convenience (host buffers). */
int se3icp_register(int device, const double* src_xyz, int64_t n_src, const double* tgt_xyz, int64_t n_tgt,
                    int method, const se3icp_params* params, se3icp_result* result);

/* ------------------------------------------------------------- stage surface
 * One entry point per reference member/free function on the hot path, operating
 * on host buffers.  They let a caller (and the parity tests) check each stage in
 * isolation.  All run on device `device`. */

/* computeAllTOLDISE3FramesOMP (ISR.cpp:318-331 -> 241-316): frames [n*16] row-major 4x4. */
int se3icp_toldi_frames(int device, const double* xyz, int64_t n, int k, double* frames);
/* KDTreeFlann::SearchKNN of every point against its own cloud: idx [n*k], sorted by (d2, idx). */
int se3icp_knn_self(int device, const double* xyz, int64_t n, int k, int32_t* idx);
/* PointCloud::EstimateNormals(KNN k) (ISR.cpp:643, :43): normals [n*3]. */
int se3icp_estimate_normals(int device, const double* xyz, int64_t n, int k, double* normals);
/* update_correspondences_raw_flann_SE3 (ISR.cpp:444-470) / update_correspondences_kd_tree_XYZ
 * (ISR.cpp:402-416): exact 1-NN of nq queries among nd points in `dim` (12 or 3)
 * dimensions (AoS rows), tie -> lowest index.  idx [nq]; d2 [nq] (may be NULL). */
int se3icp_nn(int device, const double* query, int64_t nq, const double* data, int64_t nd, int dim,
              int32_t* idx, double* d2, int32_t* num_rechecked);

/* ------------------------------------------------------------- data generators
 * The synthetic registration problems of examples/benchmark_synthetic.cpp:91-160
 * (add_noise_to_point_cloud B_SYN:13-56, RandomDownSample, T_c applied to the target),
 * generated on device `device` for n_cases cases at once: source_c = a random subset of
 * k = (int)(ratio * n) points of `base` plus N(0, noise_var I) noise, target_c = an
 * independent random subset of T_c * base plus noise.  base: host [n*3]; T: host
 * [n_cases*16] row-major.  src_out / tgt_out: [n_cases*k*3] AoS, device pointers when
 * outputs_on_device (ready for se3icp_register_batch_device with offsets c*k), host
 * pointers otherwise.  Returns k (>= 0) or a negative se3icp_status.  Counter-based
 * random streams (Philox4x32-10 keyed by `seed`, no host draws: any batch size in one pass):
 * same distributions as the reference's mt19937 draws, not the same samples (for those:
 * se3icp_synthetic_reference_device below). */
int64_t se3icp_synthetic_pairs(int device, const double* base, int64_t n, int32_t n_cases, const double* T,
                               double ratio, double noise_var, uint64_t seed, double* src_out, double* tgt_out,
                               int outputs_on_device);

/* The reference's own synthetic problems, number for number (host; no device needed):
 * examples/benchmark_synthetic.cpp:91-160 with its random streams -- Open3D's engine
 * (Seed(1), std::mt19937) for RandomDownSample, std::mt19937 gen(1) with
 * uniform_real_distribution for T (t in [-t_range, t_range]^3, rot_3d angles in
 * [-r_range, r_range]; "moderate" setup: 10, pi/2), one static std::mt19937{1} +
 * normal_distribution for the N(0, noise_var I) noise.  cloud: the full cloud in its file
 * order (stanford_bunny.ply x 50), n points.  src_out / tgt_out: [n_cases * k * 3]
 * (k = (int)(ratio * n), every case's noisy source copy and target), T_out [n_cases * 16]
 * row-major; any output may be NULL.  Returns k or a negative se3icp_status.
 * flags: SE3ICP_GEN_ARGS_LTR evaluates rot_3d's three angle draws left to right (a
 * clang-built reference) instead of GCC's right to left. */
#define SE3ICP_GEN_ARGS_LTR 1
int64_t se3icp_synthetic_reference(const double* cloud, int64_t n, int32_t n_cases, double ratio, double noise_var,
                                   double t_range, double r_range, int32_t flags, double* src_out, double* tgt_out,
                                   double* T_out);
/* The same problems, number for number, written by the GPU for a whole batch: the host
 * draws the reference's streams (as se3icp_synthetic_reference) and the device gathers,
 * transforms (Transform's arithmetic, no FMA) and adds the noise, so src_out / tgt_out equal
 * se3icp_synthetic_reference's bit for bit.  src_out / tgt_out: device pointers when
 * outputs_on_device (ready for se3icp_register_batch_device with offsets c*k), host
 * pointers otherwise; T_out: host [n_cases * 16] (may be NULL).  Returns k or a negative
 * se3icp_status. */
int64_t se3icp_synthetic_reference_device(int device, const double* cloud, int64_t n, int32_t n_cases, double ratio,
                                          double noise_var, double t_range, double r_range, int32_t flags,
                                          double* src_out, double* tgt_out, double* T_out, int outputs_on_device);
/* PointCloud::RandomDownSample(ratio) right after utility::random::Seed(seed) (Open3D 0.19):
 * the kept points in file order into out [k * 3] (may be NULL); returns k. */
int64_t se3icp_random_downsample(const double* xyz, int64_t n, double ratio, uint32_t seed, double* out);

/* ------------------------------------------------------------- diagnostics
 * Not part of the reference boundary: per-kernel GPU times (HIP events) of the
 * last batch on `device`, used by bench.py for the roofline figures.
 * (recheck_ms: ~0 since ABI 3's inline recheck -- the f64 re-resolution runs inside
 * the NN grids and is part of nn_se3_ms / nn_r3_ms.)
 * out[24] = {nn_se3_ms, nn_r3_ms, recheck_ms, trim_ms, reduce_ms, setup_ms,
 *            nn_se3_launches, nn_r3_launches, se3_dist_evals, se3_box_tests,
 *            r3_dist_evals, r3_box_tests,   (evals/tests counted per lane)
 *            lrf_ms, lrf_queries, lrf_leaves, lrf_merges, lrf_box_tests,
 *            lrf_candidates,   (kNN/TOLDI/normals kernel)
 *            nn_prep_ms, se3_queries, se3_searched, r3_queries, r3_searched,
 *            (NN certificates: queries of all iterations / those searched)
 *            lrf_fallback}  (setup queries handed to the exact one-per-wave kNN kernel) */
int se3icp_set_profiling(int device, int on);
int se3icp_last_kernel_times(int device, double* out);
/* The same record extended (ABI 4): out[SE3ICP_KERNEL_TIMES_N], n >= SE3ICP_KERNEL_TIMES_N
 * (else SE3ICP_ERR_INVALID_ARG): the 24 values above, then se3_useful_evals, r3_useful_evals --
 * the occupied (query, target) distance evaluations of the NN searches (the *_dist_evals
 * count 64-lane evaluation slots, idle lanes of partly filled sweeps included). */
#define SE3ICP_KERNEL_TIMES_N 26
int se3icp_last_kernel_times_n(int device, double* out, int n);

/* Per-iteration correspondence record of ONE pair of the next batch registered on
 * `device` (diagnostic; the parity tests compare it with the reference's loop
 * iteration by iteration).  Each row it (0-based) holds what iteration it+1 built:
 *   corr_idx / corr_dist  the pre-trim correspondence of every source point: target
 *                         index and the float distance of the pcl::Correspondence
 *                         (ISR.cpp:444-470 SE(3) phase, 402-416 R3 phase);
 *   trim_key              the trimmed rejector's cut (ISR.cpp:669-671): source point i
 *                         is kept iff (float bits of corr_dist[i]) << 32 | i <= trim_key;
 *                         UINT64_MAX when nothing is trimmed (overlap 1);
 *   T, mse                current_estimated_T_ after the iteration (normalized frame,
 *                         row-major) and the MSE it computed (ISR.cpp:684-711);
 *   phase                 1 = SE(3) correspondences, 2 = R3.
 * Any array may be NULL.  The record is armed by se3icp_set_trace (pointers are kept
 * until that batch returns, then the trace disarms itself; NULL disarms) and makes the
 * batch wait for every iteration (slower; never used by bench.py). */
typedef struct se3icp_trace {
    int32_t pair;            /* pair index within the next batch */
    int32_t max_iters;       /* rows of the arrays below */
    int32_t* corr_idx;       /* [max_iters * n_src] */
    float* corr_dist;        /* [max_iters * n_src] */
    uint64_t* trim_key;      /* [max_iters] */
    double* T;               /* [max_iters * 16] */
    double* mse;             /* [max_iters] */
    int32_t* phase;          /* [max_iters] */
    int32_t iters_recorded;  /* out: rows written */
    int32_t _reserved;
} se3icp_trace;
int se3icp_set_trace(int device, se3icp_trace* trace);

/* Diagnostic: which kernels compute the setup's kNN / TOLDI / normals on `device`:
 *   0 = the default: eight queries per wavefront (k_lrf8), the exact one-query-per-wavefront
 *       kernel for the queries it hands over, the global-buffer kernel for k > 128;
 *   1 = the exact one-query-per-wavefront kernel for every point (k <= 128);
 *   2 = the global-buffer kernel (any k) for every point.
 * All give bitwise-identical results; the tests check that. */
int se3icp_set_lrf_exact(int device, int exact_only);

/* Diagnostic: HIP events around the SE(3) NN grids of timed (non-profiled) batches, on by
 * default; they fill time_se3_correspondence_search_ms.  Each marker leaves the GPU idle a
 * few microseconds, so bench.py turns them off for its timed steps (the field is then 0). */
int se3icp_set_nn_events(int device, int on);

#ifdef __cplusplus
}
#endif
#endif /* SE3ICP_H */
