/*
 * refcpu.h — C API of the CPU restatement ("oracle") of kenahm/se3-icp.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (se3-icp_amd/) may include,
 * link or call this.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg use it, as the checker / CPU baseline.
 *
 * The restatement follows (paths relative to the reference checkout):
 *   src/iterative_SE3_registration.cpp  (ISR.cpp)
 *   include/iterative_SE3_registration.hpp (ISR.hpp)
 * and restates the third-party arithmetic the reference calls
 * (Open3D v0.19 KDTreeFlann/EstimateNormals/TransformationEstimation*,
 *  PCL 1.14 CorrespondenceRejectorTrimmed, Eigen SelfAdjointEigenSolver,
 *  umeyama, LDLT, MatrixFunctions::sqrt) — see refcpu.cpp for per-function
 * citations.  Parity is pinned end-to-end by the reference's own fixture
 * created_example_reg_problem/ (analytic ground truth) and, for kNN/NN, by
 * scipy.spatial.cKDTree (tests/test_oracle.py).
 */
#ifndef REFCPU_H
#define REFCPU_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Mirrors the public config fields of IterativeSE3Registration (ISR.hpp:80-95)
 * with the constructor defaults of ISR.cpp:334-348. */
typedef struct refcpu_params {
    int32_t max_num_iterations;     /* 150   */
    int32_t max_num_se3_iterations; /* 20    */
    int32_t number_of_nn_for_LRF;   /* 30    */
    int32_t _pad;
    double mse;                     /* 1e-5  */
    double mse_switch_error;        /* 1e-3  */
    double estimated_overlap;       /* 1.0   */
    double alpha_rot;               /* 3.0   */
    double beta_transl;             /* 1.0   */
    double scale_preprocessing;     /* 3.0   */
} refcpu_params;

/* run kinds */
enum {
    REFCPU_RUN_ICP = 0,         /* run_icp(variant)            ISR.cpp:473-552 */
    REFCPU_RUN_SE3_ICP = 1,     /* run_se3_icp(variant)        ISR.cpp:555-739 */
    REFCPU_RUN_SE3_ICP_CF = 2,  /* run_se3_icp_with_cf()       ISR.cpp:742-959 */
    REFCPU_RUN_SE3_PURE = 3     /* run_se3_pure(variant)       ISR.cpp:962-1127 */
};
/* estimator variants ("pt2pt","pt2pl","gicp") */
enum { REFCPU_PT2PT = 0, REFCPU_PT2PL = 1, REFCPU_GICP = 2 };

typedef struct refcpu_result {
    double T[16];                   /* current_estimated_T_, row-major */
    int32_t num_iterations;
    int32_t num_pure_se3_iterations;
    double scaling_factor;
    double time_setup_ms;           /* normalization + LRF + normals/covariances */
    double time_loop_ms;            /* the while(true) loop */
    double time_nn_ms;              /* correspondence search inside the loop */
    double time_toldi_ms;           /* setup: kNN + TOLDI frames of both clouds (ISR.cpp:590-591) */
    double time_normals_ms;         /* setup: normals / GICP covariances (ISR.cpp:642-648) */
    double time_trim_ms;            /* loop: trimmed rejector (ISR.cpp:669-671) */
    double time_solve_ms;           /* loop: MSE, estimator, Transform, SE(3) update (ISR.cpp:684-716) */
} refcpu_result;

/* Optional per-iteration trace.  Any pointer may be NULL.
 *   Ti        [max_trace_iters*16]  T_i of each iteration (row-major)
 *   mse       [max_trace_iters]     mse_current after each iteration
 *   n_kept    [max_trace_iters]     trimmed correspondence count
 *   corr_idx  [max_trace_iters*n_src] NN target index per source point (pre-trim)
 *   corr_dist [max_trace_iters*n_src] float distance stored in the PCL correspondence
 *   corr_d2   [max_trace_iters*n_src] squared search distance (12-D or 3-D) of the match
 *   corr_idx2 [max_trace_iters*n_src] second-nearest target (a 2-NN search when set)
 *   corr_d2b  [max_trace_iters*n_src] its squared search distance
 * (the last three measure each query's arg-min margin, so a parity test can tell a
 *  rounding-level near-tie from a wrong correspondence)
 */
typedef struct refcpu_trace {
    int32_t max_trace_iters;
    int32_t _pad;
    double* Ti;
    double* mse;
    int32_t* n_kept;
    int32_t* corr_idx;
    float* corr_dist;
    double* corr_d2;
    int32_t* corr_idx2;
    double* corr_d2b;
} refcpu_trace;

void refcpu_default_params(refcpu_params* p);
int refcpu_num_threads(void);
void refcpu_set_num_threads(int n);

/* Full registration.  src/tgt are AoS xyz f64 (n*3).  Returns 0 on success. */
int refcpu_register(const double* src, int64_t n_src, const double* tgt, int64_t n_tgt,
                    int run_kind, int variant, const refcpu_params* params,
                    refcpu_result* out, refcpu_trace* trace);

/* ---- stage entry points (each mirrors one reference function) ---- */

/* KDTreeFlann::SearchKNN for every point of the cloud against itself;
 * idx/d2 are [n*k], sorted ascending by (d2, idx).  ISR.cpp:253 */
int refcpu_knn_self(const double* pts, int64_t n, int k, int32_t* idx, double* d2);

/* computeAllTOLDISE3FramesOMP (ISR.cpp:318-331 -> 241-316).
 * frames out: [n*16] row-major 4x4 */
int refcpu_toldi_frames(const double* pts, int64_t n, int k, double* frames);

/* PointCloud::EstimateNormals(KDTreeSearchParamKNN(k)), fast normal,
 * no prior normals (ISR.cpp:643, 43).  normals out [n*3] */
int refcpu_estimate_normals(const double* pts, int64_t n, int k, double* normals);

/* InitializePointCloudForGeneralizedICP_modified covariance from normals
 * (ISR.cpp:45-51).  cov out [n*9] row-major */
int refcpu_gicp_covariances(const double* normals, int64_t n, double eps, double* cov);

/* Exact 1-NN of each query in D dims (D = 3 or 12) with nanoflann L2 arithmetic,
 * tie-break lowest index.  ISR.cpp:402-416 (D=3), 444-470 (D=12). */
int refcpu_nn(const double* query, int64_t nq, const double* data, int64_t nd, int dim,
              int32_t* idx, double* d2);

/* Estimators on explicit correspondences (pairs [k*2] = (src_idx, tgt_idx)).
 * T out row-major.  weights may be NULL (==1).  ISR.cpp:692/695/698, 57-110 */
int refcpu_estimate(int variant, const double* src_pts, const double* src_cov,
                    const double* tgt_pts, const double* tgt_normals, const double* tgt_cov,
                    const int32_t* pairs, int64_t k, const double* weights, double* T);

/* PCL CorrespondenceRejectorTrimmed on float distances: returns kept count and
 * writes the kept query indices (sorted by (dist, query idx)).  ISR.cpp:669-671 */
int64_t refcpu_trim(const float* dist, int64_t n, double overlap_ratio, int32_t* kept_query);

#ifdef __cplusplus
}
#endif
#endif
