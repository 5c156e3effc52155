// engine.hpp — host driver of the MI355X SE(3)-ICP engine.
//
// One Engine per HIP device.  register_batch() runs every pair of a batch in
// lockstep: each iteration launches one grid per stage covering all active pairs
// (pairs in the SE(3) phase and pairs already switched to the R3 phase share the
// iteration); the f64 solve and the reference's switch / convergence logic
// (ISR.cpp:654-732) run on the device at the end of the iteration (pairmath.hpp), and
// the host queues the next iteration before the previous one has finished.
#pragma once
#include <hip/hip_runtime.h>

#include <mutex>
#include <stdint.h>
#include <vector>

#include "pairmath.hpp"
#include "se3icp.h"
#include "view.hpp"

namespace se3icp {

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

// Per-kernel GPU time of the last register_batch (HIP events, ms), for bench.py.
struct KernelTimes {
    double nn_se3_ms = 0, nn_r3_ms = 0, recheck_ms = 0, trim_ms = 0, reduce_ms = 0;
    double setup_ms = 0;
    int64_t nn_se3_launches = 0, nn_r3_launches = 0;
    // work actually done by the NN kernels (device counters): lane-distance evaluations
    // in leaf sweeps and lane-box tests in the traversal
    double se3_dist_evals = 0, se3_box_tests = 0, r3_dist_evals = 0, r3_box_tests = 0;
    double se3_useful_evals = 0, r3_useful_evals = 0;  // occupied (query, target) evaluations
    // fused kNN/TOLDI/normals kernel of the setup: time, queries, leaves scanned, sorts
    double lrf_ms = 0, lrf_queries = 0, lrf_leaves = 0, lrf_merges = 0, lrf_box_tests = 0, lrf_candidates = 0;
    double lrf_fallback = 0;  // queries k_lrf8 handed to the exact kernel
    // NN certificates (k_nn_prep): its time, and per phase the queries of all iterations
    // and those that had to be searched
    double nn_prep_ms = 0, se3_queries = 0, se3_searched = 0, r3_queries = 0, r3_searched = 0;
};

class Engine {
  public:
    explicit Engine(int device);
    ~Engine();
    Engine(const Engine&) = delete;
    Engine& operator=(const Engine&) = delete;

    int device() const { return dev_; }
    std::mutex& mutex() { return mu_; }
    void set_profiling(bool on) { profile_ = on; }
    void set_trace(se3icp_trace* t) { trace_ = t; }
    void set_lrf_exact(int mode) { lrf_exact_only_ = mode; }
    void set_nn_events(bool on) { nn_events_ = on; }
    const KernelTimes& kernel_times() const { return ktimes_; }

    int register_batch(int npairs, const double* const* src, const int64_t* ns, const double* const* tgt,
                       const int64_t* nt, bool on_device, int method, const se3icp_params& prm,
                       se3icp_result* out, hipStream_t user_stream);

    // stage entry points (host buffers)
    int knn_self(const double* xyz, int64_t n, int k, int32_t* idx);
    int toldi_frames(const double* xyz, int64_t n, int k, double* frames);
    int estimate_normals(const double* xyz, int64_t n, int k, double* normals);
    int nn(const double* query, int64_t nq, const double* data, int64_t nd, int dim, int32_t* idx, double* d2,
           int32_t* num_rechecked);

  private:
    struct CloudReq {
        const double* in = nullptr;  // AoS input
        int64_t n = 0;
        CloudSetup st{};
    };
    struct TreeBufs {
        DevBuf perm, pos, vec, vec64, vec64a, blo, bhi, lo, hi, scr, vecT;  // (vecT: 12-D input columns)
        int L = 0;  // depth of the trees in these buffers
    };
    int init();
    template <class T>
    T* ensure(DevBuf& b, size_t count);
    int alloc_points(int64_t ntot, int kmax, bool knn_list = false);
    // build the D-dimensional kd-trees of every cloud over `vec` ([D][ld] f32)
    int build_tree(int D, const float* vec, hipStream_t s, const double* vec64 = nullptr);
    // ingest -> (normalize) -> 3-D kd-trees -> kNN -> frames (-> 12-D kd-trees) for a
    // list of clouds.  When `normalize_pairs` is set, clouds (2p, 2p+1) are normalized
    // together with the reference's preprocessing and scale[p] receives the factor.
    int setup_clouds(std::vector<CloudReq>& clouds, bool on_device, bool normalize_pairs, double scale_pre,
                     bool build12, std::vector<double>* centers, std::vector<double>* scales, hipStream_t s);
    int setup_chunks(int npairs, hipStream_t s);
    int read_lrf_stats();
    int sync_stream(hipStream_t s);
    View view() const;

    int dev_;
    bool ok_ = false;
    bool profile_ = false;
    std::mutex mu_;
    hipStream_t stream_ = nullptr;
    KernelTimes ktimes_;

    // geometry of the current batch
    int nclouds_ = 0, npairs_ = 0;
    int64_t ntot_ = 0;
    int ld_ = 0, kmax_ = 1, nwork_ = 0, tree_L_ = 0;
    int chunk_level_ = 0, nchunks_ = 0;  // loop NN work chunks (View::chunk_level)
    bool have12_ = false, knn_list_ = false;
    bool nn_trace_ = false;              // SE3ICP_NN_TRACE=1: per-iteration NN work on stderr
    // se3icp_set_lrf_exact: 0 k_lrf8 + hand-overs (default), 1 the exact one-query-per-wavefront
    // k_lrf for every point, 2 the global-buffer k_knn_big for every point (all bitwise equal)
    int lrf_exact_only_ = 0;
    // se3icp_set_nn_events(0): no HIP event bracket around the SE(3) NN search outside
    // profiled batches (each marker leaves the GPU idle a few us;
    // time_se3_correspondence_search_ms is then 0)
    bool nn_events_ = true;
    se3icp_trace* trace_ = nullptr;      // armed per-iteration record of one pair (se3icp_set_trace)
    int record_trace(se3icp_trace* tr, int it, int& phase_of_it, hipStream_t s);
    double trace_prev_[kStatCols] = {};
    std::vector<CloudDev> h_clouds_;
    std::vector<CloudSetup> h_setup_;
    std::vector<BlockWork> h_work_;
    std::vector<int32_t> h_wb_, h_wn_;
    std::vector<ChunkWork> h_chunks_;
    std::vector<const double*> h_inptr_;

    // device buffers
    DevBuf d_clouds_, d_setup_, d_pairs_, d_cloud_of_, d_inptr_, d_in_, d_xyz64_, d_xyz32_, d_fr64_, d_fr32_, d_nrm64_, d_tgeo_,
        d_conf64_, d_knn_, d_corr_idx_, d_corr_dist_, d_flag_count_, d_gcost_, d_cls_,
        d_trim_key_, d_red_partial_, d_red_out_, d_work_, d_wb_, d_wn_, d_chunks_, d_partial_, d_centers_,
        d_rechecked_, d_keys0_, d_vals1_, d_sort_tmp_, d_stats_, d_qlist_, d_qcount_, d_hist_, d_cert_,
        d_sqlist_, d_state_, d_trim_cand_, d_trim_ctr_, d_scales_, d_trim_hist_,
        d_lrf_fb_, d_lrf_fbn_,  // k_lrf8 -> exact k_lrf hand-over list and its count
        d_big_d_, d_big_i_;     // k_knn_big candidate buffers (neighbourhoods over kSmallK)
    TreeBufs t3_, t12_;
    // pinned host mirrors
    PairDev* h_pairs_ = nullptr;
    double* h_red_ = nullptr;
    double* h_partial_ = nullptr;
    int32_t* h_rechecked_ = nullptr;
    double* h_hist_ = nullptr;  // one pose-history row (npairs x 12)
    size_t h_pairs_cap_ = 0, h_red_cap_ = 0, h_partial_cap_ = 0, h_rechecked_cap_ = 0, h_hist_cap_ = 0;
    PairState* h_state_ = nullptr;  // loop state of every pair (read back after the loop)
    // [kLoopRing][npairs] each pair's phase in the next iteration, written by k_reduce_final
    // into coherent host memory (h_phase_ host view, d_phase_ device view)
    int32_t* h_phase_ = nullptr;
    int32_t* d_phase_ = nullptr;
    size_t h_state_cap_ = 0, h_phase_cap_ = 0;
    unsigned long long* h_lrf_stats_ = nullptr;  // k_lrf work counters (read at the next sync)
    size_t h_lrf_stats_cap_ = 0;
    unsigned long long* h_loop_stats_ = nullptr;  // loop NN work counters (pinned: an async copy, not a staged one)
    size_t h_loop_stats_cap_ = 0;
    bool lrf_stats_pending_ = false;
    // 6/7: k_lrf time; 12/13/14: batch begin / setup done / loop done (GPU-timeline phase
    // times); 15: sync_stream; the rest unused
    hipEvent_t ev_[16];
    // loop iterations in flight: kernel-time events and launched NN phases per ring slot
    static constexpr int kLoopRing = 4, kLoopEv = 7;
    hipEvent_t loop_ev_[kLoopRing * kLoopEv];
    int loop_flags_[kLoopRing] = {};
    bool loop_detail_[kLoopRing] = {};
};

// process-wide engine per device (lazily created)
Engine* engine_for(int device);

}  // namespace se3icp
