// engine.cpp — host driver (see engine.hpp).
#include "engine.hpp"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>

#include "tree.hpp"

namespace se3icp {

namespace {

#define HIPCHK(x)                                                                                   \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            std::fprintf(stderr, "se3icp: HIP error %s at %s:%d (%s)\n", hipGetErrorString(e_), __FILE__, \
                         __LINE__, #x);                                                             \
            return SE3ICP_ERR_HIP;                                                                  \
        }                                                                                           \
    } while (0)
#define SYNC_STREAM(st)                   \
    do {                                  \
        const int rc_ = sync_stream(st);  \
        if (rc_) return rc_;              \
    } while (0)

// Kind (KIND_ICP / SE3 / CF / PURE): pairmath.hpp

struct MethodInfo {
    Kind kind;
    int est;
};

bool decode_method(int method, MethodInfo* mi) {
    switch (method) {
        case SE3ICP_PT2PT: *mi = {KIND_ICP, EST_PT2PT}; return true;
        case SE3ICP_PT2PL: *mi = {KIND_ICP, EST_PT2PL}; return true;
        case SE3ICP_GICP: *mi = {KIND_ICP, EST_GICP}; return true;
        case SE3ICP_SE3_PT2PT: *mi = {KIND_SE3, EST_PT2PT}; return true;
        case SE3ICP_SE3_PT2PL: *mi = {KIND_SE3, EST_PT2PL}; return true;
        case SE3ICP_SE3_GICP: *mi = {KIND_SE3, EST_GICP}; return true;
        case SE3ICP_SE3_GICP_WITH_CF: *mi = {KIND_CF, EST_GICP}; return true;
        case SE3ICP_SE3_PURE_PT2PT: *mi = {KIND_PURE, EST_PT2PT}; return true;
        case SE3ICP_SE3_PURE_PT2PL: *mi = {KIND_PURE, EST_PT2PL}; return true;
        case SE3ICP_SE3_PURE_GICP: *mi = {KIND_PURE, EST_GICP}; return true;
        default: return false;
    }
}

template <class T>
int pinned(T*& p, size_t& cap, size_t count) {
    if (cap >= count && p) return 0;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    size_t want = std::max<size_t>(count, 16);
    if (hipHostMalloc((void**)&p, want * sizeof(T), hipHostMallocDefault) != hipSuccess) {
        cap = 0;
        return SE3ICP_ERR_OUT_OF_MEMORY;
    }
    cap = want;
    return 0;
}

// Wait for an event by polling: the loop's host side has nothing else to do, and a
// blocking wait adds the thread's wake-up latency to every step.
hipError_t spin_wait(hipEvent_t e) {
    for (;;) {
        const hipError_t r = hipEventQuery(e);
        if (r != hipErrorNotReady) return r;
    }
}

// Wait until every pair's phase of the next iteration is in the coherent host slot
// (cleared to -1 before the iteration was queued; written by the next k_nn_prep, or by
// k_reduce_final without look-ahead): the loop needs no per-iteration end event, whose
// marker leaves the GPU idle ~5 us.  The stream is queried only after 20 ms without the slot
// (a stream that completed or failed with it unwritten is reported, not waited on):
// hipStreamQuery itself puts a marker into the stream, which held the GPU idle ~6 us per
// iteration when it was called every 1,024 polls (round 3).
hipError_t spin_phases(const volatile int32_t* slot, int n, hipStream_t s) {
    auto next = std::chrono::steady_clock::now() + std::chrono::milliseconds(20);
    for (unsigned spins = 0;; ++spins) {
        int left = 0;
        for (int p = 0; p < n; ++p) left += slot[p] < 0;
        if (left == 0) return hipSuccess;
        if ((spins & 1023u) == 1023u && std::chrono::steady_clock::now() >= next) {
            const hipError_t r = hipStreamQuery(s);
            if (r == hipSuccess) {
                left = 0;
                for (int p = 0; p < n; ++p) left += slot[p] < 0;
                return left == 0 ? hipSuccess : hipErrorUnknown;
            }
            if (r != hipErrorNotReady) return r;
            next = std::chrono::steady_clock::now() + std::chrono::milliseconds(20);
        }
    }
}

constexpr int kStatSlots = 64;  // work counters: [64][kStatCols] u64 (spread against atomic contention)

}  // namespace

Engine::Engine(int device) : dev_(device) {
    for (auto& e : ev_) e = nullptr;
    for (auto& e : loop_ev_) e = nullptr;
    ok_ = init() == 0;
}

int Engine::init() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || dev_ < 0 || dev_ >= n) return SE3ICP_ERR_NO_DEVICE;
    HIPCHK(hipSetDevice(dev_));
    HIPCHK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    for (auto& e : ev_) HIPCHK(hipEventCreate(&e));
    for (auto& e : loop_ev_) HIPCHK(hipEventCreate(&e));
    if (const char* e = std::getenv("SE3ICP_NN_TRACE")) nn_trace_ = std::atoi(e) != 0;
    return 0;
}

Engine::~Engine() {
    if (!ok_) return;
    (void)hipSetDevice(dev_);
    DevBuf* all[] = {&d_clouds_, &d_setup_, &d_pairs_, &d_cloud_of_, &d_inptr_, &d_in_, &d_xyz64_, &d_xyz32_,
                     &d_fr64_, &d_fr32_, &d_nrm64_, &d_tgeo_, &d_conf64_, &d_knn_,
                     &d_corr_idx_, &d_corr_dist_, &d_flag_count_, &d_gcost_, &d_cls_, &d_trim_key_, &d_red_partial_,
                     &d_red_out_, &d_work_, &d_wb_, &d_wn_, &d_chunks_, &d_partial_, &d_centers_,
                     &d_rechecked_, &d_keys0_, &d_vals1_, &d_sort_tmp_, &d_stats_,
                     &d_qlist_, &d_qcount_, &d_hist_, &d_cert_, &d_sqlist_, &d_state_, &d_trim_cand_, &d_trim_ctr_, &d_scales_, &d_trim_hist_,
                     &d_lrf_fb_, &d_lrf_fbn_, &d_big_d_, &d_big_i_,
                     &t3_.perm, &t3_.pos, &t3_.vec, &t3_.vec64, &t3_.vec64a, &t3_.blo, &t3_.bhi, &t3_.lo, &t3_.hi, &t3_.scr,
                     &t12_.perm, &t12_.pos, &t12_.vec, &t12_.vec64, &t12_.blo, &t12_.bhi, &t12_.lo, &t12_.hi, &t12_.scr,
                     &t12_.vecT};
    for (DevBuf* b : all)
        if (b->p) (void)hipFree(b->p);
    if (h_pairs_) (void)hipHostFree(h_pairs_);
    if (h_red_) (void)hipHostFree(h_red_);
    if (h_partial_) (void)hipHostFree(h_partial_);
    if (h_rechecked_) (void)hipHostFree(h_rechecked_);
    if (h_hist_) (void)hipHostFree(h_hist_);
    if (h_lrf_stats_) (void)hipHostFree(h_lrf_stats_);
    if (h_loop_stats_) (void)hipHostFree(h_loop_stats_);
    for (auto& e : ev_)
        if (e) (void)hipEventDestroy(e);
    for (auto& e : loop_ev_)
        if (e) (void)hipEventDestroy(e);
    if (h_state_) (void)hipHostFree(h_state_);
    if (h_phase_) (void)hipHostFree(h_phase_);
    if (stream_) (void)hipStreamDestroy(stream_);
}

template <class T>
T* Engine::ensure(DevBuf& b, size_t count) {
    const size_t want = std::max<size_t>(count, 1) * sizeof(T);
    if (b.bytes >= want) return static_cast<T*>(b.p);
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
    const size_t alloc = want + want / 4;
    if (hipMalloc(&b.p, alloc) != hipSuccess) {
        b.p = nullptr;
        return nullptr;
    }
    b.bytes = alloc;
    return static_cast<T*>(b.p);
}

int Engine::alloc_points(int64_t ntot, int kmax, bool knn_list) {
    if (ntot >= (int64_t)1 << 30) return SE3ICP_ERR_INVALID_ARG;
    ntot_ = ntot;
    ld_ = (int)((std::max<int64_t>(ntot, 1) + 63) / 64 * 64);
    kmax_ = std::max(kmax, 1);
    knn_list_ = knn_list;
    const size_t L = (size_t)ld_;
    bool ok = ensure<int32_t>(d_cloud_of_, L) && ensure<double>(d_in_, 3 * L) && ensure<double>(d_xyz64_, 3 * L) &&
              ensure<float>(d_xyz32_, 3 * L) && ensure<double>(d_fr64_, 12 * L) && ensure<float>(d_fr32_, 12 * L) &&
              ensure<double>(d_nrm64_, 3 * L) && ensure<double>(d_conf64_, L) && ensure<double>(d_tgeo_, 8 * L) &&
              (!knn_list || ensure<int32_t>(d_knn_, L * kmax_)) && ensure<int32_t>(d_corr_idx_, L) && ensure<float>(d_corr_dist_, L) &&
              ensure<int32_t>(d_flag_count_, 4) &&
              ensure<uint32_t>(d_keys0_, L) &&
              ensure<int32_t>(d_vals1_, L) && ensure<unsigned long long>(d_stats_, kStatCols * kStatSlots) &&
              ensure<NNCert>(d_cert_, L) &&
              ensure<int32_t>(d_sqlist_, L);
    for (TreeBufs* t : {&t3_, &t12_})
        ok = ok && ensure<int32_t>(t->perm, L) && ensure<int32_t>(t->pos, L);
    ok = ok && ensure<float>(t3_.vec, 3 * L) && ensure<float>(t12_.vec, 12 * L);
    return ok ? 0 : SE3ICP_ERR_OUT_OF_MEMORY;
}

View Engine::view() const {
    View v{};
    v.ld = ld_;
    v.npts = (int32_t)ntot_;
    v.nclouds = nclouds_;
    v.npairs = npairs_;
    v.kmax = kmax_;
    v.clouds = (CloudDev*)d_clouds_.p;
    v.setup = (CloudSetup*)d_setup_.p;
    v.pairs = (PairDev*)d_pairs_.p;
    v.cloud_of = (int32_t*)d_cloud_of_.p;
    v.in_ptr = (const double* const*)d_inptr_.p;
    v.xyz64 = (double*)d_xyz64_.p;
    v.xyz32 = (float*)d_xyz32_.p;
    v.fr64 = (double*)d_fr64_.p;
    v.fr32 = (float*)d_fr32_.p;
    v.nrm64 = (double*)d_nrm64_.p;
    v.conf64 = (double*)d_conf64_.p;
    v.tgeo = (double*)d_tgeo_.p;
    v.knn = knn_list_ ? (int32_t*)d_knn_.p : nullptr;
    v.corr_idx = (int32_t*)d_corr_idx_.p;
    v.corr_dist = (float*)d_corr_dist_.p;
    v.stats = (unsigned long long*)d_stats_.p;
    v.flag_count = (int32_t*)d_flag_count_.p;
    v.gcost = (uint32_t*)d_gcost_.p;
    v.cls = (int32_t*)d_cls_.p;
    v.trim_key = (uint64_t*)d_trim_key_.p;
    v.trim_cand = (unsigned long long*)d_trim_cand_.p;
    v.trim_ctr = (unsigned*)d_trim_ctr_.p;
    v.trim_hist = (unsigned*)d_trim_hist_.p;
    v.red_partial = (double*)d_red_partial_.p;
    v.red_out = (double*)d_red_out_.p;
    v.work = (const BlockWork*)d_work_.p;
    v.nwork = nwork_;
    v.pair_rechecked = (int32_t*)d_rechecked_.p;
    auto ref = [&](const TreeBufs& t) {
        TreeRef r{};
        r.L = t.L;
        r.GL = tree_L_;
        r.nnodes = 2 << t.L;
        r.perm = (const int32_t*)t.perm.p;
        r.pos = (const int32_t*)t.pos.p;
        r.tvec = (const float*)t.vec.p;
        r.tvec64 = (const double*)t.vec64.p;
        r.tpt64 = (const double4*)t.vec64a.p;
        r.lo = (const float*)t.lo.p;
        r.hi = (const float*)t.hi.p;
        return r;
    };
    v.t3 = ref(t3_);
    v.t12 = ref(t12_);
    v.chunk_level = chunk_level_;
    v.nchunks = nchunks_;
    v.qlist = (int32_t*)d_qlist_.p;
    v.qcount = (int32_t*)d_qcount_.p;
    v.sq_list = (int32_t*)d_sqlist_.p;
    v.hist = (const double*)d_hist_.p;
    v.cert = (NNCert*)d_cert_.p;
    return v;
}

// ----------------------------------------------------------------------------- kd-trees
int Engine::build_tree(int D, const float* vec, hipStream_t s, const double* vec64) {
    TreeBufs& tb = (D == 12) ? t12_ : t3_;
    tb.L = tree_L_;
    const int nnodes = 2 << tb.L;
    const size_t nb = (size_t)nclouds_ * nnodes * D;
    if (!ensure<uint32_t>(tb.blo, nb) || !ensure<uint32_t>(tb.bhi, nb) || !ensure<float>(tb.lo, nb) ||
        !ensure<float>(tb.hi, nb) || !ensure<float>(tb.scr, (size_t)D * ld_) ||
        (D == 12 && !ensure<float>(tb.vecT, (size_t)12 * ld_)) ||
        (vec64 && !ensure<double>(tb.vec64, (size_t)3 * ld_)) ||
        (vec64 && D == 3 && !ensure<double4>(tb.vec64a, (size_t)ld_)))
        return SE3ICP_ERR_OUT_OF_MEMORY;
    std::vector<int32_t> host_n(nclouds_);
    int max_n = 0;
    for (int c = 0; c < nclouds_; ++c) max_n = std::max(max_n, host_n[c] = h_clouds_[c].n);
    const size_t need = tree_build_temp_bytes((int)ntot_, nclouds_, max_n, tb.L);
    if (!ensure<char>(d_sort_tmp_, std::max<size_t>(need, 256))) return SE3ICP_ERR_OUT_OF_MEMORY;
    TreeView t{};
    t.host_n = host_n.data();
    t.D = D;
    t.L = tb.L;
    t.nnodes = nnodes;
    t.nclouds = nclouds_;
    t.npts = (int32_t)ntot_;
    t.ld = ld_;
    t.clouds = (const CloudDev*)d_clouds_.p;
    t.cloud_of = (const int32_t*)d_cloud_of_.p;
    t.vec = vec;
    t.vecT = (D == 12) ? (float*)tb.vecT.p : const_cast<float*>(vec);  // (3-D: the input is columns)
    t.perm = (int32_t*)tb.perm.p;
    t.pos = (int32_t*)tb.pos.p;
    t.tvec = (float*)tb.vec.p;
    t.vec64 = vec64;
    t.tvec64 = vec64 ? (double*)tb.vec64.p : nullptr;
    t.tpt64 = (vec64 && D == 3) ? (double4*)tb.vec64a.p : nullptr;
    t.vec64_sources_only = D == 12;  // the loop reads f64 12-D vectors of source clouds (even ids) only
    t.blo = (uint32_t*)tb.blo.p;
    t.bhi = (uint32_t*)tb.bhi.p;
    t.scr = (float*)tb.scr.p;
    t.lo = (float*)tb.lo.p;
    t.hi = (float*)tb.hi.p;
    if (build_trees(t, d_sort_tmp_.p, d_sort_tmp_.bytes, (uint32_t*)d_keys0_.p, (int32_t*)d_vals1_.p, s) != 0)
        return SE3ICP_ERR_HIP;
    return 0;
}

// ----------------------------------------------------------------------------- setup
int Engine::setup_clouds(std::vector<CloudReq>& clouds, bool on_device, bool normalize_pairs, double scale_pre,
                         bool build12, std::vector<double>* centers_out, std::vector<double>* scales_out,
                         hipStream_t s) {
    nclouds_ = (int)clouds.size();
    h_clouds_.assign(nclouds_, CloudDev{});
    h_setup_.resize(nclouds_);
    h_chunks_.clear();
    h_inptr_.assign(nclouds_, nullptr);
    int64_t off = 0;
    int max_n = 1;
    for (int c = 0; c < nclouds_; ++c) {
        h_clouds_[c].off = (int32_t)off;
        h_clouds_[c].n = (int32_t)clouds[c].n;
        h_setup_[c] = clouds[c].st;
        max_n = std::max<int>(max_n, (int)clouds[c].n);
        for (int64_t p0 = 0; p0 < clouds[c].n; p0 += kChunk) h_chunks_.push_back(ChunkWork{c, (int32_t)p0});
        off += clouds[c].n;
    }
    tree_L_ = tree_depth_for(max_n);
    // inputs
    double* d_in = (double*)d_in_.p;
    for (int c = 0; c < nclouds_; ++c) {
        if (on_device) {
            h_inptr_[c] = clouds[c].in;
        } else {
            double* dst = d_in + 3 * (size_t)h_clouds_[c].off;
            HIPCHK(hipMemcpyAsync(dst, clouds[c].in, sizeof(double) * 3 * clouds[c].n, hipMemcpyHostToDevice, s));
            h_inptr_[c] = dst;
        }
    }
    const int nch = (int)h_chunks_.size();
    if (!ensure<CloudDev>(d_clouds_, nclouds_) || !ensure<CloudSetup>(d_setup_, nclouds_) ||
        !ensure<ChunkWork>(d_chunks_, nch) || !ensure<const double*>(d_inptr_, nclouds_) ||
        !ensure<double>(d_partial_, (size_t)nch * 9) || !ensure<double>(d_centers_, 3 * (size_t)nclouds_))
        return SE3ICP_ERR_OUT_OF_MEMORY;
    if (pinned(h_partial_, h_partial_cap_, (size_t)nch * 9 + 8)) return SE3ICP_ERR_OUT_OF_MEMORY;
    HIPCHK(hipMemcpyAsync(d_clouds_.p, h_clouds_.data(), sizeof(CloudDev) * nclouds_, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_setup_.p, h_setup_.data(), sizeof(CloudSetup) * nclouds_, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_chunks_.p, h_chunks_.data(), sizeof(ChunkWork) * nch, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_inptr_.p, h_inptr_.data(), sizeof(double*) * nclouds_, hipMemcpyHostToDevice, s));
    View v = view();

    // 1) ingest: SoA copy + sums + bbox
    launch_ingest(v, (const ChunkWork*)d_chunks_.p, nch, (double*)d_partial_.p, s);
    HIPCHK(hipGetLastError());
    if (normalize_pairs) {
        // 2) normalization parameters (ISR.cpp:568-574) on the device: no host round trip;
        // the centers (d_centers_) and scales (d_scales_) stay there for the loop and the
        // final de-normalization
        if (!ensure<double>(d_scales_, std::max(1, nclouds_ / 2))) return SE3ICP_ERR_OUT_OF_MEMORY;
        launch_pair_centers(v, (const ChunkWork*)d_chunks_.p, nch, (const double*)d_partial_.p, (double*)d_centers_.p,
                            s);
        launch_radius(v, (const ChunkWork*)d_chunks_.p, nch, (const double*)d_centers_.p, (double*)d_partial_.p, s);
        launch_pair_scales(v, (const ChunkWork*)d_chunks_.p, nch, (const double*)d_partial_.p,
                           (const double*)d_centers_.p, scale_pre, (double*)d_scales_.p, s);
        HIPCHK(hipGetLastError());
        for (int c = 0; c < nclouds_; ++c)  // (the device holds the normalization fields)
            for (int a = 0; a < 3; ++a) h_setup_[c].f32_center[a] = 0.0;
    } else {
        HIPCHK(hipMemcpyAsync(h_partial_, d_partial_.p, sizeof(double) * 9 * nch, hipMemcpyDeviceToHost, s));
        SYNC_STREAM(s);
        std::vector<double> cen(3 * nclouds_, 0.0);
        {
            std::vector<double> sum(3 * nclouds_, 0.0);
            for (int k = 0; k < nch; ++k) {
                const int c = h_chunks_[k].cloud;
                for (int a = 0; a < 3; ++a) sum[3 * c + a] += h_partial_[9 * k + a];
            }
            for (int c = 0; c < nclouds_; ++c)
                for (int a = 0; a < 3; ++a)
                    cen[3 * c + a] = clouds[c].n > 0 ? sum[3 * c + a] / (double)clouds[c].n : 0.0;
        }
        if (centers_out) *centers_out = cen;
        for (int c = 0; c < nclouds_; ++c) {
            // raw coordinates; f32 copies centered on the target (pairs) / own centroid (single clouds)
            const int cc = (nclouds_ % 2 == 0 && npairs_ > 0) ? (c | 1) : c;
            for (int a = 0; a < 3; ++a) {
                h_setup_[c].norm_center[a] = 0.0;
                h_setup_[c].f32_center[a] = cen[3 * cc + a];
            }
            h_setup_[c].norm_scale = 1.0;
        }
        HIPCHK(hipMemcpyAsync(d_setup_.p, h_setup_.data(), sizeof(CloudSetup) * nclouds_, hipMemcpyHostToDevice, s));
    }

    // 3) normalize in place + f32 copy
    launch_normalize(v, (const ChunkWork*)d_chunks_.p, nch, (double*)d_partial_.p, s);
    HIPCHK(hipGetLastError());

    // 4) 3-D kd-trees of every cloud (kNN for TOLDI / normals, and the R3 NN of the loop)
    int rc = build_tree(3, (const float*)d_xyz32_.p, s, (const double*)d_xyz64_.p);
    if (rc) return rc;
    v = view();
    bool any_knn = false;
    for (int c = 0; c < nclouds_; ++c) any_knn |= h_setup_[c].k_knn > 0;
    if (any_knn) {
        HIPCHK(hipMemsetAsync(d_stats_.p, 0, sizeof(unsigned long long) * kStatCols * kStatSlots, s));
        HIPCHK(hipEventRecord(ev_[6], s));
        // neighbourhoods over kSmallK (Kw = min(k, n)) go to k_knn_big, the rest to the LDS
        // kernels; the global-buffer kernel's candidate buffers are sized to the largest
        int kw_big = 0, n_big = 0;
        for (int c = 0; c < nclouds_; ++c) {
            const int kw = std::min<int>(h_setup_[c].k_knn, h_clouds_[c].n);
            if (kw > kSmallK || lrf_exact_only_ == 2) {
                kw_big = std::max(kw_big, kw);
                n_big += h_clouds_[c].n;
            }
        }
        int big_cap = 0, big_blocks = 0;
        if (n_big > 0) {
            big_cap = knn_big_cap(kw_big);
            big_blocks = knn_big_blocks(big_cap, n_big);
            if (!ensure<double>(d_big_d_, (size_t)big_blocks * big_cap) || !ensure<int32_t>(d_big_i_, (size_t)big_blocks * big_cap))
                return SE3ICP_ERR_OUT_OF_MEMORY;
        }
        auto big = [&](const int32_t* qlist, const int32_t* qcount, int k_min) {
            if (n_big > 0)
                launch_knn_big(v, knn_list_ ? 1 : 0, k_min, qlist, qcount, big_blocks, (double*)d_big_d_.p,
                               (int32_t*)d_big_i_.p, big_cap, s);
        };
        if (lrf_exact_only_ == 2) {
            big(nullptr, nullptr, 0);  // (diagnostic: every query through the global-buffer kernel)
        } else if (knn_list_ || lrf_exact_only_ == 1) {
            launch_lrf(v, knn_list_ ? 1 : 0, s);  // the sorted lists (se3icp_knn_self) need the exact kernel
            big(nullptr, nullptr, kSmallK);
        } else {
            // eight queries per wavefront; the few it cannot resolve from f32 keys (and every
            // query of a cloud whose k it cannot hold) go to the exact kernels
            // waves aligned to each cloud's first point (results independent of the batch)
            std::vector<int32_t> wb(nclouds_ + 1, 0);
            for (int c = 0; c < nclouds_; ++c) wb[c + 1] = wb[c] + (h_clouds_[c].n + 7) / 8;
            const int nw = wb[nclouds_];
            if (!ensure<int32_t>(d_lrf_fb_, (size_t)8 * nw + 64) || !ensure<int32_t>(d_lrf_fbn_, 2 + nclouds_ + 1))
                return SE3ICP_ERR_OUT_OF_MEMORY;
            int32_t* d_wb = (int32_t*)d_lrf_fbn_.p + 2;
            int32_t* fb = (int32_t*)d_lrf_fb_.p;
            int32_t* fbn = (int32_t*)d_lrf_fbn_.p;
            HIPCHK(hipMemsetAsync(fbn, 0, 2 * sizeof(int32_t), s));
            HIPCHK(hipMemcpyAsync(d_wb, wb.data(), sizeof(int32_t) * (nclouds_ + 1), hipMemcpyHostToDevice, s));
            launch_lrf8(v, d_wb, 0, nw, fb, fbn, s);
            launch_lrf_list(v, fb, fbn, s);
            big(fb, fbn, kSmallK);
        }
        HIPCHK(hipEventRecord(ev_[7], s));
        HIPCHK(hipGetLastError());
        // work counters: copied now, read at the next synchronisation (read_lrf_stats)
        if (pinned(h_lrf_stats_, h_lrf_stats_cap_, (size_t)kStatCols * kStatSlots)) return SE3ICP_ERR_OUT_OF_MEMORY;
        HIPCHK(hipMemcpyAsync(h_lrf_stats_, d_stats_.p, sizeof(unsigned long long) * kStatCols * kStatSlots,
                              hipMemcpyDeviceToHost, s));
        lrf_stats_pending_ = true;
    }
    HIPCHK(hipGetLastError());
    // 5) 12-D kd-trees over the alpha/beta-weighted SE(3) elements
    have12_ = build12;
    if (build12) {
        rc = build_tree(12, (const float*)d_fr32_.p, s, (const double*)d_fr64_.p);  // f64 source elements in tree order
        if (rc) return rc;
    }
    return 0;
}

// k_lrf time and work counters of the last setup (after the stream has passed them)
int Engine::read_lrf_stats() {
    if (!lrf_stats_pending_) return 0;
    lrf_stats_pending_ = false;
    double sum[kStatCols] = {};
    for (int i = 0; i < kStatSlots; ++i)
        for (int k = 0; k < kStatCols; ++k) sum[k] += (double)h_lrf_stats_[kStatCols * i + k];
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, ev_[6], ev_[7]));
    ktimes_.lrf_ms = ms;
    ktimes_.lrf_queries = sum[0];
    ktimes_.lrf_leaves = sum[1];
    ktimes_.lrf_merges = sum[2];
    ktimes_.lrf_box_tests = sum[3];
    ktimes_.lrf_candidates = sum[4];
    ktimes_.lrf_fallback = sum[6];
#ifdef SE3ICP_PROF
    tree_prof_report();
    std::fprintf(stderr, "[prof] k_lrf cycles/query: knn|scan %.0f sort|tighten %.0f sums|final+sums %.0f finish %.0f "
                 "(queries %.0f, wave cycles summed over the kernel's waves)\n",
                 sum[8] / sum[0], sum[9] / sum[0], sum[10] / sum[0], sum[11] / sum[0], sum[0]);
    std::fprintf(stderr, "[prof] k_lrf8 per query: tightenings %.3f (overflow %.3f, final %.3f), leaf scans %.3f\n",
                 sum[2] / sum[0], sum[3] / sum[0], sum[7] / sum[0], sum[1] / sum[0]);
    {
        unsigned long long f = 0;  // (16-bit fields, summed as integers)
        for (int i = 0; i < kStatSlots; ++i) f += h_lrf_stats_[kStatCols * i + 5];
        std::fprintf(stderr, "[prof] k_lrf8 hand-overs: waves with the leaf table full %llu, no room %llu, > 128 at the end %llu; "
                     "queries with f32-equal f64-distinct ranks %llu\n",
                     f & 0xffff, (f >> 16) & 0xffff, (f >> 32) & 0xffff, f >> 48);
    }
#endif
    return 0;
}

// Wait for everything queued on `s` (polling, see spin_wait).
int Engine::sync_stream(hipStream_t s) {
    HIPCHK(hipEventRecord(ev_[15], s));
    HIPCHK(spin_wait(ev_[15]));
    return read_lrf_stats();
}

// loop NN work chunks: nodes of level tree_L_ - 4 of every source tree (<= kChunkQ
// positions each), their query lists, the pose history and void NN certificates
int Engine::setup_chunks(int npairs, hipStream_t s) {
    chunk_level_ = std::max(0, tree_L_ - 4);
    nchunks_ = npairs << chunk_level_;
    if (!ensure<int32_t>(d_qlist_, (size_t)nchunks_ * kChunkQ) || !ensure<int32_t>(d_qcount_, (size_t)nchunks_ * (kChunkQ / 64)) ||
        !ensure<double>(d_hist_, (size_t)kHist * npairs * 12) || !ensure<uint32_t>(d_gcost_, (size_t)nchunks_ * 16) ||
        !ensure<int32_t>(d_cls_, nn_cls_words(nchunks_)))
        return SE3ICP_ERR_OUT_OF_MEMORY;
    if (pinned(h_hist_, h_hist_cap_, (size_t)npairs * 12)) return SE3ICP_ERR_OUT_OF_MEMORY;
    HIPCHK(hipMemsetAsync(d_cert_.p, 0xff, sizeof(NNCert) * ld_, s));  // iteration -1: no certificate
    HIPCHK(hipMemsetAsync(d_gcost_.p, 0, sizeof(uint32_t) * nchunks_ * 16, s));
    HIPCHK(hipMemsetAsync(d_cls_.p, 0, sizeof(int32_t) * 2 * 8 * 16, s));
    return 0;
}

// ----------------------------------------------------------------------------- batch registration
int Engine::register_batch(int npairs, const double* const* src, const int64_t* ns, const double* const* tgt,
                           const int64_t* nt, bool on_device, int method, const se3icp_params& prm,
                           se3icp_result* out, hipStream_t user_stream) {
    if (!ok_) return SE3ICP_ERR_NO_DEVICE;
    se3icp_trace* tr = trace_;  // one-shot: the record covers this batch only
    trace_ = nullptr;
    if (npairs <= 0 || !src || !tgt || !ns || !nt || !out) return SE3ICP_ERR_INVALID_ARG;
    if (tr && (tr->pair < 0 || tr->pair >= npairs || tr->max_iters < 0)) return SE3ICP_ERR_INVALID_ARG;
    if (tr) tr->iters_recorded = 0;
    MethodInfo mi;
    if (!decode_method(method, &mi)) return SE3ICP_ERR_INVALID_METHOD;
    for (int p = 0; p < npairs; ++p) {
        if (ns[p] <= 0 || nt[p] <= 0) return SE3ICP_ERR_EMPTY_CLOUD;
        if (!src[p] || !tgt[p]) return SE3ICP_ERR_INVALID_ARG;
    }
    const bool se3 = mi.kind != KIND_ICP;
    const int k_lrf = se3 ? prm.number_of_nn_for_LRF : 0;
    if (se3 && k_lrf <= 0) return SE3ICP_ERR_INVALID_ARG;
    int k_nrm_s = 0, k_nrm_t = 0;
    if (mi.est == EST_PT2PL) k_nrm_t = 30;                    // target_.EstimateNormals() default KNN(30)
    if (mi.est == EST_GICP) { k_nrm_s = 20; k_nrm_t = 20; }   // InitializePointCloudForGeneralizedICP KNN(20)
    const int kmax = std::max({k_lrf, k_nrm_s, k_nrm_t, 1});
    HIPCHK(hipSetDevice(dev_));
    hipStream_t s = user_stream ? user_stream : stream_;
    ktimes_ = KernelTimes{};
    // phase times on the GPU timeline (the host does not wait for the setup): events
    // 12 (begin), 13 (setup done), 14 (loop done)
    HIPCHK(hipEventRecord(ev_[12], s));

    npairs_ = npairs;
    int64_t ntot = 0;
    for (int p = 0; p < npairs; ++p) ntot += ns[p] + nt[p];
    // work table of k_reduce: one entry per kRedQ queries of every pair
    int64_t soff = 0;
    h_work_.clear();
    h_wb_.assign(npairs, 0);
    h_wn_.assign(npairs, 0);
    for (int p = 0; p < npairs; ++p) {
        h_wb_[p] = (int32_t)h_work_.size();
        // (clouds are laid out src 0, tgt 0, src 1, ... as setup_clouds places them)
        for (int64_t q0 = 0; q0 < ns[p]; q0 += kRedQ)
            h_work_.push_back(BlockWork{p, (int32_t)q0, (int32_t)std::min<int64_t>(q0 + kRedQ, ns[p]), (int32_t)soff,
                                        (int32_t)(soff + ns[p]), {0, 0, 0}});
        soff += ns[p] + nt[p];
        h_wn_[p] = (int32_t)h_work_.size() - h_wb_[p];
    }
    nwork_ = (int)h_work_.size();
    int rc = alloc_points(ntot, kmax);
    if (rc) return rc;
    if (!ensure<PairDev>(d_pairs_, npairs) || !ensure<BlockWork>(d_work_, nwork_) || !ensure<int32_t>(d_wb_, npairs) ||
        !ensure<int32_t>(d_wn_, npairs) || !ensure<uint64_t>(d_trim_key_, 2 * (size_t)npairs) ||
        !ensure<unsigned long long>(d_trim_cand_, (size_t)npairs * kTrimList) || !ensure<unsigned>(d_trim_ctr_, 4 * (size_t)npairs) ||
        !ensure<unsigned>(d_trim_hist_, 4096 * (size_t)npairs) ||
        !ensure<double>(d_red_partial_, (size_t)nwork_ * kRedVals) || !ensure<double>(d_red_out_, (size_t)npairs * kRedVals) ||
        !ensure<int32_t>(d_rechecked_, npairs))
        return SE3ICP_ERR_OUT_OF_MEMORY;
    if (pinned(h_pairs_, h_pairs_cap_, npairs) || pinned(h_red_, h_red_cap_, (size_t)npairs * kRedVals) ||
        pinned(h_rechecked_, h_rechecked_cap_, npairs))
        return SE3ICP_ERR_OUT_OF_MEMORY;
    HIPCHK(hipMemcpyAsync(d_work_.p, h_work_.data(), sizeof(BlockWork) * nwork_, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_wb_.p, h_wb_.data(), sizeof(int32_t) * npairs, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_wn_.p, h_wn_.data(), sizeof(int32_t) * npairs, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(d_rechecked_.p, 0, sizeof(int32_t) * npairs, s));

    // ---- setup (ISR.cpp:568-648)
    std::vector<CloudReq> clouds(2 * npairs);
    for (int p = 0; p < npairs; ++p) {
        for (int side = 0; side < 2; ++side) {
            CloudReq& r = clouds[2 * p + side];
            r.in = side == 0 ? src[p] : tgt[p];
            r.n = side == 0 ? ns[p] : nt[p];
            CloudSetup& st = r.st;
            st = CloudSetup{};
            st.k_lrf = k_lrf;
            st.k_nrm = side == 0 ? k_nrm_s : k_nrm_t;
            st.k_knn = std::max(st.k_lrf, st.k_nrm);
            st.want_cov = mi.est == EST_GICP;
            st.want_conf = mi.kind == KIND_CF;
            st.is_target = side == 1;
            st.cf_target = (mi.kind == KIND_CF && side == 1);
            st.alpha = prm.alpha_rot;
            st.beta = prm.beta_transl;
            st.norm_scale = 1.0;
        }
    }
    std::vector<double> centers;  // run_icp only (run_se3_*: normalization parameters on the device)
    rc = setup_clouds(clouds, on_device, se3, prm.scale_preprocessing, se3, &centers, nullptr, s);
    if (rc) return rc;
    rc = setup_chunks(npairs, s);
    if (rc) return rc;
    HIPCHK(hipMemsetAsync(d_corr_idx_.p, 0xff, sizeof(int32_t) * ld_, s));  // no previous match yet
    HIPCHK(hipMemsetAsync(d_stats_.p, 0, sizeof(unsigned long long) * kStatCols * kStatSlots, s));
    for (double& t : trace_prev_) t = 0;
    HIPCHK(hipEventRecord(ev_[13], s));

    // ---- per-pair loop state (ISR.cpp:629-651); iteration 1 is opened here, every later
    // one by k_reduce_final on the device (pairmath.hpp), so the host only queues work
    if (!ensure<PairState>(d_state_, npairs) || pinned(h_state_, h_state_cap_, npairs))
        return SE3ICP_ERR_OUT_OF_MEMORY;
    if (h_phase_cap_ < (size_t)npairs * kLoopRing) {  // coherent host memory the device writes directly
        if (h_phase_) (void)hipHostFree(h_phase_);
        h_phase_ = nullptr;
        h_phase_cap_ = 0;
        const size_t want = std::max<size_t>((size_t)npairs * kLoopRing, 64);
        if (hipHostMalloc((void**)&h_phase_, want * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent) !=
                hipSuccess ||
            hipHostGetDevicePointer((void**)&d_phase_, h_phase_, 0) != hipSuccess)
            return SE3ICP_ERR_OUT_OF_MEMORY;
        h_phase_cap_ = want;
    }
    const float ratio = std::min(1.0f, std::max(0.0f, (float)prm.estimated_overlap));  // PCL setOverlapRatio(float)
    int n_se3 = 0, n_r3 = 0;
    bool any_trim = false;
    for (int p = 0; p < npairs; ++p) {
        PairState& S = h_state_[p];
        std::memset(&S, 0, sizeof(S));
        S.T = M4::eye();
        S.mse_prev = S.mse_cur = S.rel = 1e7;
        S.sf = 1.0;  // run_se3_*: the device's scale, written by k_pair_norms
        S.mse = prm.mse;
        S.mse_switch = prm.mse_switch_error;
        S.kind = mi.kind;
        S.max_iter = prm.max_num_iterations;
        S.max_se3 = prm.max_num_se3_iterations;
        S.phase = PHASE_IDLE;
        S.phase_start = 1;
        const unsigned nv = (unsigned)std::floor(ratio * (float)ns[p]);
        const bool trim = (int64_t)nv < ns[p];
        S.K = trim ? (double)nv : (double)ns[p];
        PairDev& P = h_pairs_[p];
        std::memset(&P, 0, sizeof(P));
        P.src = 2 * p;
        P.tgt = 2 * p + 1;
        P.est = mi.est;
        P.cf = mi.kind == KIND_CF;
        P.trim = trim;
        P.nkeep = (int)nv;
        for (int a = 0; a < 3; ++a) P.f32_center[a] = h_setup_[2 * p].f32_center[a];
        pair_open_iteration(S, P);
        std::memcpy(h_hist_ + 12 * (size_t)p, P.T, sizeof(P.T));
        n_se3 += P.phase == PHASE_SE3;
        n_r3 += P.phase == PHASE_R3;
        any_trim |= trim;
    }
    HIPCHK(hipMemcpyAsync(d_pairs_.p, h_pairs_, sizeof(PairDev) * npairs, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_state_.p, h_state_, sizeof(PairState) * npairs, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync((double*)d_hist_.p + (size_t)(1 % kHist) * npairs * 12, h_hist_, sizeof(double) * 12 * npairs,
                          hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(d_flag_count_.p, 0, 3 * sizeof(int32_t), s));
    // norm bounds of the target search vectors (f32 error certificate) from the root
    // boxes, and the normalization scales into the loop state
    launch_pair_norms(view(), 2 << t3_.L, se3 ? 2 << t12_.L : 0, se3 ? (const double*)d_scales_.p : nullptr,
                      (double*)((char*)d_state_.p + offsetof(PairState, sf)), (int)(sizeof(PairState) / sizeof(double)),
                      s);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemsetAsync((uint64_t*)d_trim_key_.p + npairs, 0, sizeof(uint64_t) * npairs, s));  // no trim window yet
    HIPCHK(hipMemsetAsync(d_trim_ctr_.p, 0, sizeof(unsigned) * 4 * npairs, s));
    launch_geo_rows(view(), s);  // (after the setup's normals and confidences)
    HIPCHK(hipMemsetAsync(d_trim_hist_.p, 0, sizeof(unsigned) * 4096 * npairs, s));
    View v = view();
    double nn_ms = 0;
    // Iteration `it` is queued while iteration it-1 still runs; the host then waits for
    // it-1 and reads how many pairs iteration it has (counted by it-1's k_reduce_final).
    // Zero means iteration `it` is empty and the loop is over.  NN grids of a phase are
    // queued while any pair may be in it: SE(3) until a finished iteration shows none
    // left, R3 from iteration 2 on (a pair may switch after any iteration).
    // SE3ICP_NN_TRACE waits for every iteration (per-iteration work counters).
    const int lag = (nn_trace_ || tr) ? 0 : 1;
    int trace_phase = tr ? h_pairs_[tr->pair].phase : 0;  // phase of the iteration being recorded
    auto enqueue = [&](int it) -> int {
        hipEvent_t* ev = &loop_ev_[(it % kLoopRing) * kLoopEv];
        // the ring slot k_reduce_final of this iteration fills (its last reader, iteration
        // it - kLoopRing, is finished): unwritten until then (spin_phases)
        for (int p = 0; p < npairs; ++p) h_phase_[(size_t)(it % kLoopRing) * npairs + p] = -1;
        // SE(3) phase: iterations 1..max_num_se3_iterations at most (ISR.cpp:718-723, 1118)
        const bool do_se3 =
            n_se3 > 0 && (prm.max_num_se3_iterations < 1 || it <= prm.max_num_se3_iterations);
        const bool do_r3 = n_r3 > 0 || (mi.kind != KIND_ICP && mi.kind != KIND_PURE && it >= 2);
        // HIP events around the NN grids always (bench.py's roofline); around every other
        // stage only when profiling (each marker costs the stream a few microseconds)
        const bool detail = profile_ || nn_trace_;
        // (timed steps: the SE(3) NN bracket only when that grid is queued, plus the
        // iteration's end marker; profiled steps: every stage)
        const bool t_se3 = detail || (do_se3 && nn_events_);
        if (detail) HIPCHK(hipEventRecord(ev[0], s));
        // the phases of iteration it (opened by it-1's k_reduce_final) reach the host through
        // this k_nn_prep (ring slot it-1); without look-ahead, k_reduce_final writes them
        launch_nn_prep(v, (lag == 1 && it >= 2) ? d_phase_ + (size_t)((it - 1) % kLoopRing) * npairs : nullptr, s);
        // One search grid per phase (single-query waves and groups together, k_nn.hip): no
        // second stream and no cross-stream events.  ev[1] / ev[2] bracket the SE(3) search.
        if (t_se3) HIPCHK(hipEventRecord(ev[1], s));
        if (do_se3) launch_nn(v, 12, s);
        if (t_se3) HIPCHK(hipEventRecord(ev[2], s));
        if (do_r3) launch_nn(v, 3, s);
        if (detail) HIPCHK(hipEventRecord(ev[3], s));
        // (no recheck stage: the NN grids re-resolve their uncertified queries inline; the
        // ev[3] -> ev[4] bracket stays empty and time_recheck reads ~0)
        if (detail) HIPCHK(hipEventRecord(ev[4], s));
        if (any_trim) launch_trim(v, s);
        if (detail) HIPCHK(hipEventRecord(ev[5], s));
        launch_reduce(v, (const int32_t*)d_wb_.p, (const int32_t*)d_wn_.p, (PairState*)d_state_.p, (double*)d_hist_.p,
                      lag == 0 ? d_phase_ + (size_t)(it % kLoopRing) * npairs : nullptr, s);
        HIPCHK(hipGetLastError());
        if (detail) HIPCHK(hipEventRecord(ev[6], s));
        loop_detail_[it % kLoopRing] = detail;
        loop_flags_[it % kLoopRing] = (do_se3 ? 1 : 0) | (do_r3 ? 2 : 0) | (t_se3 ? 4 : 0);
        return 0;
    };
    // wait for iteration `it`, add its kernel times; returns the pairs of iteration it+1
    // (last: the loop's final, empty, iteration -- no k_nn_prep follows to publish its slot)
    auto finish = [&](int it, bool last) -> int {
        hipEvent_t* ev = &loop_ev_[(it % kLoopRing) * kLoopEv];
        // (the phase slot of iteration it is written by the next iteration's k_nn_prep, queued
        // already, or with lag 0 by this iteration's k_reduce_final -- after its end event)
        if (loop_detail_[it % kLoopRing]) HIPCHK(spin_wait(ev[6]));
        if (last && lag == 1) {
            if (!loop_detail_[it % kLoopRing]) {
                HIPCHK(hipEventRecord(ev_[15], s));
                HIPCHK(spin_wait(ev_[15]));
            }
        } else {
            HIPCHK(spin_phases(h_phase_ + (size_t)(it % kLoopRing) * npairs, npairs, s));
        }
        float ms[6] = {};
        if (loop_detail_[it % kLoopRing]) {
            for (int k = 0; k < 6; ++k) HIPCHK(hipEventElapsedTime(&ms[k], ev[k], ev[k + 1]));
        } else if (loop_flags_[it % kLoopRing] & 4) {
            HIPCHK(hipEventElapsedTime(&ms[1], ev[1], ev[2]));
        }
        ktimes_.nn_prep_ms += ms[0];
        ktimes_.nn_se3_ms += ms[1];
        ktimes_.nn_r3_ms += ms[2];
        ktimes_.recheck_ms += ms[3];
        ktimes_.trim_ms += ms[4];
        ktimes_.reduce_ms += ms[5];
        nn_ms += ms[0] + ms[1] + ms[2] + ms[3];
        const int flags = loop_flags_[it % kLoopRing];
        if (flags & 1) ktimes_.nn_se3_launches++;
        if (flags & 2) ktimes_.nn_r3_launches++;
        if (nn_trace_) {  // per-iteration NN work (diagnostics): diffs of the device counters
            unsigned long long stats[kStatCols * kStatSlots];
            HIPCHK(hipMemcpy(stats, d_stats_.p, sizeof(stats), hipMemcpyDeviceToHost));
            double sum[kStatCols] = {};
            for (int i = 0; i < kStatSlots; ++i)
                for (int k = 0; k < kStatCols; ++k) sum[k] += (double)stats[kStatCols * i + k];
            std::fprintf(stderr,
                         "[nn] iter %d: se3 %.0f/%.0f searched, evals %.3g boxes %.3g | r3 %.0f/%.0f, evals %.3g "
                         "boxes %.3g | prep %.3f nn12 %.3f nn3 %.3f recheck %.3f ms\n",
                         it, sum[5] - trace_prev_[5], sum[4] - trace_prev_[4], sum[0] - trace_prev_[0],
                         sum[1] - trace_prev_[1], sum[7] - trace_prev_[7], sum[6] - trace_prev_[6],
                         sum[2] - trace_prev_[2], sum[3] - trace_prev_[3], ms[0], ms[1], ms[2], ms[3]);
#ifdef SE3ICP_PROF
            {
                // this iteration's SE(3) group waves: count and summed duration (column 11:
                // (1 << 44) + dt per wave, 100 MHz clock), shader cycles in leaf visits (12),
                // in their target loads (14) and in the whole wave (13)
                double d[kStatCols];
                for (int k = 0; k < kStatCols; ++k) d[k] = sum[k] - trace_prev_[k];
                const double nw = std::floor(d[11] / 17592186044416.0), dt = d[11] - nw * 17592186044416.0;
                std::fprintf(stderr, "[nn] iter %d: %.0f SE(3) group waves, mean %.1f us, summed %.1f ms (100 MHz clock)\n",
                             it, nw, nw > 0 ? dt / nw / 100.0 : 0.0, dt / 1e5);
                std::fprintf(stderr, "[nn] iter %d: k_nn_prep span %.1f us\n", it, nn_prep_span());
                nn_wave_report(it);
                std::fprintf(stderr, "[nn] iter %d: wave cycles in leaf visits %.1f %% (target loads %.1f %%), "
                             "%.0f cycles per leaf visit, %.0f per box-test step\n", it, 100.0 * d[12] / std::max(1.0, d[13]),
                             100.0 * d[14] / std::max(1.0, d[13]), d[12] / std::max(1.0, d[9]),
                             (d[13] - d[12]) / std::max(1.0, d[1] / 128.0));
            }
#endif
            for (int k = 0; k < kStatCols; ++k) trace_prev_[k] = sum[k];
#ifdef SE3ICP_PROF
            std::fprintf(stderr, "[nn] iter %d: longest SE(3) group wave %.1f us (%llu box-test steps, %llu leaf visits, "
                         "%llu queries)\n", it, (double)(stats[10] >> 40) / 100.0, (stats[10] >> 20) & 0xfffffull,
                         (stats[10] >> 6) & 0x3fffull, stats[10] & 63ull);
            HIPCHK(hipMemset((unsigned long long*)d_stats_.p + 10, 0, sizeof(unsigned long long)));
#endif
        }
        if (last && lag == 1) return 0;
        const volatile int32_t* ph = h_phase_ + (size_t)(it % kLoopRing) * npairs;
        n_se3 = n_r3 = 0;
        for (int p = 0; p < npairs; ++p) {
            const int32_t f = ph[p];
            n_se3 += f == PHASE_SE3;
            n_r3 += f == PHASE_R3;
        }
        return n_se3 + n_r3;
    };
    static_assert(kLoopRing >= 2, "one iteration in flight while the previous one is read");
    int it = 1;
    if (enqueue(it)) return SE3ICP_ERR_HIP;
    for (;;) {
        if (lag == 0) {
            const int left = finish(it, false);
            if (tr) {
                rc = record_trace(tr, it, trace_phase, s);
                if (rc) return rc;
            }
            if (left == 0) break;
            ++it;
            if (enqueue(it)) return SE3ICP_ERR_HIP;
            continue;
        }
        ++it;
        if (enqueue(it)) return SE3ICP_ERR_HIP;  // phase flags as of iteration it-2
        if (finish(it - 1, false) == 0) {        // iteration `it` is empty
            (void)finish(it, true);
            break;
        }
    }
    HIPCHK(hipEventRecord(ev_[14], s));
    HIPCHK(hipMemcpyAsync(h_state_, d_state_.p, sizeof(PairState) * npairs, hipMemcpyDeviceToHost, s));
    if (se3)  // the device's GetCenter results, for the de-normalization (h_partial_ holds >= 9 * nclouds)
        HIPCHK(hipMemcpyAsync(h_partial_, d_centers_.p, sizeof(double) * 3 * nclouds_, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(h_rechecked_, d_rechecked_.p, sizeof(int32_t) * npairs, hipMemcpyDeviceToHost, s));
    {
        if (pinned(h_loop_stats_, h_loop_stats_cap_, (size_t)kStatCols * kStatSlots)) return SE3ICP_ERR_OUT_OF_MEMORY;
        const unsigned long long* stats = h_loop_stats_;
        HIPCHK(hipMemcpyAsync(h_loop_stats_, d_stats_.p, sizeof(unsigned long long) * kStatCols * kStatSlots,
                              hipMemcpyDeviceToHost, s));
        SYNC_STREAM(s);
        double sum[kStatCols] = {};
        for (int i = 0; i < kStatSlots; ++i)
            for (int k = 0; k < kStatCols; ++k) sum[k] += (double)stats[kStatCols * i + k];
        ktimes_.se3_dist_evals = sum[0];
        ktimes_.se3_box_tests = sum[1];
        ktimes_.r3_dist_evals = sum[2];
        ktimes_.r3_box_tests = sum[3];
        ktimes_.se3_queries = sum[4];
        ktimes_.se3_searched = sum[5];
        ktimes_.r3_queries = sum[6];
        ktimes_.r3_searched = sum[7];
        ktimes_.se3_useful_evals = sum[kStatUseSe3];
        ktimes_.r3_useful_evals = sum[kStatUseR3];
#ifdef SE3ICP_PROF
        {
            const double nw = std::max(1.0, std::floor(sum[11] / 17592186044416.0));
            const double mean = std::fmod(sum[11], 17592186044416.0) / nw;  // 100 MHz ticks
            const double sq = (double)stats[kStatCols + 10] / nw;
            nn_prof_report();
            trim_prof_report();
            std::fprintf(stderr, "[prof] nn12: leaf visits %.0f; %.0f group waves, %.1f us each on average (sd %.1f, "
                         "longest %.1f us; 100 MHz clock)\n",
                         sum[9], nw, mean / 100.0, std::sqrt(std::max(0.0, sq - mean * mean)) / 100.0,
                         (double)(stats[10] >> 40) / 100.0);
            std::fprintf(stderr, "[prof] nn12 longest wave: %llu box-test steps, %llu leaf visits, %llu queries\n",
                         (stats[10] >> 20) & 0xfffffull, (stats[10] >> 6) & 0x3fffull, stats[10] & 63ull);
        }
#endif
    }
    float setup_ms = 0, loop_ms = 0;
    HIPCHK(hipEventElapsedTime(&setup_ms, ev_[12], ev_[13]));
    HIPCHK(hipEventElapsedTime(&loop_ms, ev_[13], ev_[14]));
    ktimes_.setup_ms = setup_ms;

    int worst = 0;
    for (int p = 0; p < npairs; ++p) {
        const PairState& S = h_state_[p];
        M4 T = S.T;
        if (se3) {  // ISR.cpp:735-738 de-normalization
            const double* cs = &h_partial_[3 * (2 * p)];
            const double* ct = &h_partial_[3 * (2 * p + 1)];
            for (int r = 0; r < 3; ++r) {
                const double Rc = T.m[r][0] * cs[0] + T.m[r][1] * cs[1] + T.m[r][2] * cs[2];
                T.m[r][3] = (1.0 / S.sf) * T.m[r][3] - Rc + ct[r];
            }
        }
        se3icp_result& R = out[p];
        std::memset(&R, 0, sizeof(R));
        bool finite = true;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                R.T[i * 4 + j] = T.m[i][j];
                finite &= std::isfinite(T.m[i][j]);
            }
        R.num_iterations = S.iter;
        R.num_pure_se3_iterations = se3 ? S.pure : -1;
        R.status = finite ? SE3ICP_OK : SE3ICP_ERR_NONFINITE;
        R.num_rechecked = h_rechecked_[p];
        R.scaling_factor = S.sf;
        R.time_setup_ms = setup_ms;
        R.time_loop_ms = loop_ms;
        R.time_se3_correspondence_search_ms = nn_ms;
        R.time_before_pure_icp_ms = mi.kind == KIND_CF ? (double)setup_ms + (double)loop_ms : 0.0;
        if (R.status != SE3ICP_OK) worst = R.status;
    }
    return worst;
}

// Row it-1 of the armed trace after iteration `it` completed (the stream is idle: the
// trace runs the loop without look-ahead).  phase_of_it: the pair's phase in iteration
// it, updated to its phase in iteration it+1.
int Engine::record_trace(se3icp_trace* tr, int it, int& phase_of_it, hipStream_t s) {
    const int p = tr->pair;
    PairState S;
    HIPCHK(hipMemcpyAsync(&S, (const PairState*)d_state_.p + p, sizeof(S), hipMemcpyDeviceToHost, s));
    uint64_t cut = UINT64_MAX;
    if (h_pairs_[p].trim) HIPCHK(hipMemcpyAsync(&cut, (const uint64_t*)d_trim_key_.p + p, sizeof(cut), hipMemcpyDeviceToHost, s));
    const int phase = phase_of_it;
    const int r = it - 1;
    const bool active = phase != PHASE_IDLE && r < tr->max_iters;
    const CloudDev& cs = h_clouds_[2 * p];
    if (active) {
        if (tr->corr_idx)
            HIPCHK(hipMemcpyAsync(tr->corr_idx + (size_t)r * cs.n, (const int32_t*)d_corr_idx_.p + cs.off,
                                  sizeof(int32_t) * cs.n, hipMemcpyDeviceToHost, s));
        if (tr->corr_dist)
            HIPCHK(hipMemcpyAsync(tr->corr_dist + (size_t)r * cs.n, (const float*)d_corr_dist_.p + cs.off,
                                  sizeof(float) * cs.n, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    if (active) {
        // a pair that took part in iteration it has iter >= it (one that finished at j keeps j)
        if (S.iter < it) return SE3ICP_ERR_HIP;
        if (tr->trim_key) tr->trim_key[r] = cut;
        if (tr->T)
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 4; ++j) tr->T[(size_t)r * 16 + 4 * i + j] = S.T.m[i][j];
        if (tr->mse) tr->mse[r] = S.mse_cur;
        if (tr->phase) tr->phase[r] = phase;
        tr->iters_recorded = it;
    }
    phase_of_it = S.done ? PHASE_IDLE : S.phase;
    return 0;
}

// ----------------------------------------------------------------------------- stage entry points
int Engine::knn_self(const double* xyz, int64_t n, int k, int32_t* idx) {
    if (!ok_) return SE3ICP_ERR_NO_DEVICE;
    if (!xyz || !idx || n <= 0) return n <= 0 ? SE3ICP_ERR_EMPTY_CLOUD : SE3ICP_ERR_INVALID_ARG;
    if (k <= 0) return SE3ICP_ERR_INVALID_ARG;
    HIPCHK(hipSetDevice(dev_));
    npairs_ = 0;
    int rc = alloc_points(n, k, true);
    if (rc) return rc;
    std::vector<CloudReq> cl(1);
    cl[0].in = xyz;
    cl[0].n = n;
    cl[0].st.k_knn = k;
    cl[0].st.norm_scale = 1.0;
    rc = setup_clouds(cl, false, false, 1.0, false, nullptr, nullptr, stream_);
    if (rc) return rc;
    HIPCHK(hipMemcpy2DAsync(idx, sizeof(int32_t) * k, d_knn_.p, sizeof(int32_t) * kmax_, sizeof(int32_t) * k, n,
                            hipMemcpyDeviceToHost, stream_));
    SYNC_STREAM(stream_);
    return 0;
}

int Engine::toldi_frames(const double* xyz, int64_t n, int k, double* frames) {
    if (!ok_) return SE3ICP_ERR_NO_DEVICE;
    if (!xyz || !frames || n <= 0) return n <= 0 ? SE3ICP_ERR_EMPTY_CLOUD : SE3ICP_ERR_INVALID_ARG;
    if (k <= 0) return SE3ICP_ERR_INVALID_ARG;
    HIPCHK(hipSetDevice(dev_));
    npairs_ = 0;
    int rc = alloc_points(n, k);
    if (rc) return rc;
    std::vector<CloudReq> cl(1);
    cl[0].in = xyz;
    cl[0].n = n;
    cl[0].st.k_knn = k;
    cl[0].st.k_lrf = k;
    cl[0].st.alpha = 1.0;
    cl[0].st.beta = 1.0;
    cl[0].st.norm_scale = 1.0;
    rc = setup_clouds(cl, false, false, 1.0, false, nullptr, nullptr, stream_);
    if (rc) return rc;
    std::vector<double> fr(12 * (size_t)ld_);
    HIPCHK(hipMemcpyAsync(fr.data(), d_fr64_.p, sizeof(double) * 12 * ld_, hipMemcpyDeviceToHost, stream_));
    SYNC_STREAM(stream_);
    for (int64_t i = 0; i < n; ++i) {
        double* F = frames + 16 * i;
        // packing [R00 R10 R20 R01 R11 R21 R02 R12 R22 t0 t1 t2] -> row-major 4x4
        for (int r = 0; r < 3; ++r) {
            for (int c = 0; c < 3; ++c) F[r * 4 + c] = fr[(size_t)i * 12 + c * 3 + r];
            F[r * 4 + 3] = fr[(size_t)i * 12 + 9 + r];
        }
        F[12] = F[13] = F[14] = 0.0;
        F[15] = 1.0;
    }
    return 0;
}

int Engine::estimate_normals(const double* xyz, int64_t n, int k, double* normals) {
    if (!ok_) return SE3ICP_ERR_NO_DEVICE;
    if (!xyz || !normals || n <= 0) return n <= 0 ? SE3ICP_ERR_EMPTY_CLOUD : SE3ICP_ERR_INVALID_ARG;
    if (k <= 0) return SE3ICP_ERR_INVALID_ARG;
    HIPCHK(hipSetDevice(dev_));
    npairs_ = 0;
    int rc = alloc_points(n, k);
    if (rc) return rc;
    std::vector<CloudReq> cl(1);
    cl[0].in = xyz;
    cl[0].n = n;
    cl[0].st.k_knn = k;
    cl[0].st.k_nrm = k;
    cl[0].st.norm_scale = 1.0;
    rc = setup_clouds(cl, false, false, 1.0, false, nullptr, nullptr, stream_);
    if (rc) return rc;
    std::vector<double> nr(3 * (size_t)ld_);
    HIPCHK(hipMemcpyAsync(nr.data(), d_nrm64_.p, sizeof(double) * 3 * ld_, hipMemcpyDeviceToHost, stream_));
    SYNC_STREAM(stream_);
    for (int64_t i = 0; i < n; ++i)
        for (int a = 0; a < 3; ++a) normals[3 * i + a] = nr[(size_t)a * ld_ + i];
    return 0;
}

// Exact 1-NN of arbitrary query vectors among data vectors (3 or 12 dims): the vectors
// are placed in the source/target slots of a one-pair batch with the identity pose, the
// kd-trees are built over them, and the loop's NN kernels (with their inline f64 recheck) run once.
int Engine::nn(const double* query, int64_t nq, const double* data, int64_t nd, int dim, int32_t* idx, double* d2,
               int32_t* num_rechecked) {
    if (!ok_) return SE3ICP_ERR_NO_DEVICE;
    if (!query || !data || !idx || (dim != 3 && dim != 12)) return SE3ICP_ERR_INVALID_ARG;
    if (nq <= 0 || nd <= 0) return SE3ICP_ERR_EMPTY_CLOUD;
    HIPCHK(hipSetDevice(dev_));
    hipStream_t s = stream_;
    npairs_ = 1;
    nclouds_ = 2;
    const int64_t ntot = nq + nd;
    int rc = alloc_points(ntot, 1);
    if (rc) return rc;
    if (!ensure<PairDev>(d_pairs_, 1) || !ensure<CloudDev>(d_clouds_, 2) || !ensure<int32_t>(d_rechecked_, 1))
        return SE3ICP_ERR_OUT_OF_MEMORY;
    h_clouds_.assign(2, CloudDev{});
    h_clouds_[0].off = 0;
    h_clouds_[0].n = (int32_t)nq;
    h_clouds_[1].off = (int32_t)nq;
    h_clouds_[1].n = (int32_t)nd;
    tree_L_ = tree_depth_for((int)std::max(nq, nd));
    // SoA f64 masters + f32 copies, filled on the host (diagnostic entry point)
    const size_t L = ld_;
    std::vector<int32_t> cof(L, 0);
    for (int64_t i = nq; i < ntot; ++i) cof[i] = 1;
    double cen[3] = {0, 0, 0};
    if (dim == 3) {
        for (int64_t j = 0; j < nd; ++j)
            for (int a = 0; a < 3; ++a) cen[a] += data[3 * j + a];
        for (int a = 0; a < 3; ++a) cen[a] /= (double)nd;
    }
    std::vector<double> m64((size_t)dim * L, 0.0);
    std::vector<float> m32((size_t)dim * L, 0.f);
    double nb = 0;
    for (int64_t i = 0; i < ntot; ++i) {
        const double* row = i < nq ? query + dim * i : data + dim * (i - nq);
        double n2 = 0;
        for (int r = 0; r < dim; ++r) {  // (12-D vectors as rows, 3-D points as columns: tree_in_ix)
            const size_t at = dim == 12 ? (size_t)i * 12 + r : (size_t)r * L + i;
            m64[at] = row[r];
            const double c = dim == 3 ? row[r] - cen[r] : row[r];
            m32[at] = (float)c;
            n2 += c * c;
        }
        if (i >= nq) nb = std::max(nb, std::sqrt(n2));
    }
    double* dst64 = dim == 12 ? (double*)d_fr64_.p : (double*)d_xyz64_.p;
    float* dst32 = dim == 12 ? (float*)d_fr32_.p : (float*)d_xyz32_.p;
    HIPCHK(hipMemcpyAsync(dst64, m64.data(), sizeof(double) * m64.size(), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(dst32, m32.data(), sizeof(float) * m32.size(), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_cloud_of_.p, cof.data(), sizeof(int32_t) * L, hipMemcpyHostToDevice, s));
    HIPCHK(hipMemcpyAsync(d_clouds_.p, h_clouds_.data(), sizeof(CloudDev) * 2, hipMemcpyHostToDevice, s));
    rc = build_tree(dim, dst32, s, dst64);
    if (rc) return rc;
    rc = setup_chunks(1, s);
    if (rc) return rc;
    PairDev P;
    std::memset(&P, 0, sizeof(P));
    P.T[0] = P.T[5] = P.T[10] = 1.0;
    P.src = 0;
    P.tgt = 1;
    P.phase = dim == 12 ? PHASE_SE3 : PHASE_R3;
    P.iter = 1;
    P.phase_start = 1;
    P.tgt_norm12 = (float)(nb * (1 + 1e-6));
    P.tgt_norm3 = (float)(nb * (1 + 1e-6));
    for (int a = 0; a < 3; ++a) P.f32_center[a] = cen[a];
    HIPCHK(hipMemcpyAsync(d_pairs_.p, &P, sizeof(P), hipMemcpyHostToDevice, s));
    HIPCHK(hipMemsetAsync(d_flag_count_.p, 0, 3 * sizeof(int32_t), s));
    HIPCHK(hipMemsetAsync(d_rechecked_.p, 0, sizeof(int32_t), s));
    HIPCHK(hipMemsetAsync(d_corr_idx_.p, 0xff, sizeof(int32_t) * L, s));
    View v = view();
    launch_nn_prep(v, nullptr, s);
    launch_nn(v, dim, s);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(idx, d_corr_idx_.p, sizeof(int32_t) * nq, hipMemcpyDeviceToHost, s));
    int32_t rech = 0;
    HIPCHK(hipMemcpyAsync(&rech, d_rechecked_.p, sizeof(int32_t), hipMemcpyDeviceToHost, s));
    SYNC_STREAM(s);
    if (num_rechecked) *num_rechecked = rech;
    if (d2) {
        for (int64_t i = 0; i < nq; ++i) {
            const double* a = query + dim * i;
            const double* b = data + (size_t)dim * idx[i];
            double r = 0;
            if (dim == 12) {
                for (int d = 0; d < 12; d += 4) {
                    const double d0 = a[d] - b[d], d1 = a[d + 1] - b[d + 1], dd2 = a[d + 2] - b[d + 2], d3 = a[d + 3] - b[d + 3];
                    r += d0 * d0 + d1 * d1 + dd2 * dd2 + d3 * d3;
                }
            } else {
                const double d0 = a[0] - b[0], d1 = a[1] - b[1], dd2 = a[2] - b[2];
                r = (d0 * d0 + d1 * d1) + dd2 * dd2;
            }
            d2[i] = r;
        }
    }
    return 0;
}

// ----------------------------------------------------------------------------- engine registry
Engine* engine_for(int device) {
    static std::mutex reg_mu;
    static std::map<int, std::unique_ptr<Engine>> reg;
    std::lock_guard<std::mutex> lk(reg_mu);
    auto it = reg.find(device);
    if (it != reg.end()) return it->second.get();
    auto e = std::make_unique<Engine>(device & 0xff);  // (slots: see capi.cpp usable_engine)
    Engine* raw = e.get();
    reg[device] = std::move(e);
    return raw;
}

}  // namespace se3icp
