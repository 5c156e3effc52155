// capi.cpp — extern "C" boundary of libse3icp.so (declared in include/se3icp.h).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <iostream>
#include <mutex>
#include <string>
#include <vector>

#include "engine.hpp"
#include "se3icp.h"

using se3icp::Engine;
using se3icp::engine_for;

namespace {

const char* kMethodNames[SE3ICP_NUM_METHODS] = {"pt2pt",     "pt2pl",     "gicp",
                                                "se3_pt2pt", "se3_pt2pl", "se3_gicp",
                                                "se3_gicp_with_cf", "se3_pure_pt2pt", "se3_pure_pt2pl",
                                                "se3_pure_gicp"};

int variant_index(const char* v) {
    if (!v) return -1;
    if (!std::strcmp(v, "pt2pt")) return 0;
    if (!std::strcmp(v, "pt2pl")) return 1;
    if (!std::strcmp(v, "gicp")) return 2;
    return -1;
}

int current_device() {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) return 0;
    return d;
}

// device = ordinal | slot << 8: slot s > 0 is a further engine on the same GPU (its own
// stream and buffers), so independent batches can be queued side by side
Engine* usable_engine(int device) {
    int n = 0;
    const int ord = device & 0xff;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0 || device < 0 || ord >= n || (device >> 8) > 15) return nullptr;
    return engine_for(device);
}

}  // namespace

struct se3icp_registration {
    std::vector<double> src, tgt;
    se3icp_params prm;
    se3icp_result res;
};

extern "C" {

int se3icp_abi_version(void) { return SE3ICP_ABI_VERSION; }

const char* se3icp_status_string(int status) {
    switch (status) {
        case SE3ICP_OK: return "ok";
        case SE3ICP_ERR_INVALID_ARG: return "invalid argument";
        case SE3ICP_ERR_INVALID_METHOD: return "invalid method name";
        case SE3ICP_ERR_EMPTY_CLOUD: return "empty point cloud";
        case SE3ICP_ERR_K_TOO_LARGE: return "number_of_nn_for_LRF too large (unused since ABI 3: any k is taken)";
        case SE3ICP_ERR_NO_DEVICE: return "no usable HIP device (the engine has no CPU fallback)";
        case SE3ICP_ERR_HIP: return "HIP runtime error";
        case SE3ICP_ERR_NONFINITE: return "non-finite pose";
        case SE3ICP_ERR_OUT_OF_MEMORY: return "out of device memory";
        default: return "unknown status";
    }
}

int se3icp_method_from_name(const char* name) {
    if (!name) return SE3ICP_ERR_INVALID_METHOD;
    for (int m = 0; m < SE3ICP_NUM_METHODS; ++m)
        if (!std::strcmp(name, kMethodNames[m])) return m;
    return SE3ICP_ERR_INVALID_METHOD;
}

const char* se3icp_method_name(int method) {
    return (method >= 0 && method < SE3ICP_NUM_METHODS) ? kMethodNames[method] : nullptr;
}

// IterativeSE3Registration::IterativeSE3Registration()  ISR.cpp:334-348
void se3icp_default_params(se3icp_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof(*p));
    p->max_num_iterations = 150;
    p->max_num_se3_iterations = 20;
    p->number_of_nn_for_LRF = 30;
    p->mse = 0.00001;
    p->mse_switch_error = 0.001;
    p->estimated_overlap = 1.0;
    p->alpha_rot = 3.0;
    p->beta_transl = 1.0;
    p->scale_preprocessing = 3.0;
}

int se3icp_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// ------------------------------------------------------------------ batch surface
int se3icp_register_batch(int device, int32_t n_pairs, const double* const* src_xyz, const int64_t* n_src,
                          const double* const* tgt_xyz, const int64_t* n_tgt, int method,
                          const se3icp_params* params, se3icp_result* results) {
    Engine* e = usable_engine(device);
    if (!e) return SE3ICP_ERR_NO_DEVICE;
    se3icp_params p;
    if (params) p = *params; else se3icp_default_params(&p);
    std::lock_guard<std::mutex> lk(e->mutex());
    return e->register_batch(n_pairs, src_xyz, n_src, tgt_xyz, n_tgt, false, method, p, results, nullptr);
}

int se3icp_register_batch_device(int device, int32_t n_pairs, const double* d_src_xyz, const int64_t* src_off,
                                 const double* d_tgt_xyz, const int64_t* tgt_off, int method,
                                 const se3icp_params* params, se3icp_result* results, void* hip_stream) {
    Engine* e = usable_engine(device);
    if (!e) return SE3ICP_ERR_NO_DEVICE;
    if (n_pairs <= 0 || !d_src_xyz || !d_tgt_xyz || !src_off || !tgt_off) return SE3ICP_ERR_INVALID_ARG;
    std::vector<const double*> s(n_pairs), t(n_pairs);
    std::vector<int64_t> ns(n_pairs), nt(n_pairs);
    for (int i = 0; i < n_pairs; ++i) {
        s[i] = d_src_xyz + 3 * src_off[i];
        t[i] = d_tgt_xyz + 3 * tgt_off[i];
        ns[i] = src_off[i + 1] - src_off[i];
        nt[i] = tgt_off[i + 1] - tgt_off[i];
    }
    se3icp_params p;
    if (params) p = *params; else se3icp_default_params(&p);
    std::lock_guard<std::mutex> lk(e->mutex());
    return e->register_batch(n_pairs, s.data(), ns.data(), t.data(), nt.data(), true, method, p, results,
                             (hipStream_t)hip_stream);
}

int se3icp_register(int device, const double* src_xyz, int64_t n_src, const double* tgt_xyz, int64_t n_tgt,
                    int method, const se3icp_params* params, se3icp_result* result) {
    return se3icp_register_batch(device, 1, &src_xyz, &n_src, &tgt_xyz, &n_tgt, method, params, result);
}

// ------------------------------------------------------------------ object surface
se3icp_registration* se3icp_registration_new(void) {
    auto* r = new (std::nothrow) se3icp_registration;
    if (!r) return nullptr;
    se3icp_default_params(&r->prm);
    std::memset(&r->res, 0, sizeof(r->res));
    for (int i = 0; i < 4; ++i) r->res.T[i * 4 + i] = 1.0;
    r->res.num_pure_se3_iterations = -1;  // ISR.cpp:338
    return r;
}

void se3icp_registration_free(se3icp_registration* r) { delete r; }

int se3icp_set_source_cloud(se3icp_registration* r, const double* xyz, int64_t n) {
    if (!r || (n > 0 && !xyz) || n < 0) return SE3ICP_ERR_INVALID_ARG;
    r->src.insert(r->src.end(), xyz, xyz + 3 * n);  // push_back, ISR.cpp:359-362
    return 0;
}

int se3icp_set_target_cloud(se3icp_registration* r, const double* xyz, int64_t n) {
    if (!r || (n > 0 && !xyz) || n < 0) return SE3ICP_ERR_INVALID_ARG;
    r->tgt.insert(r->tgt.end(), xyz, xyz + 3 * n);
    return 0;
}

se3icp_params* se3icp_params_of(se3icp_registration* r) { return r ? &r->prm : nullptr; }

static int run_object(se3icp_registration* r, int method) {
    const int64_t ns = (int64_t)r->src.size() / 3, nt = (int64_t)r->tgt.size() / 3;
    if (ns <= 0 || nt <= 0) return SE3ICP_ERR_EMPTY_CLOUD;
    const double* s = r->src.data();
    const double* t = r->tgt.data();
    se3icp_result res;
    int rc = se3icp_register_batch(current_device(), 1, &s, &ns, &t, &nt, method, &r->prm, &res);
    if (rc == SE3ICP_OK || rc == SE3ICP_ERR_NONFINITE) r->res = res;
    return rc;
}

int se3icp_run_icp(se3icp_registration* r, const char* variant) {
    if (!r) return SE3ICP_ERR_INVALID_ARG;
    const int v = variant_index(variant);
    if (v < 0) {  // ISR.cpp:478-480
        std::cerr << "Invalid ICP variant name. Valid names are pt2pt, pt2pl and gicp.\n";
        return SE3ICP_ERR_INVALID_METHOD;
    }
    return run_object(r, SE3ICP_PT2PT + v);
}

int se3icp_run_se3_icp(se3icp_registration* r, const char* variant) {
    if (!r) return SE3ICP_ERR_INVALID_ARG;
    const int v = variant_index(variant);
    if (v < 0) {
        // ISR.cpp:561-563 then 700-703: one iteration, T_i never formed, loop breaks;
        // the de-normalized identity is [I | c_t - c_s].
        std::cerr << "Invalid variant name. Choose one of: pt2pt, pt2pl, gicp \n";
        std::cout << "Unknown optimization strategy for SE(3) \n";
        const int64_t ns = (int64_t)r->src.size() / 3, nt = (int64_t)r->tgt.size() / 3;
        if (ns <= 0 || nt <= 0) return SE3ICP_ERR_EMPTY_CLOUD;
        double cs[3] = {0, 0, 0}, ct[3] = {0, 0, 0};
        for (int64_t i = 0; i < ns; ++i)
            for (int a = 0; a < 3; ++a) cs[a] += r->src[3 * i + a];
        for (int64_t i = 0; i < nt; ++i)
            for (int a = 0; a < 3; ++a) ct[a] += r->tgt[3 * i + a];
        std::memset(r->res.T, 0, sizeof(r->res.T));
        for (int a = 0; a < 4; ++a) r->res.T[a * 4 + a] = 1.0;
        for (int a = 0; a < 3; ++a) r->res.T[a * 4 + 3] = ct[a] / (double)nt - cs[a] / (double)ns;
        r->res.num_iterations = 1;
        r->res.num_pure_se3_iterations = 1;
        r->res.status = SE3ICP_ERR_INVALID_METHOD;
        return SE3ICP_ERR_INVALID_METHOD;
    }
    return run_object(r, SE3ICP_SE3_PT2PT + v);
}

int se3icp_run_se3_icp_with_cf(se3icp_registration* r) {
    if (!r) return SE3ICP_ERR_INVALID_ARG;
    const int rc = run_object(r, SE3ICP_SE3_GICP_WITH_CF);
    if (rc == SE3ICP_OK || rc == SE3ICP_ERR_NONFINITE)  // ISR.cpp:794 (printed once the run returns)
        std::cout << "### scaling factor = " << r->res.scaling_factor << std::endl;
    return rc;
}

int se3icp_run_se3_pure(se3icp_registration* r, const char* variant) {
    if (!r) return SE3ICP_ERR_INVALID_ARG;
    const int v = variant_index(variant);
    if (v < 0) {
        std::cerr << "Invalid variant name. Choose one of: pt2pt, pt2pl, gicp \n";
        return SE3ICP_ERR_INVALID_METHOD;
    }
    const int rc = run_object(r, SE3ICP_SE3_PURE_PT2PT + v);
    if (rc == SE3ICP_OK || rc == SE3ICP_ERR_NONFINITE) std::cout << "pure se3 finished" << std::endl;  // ISR.cpp:1127
    return rc;
}

int se3icp_get_result(const se3icp_registration* r, se3icp_result* out) {
    if (!r || !out) return SE3ICP_ERR_INVALID_ARG;
    *out = r->res;
    return 0;
}

// ------------------------------------------------------------------ stage surface
int se3icp_toldi_frames(int device, const double* xyz, int64_t n, int k, double* frames) {
    Engine* e = usable_engine(device);
    if (!e) return SE3ICP_ERR_NO_DEVICE;
    std::lock_guard<std::mutex> lk(e->mutex());
    return e->toldi_frames(xyz, n, k, frames);
}

int se3icp_knn_self(int device, const double* xyz, int64_t n, int k, int32_t* idx) {
    Engine* e = usable_engine(device);
    if (!e) return SE3ICP_ERR_NO_DEVICE;
    std::lock_guard<std::mutex> lk(e->mutex());
    return e->knn_self(xyz, n, k, idx);
}

int se3icp_estimate_normals(int device, const double* xyz, int64_t n, int k, double* normals) {
    Engine* e = usable_engine(device);
    if (!e) return SE3ICP_ERR_NO_DEVICE;
    std::lock_guard<std::mutex> lk(e->mutex());
    return e->estimate_normals(xyz, n, k, normals);
}

int se3icp_nn(int device, const double* query, int64_t nq, const double* data, int64_t nd, int dim, int32_t* idx,
              double* d2, int32_t* num_rechecked) {
    Engine* e = usable_engine(device);
    if (!e) return SE3ICP_ERR_NO_DEVICE;
    std::lock_guard<std::mutex> lk(e->mutex());
    return e->nn(query, nq, data, nd, dim, idx, d2, num_rechecked);
}

// ------------------------------------------------------------------ profiling hooks (not part of the
// reference boundary; used by bench.py to read the per-kernel HIP-event times of the last batch)
int se3icp_set_profiling(int device, int on) {
    Engine* e = usable_engine(device);
    if (!e) return SE3ICP_ERR_NO_DEVICE;
    e->set_profiling(on != 0);
    return 0;
}

int se3icp_set_trace(int device, se3icp_trace* trace) {
    Engine* e = usable_engine(device);
    if (!e) return SE3ICP_ERR_NO_DEVICE;
    if (trace && (trace->max_iters < 0 || trace->pair < 0)) return SE3ICP_ERR_INVALID_ARG;
    std::lock_guard<std::mutex> lk(e->mutex());
    e->set_trace(trace);
    return 0;
}

int se3icp_set_lrf_exact(int device, int exact_only) {
    Engine* e = usable_engine(device);
    if (!e) return SE3ICP_ERR_NO_DEVICE;
    std::lock_guard<std::mutex> lk(e->mutex());
    if (exact_only < 0 || exact_only > 2) return SE3ICP_ERR_INVALID_ARG;
    e->set_lrf_exact(exact_only);
    return 0;
}

int se3icp_set_nn_events(int device, int on) {
    Engine* e = usable_engine(device);
    if (!e) return SE3ICP_ERR_NO_DEVICE;
    std::lock_guard<std::mutex> lk(e->mutex());
    e->set_nn_events(on != 0);
    return 0;
}

int se3icp_last_kernel_times(int device, double* out /* [24] */) {
    double x[SE3ICP_KERNEL_TIMES_N];
    const int rc = se3icp_last_kernel_times_n(device, x, SE3ICP_KERNEL_TIMES_N);
    if (rc == 0)
        for (int i = 0; i < 24; ++i) out[i] = x[i];
    return rc;
}

int se3icp_last_kernel_times_n(int device, double* out, int n) {
    Engine* e = usable_engine(device);
    if (!e || !out) return SE3ICP_ERR_NO_DEVICE;
    if (n < SE3ICP_KERNEL_TIMES_N) return SE3ICP_ERR_INVALID_ARG;
    const auto& k = e->kernel_times();
    out[0] = k.nn_se3_ms;
    out[1] = k.nn_r3_ms;
    out[2] = k.recheck_ms;
    out[3] = k.trim_ms;
    out[4] = k.reduce_ms;
    out[5] = k.setup_ms;
    out[6] = (double)k.nn_se3_launches;
    out[7] = (double)k.nn_r3_launches;
    out[8] = k.se3_dist_evals;
    out[9] = k.se3_box_tests;
    out[10] = k.r3_dist_evals;
    out[11] = k.r3_box_tests;
    out[12] = k.lrf_ms;
    out[13] = k.lrf_queries;
    out[14] = k.lrf_leaves;
    out[15] = k.lrf_merges;
    out[16] = k.lrf_box_tests;
    out[17] = k.lrf_candidates;
    out[18] = k.nn_prep_ms;
    out[19] = k.se3_queries;
    out[20] = k.se3_searched;
    out[21] = k.r3_queries;
    out[22] = k.r3_searched;
    out[23] = k.lrf_fallback;
    out[24] = k.se3_useful_evals;
    out[25] = k.r3_useful_evals;
    return 0;
}

}  // extern "C"
