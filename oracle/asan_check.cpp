// asan_check.cpp — TEST INFRASTRUCTURE: drives every entry point of the CPU restatement
// (refcpu.cpp) on the reference's fixture (created_example_reg_problem/, committed as
// tests/golden/fixture_*.ply) in a build instrumented with -fsanitize=address,undefined
// (`make -C oracle asan-run`, SURVEY.md §5 "race detection / sanitizers").  Any
// out-of-bounds access, use-after-free, leak-free misuse or undefined behaviour aborts the
// run; the results are also checked against the fixture's analytic ground truth
// (examples/create_and_save_reg_problem.cpp:31-37: rot_3d(pi/9, pi/8, -pi/7), t = (1,2,3)).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "refcpu.h"

namespace {

int g_fail = 0;
#define CHECK(c, ...)                                  \
    do {                                               \
        if (!(c)) {                                    \
            std::fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
            std::fprintf(stderr, __VA_ARGS__);         \
            std::fprintf(stderr, "\n");                \
            ++g_fail;                                  \
        }                                              \
    } while (0)

// binary little-endian PLY with double x, y, z vertices (the fixture's format)
std::vector<double> read_ply(const char* path) {
    std::vector<double> out;
    FILE* f = std::fopen(path, "rb");
    if (!f) return out;
    char line[256];
    long n = 0;
    bool ok = false;
    while (std::fgets(line, sizeof line, f)) {
        if (std::sscanf(line, "element vertex %ld", &n) == 1) continue;
        if (std::strncmp(line, "end_header", 10) == 0) { ok = true; break; }
    }
    if (ok && n > 0) {
        out.resize((size_t)n * 3);
        if (std::fread(out.data(), sizeof(double), out.size(), f) != out.size()) out.clear();
    }
    std::fclose(f);
    return out;
}

// T_gt = [Rz(-pi/7) Ry(pi/8) Rx(pi/9) | (1, 2, 3)]
void ground_truth(double T[16]) {
    const double r = M_PI / 9, p = M_PI / 8, y = -M_PI / 7;
    const double Rx[9] = {1, 0, 0, 0, std::cos(r), -std::sin(r), 0, std::sin(r), std::cos(r)};
    const double Ry[9] = {std::cos(p), 0, std::sin(p), 0, 1, 0, -std::sin(p), 0, std::cos(p)};
    const double Rz[9] = {std::cos(y), -std::sin(y), 0, std::sin(y), std::cos(y), 0, 0, 0, 1};
    double A[9], R[9];
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            A[3 * i + j] = 0;
            for (int k = 0; k < 3; ++k) A[3 * i + j] += Rz[3 * i + k] * Ry[3 * k + j];
        }
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) {
            R[3 * i + j] = 0;
            for (int k = 0; k < 3; ++k) R[3 * i + j] += A[3 * i + k] * Rx[3 * k + j];
        }
    std::memset(T, 0, 16 * sizeof(double));
    for (int i = 0; i < 3; ++i)
        for (int j = 0; j < 3; ++j) T[4 * i + j] = R[3 * i + j];
    T[3] = 1; T[7] = 2; T[11] = 3; T[15] = 1;
}

double frob(const double* A, const double* B) {
    double s = 0;
    for (int i = 0; i < 16; ++i) s += (A[i] - B[i]) * (A[i] - B[i]);
    return std::sqrt(s);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: %s source.ply target.ply\n", argv[0]);
        return 2;
    }
    const std::vector<double> src = read_ply(argv[1]), tgt = read_ply(argv[2]);
    CHECK(!src.empty() && src.size() == tgt.size(), "fixture not readable");
    if (g_fail) return 1;
    const int64_t n = (int64_t)src.size() / 3;
    double Tgt[16];
    ground_truth(Tgt);
    refcpu_params prm;
    refcpu_default_params(&prm);
    prm.estimated_overlap = 1.0;  // examples/run_registration_method.cpp:38-42
    prm.max_num_se3_iterations = 10;
    prm.mse = 1e-5;
    prm.mse_switch_error = 5e-5;
    prm.number_of_nn_for_LRF = 90;

    // every run kind and estimator, with a short trace (all trace arrays)
    const int kTr = 4;
    std::vector<double> Ti(kTr * 16), mse(kTr), d2((size_t)kTr * n), d2b((size_t)kTr * n);
    std::vector<int32_t> nk(kTr), ci((size_t)kTr * n), ci2((size_t)kTr * n);
    std::vector<float> cd((size_t)kTr * n);
    for (int run : {REFCPU_RUN_SE3_ICP, REFCPU_RUN_ICP, REFCPU_RUN_SE3_PURE, REFCPU_RUN_SE3_ICP_CF}) {
        for (int var : {REFCPU_PT2PT, REFCPU_PT2PL, REFCPU_GICP}) {
            if (run == REFCPU_RUN_SE3_ICP_CF && var != REFCPU_GICP) continue;
            for (double overlap : {1.0, 0.7}) {
                refcpu_params p = prm;
                p.estimated_overlap = overlap;
                refcpu_trace tr{kTr, 0, Ti.data(), mse.data(), nk.data(), ci.data(), cd.data(), d2.data(), ci2.data(), d2b.data()};
                refcpu_result r;
                const int rc = refcpu_register(src.data(), n, tgt.data(), n, run, var, &p, &r, &tr);
                CHECK(rc == 0, "register run %d variant %d overlap %.1f: rc %d", run, var, overlap, rc);
                const double e = frob(r.T, Tgt);
                std::printf("run %d variant %d overlap %.1f: iterations %d (se3 %d), |T - T_gt| = %.3e\n", run, var,
                            overlap, r.num_iterations, r.num_pure_se3_iterations, e);
                if (run != REFCPU_RUN_ICP && overlap == 1.0) CHECK(e <= 1e-6, "pose off the ground truth: %.3e", e);
            }
        }
    }
    // stage entry points
    for (int k : {30, 90, 150}) {
        std::vector<int32_t> idx((size_t)n * k);
        std::vector<double> dd((size_t)n * k);
        CHECK(refcpu_knn_self(src.data(), n, k, idx.data(), dd.data()) == 0, "knn_self k=%d", k);
        for (int64_t i = 0; i < n; ++i) {
            CHECK(idx[(size_t)i * k] >= 0 && idx[(size_t)i * k] < n, "knn index");
            for (int j = 1; j < k; ++j) CHECK(dd[(size_t)i * k + j] >= dd[(size_t)i * k + j - 1], "knn order");
        }
        std::vector<double> fr((size_t)n * 16), nr((size_t)n * 3), cov((size_t)n * 9);
        CHECK(refcpu_toldi_frames(src.data(), n, k, fr.data()) == 0, "toldi k=%d", k);
        CHECK(refcpu_estimate_normals(src.data(), n, k, nr.data()) == 0, "normals k=%d", k);
        CHECK(refcpu_gicp_covariances(nr.data(), n, 1e-3, cov.data()) == 0, "gicp covariances");
    }
    {
        std::vector<int32_t> idx(n);
        std::vector<double> dd(n);
        CHECK(refcpu_nn(tgt.data(), n, tgt.data(), n, 3, idx.data(), dd.data()) == 0, "nn 3-D");
        for (int64_t i = 0; i < n; ++i) CHECK(dd[i] == 0.0, "self nn distance");
        std::vector<double> q12((size_t)n * 12), d12((size_t)n * 12);
        for (int64_t i = 0; i < n; ++i)
            for (int a = 0; a < 12; ++a) {
                q12[(size_t)i * 12 + a] = src[(size_t)i * 3 + a % 3] * (1 + a / 3);
                d12[(size_t)i * 12 + a] = tgt[(size_t)i * 3 + a % 3] * (1 + a / 3);
            }
        CHECK(refcpu_nn(q12.data(), n, d12.data(), n, 12, idx.data(), dd.data()) == 0, "nn 12-D");
    }
    {
        std::vector<int32_t> pairs((size_t)n * 2);
        for (int64_t i = 0; i < n; ++i) { pairs[2 * i] = (int32_t)i; pairs[2 * i + 1] = (int32_t)i; }
        std::vector<double> nr((size_t)n * 3), cs((size_t)n * 9), ct((size_t)n * 9), w(n, 0.5);
        refcpu_estimate_normals(tgt.data(), n, 20, nr.data());
        refcpu_gicp_covariances(nr.data(), n, 1e-3, ct.data());
        refcpu_estimate_normals(src.data(), n, 20, nr.data());
        refcpu_gicp_covariances(nr.data(), n, 1e-3, cs.data());
        refcpu_estimate_normals(tgt.data(), n, 30, nr.data());
        // the source moved onto the target by T_gt: every estimator's step is the identity
        // (pt2pt also recovers T_gt in one closed-form step from the raw source)
        std::vector<double> moved((size_t)n * 3);
        for (int64_t i = 0; i < n; ++i)
            for (int a = 0; a < 3; ++a)
                moved[3 * i + a] = Tgt[4 * a] * src[3 * i] + Tgt[4 * a + 1] * src[3 * i + 1] +
                                   Tgt[4 * a + 2] * src[3 * i + 2] + Tgt[4 * a + 3];
        double T[16], I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
        for (int var : {REFCPU_PT2PT, REFCPU_PT2PL, REFCPU_GICP}) {
            CHECK(refcpu_estimate(var, moved.data(), cs.data(), tgt.data(), nr.data(), ct.data(), pairs.data(), n,
                                  var == REFCPU_GICP ? w.data() : nullptr, T) == 0, "estimate %d", var);
            CHECK(frob(T, I) <= 1e-9, "estimator %d on aligned true correspondences: %.3e", var, frob(T, I));
        }
        CHECK(refcpu_estimate(REFCPU_PT2PT, src.data(), cs.data(), tgt.data(), nr.data(), ct.data(), pairs.data(), n,
                              nullptr, T) == 0, "estimate pt2pt");
        CHECK(frob(T, Tgt) <= 1e-9, "umeyama on the true correspondences: %.3e", frob(T, Tgt));
    }
    {
        std::vector<float> dist(n);
        for (int64_t i = 0; i < n; ++i) dist[i] = (float)((i * 7919) % 1000) * 0.01f;
        std::vector<int32_t> kept(n);
        const int64_t k = refcpu_trim(dist.data(), n, 0.7, kept.data());
        CHECK(k == (int64_t)std::floor(0.7f * (float)n), "trim count %ld", (long)k);
    }
    std::printf("%s: %d failures\n", g_fail ? "FAILED" : "ok", g_fail);
    return g_fail ? 1 : 0;
}
