// FETCH_SIZE calibration for gather patterns on gfx950 ("What's weak" #5).
//
// MI355X_MICROARCH.md §HBM establishes that FETCH_SIZE reports 1/2 of the bytes of a wide
// coalesced streaming read and leaves other widths uncalibrated.  The engine's loop kernels
// are gather-dominated (k_reduce: 8-B SoA rows by correspondence index; k_nn_search /
// k_tree_local: 48-B f32 SE(3) rows; k_nn_prep: 4-B and 48-B records), so this program runs
// each access pattern once over a 1 GiB table (4x the 256 MiB Infinity Cache, so re-reads
// are rare and every access is a fabric request) with a known number of accesses:
//
//   k_stream16      coalesced 16 B per lane over the whole table (the guide's reference case)
//   k_gather<W>     W = 4, 8, 16, 48: one W-byte row per thread at a hashed row index
//   k_gather_soa3   three 8-B loads per thread at one hashed index from three columns
//                   (k_reduce's xt / nt rows)
//   k_gather_local  8-B loads at hashed indices inside 4-KiB windows (one window per wave:
//                   the spatial locality of correspondences of neighbouring source points)
//
// Each kernel prints its access count, requested bytes and HIP-event time; the FETCH_SIZE /
// TCC_* counters come from rocprofv3 --pmc passes over this program
// (tools/fetch_calib.sh), and tools/pmc_summary.py --calib turns them into the per-pattern
// ratios (profiles/r05_fetch_calib.json).  Loads only: the kernels store nothing unless an
// impossible sum appears, so WRITE_SIZE stays ~0.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                \
        }                                                                           \
    } while (0)

__device__ __forceinline__ unsigned mix32(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

__device__ __forceinline__ void sink(float acc, float* out) {
    if (acc == -1.2345e-30f) out[threadIdx.x] = acc;  // (never taken)
}

__global__ __launch_bounds__(256) void k_stream16(const float4* __restrict__ t, size_t n4, float* out) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = t[i];
        acc += v.x + v.y + v.z + v.w;
    }
    sink(acc, out);
}

template <int W>
__global__ __launch_bounds__(256) void k_gather(const char* __restrict__ t, unsigned nrows, int per, unsigned salt,
                                                float* out) {
    float acc = 0.f;
    const unsigned base = (blockIdx.x * blockDim.x + threadIdx.x) * (unsigned)per;
    for (int k = 0; k < per; ++k) {
        const unsigned r = mix32((base + k) ^ salt) % nrows;
        const char* p = t + (size_t)r * W;
        if constexpr (W == 4) {
            acc += *reinterpret_cast<const float*>(p);
        } else if constexpr (W == 8) {
            const float2 v = *reinterpret_cast<const float2*>(p);
            acc += v.x + v.y;
        } else if constexpr (W == 16) {
            const float4 v = *reinterpret_cast<const float4*>(p);
            acc += v.x + v.y + v.z + v.w;
        } else {
            static_assert(W == 48, "row widths 4, 8, 16, 48");
            const float4* q = reinterpret_cast<const float4*>(p);
            const float4 a = q[0], b = q[1], c = q[2];
            acc += a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w + c.x + c.y + c.z + c.w;
        }
    }
    sink(acc, out);
}

__global__ __launch_bounds__(256) void k_gather_soa3(const double* __restrict__ t, unsigned ld, int per, unsigned salt,
                                                     float* out) {
    double acc = 0.0;
    const unsigned base = (blockIdx.x * blockDim.x + threadIdx.x) * (unsigned)per;
    for (int k = 0; k < per; ++k) {
        const unsigned r = mix32((base + k) ^ salt) % ld;
        acc += t[r] + t[(size_t)ld + r] + t[2 * (size_t)ld + r];
    }
    sink((float)acc, out);
}

// 8-B loads at hashed indices inside one 4-KiB window per wave and iteration
__global__ __launch_bounds__(256) void k_gather_local(const double* __restrict__ t, unsigned nwin, int per,
                                                      unsigned salt, float* out) {
    double acc = 0.0;
    const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const unsigned lane = threadIdx.x & 63;
    for (int k = 0; k < per; ++k) {
        const unsigned w = mix32((wave * (unsigned)per + k) ^ salt) % nwin;
        const unsigned r = mix32(((wave * (unsigned)per + k) << 6 | lane) ^ (salt * 3u)) & 511u;
        acc += t[(size_t)w * 512 + r];
    }
    sink((float)acc, out);
}

int main(int argc, char** argv) {
    const size_t bytes = (size_t)1 << 30;  // 1 GiB table
    const int per = 8;                       // accesses per thread
    const int threads = 256;
    const int blocks = 16384;                // 4.2 M threads, 33.5 M accesses per gather kernel
    const double nacc = (double)blocks * threads * per;
    char* t;
    float* out;
    CK(hipMalloc(&t, bytes));
    CK(hipMalloc(&out, 4096));
    CK(hipMemset(t, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto timed = [&](const char* name, double accesses, double req_bytes, auto launch) {
        launch(0u);  // warm (page tables / code; other rows than the timed launch)
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        launch(1u);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"kernel\": \"%s\", \"launches\": 2, \"accesses\": %.0f, \"requested_bytes\": %.0f, \"ms\": %.4f, "
               "\"requested_GBps\": %.1f}\n",
               name, accesses, req_bytes, ms, req_bytes / (ms * 1e-3) / 1e9);
        fflush(stdout);
    };
    timed("k_stream16", (double)(bytes / 16), (double)bytes,
          [&](unsigned s) { (void)s;
              k_stream16<<<8192, threads>>>(reinterpret_cast<const float4*>(t), bytes / 16, out); });
    timed("k_gather<4>", nacc, nacc * 4,
          [&](unsigned s) { k_gather<4><<<blocks, threads>>>(t, (unsigned)(bytes / 4), per, 0x1234u + 0x9e3779b9u * s, out); });
    timed("k_gather<8>", nacc, nacc * 8,
          [&](unsigned s) { k_gather<8><<<blocks, threads>>>(t, (unsigned)(bytes / 8), per, 0x2345u + 0x9e3779b9u * s, out); });
    timed("k_gather<16>", nacc, nacc * 16,
          [&](unsigned s) { k_gather<16><<<blocks, threads>>>(t, (unsigned)(bytes / 16), per, 0x3456u + 0x9e3779b9u * s, out); });
    timed("k_gather<48>", nacc, nacc * 48,
          [&](unsigned s) { k_gather<48><<<blocks, threads>>>(t, (unsigned)(bytes / 48), per, 0x4567u + 0x9e3779b9u * s, out); });
    timed("k_gather_soa3", nacc * 3, nacc * 24, [&](unsigned s) {
        k_gather_soa3<<<blocks, threads>>>(reinterpret_cast<const double*>(t), (unsigned)(bytes / 24), per, 0x5678u + 0x9e3779b9u * s, out);
    });
    timed("k_gather_local", nacc, nacc * 8, [&](unsigned s) {
        k_gather_local<<<blocks, threads>>>(reinterpret_cast<const double*>(t), (unsigned)(bytes / 4096), per, 0x6789u + 0x9e3779b9u * s,
                                            out);
    });
    CK(hipFree(t));
    CK(hipFree(out));
    return 0;
}
