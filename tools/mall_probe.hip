// Measurement probe (not product code): does the config-5 step's working set (n rows of 2*d SoA
// fp64 columns + w + A, d = 50: 832 B per row, 416 MB at n = 5e5) gain from the MI355X memory-side
// cache (256 MB Infinity Cache / MALL) when the same columns are streamed step after step?
//   part 1: back-to-back launches over n rows, default cache policy, n = 1e5 .. 5e5
//   part 2: n = 5e5, rows >= split loaded with a cache-policy aux (buffer loads), rows < split
//           with the default policy -- can a subset stay MALL-resident while the rest streams?
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

template <int AUX>
__device__ __forceinline__ double ld_buf(__amdgpu_buffer_rsrc_t r, int64_t i) {
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(i * 8), 0, AUX);
    return __longlong_as_double((long long)(((uint64_t)v.y << 32) | v.x));
}

template <int D, int AUX>
__global__ __launch_bounds__(256) void stream_rows(const double* __restrict__ x, const double* __restrict__ g,
                                                   const double* __restrict__ w, double* __restrict__ A,
                                                   int64_t n, int64_t ld, int64_t split) {
    const auto rx = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(x), 0, 0x7FFFFFFF, 0x00020000);
    const auto rg = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(g), 0, 0x7FFFFFFF, 0x00020000);
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        double s = 0.0;
        const bool pol = i >= split;
#pragma unroll 1
        for (int k0 = 0; k0 < D; k0 += 8) {
            double xv[8], gv[8];
            if (pol) {
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const int k = k0 + c < D ? k0 + c : D - 1;
                    xv[c] = ld_buf<AUX>(rx, k * ld + i);
                    gv[c] = ld_buf<AUX>(rg, k * ld + i);
                }
            } else {
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const int k = k0 + c < D ? k0 + c : D - 1;
                    xv[c] = ld_buf<0>(rx, k * ld + i);
                    gv[c] = ld_buf<0>(rg, k * ld + i);
                }
            }
#pragma unroll
            for (int c = 0; c < 8; ++c) s += xv[c] * gv[c];
        }
        A[i] = A[i] + s * w[i];
    }
}

int main() {
    constexpr int D = 50;
    const int64_t nmax = 500000, ld = 500032;
    double *x, *g, *w, *A, *junk;
    hipMalloc(&x, 8 * D * ld); hipMalloc(&g, 8 * D * ld); hipMalloc(&w, 8 * ld); hipMalloc(&A, 8 * ld);
    const size_t junk_bytes = (size_t)1 << 30;   // 1 GB write between cases: flushes the MALL
    hipMalloc(&junk, junk_bytes);
    hipMemset(x, 0, 8 * D * ld); hipMemset(g, 0, 8 * D * ld); hipMemset(w, 0, 8 * ld); hipMemset(A, 0, 8 * ld);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const int blocks = 1024, reps = 50;
    auto timeit = [&](auto launch, int64_t n, const char* what) {
        hipMemset(junk, 1, junk_bytes);
        for (int i = 0; i < 5; ++i) launch();
        hipEventRecord(e0);
        for (int i = 0; i < reps; ++i) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        const double us = ms * 1e3 / reps, bytes = (double)n * (16 * D + 24);
        printf("%-44s n=%7lld  %8.2f us/step  %7.1f GB/s (%.0f MB per step)\n", what, (long long)n, us,
               bytes / (us * 1e-6) / 1e9, bytes / 1e6);
        fflush(stdout);
    };
    for (int64_t n : {100000ll, 200000ll, 250000ll, 300000ll, 350000ll, 400000ll, 500000ll})
        timeit([&]() { stream_rows<D, 0><<<blocks, 256>>>(x, g, w, A, n, ld, n); }, n, "default policy");
    const int64_t n = nmax;
    for (int64_t split : {0ll, 150000ll, 200000ll, 250000ll, 300000ll, 500000ll}) {
        char buf[96];
        snprintf(buf, sizeof buf, "rows >= %lld nt (aux 2)", (long long)split);
        timeit([&]() { stream_rows<D, 2><<<blocks, 256>>>(x, g, w, A, n, ld, split); }, n, buf);
        snprintf(buf, sizeof buf, "rows >= %lld sc1 nt (aux 18)", (long long)split);
        timeit([&]() { stream_rows<D, 18><<<blocks, 256>>>(x, g, w, A, n, ld, split); }, n, buf);
        snprintf(buf, sizeof buf, "rows >= %lld sc0 sc1 (aux 17)", (long long)split);
        timeit([&]() { stream_rows<D, 17><<<blocks, 256>>>(x, g, w, A, n, ld, split); }, n, buf);
    }
    return 0;
}
