// Achievable HBM read bandwidth for the config-5 step's access pattern: 2*d SoA columns of ld
// doubles (+ w, + A read/write), one row per thread, coordinates loaded in chunks of 8.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int D, int CH>
__global__ __launch_bounds__(256) void stream_rows(const double* __restrict__ x, const double* __restrict__ g,
                                                   const double* __restrict__ w, double* __restrict__ A,
                                                   int64_t n, int64_t ld) {
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        double s = 0.0;
#pragma unroll 1
        for (int k0 = 0; k0 < D; k0 += CH) {
            double xv[CH], gv[CH];
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                const int k = k0 + c < D ? k0 + c : D - 1;
                xv[c] = x[k * ld + i];
                gv[c] = g[k * ld + i];
            }
#pragma unroll
            for (int c = 0; c < CH; ++c) s += xv[c] * gv[c];
        }
        A[i] = A[i] + s * w[i];
    }
}

int main() {
    const int64_t n = 500000, ld = 500032;
    constexpr int D = 50;
    double *x, *g, *w, *A;
    hipMalloc(&x, 8 * D * ld); hipMalloc(&g, 8 * D * ld); hipMalloc(&w, 8 * ld); hipMalloc(&A, 8 * ld);
    hipMemset(x, 0, 8 * D * ld); hipMemset(g, 0, 8 * D * ld); hipMemset(w, 0, 8 * ld); hipMemset(A, 0, 8 * ld);
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    const double bytes = (double)n * (16 * D + 24);
    for (int blocks : {256, 512, 1024, 2048, 1954}) {
        for (int ch : {4, 8, 16}) {
            auto run = [&]() {
                if (ch == 4) stream_rows<D, 4><<<blocks, 256>>>(x, g, w, A, n, ld);
                else if (ch == 8) stream_rows<D, 8><<<blocks, 256>>>(x, g, w, A, n, ld);
                else stream_rows<D, 16><<<blocks, 256>>>(x, g, w, A, n, ld);
            };
            for (int r = 0; r < 5; ++r) run();
            hipEventRecord(e0);
            for (int r = 0; r < 50; ++r) run();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = ms * 1e3 / 50;
            printf("blocks=%5d ch=%2d  %7.2f us  %6.2f TB/s\n", blocks, ch, us, bytes / (us * 1e-6) / 1e12);
        }
    }
    return 0;
}
