// Throughput of v_mfma_f64_16x16x4_f64 on one GPU: W waves per block x B blocks, each wave runs
// ITER iterations of 8 independent 16x16x4 MFMAs.  Prints TFLOP/s and cycles per MFMA per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef double dbl4 __attribute__((ext_vector_type(4)));

__global__ void probe(double* out, int iters, double a0, double b0) {
    dbl4 acc[8];
    for (int u = 0; u < 8; ++u) acc[u] = dbl4{0, 0, 0, 0};
    double a = a0 + threadIdx.x * 1e-9, b = b0 - threadIdx.x * 1e-9;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[u], 0, 0, 0);
    }
    double s = 0;
    for (int u = 0; u < 8; ++u) s += acc[u][0] + acc[u][1] + acc[u][2] + acc[u][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void probe_valu(double* out, int iters, double a0, double b0) {
    double acc[8];
    for (int u = 0; u < 8; ++u) acc[u] = 0;
    double a = a0 + threadIdx.x * 1e-9, b = b0 - threadIdx.x * 1e-9;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 8; ++u) acc[u] = fma(a, b, acc[u]);
    }
    double s = 0;
    for (int u = 0; u < 8; ++u) s += acc[u];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main(int argc, char** argv) {
    const int iters = 20000;
    double* out;
    hipMalloc(&out, 1024 * 1024 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    int cus = 256;
    for (int kind = 0; kind < 2; ++kind)
    for (int wps = 1; wps <= 4; wps *= 2) {   // waves per SIMD
        const int threads = 256;              // 4 waves / block = 1 per SIMD
        const int blocks = cus * wps;
        for (int rep = 0; rep < 2; ++rep) {
            hipEventRecord(e0, 0);
            if (kind == 0) probe<<<blocks, threads>>>(out, iters, 1.0, 1.0);
            else probe_valu<<<blocks, threads>>>(out, iters, 1.0, 1.0);
            hipEventRecord(e1, 0);
            hipEventSynchronize(e1);
        }
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        const double flop = kind == 0 ? (double)blocks * 4 * iters * 8 * 2048.0 : (double)blocks * threads * iters * 8 * 2.0;
        const double tf = flop / (ms * 1e-3) / 1e12;
        const double per_simd_ops = (double)wps * iters * 8;   // instructions per SIMD
        printf("%s waves/SIMD=%d: %.3f ms, %.1f TFLOP/s, %.1f ns per instr per SIMD (%.1f cycles @2.4GHz)\n",
               kind == 0 ? "mfma_f64_16x16x4" : "v_fma_f64       ", wps, ms, tf, ms * 1e6 / per_simd_ops,
               ms * 1e6 / per_simd_ops * 2.4);
    }
    return 0;
}
