// Measurement probe (not product code): fp64 VALU issue rate on gfx950 for one / two waves per
// SIMD, independent vs dependent chains, and the cost of the IEEE division sequence.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/fp64_rate tools/fp64_rate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

template <int CH>
__global__ void fma_chains(double* out, double a, double b, int iters) {
    double acc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) acc[c] = __builtin_fma(acc[c], a, b);
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += acc[c];
    if (s == 12345.678) out[threadIdx.x] = s;
}

template <int CH, int OP>
__global__ void op_chains(double* out, double a, double b, int iters) {
    double acc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) acc[c] = OP == 0 ? acc[c] * a : acc[c] + b;
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += acc[c];
    if (s == 12345.678) out[threadIdx.x] = s;
}

// shader clock: s_memtime (core clock) vs s_memrealtime (100 MHz) around a long fma loop
__global__ void clock_probe(double* out, double a, double b, int iters) {
    const uint64_t c0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    double acc[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) acc[c] = threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < 16; ++c) acc[c] = __builtin_fma(acc[c], a, b);
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += acc[c];
    asm volatile("" ::"v"(s));
    const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0 && blockIdx.x == 0) { out[0] = (double)(c1 - c0); out[1] = (double)(r1 - r0); }
    if ((threadIdx.x & 63) == 0) {   // one record per wave: {start, end, HW_ID}
        uint32_t hw;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        const int w = blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        out[1024 + 3 * w + 0] = (double)r0;
        out[1024 + 3 * w + 1] = (double)r1;
        out[1024 + 3 * w + 2] = (double)hw;
    }
}

template <int CH>
__global__ void div_chains(double* out, double a, int iters) {
    double acc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x * 1e-3 + c + 1.5;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) acc[c] = a / acc[c] + 1.0;
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += acc[c];
    if (s == 12345.678) out[threadIdx.x] = s;
}

constexpr size_t kOneBlockLds = 96 * 1024;   // > half the CU's LDS: exactly one block per CU

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    double* out;
    CK(hipMalloc(&out, 1 << 22));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int dev, cus, clk;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev));
    printf("CUs %d  max clock %.0f MHz\n", cus, clk / 1e3);
    const int iters = 20000;
    for (const void* f : {(const void*)fma_chains<1>, (const void*)fma_chains<4>, (const void*)fma_chains<16>,
                          (const void*)op_chains<16, 0>, (const void*)op_chains<16, 1>, (const void*)clock_probe,
                          (const void*)div_chains<1>, (const void*)div_chains<8>})
        CK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kOneBlockLds));
    auto run = [&](const char* name, auto kern, int threads, int ops_per_iter, auto... args) {
        for (int rep = 0; rep < 2; ++rep) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(cus), dim3(threads), kOneBlockLds, 0, out, args..., iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double waves_per_simd = threads / 256.0;
            const double instr = (double)iters * ops_per_iter;         // per wave
            const double ns_per_instr_simd = ms * 1e6 / (instr * waves_per_simd);
            if (rep) printf("%-28s threads=%4d  %.3f ms  %.3f ns per wave-instr per SIMD  (%.2f cyc @2.4GHz)  %.1f TFLOP/s\n",
                            name, threads, ms, ns_per_instr_simd, ns_per_instr_simd * 2.4,
                            2.0 * instr * 64 * (threads / 64) * cus / (ms * 1e-3) / 1e12);
        }
    };
    run("fma 1 chain", fma_chains<1>, 256, 1, 1.0000001, 1e-9);
    run("fma 4 chains", fma_chains<4>, 256, 4, 1.0000001, 1e-9);
    run("fma 16 chains", fma_chains<16>, 256, 16, 1.0000001, 1e-9);
    run("fma 1 chain", fma_chains<1>, 512, 1, 1.0000001, 1e-9);
    run("fma 4 chains", fma_chains<4>, 512, 4, 1.0000001, 1e-9);
    run("fma 16 chains", fma_chains<16>, 512, 16, 1.0000001, 1e-9);
    run("fma 16 chains", fma_chains<16>, 1024, 16, 1.0000001, 1e-9);
    run("mul 16 chains", op_chains<16, 0>, 256, 16, 1.0000001, 1e-9);
    run("add 16 chains", op_chains<16, 1>, 256, 16, 1.0000001, 1e-9);
    run("mul 16 chains", op_chains<16, 0>, 512, 16, 1.0000001, 1e-9);
    run("add 16 chains", op_chains<16, 1>, 512, 16, 1.0000001, 1e-9);
    run("mul 16 chains", op_chains<16, 0>, 1024, 16, 1.0000001, 1e-9);
    run("add 16 chains", op_chains<16, 1>, 1024, 16, 1.0000001, 1e-9);
    run("fma 4 chains", fma_chains<4>, 1024, 4, 1.0000001, 1e-9);
    for (int thr : {256, 512, 1024}) {
        hipLaunchKernelGGL(clock_probe, dim3(cus), dim3(thr), kOneBlockLds, 0, out, 1.0000001, 1e-9, iters);
        CK(hipDeviceSynchronize());
        double h[2];
        CK(hipMemcpy(h, out, 16, hipMemcpyDeviceToHost));
        printf("clock under fp64 fma load (%d threads/CU): %.0f MHz (s_memtime %.0f / s_memrealtime %.0f ticks)\n",
               thr, h[0] / (h[1] / 100.0), h[0], h[1]);
        const int wpb = thr / 64;
        std::vector<double> b(3 * cus * wpb);
        CK(hipMemcpy(b.data(), out + 1024, 8 * b.size(), hipMemcpyDeviceToHost));
        for (int blk = 0; blk < 2; ++blk) {
            printf("   block %d:", blk);
            for (int w = 0; w < wpb; ++w) {
                const double* r = &b[3 * (blk * wpb + w)];
                const unsigned hw = (unsigned)r[2];
                printf(" [w%d simd%u %.0fus]", w, (hw >> 4) & 3, (r[1] - r[0]) / 100);
            }
            printf("\n");
        }
        double mx = 0;
        for (int i = 0; i < cus * wpb; ++i) mx = std::max(mx, b[3 * i + 1] - b[3 * i]);
        printf("   slowest wave %.0f us\n", mx / 100);
    }
    run("div 1 chain (per div)", div_chains<1>, 256, 1, 3.0);
    run("div 8 chains (per div)", div_chains<8>, 256, 8, 3.0);
    run("div 8 chains (per div)", div_chains<8>, 512, 8, 3.0);
    return 0;
}
