// Measurement probe (not product code): issue cost of the fp64 transcendentals (v_rcp_f64,
// v_rsq_f64) next to v_fma_f64 at one and two waves per SIMD, and their accuracy on [1, 2^185]
// (the persistent kernel's fast range for qf) -- the inputs for replacing the three reciprocal
// seeds of the Stein pair's divisions.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/_diag/trans_rate tools/trans_rate.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>

#include <algorithm>
#include <vector>

template <int CH, int OP>   // OP 0: 2 fma per iter; 1: rcp + fma; 2: rsq + fma; 3: 3 fma + rcp (pair-like mix)
__global__ void chains(double* out, double a, double b, int iters) {
    double acc[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) acc[c] = 1.5 + threadIdx.x * 1e-3 + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            if constexpr (OP == 0) acc[c] = __builtin_fma(__builtin_fma(acc[c], a, b), a, b);
            else if constexpr (OP == 1) acc[c] = __builtin_fma(__builtin_amdgcn_rcp(acc[c]), a, b);
            else if constexpr (OP == 2) acc[c] = __builtin_fma(__builtin_amdgcn_rsq(acc[c]), a, b);
            else acc[c] = __builtin_fma(__builtin_fma(__builtin_fma(__builtin_amdgcn_rcp(acc[c]), a, b), a, b), a, b);
        }
    }
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += acc[c];
    if (s == 12345.678) out[threadIdx.x] = s;
}

__global__ void accuracy(const double* x, double* r, double* q, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { r[i] = __builtin_amdgcn_rcp(x[i]); q[i] = __builtin_amdgcn_rsq(x[i]); }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    double* out;
    CK(hipMalloc(&out, 1 << 20));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int dev, cus;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    const int iters = 20000;
    auto run = [&](const char* name, auto kern, int threads, double slots_per_iter) {
        float best = 1e30f;
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(cus), dim3(threads), 96 * 1024, 0, out, 1.0000001, 1e-9, iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            best = std::min(best, ms);
        }
        const double per_iter_ns = best * 1e6 / ((double)iters * 16 * threads / 256.0);   // per wave-iteration per SIMD
        printf("%-34s threads=%4d  %.3f ms  %.3f ns per chain-iteration per SIMD\n", name, threads, best, per_iter_ns);
        return per_iter_ns;
    };
    for (const void* f : {(const void*)chains<16, 0>, (const void*)chains<16, 1>, (const void*)chains<16, 2>, (const void*)chains<16, 3>})
        CK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024));
    for (int threads : {256, 512}) {
        const double f2 = run("2 fma", chains<16, 0>, threads, 2);
        const double rc = run("rcp + fma", chains<16, 1>, threads, 2);
        const double rs = run("rsq + fma", chains<16, 2>, threads, 2);
        const double mix = run("rcp + 3 fma", chains<16, 3>, threads, 4);
        printf("  => at %d threads/CU: fma %.3f ns, rcp ~ %.2f fma, rsq ~ %.2f fma (rcp + 3 fma = %.2f fma)\n", threads,
               f2 / 2, rc / (f2 / 2) - 1, rs / (f2 / 2) - 1, mix / (f2 / 2));
    }
    // accuracy on [1, 2^185] log-uniform
    const int n = 1 << 22;
    std::vector<double> hx(n), hr(n), hq(n);
    uint64_t z = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {
        z ^= z << 13; z ^= z >> 7; z ^= z << 17;
        const double u = (double)(z >> 11) * 0x1.0p-53;
        hx[i] = ldexp(1.0 + u, (int)((z >> 3) % 185));
    }
    double *dx, *dr, *dq;
    CK(hipMalloc(&dx, n * 8)); CK(hipMalloc(&dr, n * 8)); CK(hipMalloc(&dq, n * 8));
    CK(hipMemcpy(dx, hx.data(), n * 8, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(accuracy, dim3(n / 256), dim3(256), 0, 0, dx, dr, dq, n);
    CK(hipMemcpy(hr.data(), dr, n * 8, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hq.data(), dq, n * 8, hipMemcpyDeviceToHost));
    long double mr = 0, mq = 0;
    for (int i = 0; i < n; ++i) {
        const long double x = hx[i];
        mr = std::max(mr, fabsl((long double)hr[i] * x - 1.0L));
        mq = std::max(mq, fabsl((long double)hq[i] * (long double)hq[i] * x - 1.0L) / 2);
    }
    printf("max relative error on [1, 2^185]: v_rcp_f64 %.3Le (2^%.1f)  v_rsq_f64 %.3Le (2^%.1f)\n", mr,
           (double)log2l(mr), mq, (double)log2l(mq));
    return 0;
}
