// Measurement probe (not product code): fp64 throughput of the persistent kernel's register-row
// inner loop (pair_value_ct<4, FAST> or the compact pair_compact_ct<4> + running-sum fma + argmin
// scan) at 1 / 2 / 3 / 4 waves per SIMD and IL rows per scheduling group (sched_barrier every IL
// rows), with no exchange: every "step" reads the next winner row from a small table (block-uniform)
// and sweeps the thread's RT register rows.  Reports ns per row-step per CU.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -o tools/pair_rate tools/pair_rate.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "../gradient-free-mcmc-postprocessing_amd/csrc/stein_math.hpp"

using namespace st;

template <int NT, int RT, bool CMP, int IL>
__global__ __launch_bounds__(NT, 1) void rows_kernel(const double* x, const double* g, const double* wins,
                                                     int steps, double l, double tr, double* out) {
    constexpr int D = 4;
    double xr[RT][D], gr[RT][D], ar[RT];
    const int tid = threadIdx.x;
#pragma unroll
    for (int q = 0; q < RT; ++q) {
        const int64_t row = ((int64_t)blockIdx.x * RT + q) * NT + tid;
#pragma unroll
        for (int k = 0; k < D; ++k) { xr[q][k] = x[row * D + k]; gr[q][k] = g[row * D + k]; }
        ar[q] = 1.0;
    }
    const double l2 = l * l, m3l2 = -3.0 * l2;
    double bv = 0;
    uint32_t bq = 0;
    for (int t = 0; t < steps; ++t) {
        double xj[D], gj[D];
        const double* wr = wins + (t & 63) * 2 * D;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            xj[k] = wr[k];
            gj[k] = wr[D + k];
        }
#pragma unroll
        for (int q = 0; q < RT; ++q) {
            const double kv = CMP ? pair_compact_ct<D>(xr[q], gr[q], xj, gj, l, m3l2, tr)
                                  : pair_value_ct<D, true>(xr[q], gr[q], xj, gj, l, l2, tr);
            ar[q] = add_twice<true>(ar[q], kv);
            if (q == 0) { bv = ar[q]; bq = 0; }
            else { const bool tk = ar[q] < bv; bv = tk ? ar[q] : bv; bq = tk ? q : bq; }
            if ((q % IL) == IL - 1) __builtin_amdgcn_sched_barrier(0);
        }
        if (bv == -1.0) out[tid] = bq;   // keep the scan live
    }
    double s = 0;
#pragma unroll
    for (int q = 0; q < RT; ++q) s += ar[q];
    out[(int64_t)blockIdx.x * NT + tid] = s + bv + bq;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

template <int NT, int RT, bool CMP, int IL>
static int run(const double* x, const double* g, const double* w, double* out, int steps) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    rows_kernel<NT, RT, CMP, IL><<<256, NT>>>(x, g, w, 10, 0.37, 1.48, out);
    CK(hipDeviceSynchronize());
    hipEventRecord(a);
    rows_kernel<NT, RT, CMP, IL><<<256, NT>>>(x, g, w, steps, 0.37, 1.48, out);
    hipEventRecord(b);
    CK(hipEventSynchronize(b));
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double rows_per_cu = (double)NT * RT;
    printf("%s NT=%4d RT=%2d IL=%d rows/CU=%5.0f  %8.3f ms  %6.3f ns per row-step per CU  %.3f us per 7812-row step\n",
           CMP ? "compact" : "exact  ", NT, RT, IL, rows_per_cu, ms, ms * 1e6 / steps / rows_per_cu,
           ms * 1e3 / steps / rows_per_cu * 7812);
    return 0;
}

__global__ void fill(double* p, int64_t n, uint64_t seed, double scale) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        p[i] = ((double)(z >> 11) * 0x1.0p-53 - 0.5) * scale;
    }
}

int main() {
    const int64_t n = 256ll * 4096 * 2;
    double *x, *g, *w, *out;
    CK(hipMalloc(&x, n * 4 * 8));
    CK(hipMalloc(&g, n * 4 * 8));
    CK(hipMalloc(&w, 64 * 8 * 8));
    CK(hipMalloc(&out, n * 8));
    fill<<<1024, 256>>>(x, n * 4, 1, 4.0);
    fill<<<1024, 256>>>(g, n * 4, 2, 6.0);
    fill<<<8, 64>>>(w, 64 * 8, 3, 4.0);
    CK(hipDeviceSynchronize());
    const int steps = 2000;
    run<512, 8, false, 2>(x, g, w, out, steps);
    run<256, 16, true, 1>(x, g, w, out, steps);
    run<256, 16, true, 2>(x, g, w, out, steps);
    run<256, 16, true, 4>(x, g, w, out, steps);
    run<256, 16, true, 8>(x, g, w, out, steps);
    run<512, 8, true, 1>(x, g, w, out, steps);
    run<512, 8, true, 2>(x, g, w, out, steps);
    run<512, 8, true, 4>(x, g, w, out, steps);
    run<512, 8, true, 8>(x, g, w, out, steps);
    run<768, 5, true, 1>(x, g, w, out, steps);
    run<768, 5, true, 5>(x, g, w, out, steps);
    run<1024, 4, true, 1>(x, g, w, out, steps);
    run<1024, 4, true, 2>(x, g, w, out, steps);
    return 0;
}
