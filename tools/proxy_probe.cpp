// Diagnostic timing of the proxy kernels at the config-5 shape (n = 5e5, d = 50) outside Python:
// builds proxy.hip with -DST_PROXY_DIAG=<0..3> (scripts/build_probes.sh) and times every st_tune
// key-7 mode with hipEvents.  Inputs are synthetic; results are not checked (tests do that).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../gradient-free-mcmc-postprocessing_amd/csrc/stein_internal.hpp"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 500000;
    const int d = argc > 2 ? atoi(argv[2]) : 50;
    std::vector<double> hx(n * d), hp(d * d), hl(d);
    for (int64_t i = 0; i < n * d; ++i) hx[i] = (double)((i * 2654435761u) % 1000) / 500.0 - 1.0;
    for (int i = 0; i < d * d; ++i) hp[i] = (i % (d + 1) == 0) ? 2.0 : 0.01;
    for (int i = 0; i < d; ++i) hl[i] = 0.01 * i;
    double *x, *P, *loc, *lq, *g;
    CK(hipMalloc(&x, n * d * 8)); CK(hipMalloc(&P, d * d * 8)); CK(hipMalloc(&loc, d * 8));
    CK(hipMalloc(&lq, n * 8)); CK(hipMalloc(&g, n * d * 8));
    CK(hipMemcpy(x, hx.data(), n * d * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(P, hp.data(), d * d * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(loc, hl.data(), d * 8, hipMemcpyHostToDevice));
    st::ProxyArgs a{};
    a.x = x; a.loc = loc; a.U = P; a.P = P; a.n = n; a.d = d; a.df = 0.0; a.c_log = 1.0; a.log_q = lq; a.grad = g;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    printf("diag %d  n %lld  d %d  bytes %.1f MB\n", ST_PROXY_DIAG, (long long)n, d, (16.0 * d + 8) * n / 1e6);
    for (int mode : {2, 3, 4}) {
        if (st::proxy_tune(mode) != 0) continue;
        for (int w = 0; w < 3; ++w) CK(st::launch_proxy(a, nullptr));
        CK(hipDeviceSynchronize());
        std::vector<float> t;
        for (int r = 0; r < 20; ++r) {
            CK(hipEventRecord(e0, nullptr));
            CK(st::launch_proxy(a, nullptr));
            CK(hipEventRecord(e1, nullptr));
            CK(hipEventSynchronize(e1));
            float ms; CK(hipEventElapsedTime(&ms, e0, e1)); t.push_back(ms * 1e3f);
        }
        std::sort(t.begin(), t.end());
        printf("mode %d: median %.1f us  (%.2f TB/s)\n", mode, t[t.size() / 2], (16.0 * d + 8) * n / (t[t.size() / 2] * 1e-6) / 1e12);
    }
    return 0;
}
