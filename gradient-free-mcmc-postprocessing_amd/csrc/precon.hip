// Pairwise distances of the 'med' preconditioner's subsample on the GPU (stein_thinning.kernel
// make_precon: med = np.median(scipy.spatial.distance.pdist(sub)), the reference's median heuristic,
// report.tex:432).  scipy 1.15's euclidean pdist sums (u_k - v_k)^2 over k in order and takes the
// correctly rounded square root; this kernel does the same operations in the same order (built with
// -ffp-contract=off, so no fma), so every distance is bit-identical (tests/test_gpu_precon.py), in
// scipy's condensed order: pair (i, j), i < j, at i k - i (i + 1) / 2 + j - i - 1.
// One block per row i, threads over j; the rows are row-major (k, d) and small (k <= a few 1000).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "stein_internal.hpp"

namespace st {

namespace {

constexpr int kPdistBlock = 256;

__global__ __launch_bounds__(kPdistBlock) void pdist_kernel(const double* __restrict__ rows, int64_t k, int d,
                                                            double* __restrict__ out) {
    const int64_t i = blockIdx.x;
    const int64_t base = i * k - i * (i + 1) / 2 - i - 1;   // + j: the condensed index of (i, j)
    const double* u = rows + i * d;
    for (int64_t j = i + 1 + threadIdx.x; j < k; j += kPdistBlock) {
        const double* v = rows + j * d;
        double s = 0.0;
        for (int q = 0; q < d; ++q) {
            const double t = u[q] - v[q];
            s = s + t * t;
        }
        out[base + j] = __builtin_sqrt(s);
    }
}

}  // namespace

hipError_t launch_pdist(const double* rows, int64_t k, int d, double* out, hipStream_t s) {
    pdist_kernel<<<(unsigned)k, kPdistBlock, 0, s>>>(rows, k, d, out);
    return hipGetLastError();
}

}  // namespace st
