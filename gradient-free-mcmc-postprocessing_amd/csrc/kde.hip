// KDE proxy for the gradient-free operator: log q and grad log q of a Gaussian kernel density
// estimate at every query point -- what the reference's Gaussian-mixture study feeds thin_gf
// (Gaussian_mixture.ipynb cells 42-48: jax.scipy.stats.gaussian_kde(sample.T, bw_method='silverman'),
// log q = kde.logpdf, grad log q = jax.grad of it; cell 51 the weighted KDE).  With the whitening
// factor L (Cholesky of the KDE precision, lower) and whitened data p_i = x_i L, queries q_j = y_j L:
//   a_ij  = log w_i + log_norm - 0.5 |p_i - q_j|^2
//   log q_j = logsumexp_i a_ij
//   grad_j  = (sum_i s_ij p_i - q_j) L^T,   s_ij = exp(a_ij - log q_j)      (the autodiff of log q)
// Two sweeps over the data per query tile: the row maximum of a_ij, then the shifted exponential
// sums (one exp per pair).  One query per thread; data points staged 256 at a time in LDS and read
// as block-uniform broadcasts (as the energy-distance kernel K7).  Sums are sequential in i
// (scipy's logsumexp sums pairwise: fp64 tolerance).
#include <hip/hip_runtime.h>

#include "stein_internal.hpp"

namespace st {
namespace {

constexpr int kKdeBlock = 256;

struct KdeArgs {
    const double* p;      // whitened data, SoA (d, ldp)
    int64_t ldp, n;
    const double* logw;   // (n) log weights, or nullptr: logw0 for every point
    double logw0;
    const double* q;      // whitened queries, SoA (d, ldq)
    int64_t ldq, m;
    double log_norm;
    const double* L;      // (d, d) row-major whitening factor (grad = v L^T)
    double* log_q;        // (m)
    double* grad;         // (m, d) row-major
};

template <int D>
__global__ __launch_bounds__(kKdeBlock) void kde_kernel(KdeArgs a) {
    constexpr int R = kKdeBlock;
    __shared__ double sp[D][R];
    __shared__ double sw[R];
    const int tid = threadIdx.x;
    const int64_t j = (int64_t)blockIdx.x * R + tid;
    const bool live = j < a.m;
    double qj[D];
#pragma unroll
    for (int k = 0; k < D; ++k) qj[k] = live ? a.q[k * a.ldq + j] : 0.0;
    auto stage = [&](int64_t i0) -> int {
        __syncthreads();
        const int64_t i = i0 + tid;
        if (i < a.n) {
#pragma unroll
            for (int k = 0; k < D; ++k) sp[k][tid] = a.p[k * a.ldp + i];
            sw[tid] = a.logw ? a.logw[i] : a.logw0;
        }
        __syncthreads();
        return (int)((a.n - i0) < R ? (a.n - i0) : R);
    };
    auto arg = [&](int e) {
        double ss = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const double dk = sp[k][e] - qj[k];
            ss += dk * dk;
        }
        return sw[e] + (a.log_norm - 0.5 * ss);
    };
    double mx = -INFINITY;
    for (int64_t i0 = 0; i0 < a.n; i0 += R) {
        const int cnt = stage(i0);
        for (int e = 0; e < cnt; ++e) mx = fmax(mx, arg(e));
    }
    const double shift = mx == -INFINITY ? 0.0 : mx;   // all weights zero: log q = -inf
    double s = 0.0, sm[D];
#pragma unroll
    for (int k = 0; k < D; ++k) sm[k] = 0.0;
    for (int64_t i0 = 0; i0 < a.n; i0 += R) {
        const int cnt = stage(i0);
        for (int e = 0; e < cnt; ++e) {
            const double t = exp(arg(e) - shift);
            s += t;
#pragma unroll
            for (int k = 0; k < D; ++k) sm[k] = fma(t, sp[k][e], sm[k]);
        }
    }
    if (!live) return;
    a.log_q[j] = log(s) + shift;
    double v[D];
#pragma unroll
    for (int k = 0; k < D; ++k) v[k] = sm[k] / s - qj[k];
#pragma unroll
    for (int k = 0; k < D; ++k) {
        double gk = 0.0;
#pragma unroll
        for (int l = 0; l < D; ++l) gk = fma(v[l], a.L[k * D + l], gk);
        a.grad[j * D + k] = gk;
    }
}

// runtime d (9 .. kMaxDim): coordinates of the query re-read from L1/L2, data staged 32 at a time
constexpr int kKdeRowsRt = 32;

__global__ __launch_bounds__(kKdeBlock) void kde_rt_kernel(KdeArgs a, int d, double* scratch) {
    constexpr int R = kKdeRowsRt;
    __shared__ double sp[kMaxDim][R];
    __shared__ double sw[R];
    const int tid = threadIdx.x;
    const int64_t j = (int64_t)blockIdx.x * kKdeBlock + tid;
    const bool live = j < a.m;
    const int64_t jc = live ? j : 0;
    double* smj = scratch + jc * d;   // (m, d) per-query weighted sums
    auto stage = [&](int64_t i0) -> int {
        const int cnt = (int)((a.n - i0) < R ? (a.n - i0) : R);
        __syncthreads();
        for (int e = tid; e < d * R; e += kKdeBlock) {
            const int k = e / R, r = e % R;
            if (r < cnt) sp[k][r] = a.p[(int64_t)k * a.ldp + i0 + r];
        }
        if (tid < cnt) sw[tid] = a.logw ? a.logw[i0 + tid] : a.logw0;
        __syncthreads();
        return cnt;
    };
    auto arg = [&](int e) {
        double ss = 0.0;
        for (int k = 0; k < d; ++k) {
            const double dk = sp[k][e] - a.q[(int64_t)k * a.ldq + jc];
            ss += dk * dk;
        }
        return sw[e] + (a.log_norm - 0.5 * ss);
    };
    double mx = -INFINITY;
    for (int64_t i0 = 0; i0 < a.n; i0 += R) {
        const int cnt = stage(i0);
        for (int e = 0; e < cnt; ++e) mx = fmax(mx, arg(e));
    }
    const double shift = mx == -INFINITY ? 0.0 : mx;
    if (live)
        for (int k = 0; k < d; ++k) smj[k] = 0.0;
    double s = 0.0;
    for (int64_t i0 = 0; i0 < a.n; i0 += R) {
        const int cnt = stage(i0);
        for (int e = 0; e < cnt; ++e) {
            const double t = exp(arg(e) - shift);
            s += t;
            if (live)
                for (int k = 0; k < d; ++k) smj[k] = fma(t, sp[k][e], smj[k]);
        }
    }
    if (!live) return;
    a.log_q[j] = log(s) + shift;
    for (int k = 0; k < d; ++k) smj[k] = smj[k] / s - a.q[(int64_t)k * a.ldq + j];
    for (int k = 0; k < d; ++k) {
        double gk = 0.0;
        for (int l = 0; l < d; ++l) gk = fma(smj[l], a.L[k * d + l], gk);
        a.grad[j * d + k] = gk;
    }
}

}  // namespace

int64_t kde_workspace_bytes(int64_t m, int d) { return d > 8 ? m * d * (int64_t)sizeof(double) : 0; }

hipError_t launch_kde(const double* p, int64_t ldp, int64_t n, const double* logw, double logw0,
                      const double* q, int64_t ldq, int64_t m, int d, double log_norm, const double* L,
                      double* log_q, double* grad, double* ws, hipStream_t s) {
    KdeArgs a{p, ldp, n, logw, logw0, q, ldq, m, log_norm, L, log_q, grad};
    const unsigned grid = (unsigned)((m + kKdeBlock - 1) / kKdeBlock);
    switch (d) {
        case 1: kde_kernel<1><<<grid, kKdeBlock, 0, s>>>(a); break;
        case 2: kde_kernel<2><<<grid, kKdeBlock, 0, s>>>(a); break;
        case 3: kde_kernel<3><<<grid, kKdeBlock, 0, s>>>(a); break;
        case 4: kde_kernel<4><<<grid, kKdeBlock, 0, s>>>(a); break;
        case 5: kde_kernel<5><<<grid, kKdeBlock, 0, s>>>(a); break;
        case 6: kde_kernel<6><<<grid, kKdeBlock, 0, s>>>(a); break;
        case 7: kde_kernel<7><<<grid, kKdeBlock, 0, s>>>(a); break;
        case 8: kde_kernel<8><<<grid, kKdeBlock, 0, s>>>(a); break;
        default: kde_rt_kernel<<<grid, kKdeBlock, 0, s>>>(a, d, ws); break;
    }
    return hipGetLastError();
}

}  // namespace st
