// Proxy producers for the gradient-free operator: log q and grad log q of a Gaussian or Student-t
// proxy at every sample row, the O(n d^2) host prep before thin_gf.
//
//   Gaussian  (code/src/thinning.py:15-16, gaussian_thin):
//     log_q = scipy.stats.multivariate_normal.logpdf(x, mean, cov)
//           = -0.5 * (rank * log(2 pi) + log_pdet + |(x - mean) @ U|^2)          (c_log = rank*log2pi + log_pdet)
//     grad  = -inv(cov) @ (x - mean)
//   Student-t (Gradient_free_Student_t.ipynb cells 29/31/40, thin_gf_t):
//     log_q = scipy.stats.multivariate_t.logpdf(x, loc, shape, df)
//           = (A - B - C - D) - t * log(1 + (1/df) * |(x - loc) @ U|^2),  t = (df + d) / 2
//     grad  = (-(df + d) / df) / (1 + m / df) * (inv(shape) @ (x - loc)),   m = (x-loc).inv(shape).(x-loc)
// U is scipy's _PSD factor (U U^T = pinv(cov)), computed on the host like the reference does; P =
// np.linalg.inv(cov).  Constant parts are computed on the host with the reference's operation order;
// the per-row dot products differ from NumPy/BLAS in summation order only (fp64 tolerance).
//
// Layout: x, grad row-major (n, d) exactly as the caller's NumPy arrays; one block = 64 rows
// (lane = row) x 4 waves (column groups).  The block stages its (64, d) tile of x - loc transposed
// in LDS (pitch 65: conflict-free both ways), each wave computes 4 output columns at a time for all
// 64 rows with U / P entries as wave-uniform scalar operands, and the tile of inv(P) dev goes back
// through LDS so the grad rows are written contiguously.  Bound: fp64 VALU for d >~ 8 (4 d^2 flop per
// row vs 16 d + 8 bytes), HBM below.
#include <hip/hip_runtime.h>

#include "stein_internal.hpp"

namespace st {
namespace {

constexpr int kRows = 64;
constexpr int kPitch = kRows + 1;
constexpr int kThreads = 256;

__global__ __launch_bounds__(kThreads) void proxy_kernel(ProxyArgs a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int d = a.d;
    double* s_dev = lds;                   // [d][kPitch]
    double* s_y = lds + d * kPitch;        // [d][kPitch]
    double* s_part = s_y + d * kPitch;     // [4][kRows]
    const int64_t r0 = (int64_t)blockIdx.x * kRows;
    const int rows = (int)min<int64_t>(kRows, a.n - r0);
    const int tid = threadIdx.x;
    const double* xb = a.x + r0 * d;
    for (int e = tid; e < kRows * d; e += kThreads) {
        const int r = e / d;
        const int k = e - r * d;
        s_dev[k * kPitch + r] = r < rows ? xb[e] - a.loc[k] : 0.0;
    }
    __syncthreads();
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    double mz = 0.0;
    for (int j0 = 4 * w; j0 < d; j0 += 16) {
        double z0 = 0.0, z1 = 0.0, z2 = 0.0, z3 = 0.0;
        double y0 = 0.0, y1 = 0.0, y2 = 0.0, y3 = 0.0;
        const int nc = min(4, d - j0);
        if (nc == 4) {
            for (int k = 0; k < d; ++k) {
                const double dv = s_dev[k * kPitch + lane];
                const double* u = a.U + (int64_t)k * d + j0;
                z0 = fma(dv, u[0], z0);
                z1 = fma(dv, u[1], z1);
                z2 = fma(dv, u[2], z2);
                z3 = fma(dv, u[3], z3);
                y0 = fma(a.P[(int64_t)(j0 + 0) * d + k], dv, y0);
                y1 = fma(a.P[(int64_t)(j0 + 1) * d + k], dv, y1);
                y2 = fma(a.P[(int64_t)(j0 + 2) * d + k], dv, y2);
                y3 = fma(a.P[(int64_t)(j0 + 3) * d + k], dv, y3);
            }
        } else {
            for (int k = 0; k < d; ++k) {
                const double dv = s_dev[k * kPitch + lane];
                const double* u = a.U + (int64_t)k * d + j0;
                z0 = fma(dv, u[0], z0);
                y0 = fma(a.P[(int64_t)j0 * d + k], dv, y0);
                if (nc > 1) { z1 = fma(dv, u[1], z1); y1 = fma(a.P[(int64_t)(j0 + 1) * d + k], dv, y1); }
                if (nc > 2) { z2 = fma(dv, u[2], z2); y2 = fma(a.P[(int64_t)(j0 + 2) * d + k], dv, y2); }
            }
        }
        mz = fma(z0, z0, mz);
        s_y[j0 * kPitch + lane] = y0;
        if (nc > 1) { mz = fma(z1, z1, mz); s_y[(j0 + 1) * kPitch + lane] = y1; }
        if (nc > 2) { mz = fma(z2, z2, mz); s_y[(j0 + 2) * kPitch + lane] = y2; }
        if (nc > 3) { mz = fma(z3, z3, mz); s_y[(j0 + 3) * kPitch + lane] = y3; }
    }
    s_part[w * kRows + lane] = mz;
    __syncthreads();
    if (w == 0) {
        const double maha = ((s_part[lane] + s_part[kRows + lane]) + s_part[2 * kRows + lane]) +
                            s_part[3 * kRows + lane];
        double lq, coef;
        if (a.df > 0.0) {
            double my = 0.0;
            for (int k = 0; k < d; ++k) my = fma(s_dev[k * kPitch + lane], s_y[k * kPitch + lane], my);
            const double t = 0.5 * (a.df + (double)d);
            lq = a.c_log + -t * log(1.0 + (1.0 / a.df) * maha);
            coef = (-(a.df + (double)d) / a.df) / (1.0 + my / a.df);
        } else {
            lq = -0.5 * (a.c_log + maha);
            coef = -1.0;
        }
        if (lane < rows) a.log_q[r0 + lane] = lq;
        s_part[lane] = coef;   // wave 0 only: rows' coefficients (read after the barrier)
    }
    __syncthreads();
    double* gb = a.grad + r0 * d;
    for (int e = tid; e < rows * d; e += kThreads) {
        const int r = e / d;
        const int k = e - r * d;
        const double y = s_y[k * kPitch + r];
        const double c = s_part[r];
        gb[e] = c == -1.0 ? -y : c * y;   // Gaussian: exact negation, as -np.einsum(...)
    }
}

}  // namespace

int64_t proxy_lds_bytes(int d) { return ((int64_t)2 * d * kPitch + 4 * kRows) * 8; }

hipError_t launch_proxy(const ProxyArgs& a, hipStream_t s) {
    if (a.n <= 0) return hipSuccess;
    const int64_t lds = proxy_lds_bytes(a.d);
    static int64_t s_lds_set = 0;   // raise the dynamic-LDS ceiling once (up to 130 KB at d = 128)
    if (lds > 65536 && lds > s_lds_set) {
        const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(proxy_kernel),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
        s_lds_set = lds;
    }
    const int64_t blocks = (a.n + kRows - 1) / kRows;
    proxy_kernel<<<dim3((unsigned)blocks), kThreads, (size_t)lds, s>>>(a);
    return hipGetLastError();
}

}  // namespace st
