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

// Stage the (rows, d) row-major tile at xb into LDS as dev[r][k] = x - loc at s[r * rs + k * ks]:
// CH coalesced loads per thread are issued before any is consumed (one wait per batch, not one per
// element).
template <int CH>
__device__ inline void stage_tile(const double* __restrict__ xb, int rows, int d, const double* s_loc,
                                  double* s, int rs, int ks) {
    const int total = rows * d;
    for (int base = 0; base < total; base += kThreads * CH) {
        double v[CH];
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            const int e = base + threadIdx.x + kThreads * i;
            v[i] = e < total ? xb[e] : 0.0;
        }
#pragma unroll
        for (int i = 0; i < CH; ++i) {
            const int e = base + threadIdx.x + kThreads * i;
            if (e < total) {
                const int r = e / d;
                const int k = e - r * d;
                s[r * rs + k * ks] = v[i] - s_loc[k];
            }
        }
    }
}

__global__ __launch_bounds__(kThreads) void proxy_kernel(ProxyArgs a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int d = a.d;
    double* s_dev = lds;                   // [d][kPitch]
    double* s_y = lds + d * kPitch;        // [d][kPitch]
    double* s_part = s_y + d * kPitch;     // [4][kRows]
    double* s_loc = s_part + 4 * kRows;    // [d]
    const int64_t r0 = (int64_t)blockIdx.x * kRows;
    const int rows = (int)min<int64_t>(kRows, a.n - r0);
    const int tid = threadIdx.x;
    for (int k = tid; k < d; k += kThreads) s_loc[k] = a.loc[k];
    __syncthreads();
    stage_tile<8>(a.x + r0 * d, rows, d, s_loc, s_dev, 1, kPitch);   // rows >= `rows`: unused garbage
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

// ---- 16 < d <= 64: the (64, d) x (d, d) product of a row tile on the matrix cores ----------------
// v_mfma_f64_16x16x4_f64 (gfx950 maps, cdna_hip_programming.md: A[l&15][k=l>>4], B[k=l>>4][l&15],
// D col = l&15, row = (l>>4) + 4 reg).  One product per tile: y = dev @ P^T in T = ceil(d/16) column
// tiles of 16, wave w owning tile w (its B fragments, all k-steps, in VGPRs for the life of the
// block, which loops over 64-row tiles: persistent grid).  The Mahalanobis term is dev . y (the
// same quadratic form as scipy's |dev @ U|^2, U U^T = pinv(cov) = P for the full-rank covariances
// the proxies use; fp64 tolerance like the other summation-order differences), reduced across the
// 16 column lanes with DPP and across the waves through LDS -- one matrix product per row instead
// of two.  Per tile: the x tile is staged (coalesced) into LDS as dev = x - loc, each wave runs
// S = ceil(d/4) k-steps x 4 row subtiles of MFMAs, y goes back through LDS and out as contiguous
// grad rows.
constexpr int kMfmaMaxD = 64;
constexpr int kMfmaMaxS = kMfmaMaxD / 4;
typedef double dbl4 __attribute__((ext_vector_type(4)));

// one DPP lane permutation of a double (quad_perm controls: VALU data movement, no LDS permute)
template <int CTRL>
__device__ inline double dpp_f64(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)b, CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__host__ __device__ inline int mfma_pitch(int dk) { return ((dk + 27) / 32) * 32 + 4; }   // = 4 mod 32 doubles

__global__ __launch_bounds__(kThreads, 2) void proxy_mfma_kernel(ProxyArgs a) {
    extern __shared__ __attribute__((aligned(16))) double lds[];
    const int d = a.d;
    const int S = (d + 3) / 4;
    const int dk = 4 * S;
    const int PD = mfma_pitch(dk);
    const int PY = d + 1;
    const int tz = (d + 15) / 16;            // y column tiles of 16
    double* s_dev = lds;                      // [64][PD]
    double* s_y = s_dev + kRows * PD;         // [64][PY]
    double* s_part = s_y + kRows * PY;        // [4][64]
    double* s_coef = s_part + 4 * kRows;      // [64]
    double* s_loc = s_coef + kRows;           // [d]
    const int tid = threadIdx.x;
    for (int k = tid; k < d; k += kThreads) s_loc[k] = a.loc[k];
    for (int e = tid; e < kRows * (dk - d); e += kThreads) {   // k-padding columns: zero for good
        const int r = e / (dk - d);
        s_dev[r * PD + d + (e - r * (dk - d))] = 0.0;
    }
    const int lane = tid & 63;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int li = lane & 15, lk = lane >> 4;
    const bool has = w < tz;                  // wave w owns y tile w (tz <= 4 for d <= 64)
    const int jcol = 16 * w + li;             // this lane's output column
    double bf[kMfmaMaxS];
#pragma unroll
    for (int s = 0; s < kMfmaMaxS; ++s) {
        const int k = 4 * s + lk;
        bf[s] = (has && s < S && k < d && jcol < d) ? a.P[(int64_t)jcol * d + k] : 0.0;
    }
    const float inv_d = 1.0f / (float)d;
    const int64_t ntiles = (a.n + kRows - 1) / kRows;
    constexpr int kPf = kRows * kMfmaMaxD / kThreads;   // 16 prefetched doubles per thread
    double pf[kPf];
    auto prefetch = [&](int64_t tile) {   // issue the loads of a tile's x rows (consumed later)
        const int64_t r0 = tile * kRows;
        const int total = (int)min<int64_t>(kRows, a.n - r0) * d;
        const double* xb = a.x + r0 * d;
#pragma unroll
        for (int i = 0; i < kPf; ++i) {
            const int e = tid + kThreads * i;
            pf[i] = e < total ? xb[e] : 0.0;
        }
    };
    if (blockIdx.x < ntiles) prefetch(blockIdx.x);
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
        const int64_t r0 = tile * kRows;
        const int rows = (int)min<int64_t>(kRows, a.n - r0);
        __syncthreads();   // s_loc / padding (first tile); the previous tile's readers are done
#pragma unroll
        for (int i = 0; i < kPf; ++i) {
            const int e = tid + kThreads * i;
            if (e < rows * d) {
                const int r = (int)(((float)e + 0.5f) * inv_d);   // exact: e < 4096, d <= 64
                const int k = e - r * d;
                s_dev[r * PD + k] = pf[i] - s_loc[k];
            }
        }
        __syncthreads();
        if (tile + gridDim.x < ntiles) prefetch(tile + gridDim.x);   // overlaps this tile's MFMAs
        // all four 16-row subtiles in one pass: four independent accumulator chains
        dbl4 acc[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] = dbl4{0, 0, 0, 0};
        if (has) {
#pragma unroll
            for (int s = 0; s < kMfmaMaxS; ++s) {
                if (s < S) {
                    double av[4];
#pragma unroll
                    for (int u = 0; u < 4; ++u) av[u] = s_dev[(16 * u + li) * PD + 4 * s + lk];
#pragma unroll
                    for (int u = 0; u < 4; ++u) acc[u] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u], bf[s], acc[u], 0, 0, 0);
                }
            }
        }
        // epilogue: y -> s_y; then every thread takes a quarter of one row's dot dev . y (columns
        // j = q, q + 4, ...; row = tid / 4), the four partials summed with two quad DPP steps
        if (has && jcol < d) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
#pragma unroll
                for (int r = 0; r < 4; ++r) s_y[(16 * u + lk + 4 * r) * PY + jcol] = acc[u][r];
        }
        __syncthreads();
        {
            const int row = tid >> 2, q = tid & 3;
            double part = 0.0;
            for (int j = q; j < d; j += 4) part = fma(s_dev[row * PD + j], s_y[row * PY + j], part);
            part += dpp_f64<0xB1>(part);    // quad_perm [1,0,3,2]
            const double maha = part + dpp_f64<0x4E>(part);   // quad_perm [2,3,0,1]
            if (q == 0) {
                double lq, coef;
                if (a.df > 0.0) {
                    const double t = 0.5 * (a.df + (double)d);
                    lq = a.c_log + -t * log(1.0 + (1.0 / a.df) * maha);
                    coef = (-(a.df + (double)d) / a.df) / (1.0 + maha / a.df);
                } else {
                    lq = -0.5 * (a.c_log + maha);
                    coef = -1.0;
                }
                if (row < rows) a.log_q[r0 + row] = lq;
                s_coef[row] = coef;
            }
        }
        __syncthreads();
        double* gb = a.grad + r0 * d;
        for (int base = 0; base < rows * d; base += 4 * kThreads) {   // LDS reads batched, then stores
            double y[4], c[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int e = min(base + tid + kThreads * i, rows * d - 1);
                const int r = (int)(((float)e + 0.5f) * inv_d);
                y[i] = s_y[r * PY + (e - r * d)];
                c[i] = s_coef[r];
            }
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int e = base + tid + kThreads * i;
                if (e < rows * d) gb[e] = c[i] == -1.0 ? -y[i] : c[i] * y[i];
            }
        }
    }
}

// ---- 16 < d <= 64, streaming form: every wave on its own 16-row blocks, no tiles, no barriers ----
// The transposed product y^T = P dev^T on v_mfma_f64_16x16x4_f64: A = P (16 output columns x 4 k per
// MFMA, register-resident for the whole kernel), B = dev^T (4 k x 16 sample rows), so lane l holds
// sample row l & 15 throughout.  The contraction index k and the output columns are permuted (kmap /
// jmap) such that
//   * the B fragment of MFMA step s for lane group lk = l >> 4 is k = 8(s >> 1) + 2 lk + (s & 1): the
//     lane loads its row's k pairs {8t + 2 lk, +1} with ONE 16-byte load each (16 rows x 64 B per
//     wave instruction), straight from the row-major (n, d) input into registers;
//   * the output column of D row i = lk + 4r in tile c is 16c + 8(r >> 1) + 2 lk + (r & 1), i.e.
//     exactly the input column of step s = 4c + r: each lane already holds dev at every column whose
//     y it holds, so the Mahalanobis term dev . y is a register dot plus two cross-lane adds.
// Summation order differs from NumPy's einsum / scipy's BLAS (fp64 tolerance, as the other kernels).
//
// Two forms (st_tune key 7; profiles/r02_proxy_variants.log has the measured alternatives):
//   * proxy_mfma_buf_kernel (even d, the default): every global access is a buffer instruction whose
//     descriptor covers exactly the current 16-row block, so padding columns and rows past n are
//     out-of-range lanes (loads return 0, stores are dropped) -- no exec-masked branches, a fixed
//     number of memory instructions per iteration, and the compiler's vmcnt waits count exactly
//     (the guarded form's loop waits vmcnt(0) every iteration).  The block's grad rows go through a
//     wave-private LDS slab and out as contiguous 16-B-per-lane stores (whole lines: the fragment
//     layout's own 64-B row pieces straddle lines and cost 91 vs 81 us of memory time).  The next
//     block's loads are issued as soon as dev is formed, under this block's MFMAs; two waves per SIMD.
//   * proxy_mfma_stream_kernel (odd d): 8-B loads/stores guarded per lane, one wave per SIMD with a
//     two-block prefetch.
// Diagnostic builds only (tools/proxy_probe.cpp, never the product library): ST_PROXY_DIAG 1 = no
// MFMAs (memory traffic and epilogue alone), 2 = no grad stores, 3 = neither.
#ifndef ST_PROXY_DIAG
#define ST_PROXY_DIAG 0
#endif

__device__ __forceinline__ int kmap(int s, int lk) { return 8 * (s >> 1) + 2 * lk + (s & 1); }
__device__ __forceinline__ int jmap(int c, int i) { return 16 * c + 8 * (i >> 3) + 2 * (i & 3) + ((i >> 2) & 1); }

// A fragments of P for this lane: pa[c][s] = P[jmap(c, l & 15)][kmap(s, l >> 4)] (zero past d)
template <int T, int S>
__device__ __forceinline__ void load_p_fragments(const ProxyArgs& a, int li, int lk, double (&pa)[T][S]) {
#pragma unroll
    for (int c = 0; c < T; ++c) {
        const int j = jmap(c, li);
#pragma unroll
        for (int s = 0; s < S; ++s) {
            const int k = kmap(s, lk);
            pa[c][s] = (j < a.d && k < a.d) ? a.P[(int64_t)j * a.d + k] : 0.0;
        }
    }
}

// acc[c] = y for this lane's row at output columns jmap(c, lk + 4r), r = 0..3
template <int T, int S>
__device__ __forceinline__ void mfma_rows(const double (&pa)[T][S], const double (&dev)[S], dbl4 (&acc)[T]) {
#pragma unroll
    for (int c = 0; c < T; ++c) acc[c] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < S; ++s)
#pragma unroll
        for (int c = 0; c < T; ++c) {
            if constexpr (ST_PROXY_DIAG & 1) acc[c][s & 3] += pa[c][s] * dev[s];
            else acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(pa[c][s], dev[s], acc[c], 0, 0, 0);
        }
}

// Mahalanobis term of the lane's row (dev . y, step 4c + r <-> output (c, r), then the 4 lanes of the
// row), and the row's log q and grad coefficient
template <int T, int S>
__device__ __forceinline__ void row_terms(const ProxyArgs& a, const double (&dev)[S], const dbl4 (&acc)[T],
                                          double& lq, double& coef) {
    double part = 0.0;
#pragma unroll
    for (int c = 0; c < T; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r)
            if (4 * c + r < S) part = fma(dev[4 * c + r], acc[c][r], part);
    part += __shfl_xor(part, 16);
    const double maha = part + __shfl_xor(part, 32);
    if (a.df > 0.0) {
        const double t = 0.5 * (a.df + (double)a.d);
        lq = a.c_log + -t * log(1.0 + (1.0 / a.df) * maha);
        coef = (-(a.df + (double)a.d) / a.df) / (1.0 + maha / a.df);
    } else {
        lq = -0.5 * (a.c_log + maha);
        coef = -1.0;
    }
}

__device__ __forceinline__ double scaled(double coef, double y) { return coef == -1.0 ? -y : coef * y; }   // Gaussian: exact negation

template <int T, int S>
__global__ __launch_bounds__(kThreads, 2) void proxy_mfma_buf_kernel(ProxyArgs a) {
    static_assert(S % 2 == 0 && S <= 4 * T, "k steps pair up; every step has an output tile");
    typedef double dbl2 __attribute__((ext_vector_type(2)));
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    constexpr int kPairs = S / 2;      // 16-B loads per lane per block; also its 16-B output chunks
    constexpr uint32_t kOob = 0x80000000u;
    const int d = a.d;
    const int lane = threadIdx.x & 63;
    const int li = lane & 15, lk = lane >> 4;
    double pa[T][S];
    load_p_fragments(a, li, lk, pa);
    __shared__ __attribute__((aligned(16))) double s_loc[8 * kPairs];
    __shared__ __attribute__((aligned(16))) double s_out[(kThreads / 64) * 16 * 8 * kPairs];
    double* slab = s_out + (threadIdx.x >> 6) * 16 * d;   // this wave's 16 x d block
    for (int k = threadIdx.x; k < 8 * kPairs; k += kThreads) s_loc[k] = k < d ? a.loc[k] : 0.0;
    __syncthreads();   // the kernel's only barrier
    const int64_t nsub = (a.n + 15) >> 4;
    const int64_t wstride = (int64_t)gridDim.x * (kThreads / 64);
    // wave-uniform (SGPR) block index: the descriptors built from it are scalar, no waterfall loops
    const int64_t sub0 = (int64_t)blockIdx.x * (kThreads / 64) + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // descriptor over block sb's valid rows (none past the end of the array)
    auto block_rsrc = [&](const double* base, int64_t sb, int per_row) {
        const int64_t r0 = sb * 16;
        const int64_t rows = r0 < a.n ? min<int64_t>(16, a.n - r0) : 0;
        const double* p = base + (r0 < a.n ? r0 : 0) * per_row;
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(p), 0, (int)(rows * per_row * 8), 0x00020000);
    };
    auto load = [&](int64_t sb, dbl2 (&v)[kPairs]) {   // row li, column pairs k0 = 8t + 2 lk
        const auto rs = block_rsrc(a.x, sb, d);
#pragma unroll
        for (int t = 0; t < kPairs; ++t) {
            const int k0 = 8 * t + 2 * lk;
            const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(rs, k0 < d ? (uint32_t)((li * d + k0) * 8) : kOob, 0, 0);
            v[t] = dbl2{__builtin_bit_cast(double, u32x2{q.x, q.y}), __builtin_bit_cast(double, u32x2{q.z, q.w})};
        }
    };
    dbl2 buf[kPairs];
    load(sub0, buf);
    for (int64_t sb = sub0; sb < nsub; sb += wstride) {
        double dev[S];
#pragma unroll
        for (int t = 0; t < kPairs; ++t) {
            const dbl2 lp = *reinterpret_cast<const dbl2*>(s_loc + 8 * t + 2 * lk);
            dev[2 * t] = buf[t].x - lp.x;
            dev[2 * t + 1] = buf[t].y - lp.y;
        }
        load(sb + wstride, buf);   // past the end: an empty descriptor, no traffic
        dbl4 acc[T];
        mfma_rows(pa, dev, acc);
        double lq, coef;
        row_terms(a, dev, acc, lq, coef);
        {   // log q from the lk == 0 lanes; rows past n are out of range
            const auto rs = block_rsrc(a.log_q, sb, 1);
            const uint64_t lb = (uint64_t)__double_as_longlong(lq);
            __builtin_amdgcn_raw_buffer_store_b64(u32x2{(unsigned)lb, (unsigned)(lb >> 32)}, rs,
                                                  lk == 0 ? (uint32_t)(li * 8) : kOob, 0, 0);
        }
        if constexpr (ST_PROXY_DIAG & 2) continue;
        // grad rows into the slab at their global layout (row li at slab[li d]) ...
#pragma unroll
        for (int c = 0; c < T; ++c)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int j0 = 16 * c + 8 * h + 2 * lk;
                if (j0 < d)
                    *reinterpret_cast<dbl2*>(slab + li * d + j0) =
                        dbl2{scaled(coef, acc[c][2 * h]), scaled(coef, acc[c][2 * h + 1])};
            }
        __builtin_amdgcn_wave_barrier();
        // ... and out as contiguous 16-B-per-lane stores of the whole 16 d-double block
        const auto rs = block_rsrc(a.grad, sb, d);
#pragma unroll
        for (int i = 0; i < kPairs; ++i) {
            const int e = 2 * (lane + 64 * i);
            const bool in = e < 16 * d;
            const dbl2 v = *reinterpret_cast<const dbl2*>(slab + (in ? e : 0));
            const uint64_t v0 = (uint64_t)__double_as_longlong(v.x), v1 = (uint64_t)__double_as_longlong(v.y);
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{(unsigned)v0, (unsigned)(v0 >> 32), (unsigned)v1, (unsigned)(v1 >> 32)},
                                                   rs, in ? (uint32_t)(e * 8) : kOob, 0, 0);
        }
        __builtin_amdgcn_wave_barrier();   // the slab's reads are issued before the next block's writes
    }
}

template <int T, int S>
__global__ __launch_bounds__(kThreads, 1) void proxy_mfma_stream_kernel(ProxyArgs a) {
    static_assert(S % 2 == 0 && S <= 4 * T, "k steps pair up; every step has an output tile");
    constexpr int kDepth = 2;   // blocks in flight per wave
    const int d = a.d;
    const int lane = threadIdx.x & 63;
    const int li = lane & 15, lk = lane >> 4;
    double pa[T][S];
    load_p_fragments(a, li, lk, pa);
    __shared__ __attribute__((aligned(16))) double s_loc[8 * (S / 2)];
    for (int k = threadIdx.x; k < 8 * (S / 2); k += kThreads) s_loc[k] = k < d ? a.loc[k] : 0.0;
    __syncthreads();   // the kernel's only barrier
    const int64_t nsub = (a.n + 15) >> 4;
    const int64_t wstride = (int64_t)gridDim.x * (kThreads / 64);
    int64_t sub = (int64_t)blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
    auto load = [&](int64_t sb, double (&v)[S]) {
        int64_t row = sb * 16 + li;
        row = row < a.n ? row : a.n - 1;   // rows past n: a valid row, results dropped
        const double* xr = a.x + row * d;
#pragma unroll
        for (int t = 0; t < S / 2; ++t) {
            const int k0 = 8 * t + 2 * lk;
            v[2 * t] = k0 < d ? xr[k0] : 0.0;
            v[2 * t + 1] = k0 + 1 < d ? xr[k0 + 1] : 0.0;
        }
    };
    double nx[kDepth][S];
#pragma unroll
    for (int q = 0; q < kDepth; ++q)
        if (sub + q * wstride < nsub) load(sub + q * wstride, nx[q]);
    for (; sub < nsub; sub += wstride) {
        double dev[S];
#pragma unroll
        for (int s = 0; s < S; ++s) dev[s] = nx[0][s] - s_loc[kmap(s, lk)];
#pragma unroll
        for (int q = 0; q + 1 < kDepth; ++q)
#pragma unroll
            for (int s = 0; s < S; ++s) nx[q][s] = nx[q + 1][s];
        if (sub + kDepth * wstride < nsub) load(sub + kDepth * wstride, nx[kDepth - 1]);
        dbl4 acc[T];
        mfma_rows(pa, dev, acc);
        double lq, coef;
        row_terms(a, dev, acc, lq, coef);
        const int64_t row = sub * 16 + li;
        if (row < a.n) {
            if (lk == 0) a.log_q[row] = lq;
            if constexpr (ST_PROXY_DIAG & 2) continue;
            double* gr = a.grad + row * d;
#pragma unroll
            for (int c = 0; c < T; ++c)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const int j0 = 16 * c + 8 * h + 2 * lk;
                    if (j0 < d) gr[j0] = scaled(coef, acc[c][2 * h]);
                    if (j0 + 1 < d) gr[j0 + 1] = scaled(coef, acc[c][2 * h + 1]);
                }
        }
    }
}

}  // namespace

int64_t proxy_lds_bytes(int d) { return ((int64_t)2 * d * kPitch + 4 * kRows + d) * 8; }

static int64_t proxy_mfma_lds_bytes(int d) {
    const int dk = 4 * ((d + 3) / 4);
    return ((int64_t)kRows * mfma_pitch(dk) + (int64_t)kRows * (d + 1) + 5 * kRows + d) * 8;
}

// st_tune key 7: 0 auto (16 < d <= 64: the buffer form for even d, the guarded streaming form for
// odd d), 1 always the VALU kernel, 2 the LDS-tiled matrix-core kernel (round 1), 3 the guarded
// streaming form for any d, 4 the buffer form (even d; odd d runs 3)
static int g_proxy_mode = 0;

int proxy_tune(int value) {
    if (value < 0 || value > 4) return -1;
    g_proxy_mode = value;
    return 0;
}

static hipError_t grid_for(const ProxyArgs& a, int bpc, int64_t& grid) {
    int dev = 0, cus = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
    const int64_t waves = ((a.n + 15) / 16 + 1) / 2;   // at least two blocks per wave
    grid = (waves + kThreads / 64 - 1) / (kThreads / 64);
    if (grid > (int64_t)cus * bpc) grid = (int64_t)cus * bpc;
    if (grid < 1) grid = 1;
    return hipSuccess;
}

template <int T, int S>
static hipError_t launch_stream_ts(const ProxyArgs& a, hipStream_t s, bool buffered) {
    int64_t grid = 0;
    hipError_t e = grid_for(a, buffered ? 2 : 1, grid);
    if (e != hipSuccess) return e;
    if (buffered) proxy_mfma_buf_kernel<T, S><<<dim3((unsigned)grid), kThreads, 0, s>>>(a);
    else proxy_mfma_stream_kernel<T, S><<<dim3((unsigned)grid), kThreads, 0, s>>>(a);
    return hipGetLastError();
}

// T = ceil(d / 16) output tiles, S = 2 ceil(d / 8) k steps
static hipError_t launch_stream(const ProxyArgs& a, hipStream_t s, bool buffered) {
    switch ((a.d + 7) / 8) {
        case 3: return launch_stream_ts<2, 6>(a, s, buffered);
        case 4: return launch_stream_ts<2, 8>(a, s, buffered);
        case 5: return launch_stream_ts<3, 10>(a, s, buffered);
        case 6: return launch_stream_ts<3, 12>(a, s, buffered);
        case 7: return launch_stream_ts<4, 14>(a, s, buffered);
        default: return launch_stream_ts<4, 16>(a, s, buffered);
    }
}

hipError_t launch_proxy(const ProxyArgs& a, hipStream_t s) {
    if (a.n <= 0) return hipSuccess;
    if (g_proxy_mode != 1 && g_proxy_mode != 2 && a.d > 16 && a.d <= kMfmaMaxD)
        return launch_stream(a, s, a.d % 2 == 0 && g_proxy_mode != 3);
    if (g_proxy_mode == 2 && a.d > 16 && a.d <= kMfmaMaxD) {
        const int64_t lds = proxy_mfma_lds_bytes(a.d);   // <= 69 KB at d = 64
        static bool s_set = false;
        if (!s_set) {
            const hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(proxy_mfma_kernel),
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
            if (e != hipSuccess) return e;
            s_set = true;
        }
        const int64_t tiles = (a.n + kRows - 1) / kRows;
        const int64_t grid = tiles < 2 * 256 ? tiles : 2 * 256;
        proxy_mfma_kernel<<<dim3((unsigned)grid), kThreads, (size_t)lds, s>>>(a);
        return hipGetLastError();
    }
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
