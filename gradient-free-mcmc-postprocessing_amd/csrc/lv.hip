// Lotka-Volterra posterior inputs for Stein thinning, batched over parameter points: the gradient
// of the log posterior from the forward sensitivity equations, and the log target density.
//
// Reference (code/src/lotka_volterra.py; Sensitivity_analysis.ipynb cells 16, 40, 46):
//   grad_log_posterior(theta) = sum_k J_k^T C^-1 (y_k - u(t_k)) - log(theta) / theta
//     u, J = du/dtheta from solve_ivp(lotka_volterra_sensitivity, [0, 25], [1, 1, 0 x 8],
//     dense_output=True).sol(t): RK45 (Dormand-Prince), rtol 1e-3, atol 1e-6 (scipy defaults)
//   log_target_density(log_theta) = sum_k mvn.logpdf(y_k - u(t_k), 0, C) + sum_j norm.logpdf(log_theta_j)
//     u from solve_ivp(lotka_volterra, ...) (the 2-state system: its own step sequence)
// One thread integrates one parameter point with scipy's algorithm step for step: initial step
// selection (common.select_initial_step), the accept / reject loop of RungeKutta._step_impl
// (SAFETY 0.9, factors in [0.2, 10], error exponent -1/5, RMS error norm), the tableau as scipy
// holds it (rk45_tableau.hpp, generated), and dense output y = h Q p(x) + y_old per accepted step
// with OdeSolution's segment rule (t in (t_j, t_j+1] -> segment j).  The observation points are
// consumed in time order while the integration proceeds, so no trajectory is stored; the gradient
// sums over time points sequentially (np.sum(axis=0) of the (t_n, 4) terms).  Summation orders
// inside the BLAS products scipy uses (np.dot of stages) are not reproducible bit for bit:
// results agree with scipy to rounding as long as the step sequences coincide.
#include <hip/hip_runtime.h>

#include "rk45_tableau.hpp"
#include "stein_internal.hpp"

namespace st {
namespace {

constexpr int kLvThreads = 64;
constexpr int kLvOverflow = 3;     // status: more accepted steps than the step table holds (internal)
constexpr int kLvStepRec = 56;     // doubles per recorded step: t_old, 1/h, k_begin, k_end, y[10], hQ[10][4], pad

template <int NS>
__device__ inline void lv_rhs(const double th[4], const double* y, double* f) {
    const double th1 = th[0], th2 = th[1], th3 = th[2], th4 = th[3];
    const double u1 = y[0], u2 = y[1];
    f[0] = th1 * u1 - th2 * u1 * u2;
    f[1] = th4 * u1 * u2 - th3 * u2;
    if constexpr (NS == 10) {
        const double w1 = y[2], w2 = y[3], w3 = y[4], w4 = y[5];
        const double w5 = y[6], w6 = y[7], w7 = y[8], w8 = y[9];
        f[2] = u1 + (th1 - th2 * u2) * w1 - th2 * u1 * w5;
        f[3] = -u1 * u2 + (th1 - th2 * u2) * w2 - th2 * u1 * w6;
        f[4] = (th1 - th2 * u2) * w3 - th2 * u1 * w7;
        f[5] = (th1 - th2 * u2) * w4 - th2 * u1 * w8;
        f[6] = th4 * u2 * w1 + (th4 * u1 - th3) * w5;
        f[7] = th4 * u2 * w2 + (th4 * u1 - th3) * w6;
        f[8] = -u2 + th4 * u2 * w3 + (th4 * u1 - th3) * w7;
        f[9] = u1 * u2 + th4 * u2 * w4 + (th4 * u1 - th3) * w8;
    }
}

// scipy common.norm: np.linalg.norm(x) / x.size ** 0.5
template <int NS>
__device__ inline double rms(const double* v) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NS; ++i) s += v[i] * v[i];
    return sqrt(s) / sqrt((double)NS);
}

// NS = 10: gradient of the log posterior -> out[4 i + j]; NS = 2: per-time log-likelihood terms ->
// work[k n + i] (summed by lv_logdens_finish).
// RECORD (NS = 10, two-phase gradient): instead of evaluating the observation points while it
// integrates, the thread stores every accepted step's dense-output polynomial (t_old, 1/h, the
// observation range, y_old, hQ) in the step table a.steps[i][s] and leaves the points to
// lv_dense_kernel (one wave per parameter point); a point with more than a.step_cap accepted
// steps gets status kLvOverflow and is recomputed by the single-phase kernel (ONLY_OVERFLOW).
template <int NS, bool RECORD = false, bool ONLY_OVERFLOW = false>
__global__ __launch_bounds__(kLvThreads) void lv_kernel(LvArgs a) {
    const int64_t i = (int64_t)blockIdx.x * kLvThreads + threadIdx.x;
    if (i >= a.n) return;
    if constexpr (ONLY_OVERFLOW) {
        if (a.status[i] != kLvOverflow) return;
    }
    double th[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) th[j] = a.theta[4 * i + j];
    const double rtol = a.rtol, atol = a.atol;
    double y[NS], f[NS], K[rk45::kStages + 1][NS];
#pragma unroll
    for (int c = 0; c < NS; ++c) y[c] = c < 2 ? a.u0[c] : 0.0;
    double t = a.t0;
    const double t_bound = a.t1;
    lv_rhs<NS>(th, y, f);
    // ---- select_initial_step (order = error estimator order 4, max_step = inf, direction +1)
    double h_abs;
    {
        const double interval = fabs(t_bound - t);
        double sc[NS], v[NS];
#pragma unroll
        for (int c = 0; c < NS; ++c) sc[c] = atol + fabs(y[c]) * rtol;
#pragma unroll
        for (int c = 0; c < NS; ++c) v[c] = y[c] / sc[c];
        const double d0 = rms<NS>(v);
#pragma unroll
        for (int c = 0; c < NS; ++c) v[c] = f[c] / sc[c];
        const double d1 = rms<NS>(v);
        double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
        h0 = fmin(h0, interval);
        double y1[NS], f1[NS];
#pragma unroll
        for (int c = 0; c < NS; ++c) y1[c] = y[c] + h0 * 1.0 * f[c];
        lv_rhs<NS>(th, y1, f1);
#pragma unroll
        for (int c = 0; c < NS; ++c) v[c] = (f1[c] - f[c]) / sc[c];
        const double d2 = rms<NS>(v) / h0;
        double h1;
        if (d1 <= 1e-15 && d2 <= 1e-15) h1 = fmax(1e-6, h0 * 1e-3);
        else h1 = pow(0.01 / fmax(d1, d2), 1.0 / (rk45::kOrder + 1));
        h_abs = fmin(fmin(100 * h0, h1), interval);   // max_step = inf
    }
    int kk = 0;                       // next observation point
    int nrec = 0;                     // RECORD: accepted steps stored
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    int32_t status = 0;
    for (int64_t step = 0;; ++step) {
        if (t == t_bound) break;      // OdeSolver.step: finished
        if (step >= a.max_steps) { status = 2; break; }
        const double min_step = 10 * fabs(nextafter(t, INFINITY) - t);
        if (h_abs < min_step) h_abs = min_step;   // (h_abs > max_step = inf never)
        bool rejected = false;
        double t_new, h, y_new[NS], f_new[NS];
        for (;;) {
            if (h_abs < min_step) { status = 1; break; }
            h = h_abs;
            t_new = t + h;
            if (t_new - t_bound > 0) t_new = t_bound;
            h = t_new - t;
            h_abs = fabs(h);
            // rk_step
#pragma unroll
            for (int c = 0; c < NS; ++c) K[0][c] = f[c];
#pragma unroll
            for (int s = 1; s < rk45::kStages; ++s) {
                double ys[NS];
#pragma unroll
                for (int c = 0; c < NS; ++c) {
                    double dy = K[0][c] * rk45::A[s][0];
#pragma unroll
                    for (int j = 1; j < s; ++j) dy += K[j][c] * rk45::A[s][j];
                    ys[c] = y[c] + dy * h;
                }
                lv_rhs<NS>(th, ys, K[s]);
            }
#pragma unroll
            for (int c = 0; c < NS; ++c) {
                double bsum = K[0][c] * rk45::B[0];
#pragma unroll
                for (int j = 1; j < rk45::kStages; ++j) bsum += K[j][c] * rk45::B[j];
                y_new[c] = y[c] + h * bsum;
            }
            lv_rhs<NS>(th, y_new, f_new);
#pragma unroll
            for (int c = 0; c < NS; ++c) K[rk45::kStages][c] = f_new[c];
            double ev[NS];
#pragma unroll
            for (int c = 0; c < NS; ++c) {
                double e = K[0][c] * rk45::E[0];
#pragma unroll
                for (int j = 1; j <= rk45::kStages; ++j) e += K[j][c] * rk45::E[j];
                const double scale = atol + fmax(fabs(y[c]), fabs(y_new[c])) * rtol;
                ev[c] = e * h / scale;
            }
            const double error_norm = rms<NS>(ev);
            if (error_norm < 1) {
                double factor = error_norm == 0 ? rk45::kMaxFactor
                                                : fmin(rk45::kMaxFactor, rk45::kSafety * pow(error_norm, rk45::kErrorExponent));
                if (rejected) factor = fmin(1.0, factor);
                h_abs *= factor;
                break;
            }
            h_abs *= fmax(rk45::kMinFactor, rk45::kSafety * pow(error_norm, rk45::kErrorExponent));
            rejected = true;
        }
        if (status) break;
        // dense output of this step: Q = K^T P; points t in (t_old, t_new] (all remaining at the end).
        // scipy evaluates h Q p(x) + y_old with p = (x, x^2, x^3, x^4); here hQ is formed once per
        // step and p is applied in Horner form, x = (t - t_old) * (1 / h): the dense output feeds
        // nothing back into the step sequence, so these roundings only move the result within the
        // 1e-8 tolerance of the BLAS-ordered reference (tests/test_gpu_lv.py), at ~45 instead of
        // ~110 fp64 instructions per observation point
        const double t_old = t;
        const double hd = t_new - t_old;
        const double inv_hd = 1.0 / hd;
        double Q[NS][rk45::kDenseOrder];
#pragma unroll
        for (int c = 0; c < NS; ++c)
#pragma unroll
            for (int q = 0; q < rk45::kDenseOrder; ++q) {
                double s = K[0][c] * rk45::P[0][q];
#pragma unroll
                for (int j = 1; j <= rk45::kStages; ++j) s += K[j][c] * rk45::P[j][q];
                Q[c][q] = hd * s;
            }
        static_assert(rk45::kDenseOrder == 4, "Horner form below is written for RK45's quartic");
        const bool last = t_new - t_bound >= 0;
        if constexpr (RECORD) {
            // observation range of this step: (t_old, t_new], everything left at the last step
            int k_end = a.t_n;
            if (!last) {
                int lo = kk, hi = a.t_n;   // first index with t_eval > t_new
                while (lo < hi) {
                    const int mid = (lo + hi) >> 1;
                    if (a.t_eval[mid] <= t_new) lo = mid + 1; else hi = mid;
                }
                k_end = lo;
            }
            if (k_end > kk) {
                if (nrec >= a.step_cap) { status = kLvOverflow; break; }
                double* r = a.steps + ((int64_t)i * a.step_cap + nrec) * kLvStepRec;
                r[0] = t_old;
                r[1] = inv_hd;
                r[2] = (double)kk;
                r[3] = (double)k_end;
#pragma unroll
                for (int c = 0; c < NS; ++c) {
                    r[4 + c] = y[c];
#pragma unroll
                    for (int q = 0; q < rk45::kDenseOrder; ++q) r[4 + NS + 4 * c + q] = Q[c][q];
                }
                ++nrec;
                kk = k_end;
            }
        }
        while (!RECORD && kk < a.t_n && (last || a.t_eval[kk] <= t_new)) {
            const double x = (a.t_eval[kk] - t_old) * inv_hd;
            double u[NS];
#pragma unroll
            for (int c = 0; c < NS; ++c)
                u[c] = __builtin_fma(x, __builtin_fma(x, __builtin_fma(x, __builtin_fma(x, Q[c][3], Q[c][2]), Q[c][1]),
                                                      Q[c][0]), y[c]);
            const double r0 = a.y_obs[2 * kk] - u[0], r1 = a.y_obs[2 * kk + 1] - u[1];
            if constexpr (NS == 10) {
                const double g0 = a.cinv[0] * r0 + a.cinv[1] * r1;
                const double g1 = a.cinv[2] * r0 + a.cinv[3] * r1;
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[j] += u[2 + j] * g0 + u[6 + j] * g1;
            } else {
                const double z0 = r0 * a.U[0] + r1 * a.U[2];
                const double z1 = r0 * a.U[1] + r1 * a.U[3];
                a.work[(int64_t)kk * a.n + i] = -0.5 * (a.c_log + (z0 * z0 + z1 * z1));
            }
            ++kk;
        }
        t = t_new;
#pragma unroll
        for (int c = 0; c < NS; ++c) { y[c] = y_new[c]; f[c] = f_new[c]; }
    }
    a.status[i] = status;
    if constexpr (RECORD) {
        a.nsteps[i] = nrec;
        if (status == kLvOverflow) return;
        if (status) {
#pragma unroll
            for (int j = 0; j < 4; ++j) a.out[4 * i + j] = NAN;
        }
        return;
    }
    if constexpr (NS == 10) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            a.out[4 * i + j] = status ? NAN : acc[j] - log(th[j]) / th[j];
    } else if (status) {
        for (; kk < a.t_n; ++kk) a.work[(int64_t)kk * a.n + i] = NAN;
    }
}

// numpy pairwise_sum (loops_utils.h.src, PW_BLOCKSIZE 128) over a strided column: the recursion
// (sum(first n2) + sum(rest), n2 = n/2 rounded down to a multiple of 8, leaves <= 128) walked
// post-order with an explicit stack
__device__ inline double pairwise_leaf(const double* a, int64_t n, int64_t stride) {
    if (n < 8) {
        double res = -0.0;
        for (int64_t k = 0; k < n; ++k) res += a[k * stride];
        return res;
    }
    double r[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) r[q] = a[q * stride];
    int64_t k;
    for (k = 8; k < n - (n % 8); k += 8)
#pragma unroll
        for (int q = 0; q < 8; ++q) r[q] += a[(k + q) * stride];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; k < n; ++k) res += a[k * stride];
    return res;
}

__device__ double pairwise_sum_strided(const double* a, int64_t n, int64_t stride) {
    struct Frame { int64_t off, cnt; int state; double left; };
    Frame st[40];   // depth <= log2(n / 128) + 1
    int sp = 0;
    st[0] = {0, n, 0, 0.0};
    double ret = 0.0;
    while (sp >= 0) {
        Frame& f = st[sp];
        if (f.cnt <= 128) {
            ret = pairwise_leaf(a + f.off * stride, f.cnt, stride);
            --sp;
            continue;
        }
        int64_t n2 = f.cnt / 2;
        n2 -= n2 % 8;
        if (f.state == 0) {
            f.state = 1;
            st[sp + 1] = {f.off, n2, 0, 0.0};
            ++sp;
        } else if (f.state == 1) {
            f.left = ret;
            f.state = 2;
            st[sp + 1] = {f.off + n2, f.cnt - n2, 0, 0.0};
            ++sp;
        } else {
            ret = f.left + ret;
            --sp;
        }
    }
    return ret;
}

// log_likelihood = np.sum(per-time terms) (0.0 + pairwise), log_prior = np.sum(norm.logpdf(log_theta))
__global__ __launch_bounds__(kLvThreads) void lv_logdens_finish(LvArgs a) {
    const int64_t i = (int64_t)blockIdx.x * kLvThreads + threadIdx.x;
    if (i >= a.n) return;
    const double ll = 0.0 + pairwise_sum_strided(a.work + i, a.t_n, a.n);
    double lp = -0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const double x = a.log_theta[4 * i + j];
        lp += -(x * x) / 2.0 - a.norm_logc;
    }
    lp = 0.0 + lp;
    a.out[i] = ll + lp;
}

__device__ __forceinline__ int wave_sum_int(int v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// Phase B of the two-phase gradient: one wave per parameter point.  Each recorded step's
// observation range is cut into pieces of at most P points, P the smallest piece length that
// yields at most 64 pieces (one per lane, one round); lane L takes piece L, loads its step record
// once (y_old, hQ, t_old, 1/h: no search or reload inside a piece) and accumulates
// J^T C^-1 (y_k - u(t_k)) over the piece in its own partial sums; the wave then adds the 64 partial
// sums.  The per-point sum is thus reassociated (pieces, then a tree) against the reference's
// sequential np.sum -- within the same 1e-8 tolerance as the BLAS-ordered stages
// (tests/test_gpu_lv.py).
// LDS: the observation times and data (3 t_n doubles, shared by every parameter point) are staged in
// LDS once per block of WPB points and read from there.  Round 4, PMC (profiles/r04_lv_stall.json):
// with each lane of a wave at a different observation index, every t_eval / y_obs load touched 64
// cache lines and the texture address unit was busy ~80 % of the kernel while the VALU issued on
// ~60 % of SIMD cycles.
template <int WPB, bool LDS, int KP>
__global__ __launch_bounds__(64 * WPB) void lv_dense_kernel(LvArgs a) {
    const int64_t i = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    __shared__ int pstart_sh[WPB][65];
    extern __shared__ double obs_sh[];      // LDS: t[t_n], y0[t_n], y1[t_n]
    if constexpr (LDS) {
        for (int e = threadIdx.x; e < a.t_n; e += 64 * WPB) {
            obs_sh[e] = a.t_eval[e];
            obs_sh[a.t_n + e] = a.y_obs[2 * e];
            obs_sh[2 * a.t_n + e] = a.y_obs[2 * e + 1];
        }
        __syncthreads();
    }
    if (i >= a.n) return;                   // (wave-uniform: the whole wave leaves)
    if (a.status[i] != 0) return;          // NaN already written, or the overflow kernel's point
    const int ns = a.nsteps[i];            // <= step_cap <= 64
    const double* tab = a.steps + (int64_t)i * a.step_cap * kLvStepRec;
    int* pstart = pstart_sh[threadIdx.x >> 6];
    int kb_s = 0, len = 0;                  // step `lane`: first observation, count
    if (lane < ns) {
        const double* r = tab + (int64_t)lane * kLvStepRec;
        kb_s = (int)r[2];
        len = (int)r[3] - kb_s;
    }
    // smallest P with sum_s ceil(len_s / P) <= 64 KP (ns <= 64 guarantees P = max len qualifies)
    constexpr int kPieces = 64 * KP;
    int plo = (a.t_n + kPieces - 1) / kPieces, phi = len;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) phi = max(phi, __shfl_xor(phi, off));
    if (plo > phi) plo = phi;
    while (plo < phi) {
        const int mid = (plo + phi) >> 1;
        if (wave_sum_int((len + mid - 1) / mid) <= kPieces) phi = mid; else plo = mid + 1;
    }
    const int P = plo > 0 ? plo : 1;
    const int np = (len + P - 1) / P;
    int incl = np;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const int o = __shfl_up(incl, off);
        if (lane >= off) incl += o;
    }
    pstart[lane + 1] = incl;
    if (lane == 0) pstart[0] = 0;
    __builtin_amdgcn_wave_barrier();
    const int total = __shfl(incl, 63);   // <= 64 KP
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    const double c0 = a.cinv[0], c1 = a.cinv[1], c2 = a.cinv[2], c3 = a.cinv[3];
    // KP pieces per lane, dealt in a snake (round u: lane L takes piece 64u + L, or 64u + 63 - L
    // in odd rounds), so a lane whose first piece is a step's short remainder tends to get a long one
    // next (round 4: KP = 2 cuts the busiest lane's share of a point from 1 / 0.75 of the even split
    // to 1 / 0.86, tools/lv_piece_balance.py)
#pragma unroll 1
    for (int u = 0; u < KP; ++u) {
        const int pc = 64 * u + ((u & 1) ? 63 - lane : lane);
        if (pc >= total) continue;
        int lo = 0, hi = ns - 1;           // step s with pstart[s] <= pc < pstart[s + 1]
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (pstart[mid] <= pc) lo = mid; else hi = mid - 1;
        }
        const double* r = tab + (int64_t)lo * kLvStepRec;
        const double2* r2 = reinterpret_cast<const double2*>(r);
        const double2 h0 = r2[0], h1 = r2[1];
        const double t_old = h0.x, inv_hd = h0.y;
        const int kb = (int)h1.x + (pc - pstart[lo]) * P;
#if defined(ST_LV_DIAG) && ST_LV_DIAG == 1   // diagnostic build: preamble and record loads only
        const int ke = kb + 1;
#else
        const int ke = kb + P < (int)h1.y ? kb + P : (int)h1.y;
#endif
        double y[10], Q[10][4];
#pragma unroll
        for (int c = 0; c < 10; c += 2) {
            const double2 v = r2[2 + c / 2];
            y[c] = v.x;
            y[c + 1] = v.y;
        }
#pragma unroll
        for (int c = 0; c < 10; ++c) {
            const double2 v0 = r2[7 + 2 * c], v1 = r2[8 + 2 * c];
            Q[c][0] = v0.x; Q[c][1] = v0.y; Q[c][2] = v1.x; Q[c][3] = v1.y;
        }
        // the observation (t_k, y_k) loads of the next two points are in flight while this pair
        // computes (L2-served, shared by every parameter point: without the prefetch each
        // iteration waited a full load latency at three waves per SIMD); same order of the sums
        auto obs = [&](int k, double& tk, double& o0, double& o1) {
            const int kc = k < ke ? k : ke - 1;    // past the piece: a harmless reload, unused
            if constexpr (LDS) {
                tk = obs_sh[kc];
                o0 = obs_sh[a.t_n + kc];
                o1 = obs_sh[2 * a.t_n + kc];
            } else {
                tk = a.t_eval[kc];
                o0 = a.y_obs[2 * kc];
                o1 = a.y_obs[2 * kc + 1];
            }
        };
        auto point = [&](double tk, double o0, double o1) {
            const double x = (tk - t_old) * inv_hd;
            double u[10];
#pragma unroll
            for (int c = 0; c < 10; ++c)
                u[c] = __builtin_fma(x, __builtin_fma(x, __builtin_fma(x, __builtin_fma(x, Q[c][3], Q[c][2]),
                                                                       Q[c][1]), Q[c][0]), y[c]);
            const double r0 = o0 - u[0], r1 = o1 - u[1];
            const double g0 = c0 * r0 + c1 * r1;
            const double g1 = c2 * r0 + c3 * r1;
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] += u[2 + j] * g0 + u[6 + j] * g1;
        };
        double ta, a0, a1, tb, b0, b1;
        obs(kb, ta, a0, a1);
        obs(kb + 1, tb, b0, b1);
        int k = kb;
        for (; k + 1 < ke; k += 2) {
            const double t0 = ta, p0 = a0, p1 = a1, t1 = tb, q0 = b0, q1 = b1;
            obs(k + 2, ta, a0, a1);
            obs(k + 3, tb, b0, b1);
            point(t0, p0, p1);
            point(t1, q0, q1);
        }
        if (k < ke) point(ta, a0, a1);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        double v = acc[j];
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
        acc[j] = v;
    }
    if (lane == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const double th = a.theta[4 * i + j];
            a.out[4 * i + j] = acc[j] - log(th) / th;
        }
    }
}

}  // namespace

// st_tune key 17: phase B variant -- 0 / -1 auto (observations in LDS, 8 points per block: 1.31-1.32 ms
// for 113 143 points against 1.43 with 12 per block), 1 = the observations read from global memory
// (the round-3 kernel, 1.59-1.61 ms; profiles/r04_lv_obs_lds_ab.log)
static int g_lv_global_obs = 0;
int lv_tune(int value) {
    if (value < -1 || value > 1) return -1;
    g_lv_global_obs = value < 0 ? 0 : value;
    return 0;
}

// st_tune key 18: phase-B pieces per lane (1, 2, 3; -1 = automatic)
static int g_lv_pieces = -1;
int lv_pieces_tune(int value) {
    if (value != -1 && (value < 1 || value > 3)) return -1;
    g_lv_pieces = value;
    return 0;
}

int64_t lv_grad_workspace_bytes(int64_t n, int step_cap) {
    return n * ((int64_t)step_cap * kLvStepRec * 8 + 8);
}

hipError_t launch_lv(const LvArgs& a, bool gradient, hipStream_t s) {
    if (a.n <= 0) return hipSuccess;
    const unsigned blocks = (unsigned)((a.n + kLvThreads - 1) / kLvThreads);
    if (gradient && a.steps) {   // two-phase: record, dense per wave, overflowed points single-phase
        if (a.step_cap < 1 || a.step_cap > 64) return hipErrorInvalidValue;   // one step per lane in lv_dense_kernel
        lv_kernel<10, true><<<blocks, kLvThreads, 0, s>>>(a);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return e;
        // observations in LDS when they fit next to the kernel's static LDS (pstart_sh: 8 x 65 ints) in
        // the default 64 KB per block (t_n <= 2643; ADVICE r04: the static part counts too)
        const size_t obs_bytes = (size_t)a.t_n * 3 * sizeof(double);
        const int kp = g_lv_pieces > 0 ? g_lv_pieces : 1;
        if (obs_bytes + sizeof(int) * 8 * 65 <= 65536 && g_lv_global_obs != 1) {
            const unsigned nb = (unsigned)((a.n + 7) / 8);
            if (kp == 2) lv_dense_kernel<8, true, 2><<<nb, 512, obs_bytes, s>>>(a);
            else if (kp == 3) lv_dense_kernel<8, true, 3><<<nb, 512, obs_bytes, s>>>(a);
            else lv_dense_kernel<8, true, 1><<<nb, 512, obs_bytes, s>>>(a);
        } else {
            lv_dense_kernel<4, false, 1><<<(unsigned)((a.n + 3) / 4), 256, 0, s>>>(a);
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
        lv_kernel<10, false, true><<<blocks, kLvThreads, 0, s>>>(a);
        return hipGetLastError();
    }
    if (gradient) {
        lv_kernel<10><<<blocks, kLvThreads, 0, s>>>(a);
        return hipGetLastError();
    }
    lv_kernel<2><<<blocks, kLvThreads, 0, s>>>(a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    lv_logdens_finish<<<blocks, kLvThreads, 0, s>>>(a);
    return hipGetLastError();
}

}  // namespace st
