// Per-pair IMQ Stein-kernel arithmetic for gfx950 (fp64, VALU; no MFMA: pairwise scalar work).
//
// Reproduces, rounding for rounding, NumPy's evaluation of the reference's vfk0_imq
// (restated at JAX_Stein_Thinning.ipynb cell 27, json ~354-361; maths report.tex:853-868) with an
// isotropic preconditioner Gamma^-1 = l*I:
//   qf  = 1 + SEQ_k fl(fl(l*dk)*dk)      t1 = fl(-3*SEQ_k fl(fl(l2*dk)*dk)) / qf^2.5
//   t2  = fl(tr + SEQ_k fl(fl(l*(sa_k-sb_k))*dk)) / qf^1.5
//   t3  = PAIRWISE_k fl(sa_k*sb_k) / sqrt(qf)        k = fl(fl(t1+t2)+t3)
// SEQ = left-to-right (NumPy C-order axis-0 reduction), PAIRWISE = NumPy pairwise_sum.
// The bit model is oracle/stein_ref.c; this file must stay in lock-step with it.
// Compile with -ffp-contract=off: every mul/add above is a separately rounded op.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang fp contract(off)

namespace st {

// qf^1.5 and qf^2.5 correctly rounded to ~2^-100 (then rounded once), from s = sqrt(qf) (correctly
// rounded) and its exact residual e = qf - s^2 (fma).  sqrt(qf) = s + e/(2s) + O(2^-106 s), and the
// correction term q * e/(2s) equals (s/2) e to 2^-53 relative of a term that is itself ~2^-53 of the
// result -- so no division is needed: q^1.5 = hi + lo (double-double, hi = fl(q s)).  q^2.5 is
// q (hi + lo) as a second double-double product (q hi exactly by fma, + q lo), rounded once.  An
// overflowing power is +inf (the double-double tail would turn it into inf - inf).
__device__ __forceinline__ void pow_15_25(double q, double& p15, double& p25, double& s) {
    s = __builtin_sqrt(q);
    const double e = __builtin_fma(-s, s, q);
    const double hi = q * s;
    double lo = __builtin_fma(q, s, -hi);
    lo = __builtin_fma(0.5 * s, e, lo);
    p15 = __builtin_isinf(hi) ? hi : hi + lo;
    const double hi2 = q * hi;
    double lo2 = __builtin_fma(q, hi, -hi2);
    lo2 = __builtin_fma(q, lo, lo2);
    p25 = __builtin_isinf(hi2) ? hi2 : hi2 + lo2;
}

__device__ __forceinline__ double finish_pair(double qs, double t1s, double t2s, double t3s,
                                              double tr) {
    const double qf = 1.0 + qs;
    double p15, p25, s;
    pow_15_25(qf, p15, p25, s);
    const double t1 = (-3.0 * t1s) / p25;
    const double t2 = (tr + t2s) / p15;
    const double t3 = t3s / s;
    return (t1 + t2) + t3;
}

// ---- range-guarded fast path ---------------------------------------------------------------
// When every coordinate and score component of BOTH points is 0 or has magnitude in
// [2^-60, 2^60], and l is in [2^-60, 2^60] (fast_range_ok), every intermediate of the pair is 0 or
// a normal number far from the limits: differences are 0 or >= 2^-112 (multiples of 2^-112),
// per-k products 0 or in [2^-344, 2^242], their sums 0 or >= 2^-396 (multiples of the smallest
// ulp), qf in [1, 2^185], p25 <= 2^463, and every quotient is normal.  In that range
//   * the IEEE f64 division a / b needs no scaling and no special-case fix-up: the quotient is
//     q0 + rem r rounded once with r = RN(1/b) (div_by_recip), all intermediates normal;
//   * its sqrt sequence (scale-if-below-2^-767, v_rsq, Goldschmidt + 2 residual corrections,
//     +0/-0/+inf class fix-up) never scales and never takes the fix-up;
// (|k| < 2^190 there, so the running-sum update A + 2k may also be the single fma(2, k, A): 2k is
// exact.)  So fast_sqrt and div_by_recip below (no scaling / fix-up steps) return the same bits
// as '/' and sqrt, correctly rounded.  The only deviations are signs of zero: a -0 numerator gives
// +0 instead of -0 in t1/t3, and t3s drops the leading "0.0 +".  k = fl(fl(t1 + t2) + t3) is
// unaffected because t2 = fl(tr + t2s) / p15 is never -0 (tr > 0), so a zero t1 or t3 only ever
// meets a t2 (or t1 + t2) that is +0 or non-zero.
// A + 2k: fl(A + fl(2k)); in the fast range 2k is exact, so one fma gives the same bits
template <bool FAST>
__device__ __forceinline__ double add_twice(double A, double k) {
    if constexpr (FAST) return __builtin_fma(2.0, k, A);
    else return A + 2.0 * k;
}

__device__ __forceinline__ int fast_range_ok(double v) {   // 1 / 0, branch-free
    const double a = __builtin_fabs(v);
    return (int)(a == 0.0) | ((int)(a >= 0x1p-60) & (int)(a <= 0x1p60));
}

// sqrt of x in [1, 2^185], correctly rounded (the compiler's sequence without its scaling and
// class fix-up); h ~ 1 / (2 sqrt x) to ~2^-48 comes out as a by-product
__device__ __forceinline__ double fast_sqrt(double x, double& h_out) {
    double g = x * __builtin_amdgcn_rsq(x);
    double h = __builtin_amdgcn_rsq(x) * 0.5;
    const double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double dd = __builtin_fma(-g, g, x);
    g = __builtin_fma(dd, h, g);
    dd = __builtin_fma(-g, g, x);
    h_out = h;
    return __builtin_fma(dd, h, g);
}

// RN(1/b) from a seed y0 within ~2^-48 of 1/b: two Newton steps (error 2^-96, then 2^-150 before the
// final rounding -- far inside the >= 2^-106 relative gap between 1/b and any rounding midpoint, so
// the result is the correctly rounded reciprocal whatever the seed's exact bits)
__device__ __forceinline__ double recip2(double b, double y0) {
    double e = __builtin_fma(-b, y0, 1.0);
    double y = __builtin_fma(y0, e, y0);
    e = __builtin_fma(-b, y, 1.0);
    return __builtin_fma(y, e, y);
}

// a / b from r = RN(1/b): q0 = fl(a r) is within an ulp of a/b, the remainder a - b q0 is exact, and
// q0 + rem r rounded once is the correctly rounded quotient (Markstein) -- the IEEE result of '/'
__device__ __forceinline__ double div_by_recip(double a, double b, double r) {
    const double q = a * r;
    const double rem = __builtin_fma(-b, q, a);
    return __builtin_fma(rem, r, q);
}

// Fast range (see above): the same bits as finish_pair.  The three reciprocals need no v_rcp_f64
// (a quarter-rate transcendental with 2^-24 accuracy: ~3.3 fma issue slots each at two waves per
// SIMD, profiles/r02_trans_rate.log): 1/s is seeded by the sqrt's own h (2h ~ 1/s to 2^-48), and
// 1/p15, 1/p25 by rs^3, rs^5 (within ~2^-50 of them since p15, p25 are the correctly rounded
// s^3-, s^5-sized powers); each seed is refined by recip2 to the correctly rounded reciprocal.
__device__ __forceinline__ double finish_pair_fast(double qs, double t1s, double t2s, double t3s,
                                                   double tr) {
    const double q = 1.0 + qs;
    double h;
    const double s = fast_sqrt(q, h);
    const double e = __builtin_fma(-s, s, q);
    // e is a multiple of 2^-104 (s >= 1), so 0.5*e is exact and (0.5*s)*e == s*(0.5*e) exactly
    const double he = 0.5 * e;
    const double hi = q * s;
    double lo = __builtin_fma(q, s, -hi);
    lo = __builtin_fma(s, he, lo);
    const double p15 = hi + lo;
    const double hi2 = q * hi;
    double lo2 = __builtin_fma(q, hi, -hi2);
    lo2 = __builtin_fma(q, lo, lo2);
    const double p25 = hi2 + lo2;
    const double rs = recip2(s, h + h);
    const double rs2 = rs * rs;
    const double rs3 = rs2 * rs;
    const double r15 = recip2(p15, rs3);
    const double r25 = recip2(p25, rs3 * rs2);
    const double t1 = div_by_recip(-3.0 * t1s, p25, r25);
    const double t2 = div_by_recip(tr + t2s, p15, r15);
    const double t3 = div_by_recip(t3s, s, rs);
    return (t1 + t2) + t3;
}

// ---- compact arithmetic (d <= 8 greedy kernels; default since round 3) --------------------------
// The same kernel value by the shortest route that stays a few ulps from NumPy's evaluation
// (bit model: oracle/stein_ref.c pair_compact; pinned to every reference fixture in
// tests/test_oracle_compact.py).  With S = SEQ_FMA dk^2, G = SEQ_FMA (gi_k - gj_k) dk,
// P = SEQ_FMA gi_k gj_k (first term a product, then one fma per coordinate):
//   qf = fma(l, S, 1),  y = RN(1 / RN(sqrt(qf))),  k = y * fma(y^2, fma(y^2, fl(-3 l^2) S, fma(l, G, tr)), P)
// i.e. t3 + t2 + t1 = P / qf^0.5 + (tr + l G) / qf^1.5 - 3 l^2 S / qf^2.5 regrouped around one
// reciprocal square root: 20 + 23 fp64 instructions per pair at d = 4 instead of 101.  Applies to a
// pair only when both rows are in the fast range (row_in_range) and l, tr are (the same guard as
// finish_pair_fast: qf in [1, 2^185], nothing overflows or underflows); other pairs take the exact
// arithmetic -- a per-pair rule, so the result does not depend on how rows are split over blocks,
// kernels or ranks.  y is correctly rounded: fast_sqrt is the IEEE sqrt in this range and recip2
// from its h is RN(1/s) (above).
template <int D>
__device__ __forceinline__ double pair_compact_ct(const double (&xi)[D], const double (&gi)[D],
                                                  const double* xj, const double* gj, double l,
                                                  double m3l2, double tr) {
    double S = 0.0, G = 0.0, P = 0.0;
#pragma unroll
    for (int k = 0; k < D; ++k) {
        const double dl = xi[k] - xj[k];
        const double gd = gi[k] - gj[k];
        if (k == 0) {
            S = dl * dl; G = gd * dl; P = gi[0] * gj[0];
        } else {
            S = __builtin_fma(dl, dl, S); G = __builtin_fma(gd, dl, G); P = __builtin_fma(gi[k], gj[k], P);
        }
    }
    const double q = __builtin_fma(l, S, 1.0);
    double h;
    const double s = fast_sqrt(q, h);
    const double y = recip2(s, h + h);
    const double y2 = y * y;
    const double in = __builtin_fma(y2, m3l2 * S, __builtin_fma(l, G, tr));
    return y * __builtin_fma(y2, in, P);
}

// k(x, x) in the compact arithmetic: S = G = 0, qf = 1, y = 1 -> fl(tr + P)
template <int D>
__device__ __forceinline__ double diag_compact_ct(const double (&gi)[D], double tr) {
    double P = gi[0] * gi[0];
#pragma unroll
    for (int k = 1; k < D; ++k) P = __builtin_fma(gi[k], gi[k], P);
    return tr + P;
}

// 1 if every coordinate of the row (x and g) is 0 or of magnitude in [2^-60, 2^60]
template <int D>
__device__ __forceinline__ int row_in_range(const double (&xi)[D], const double (&gi)[D]) {
    int ok = 1;
#pragma unroll
    for (int k = 0; k < D; ++k) ok &= fast_range_ok(xi[k]) & fast_range_ok(gi[k]);
    return ok;
}

// l and tr admit the fast / compact arithmetic (the kernels' per-problem part of the guard)
__device__ __forceinline__ int scale_in_range(double l, double tr) {
    return fast_range_ok(l) & (int)(l > 0.0) & (int)(tr > 0.0) & (int)(tr <= 0x1p64);
}

// t3 follows NumPy pairwise_sum streamed over k (no product array): 0 + e0 + ... for d < 8;
// 8 partial sums for 8 <= d <= 128.  (d > 128 rejected at the ABI.)

// Compile-time d (D >= 1): everything unrolled, vectors in registers.
// FAST: caller guarantees fast_range_ok for both points' components and for l (see above).
template <int D, bool FAST = false>
__device__ __forceinline__ double pair_value_ct(const double (&xi)[D], const double (&gi)[D],
                                                const double* xj, const double* gj, double l,
                                                double l2, double tr) {
    double qs = 0.0, t1s = 0.0, t2s = 0.0;
#pragma unroll
    for (int k = 0; k < D; ++k) {
        const double dl = xi[k] - xj[k];
        const double gd = gi[k] - gj[k];
        const double q = (l * dl) * dl;
        const double u = (l2 * dl) * dl;
        const double v = (l * gd) * dl;
        if (k == 0) {
            qs = q; t1s = u; t2s = v;
        } else {
            qs = qs + q; t1s = t1s + u; t2s = t2s + v;
        }
    }
    double t3s;
    if constexpr (D < 8 && FAST) {
        t3s = gi[0] * gj[0];   // "0.0 +" dropped: differs only in the sign of a zero t3s
#pragma unroll
        for (int k = 1; k < D; ++k) t3s += gi[k] * gj[k];
    } else if constexpr (D < 8) {
        t3s = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k) t3s += gi[k] * gj[k];
    } else {
        static_assert(D <= 128, "pairwise_sum recursion not modelled beyond 128");
        double r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = gi[k] * gj[k];
        constexpr int full = D - (D % 8);
#pragma unroll
        for (int k = 8; k < full; ++k) r[k % 8] += gi[k] * gj[k];
        t3s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
        for (int k = full; k < D; ++k) t3s += gi[k] * gj[k];
    }
    if constexpr (FAST) return finish_pair_fast(qs, t1s, t2s, t3s, tr);
    else return finish_pair(qs, t1s, t2s, t3s, tr);
}

// Diagonal k(x, x) = fl(tr + PAIRWISE fl(g_k*g_k)) (dk = 0: qf = 1, t1 = -0, pow(1, .) = 1).
template <int D>
__device__ __forceinline__ double diag_value_ct(const double (&gi)[D], double tr) {
    double t3s;
    if constexpr (D < 8) {
        t3s = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k) t3s += gi[k] * gi[k];
    } else {
        double r[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) r[k] = gi[k] * gi[k];
        constexpr int full = D - (D % 8);
#pragma unroll
        for (int k = 8; k < full; ++k) r[k % 8] += gi[k] * gi[k];
        t3s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
#pragma unroll
        for (int k = full; k < D; ++k) t3s += gi[k] * gi[k];
    }
    // finish_pair(0, 0, 0, t3s): t1 = -0/1, t2 = tr/1, t3 = t3s/1 -> (-0 + tr) + t3s
    return finish_pair(0.0, 0.0, 0.0, t3s, tr);
}

// The d <= 8 kernels' per-pair rule: the compact arithmetic when cok (l, tr and both rows in range,
// see pair_compact_ct), the exact one otherwise.  A real branch (not compute-both-and-select).
template <int D>
__device__ __forceinline__ double pair_value_sel(bool cok, const double (&xi)[D], const double (&gi)[D],
                                                 const double* xj, const double* gj, double l, double l2,
                                                 double m3l2, double tr) {
    if (cok) return pair_compact_ct<D>(xi, gi, xj, gj, l, m3l2, tr);
    return pair_value_ct<D>(xi, gi, xj, gj, l, l2, tr);
}

template <int D>
__device__ __forceinline__ double diag_value_sel(bool cok, const double (&gi)[D], double tr) {
    if (cok) return diag_compact_ct<D>(gi, tr);
    return diag_value_ct<D>(gi, tr);
}

// Runtime d (1..128): point a strided by sa (SoA column: sa = ld), point b strided by sb.
__device__ __forceinline__ double pair_value_rt(const double* __restrict__ xa,
                                               const double* __restrict__ ga, int64_t sa,
                                               const double* xb, const double* gb, int64_t sb,
                                               int d, double l, double l2, double tr) {
    double qs = 0.0, t1s = 0.0, t2s = 0.0;
    double r[8];
    double t3s = 0.0;
    const int full = (d >= 8) ? d - (d % 8) : 0;
    for (int k = 0; k < d; ++k) {
        const double xak = xa[k * sa];
        const double gak = ga[k * sa];
        const double gbk = gb[k * sb];
        const double dl = xak - xb[k * sb];
        const double gd = gak - gbk;
        const double q = (l * dl) * dl;
        const double u = (l2 * dl) * dl;
        const double v = (l * gd) * dl;
        if (k == 0) {
            qs = q; t1s = u; t2s = v;
        } else {
            qs = qs + q; t1s = t1s + u; t2s = t2s + v;
        }
        const double p = gak * gbk;
        if (d < 8) {
            t3s += p;
        } else if (k < 8) {
            r[k] = p;
        } else if (k < full) {
            r[k & 7] += p;
        } else {
            if (k == full) t3s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
            t3s += p;
        }
    }
    if (d >= 8 && full == d) t3s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    return finish_pair(qs, t1s, t2s, t3s, tr);
}

// Columns streamed once per step: non-temporal loads (`nt`) when a step's working set exceeds the
// 256 MB memory-side cache (MALL) -- the config-5 pattern (412 MB) runs 71.8 -> 62.4 us per pass
// (profiles/r02_mall_nt_probe.log) -- and default loads when it fits, so that the MALL serves the
// next step (d = 4, n = 2e6: 160 MB per step, nt measured 4-40 % slower).
template <bool NTL, typename T>
__device__ __forceinline__ T stream_load(const T* p) {
    if constexpr (NTL) return __builtin_nontemporal_load(p);
    else return *p;
}

// Runtime d >= 8 (the high-dimensional streaming step): the candidate's coordinates are loaded
// eight at a time (16 independent loads in flight per lane; 4 waves per SIMD hide the rest),
// matching NumPy's pairwise_sum lane structure for t3 (r[k % 8]); NTL: non-temporal loads.
// The selected point (xb, gb) is block-uniform (LDS broadcast reads).  Same bits as pair_value_rt.
template <bool NTL>
__device__ __forceinline__ double pair_value_rt8(const double* __restrict__ xa,
                                                const double* __restrict__ ga, int64_t sa,
                                                const double* xb, const double* gb, int d,
                                                double l, double l2, double tr) {
    double qs = 0.0, t1s = 0.0, t2s = 0.0;
    double r[8];
    const int full = d - (d % 8);
    for (int k0 = 0; k0 < full; k0 += 8) {
        double cx[8], cg[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            cx[j] = stream_load<NTL>(xa + (k0 + j) * sa);
            cg[j] = stream_load<NTL>(ga + (k0 + j) * sa);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = k0 + j;
            const double xbk = xb[k], gbk = gb[k];
            const double dl = cx[j] - xbk;
            const double gd = cg[j] - gbk;
            const double q = (l * dl) * dl;
            const double u = (l2 * dl) * dl;
            const double v = (l * gd) * dl;
            if (k0 == 0 && j == 0) {
                qs = q; t1s = u; t2s = v;
            } else {
                qs = qs + q; t1s = t1s + u; t2s = t2s + v;
            }
            const double p = cg[j] * gbk;
            r[j] = k0 == 0 ? p : r[j] + p;
        }
    }
    double t3s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (int k = full; k < d; ++k) {
        const double xak = stream_load<NTL>(xa + k * sa), gak = stream_load<NTL>(ga + k * sa);
        const double xbk = xb[k], gbk = gb[k];
        const double dl = xak - xbk;
        const double gd = gak - gbk;
        qs = qs + (l * dl) * dl;
        t1s = t1s + (l2 * dl) * dl;
        t2s = t2s + (l * gd) * dl;
        t3s += gak * gbk;
    }
    return finish_pair(qs, t1s, t2s, t3s, tr);
}

__device__ __forceinline__ double diag_value_rt(const double* __restrict__ gi_col, int64_t ld,
                                                int d, double tr) {
    double r[8];
    double t3s = 0.0;
    const int full = (d >= 8) ? d - (d % 8) : 0;
    for (int k = 0; k < d; ++k) {
        const double gik = gi_col[k * ld];
        const double p = gik * gik;
        if (d < 8) {
            t3s += p;
        } else if (k < 8) {
            r[k] = p;
        } else if (k < full) {
            r[k & 7] += p;
        } else {
            if (k == full) t3s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
            t3s += p;
        }
    }
    if (d >= 8 && full == d) t3s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    return finish_pair(0.0, 0.0, 0.0, t3s, tr);
}

// np.argmin order: NaN is the minimum (first NaN wins), otherwise smaller value, ties -> lower index.
// Branch-free (selects, no exec-mask branches in the per-candidate hot loop).
__device__ __forceinline__ bool better(double a, int64_t ia, double b, int64_t ib) {
    const bool na = __builtin_isnan(a), nb = __builtin_isnan(b);
    const bool il = ia < ib;
    const bool num = (a < b) | ((a == b) & il);
    const bool nan = na & (!nb | il);
    return (na | nb) ? nan : num;
}

// Wave64 MINLOC of (value, index) in np.argmin order; every lane receives the wave result.
// DPP row rotations (quad xor-1, xor-2, row_ror 4, row_ror 8: ~4 cycles each, no LDS) reduce each
// 16-lane row; v_readlane of lanes 0/16/32/48 combines the four rows.  Replaces a 24-deep
// ds_bpermute (__shfl_xor) chain (~1 us per reduction on gfx950).
template <int CTRL>
__device__ __forceinline__ void dpp_pair(double v, int64_t i, double& ov, int64_t& oi) {
    const uint64_t vb = (uint64_t)__double_as_longlong(v);
    const uint64_t ib = (uint64_t)i;
    const uint32_t v0 = __builtin_amdgcn_update_dpp(0u, (uint32_t)vb, CTRL, 0xF, 0xF, false);
    const uint32_t v1 = __builtin_amdgcn_update_dpp(0u, (uint32_t)(vb >> 32), CTRL, 0xF, 0xF, false);
    const uint32_t i0 = __builtin_amdgcn_update_dpp(0u, (uint32_t)ib, CTRL, 0xF, 0xF, false);
    const uint32_t i1 = __builtin_amdgcn_update_dpp(0u, (uint32_t)(ib >> 32), CTRL, 0xF, 0xF, false);
    ov = __longlong_as_double((long long)(((uint64_t)v1 << 32) | v0));
    oi = (int64_t)(((uint64_t)i1 << 32) | i0);
}

__device__ __forceinline__ void take_if_better(double ov, int64_t oi, double& v, int64_t& i) {
    const bool b = better(ov, oi, v, i);
    v = b ? ov : v;
    i = b ? oi : i;
}

__device__ __forceinline__ void wave_minloc_dpp(double& v, int64_t& i) {
    double ov;
    int64_t oi;
    dpp_pair<0xB1>(v, i, ov, oi);   // quad_perm [1,0,3,2]
    take_if_better(ov, oi, v, i);
    dpp_pair<0x4E>(v, i, ov, oi);   // quad_perm [2,3,0,1]
    take_if_better(ov, oi, v, i);
    dpp_pair<0x124>(v, i, ov, oi);  // row_ror:4
    take_if_better(ov, oi, v, i);
    dpp_pair<0x128>(v, i, ov, oi);  // row_ror:8
    take_if_better(ov, oi, v, i);
    const uint64_t vb = (uint64_t)__double_as_longlong(v);
    const uint64_t ib = (uint64_t)i;
    double bv = INFINITY;
    int64_t bi = INT64_MAX;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint32_t v0 = __builtin_amdgcn_readlane((uint32_t)vb, 16 * r);
        const uint32_t v1 = __builtin_amdgcn_readlane((uint32_t)(vb >> 32), 16 * r);
        const uint32_t i0 = __builtin_amdgcn_readlane((uint32_t)ib, 16 * r);
        const uint32_t i1 = __builtin_amdgcn_readlane((uint32_t)(ib >> 32), 16 * r);
        take_if_better(__longlong_as_double((long long)(((uint64_t)v1 << 32) | v0)),
                       (int64_t)(((uint64_t)i1 << 32) | i0), bv, bi);
    }
    v = bv;
    i = bi;
}

// Wave MINLOC in np.argmin order, common case first: when no lane holds a NaN (one ballot), a
// plain v_min_f64 butterfly (DPP inside 16-lane rows, readlane across rows) gives the minimum m,
// a ballot of v == m finds the lanes holding it, and a single such lane gives the index directly;
// ties (several lanes equal to m, -0 == +0 included) and NaNs take the full compare chain.
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    const uint64_t vb = (uint64_t)__double_as_longlong(v);
    const uint32_t v0 = __builtin_amdgcn_update_dpp(0u, (uint32_t)vb, CTRL, 0xF, 0xF, false);
    const uint32_t v1 = __builtin_amdgcn_update_dpp(0u, (uint32_t)(vb >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((uint64_t)v1 << 32) | v0));
}

__device__ __forceinline__ uint64_t readlane_u64(uint64_t x, int lane) {
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)x, lane);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(x >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ void wave_minloc(double& v, int64_t& i) {
    if (__builtin_amdgcn_ballot_w64(__builtin_isnan(v)) != 0) {   // rare: NaN-aware chain
        wave_minloc_dpp(v, i);
        return;
    }
    double m = v;
    m = __builtin_fmin(m, dpp_f64<0xB1>(m));    // quad_perm [1,0,3,2]
    m = __builtin_fmin(m, dpp_f64<0x4E>(m));    // quad_perm [2,3,0,1]
    m = __builtin_fmin(m, dpp_f64<0x124>(m));   // row_ror:4
    m = __builtin_fmin(m, dpp_f64<0x128>(m));   // row_ror:8
    const uint64_t mb = (uint64_t)__double_as_longlong(m);
    const double r0 = __longlong_as_double((long long)readlane_u64(mb, 0));
    const double r1 = __longlong_as_double((long long)readlane_u64(mb, 16));
    const double r2 = __longlong_as_double((long long)readlane_u64(mb, 32));
    const double r3 = __longlong_as_double((long long)readlane_u64(mb, 48));
    m = __builtin_fmin(__builtin_fmin(r0, r1), __builtin_fmin(r2, r3));
    const uint64_t tied = __builtin_amdgcn_ballot_w64(v == m);
    if (__builtin_popcountll(tied) == 1) {
        i = (int64_t)readlane_u64((uint64_t)i, __builtin_ctzll(tied));
        v = m;
        return;
    }
    // ties (duplicate MCMC rows have bit-identical sums): lowest index among the tied lanes, as
    // a u32 min (indices < 2^32 - 1; the INT64_MAX "no row" sentinel maps to 0xFFFFFFFF)
    uint32_t u = v == m ? (i == INT64_MAX ? 0xFFFFFFFFu : (uint32_t)i) : 0xFFFFFFFFu;
    u = __builtin_elementwise_min(u, (uint32_t)__builtin_amdgcn_update_dpp(0u, u, 0xB1, 0xF, 0xF, false));
    u = __builtin_elementwise_min(u, (uint32_t)__builtin_amdgcn_update_dpp(0u, u, 0x4E, 0xF, 0xF, false));
    u = __builtin_elementwise_min(u, (uint32_t)__builtin_amdgcn_update_dpp(0u, u, 0x124, 0xF, 0xF, false));
    u = __builtin_elementwise_min(u, (uint32_t)__builtin_amdgcn_update_dpp(0u, u, 0x128, 0xF, 0xF, false));
    const uint32_t u0 = __builtin_amdgcn_readlane(u, 0), u1 = __builtin_amdgcn_readlane(u, 16);
    const uint32_t u2 = __builtin_amdgcn_readlane(u, 32), u3 = __builtin_amdgcn_readlane(u, 48);
    const uint32_t um = __builtin_elementwise_min(__builtin_elementwise_min(u0, u1),
                                                  __builtin_elementwise_min(u2, u3));
    v = m;
    i = um == 0xFFFFFFFFu ? INT64_MAX : (int64_t)um;
}

}  // namespace st
