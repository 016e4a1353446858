/*
 * C restatement of the reference Stein-thinning hot path -- TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this (as the
 * checker).  It is the *bit model* of the HIP kernels: the per-pair arithmetic follows NumPy's
 * evaluation order of the reference's vfk0_imq (JAX_Stein_Thinning.ipynb cell 27, json ~354-361;
 * see oracle/stein_numpy.py), verified bit-for-bit against NumPy in tests/test_oracle_bitmodel.py:
 *
 *   delta_k = a_k - b_k
 *   qf  = 1 + SEQ_k fl(fl(l  * delta_k) * delta_k)          np.sum(np.dot(linv, amb) * amb, axis=0)
 *   t1s =     SEQ_k fl(fl(l2 * delta_k) * delta_k)          l2 = fl(l*l) = diag(linv @ linv)
 *   t2s =     SEQ_k fl(fl(l * (sa_k - sb_k)) * delta_k)
 *   t3s =     PAIRWISE_k fl(sa_k * sb_k)                     (NumPy pairwise_sum: 8 lanes, d >= 8)
 *   k   = fl(fl(fl(-3*t1s) / qf^2.5) + fl(fl(tr + t2s) / qf^1.5)) + fl(t3s / sqrt(qf))
 *
 * SEQ = sequential left-to-right adds (C-contiguous axis-0 reduction); PAIRWISE = NumPy's
 * pairwise_sum (res = 0 + e0 + ... for d < 8; 8 partial sums, ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)),
 * then the remainder, for 8 <= d <= 128).  qf^1.5 and qf^2.5 are evaluated correctly rounded
 * (double-double around the correctly rounded sqrt); NumPy's own SIMD pow is within 1 ulp of that
 * (it is not bit-reproducible across CPUs either -- DESIGN.md "pow").
 *
 * Gradient-free: k_PQ(i, j) = fl(fl(k * w_i) * w_j) (reference integrand * weights[ind1] * weights[ind2]).
 * Greedy: A = diag; idx0 = argmin A; A = fl(A + 2*col); first minimum, NaN counts as minimum
 * (np.argmin) -- JAX_Stein_Thinning.ipynb cell 22 (~281-295), report.tex:413-426.
 *
 * Compact arithmetic (arith = 1; the kernels' default for d <= 8 since round 3): the same kernel value
 * by the shortest exact-enough route -- with S = SEQ_FMA_k delta_k^2, G = SEQ_FMA_k (sa_k - sb_k) delta_k,
 * P = SEQ_FMA_k sa_k sb_k (first term a product, then one fma per coordinate):
 *   qf = fma(l, S, 1)   y = RN(1 / RN(sqrt(qf)))   T1 = fl(-3 l^2) S   T2 = fma(l, G, tr)
 *   k  = y * fma(y^2, fma(y^2, T1, T2), P)            (= t1 + t2 + t3 of the reference, regrouped)
 * a few ulps from the NumPy evaluation instead of bit-identical to it; it applies to a pair (d <= 8)
 * only when every coordinate of both rows (x and g) is 0 or of magnitude in [2^-60, 2^60], l is in
 * [2^-60, 2^60] and 0 < tr <= 2^64 (no intermediate can overflow, underflow or be NaN); other pairs
 * take the exact arithmetic (pair_any: a per-pair rule, independent of any row partition).  Index
 * parity with the reference then rests on argmin margins (tests/golden/config*_numpy_indices.json:
 * >= 1.2e9 ulps), like the NumPy path's own 1-ulp pow differences across CPUs.
 *
 * Build: gcc -O2 -fPIC -shared -ffp-contract=off -pthread -o oracle/_build/libstein_ref.so oracle/stein_ref.c -lm
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static double pairwise_sum(const double *v, int64_t n) {
    if (n < 8) {
        double res = 0.;
        for (int64_t i = 0; i < n; i++) res += v[i];
        return res;
    } else if (n <= 128) {
        double r[8], res;
        int64_t i;
        for (int j = 0; j < 8; j++) r[j] = v[j];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += v[i + j];
        res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += v[i];
        return res;
    } else {
        int64_t n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise_sum(v, n2) + pairwise_sum(v + n2, n - n2);
    }
}

/* correctly rounded (to ~2^-100, then rounded once) qf^1.5, qf^2.5 from s = sqrt(qf) and its exact
 * residual e = qf - s^2: the correction term q*e/(2s) is evaluated as (s/2)*e (equal to 2^-53
 * relative of a 2^-53-relative term); q^1.5 = hi + lo as a double-double, q^2.5 = q * (hi + lo) as a
 * second double-double product -- the kernels' exact op sequence (an overflowing power is +inf) */
static void pow_15_25(double q, double *p15, double *p25, double *sq) {
    double s = sqrt(q);
    double e = fma(-s, s, q);
    double hi = q * s;
    double lo = fma(q, s, -hi);
    lo = fma(0.5 * s, e, lo);
    *p15 = isinf(hi) ? hi : hi + lo;
    double hi2 = q * hi;
    double lo2 = fma(q, hi, -hi2);
    lo2 = fma(q, lo, lo2);
    *p25 = isinf(hi2) ? hi2 : hi2 + lo2;
    *sq = s;
}

/* one Stein-kernel value; a/b/sa/sb are d-vectors with strides */
static double pair_value(const double *a, int64_t sa_stride, const double *b, int64_t sb_stride,
                         const double *ga, const double *gb, int d, double l, double tr) {
    double l2 = l * l;
    double prod[128];
    double qs = 0, t1s = 0, t2s = 0;
    for (int k = 0; k < d; k++) {
        double dl = a[k * sa_stride] - b[k * sb_stride];
        double gd = ga[k * sa_stride] - gb[k * sb_stride];
        double q = (l * dl) * dl;
        double u = (l2 * dl) * dl;
        double v = (l * gd) * dl;
        if (k == 0) { qs = q; t1s = u; t2s = v; }
        else { qs = qs + q; t1s = t1s + u; t2s = t2s + v; }
        prod[k] = ga[k * sa_stride] * gb[k * sb_stride];
    }
    double t3s = pairwise_sum(prod, d);
    double qf = 1.0 + qs;
    double p15, p25, s;
    pow_15_25(qf, &p15, &p25, &s);
    double t1 = (-3.0 * t1s) / p25;
    double t2 = (tr + t2s) / p15;
    double t3 = t3s / s;
    return (t1 + t2) + t3;
}

/* compact arithmetic (header); y2 = y*y, m3l2 = fl(-3 * fl(l*l)) */
static double pair_compact(const double *a, int64_t sa_stride, const double *b, int64_t sb_stride,
                           const double *ga, const double *gb, int d, double l, double tr) {
    double S = 0, G = 0, P = 0;
    for (int k = 0; k < d; k++) {
        double dl = a[k * sa_stride] - b[k * sb_stride];
        double gd = ga[k * sa_stride] - gb[k * sb_stride];
        double pa = ga[k * sa_stride], pb = gb[k * sb_stride];
        if (k == 0) { S = dl * dl; G = gd * dl; P = pa * pb; }
        else { S = fma(dl, dl, S); G = fma(gd, dl, G); P = fma(pa, pb, P); }
    }
    double m3l2 = -3.0 * (l * l);
    double q = fma(l, S, 1.0);
    double y = 1.0 / sqrt(q);
    double y2 = y * y;
    double in = fma(y2, m3l2 * S, fma(l, G, tr));
    return y * fma(y2, in, P);
}

static int in_range(double v) {
    double a = fabs(v);
    return a == 0.0 || (a >= 0x1p-60 && a <= 0x1p60);
}

static int scale_ok(double l, double tr) { return in_range(l) && l > 0.0 && tr > 0.0 && tr <= 0x1p64; }

static int row_ok(const double *x, const double *g, int64_t stride, int d) {
    for (int k = 0; k < d; k++)
        if (!in_range(x[k * stride]) || !in_range(g[k * stride])) return 0;
    return 1;
}

/* the kernels' per-pair rule (stein_math.hpp pair_value_sel): compact arithmetic when arith = 1,
 * d <= 8, l and tr in range and both rows in range; the exact arithmetic otherwise */
static double pair_any(int arith, const double *a, int64_t sa_stride, const double *b, int64_t sb_stride,
                       const double *ga, const double *gb, int d, double l, double tr) {
    if (arith == 1 && d <= 8 && scale_ok(l, tr) && row_ok(a, ga, sa_stride, d) && row_ok(b, gb, sb_stride, d))
        return pair_compact(a, sa_stride, b, sb_stride, ga, gb, d, l, tr);
    return pair_value(a, sa_stride, b, sb_stride, ga, gb, d, l, tr);
}

/* 1 if every pair of the problem takes the compact arithmetic (tests) */
int sr_compact_ok(const double *x, const double *g, int64_t n, int d, double l, double tr) {
    if (d > 8 || !scale_ok(l, tr)) return 0;
    for (int64_t i = 0; i < n; i++)
        if (!row_ok(x + i * d, g + i * d, 1, d)) return 0;
    return 1;
}

/* running-sum update: fl(A + 2k) (2k exact); the kernels' fma(2, k, A) is the same bits */
static int better(double a, int64_t ia, double b, int64_t ib) {
    if (isnan(a)) return isnan(b) ? (ia < ib) : 1;
    if (isnan(b)) return 0;
    return (a < b) || (a == b && ia < ib);
}

/*
 * x, g: row-major (n, d); w: weights or NULL; A: (n) running sums (out); idx: (m) out.
 * Returns 0 on success, -1 on unsupported d.
 */
int sr_greedy(const double *x, const double *g, const double *w, int64_t n, int d,
              double l, double tr, int64_t m, uint32_t *idx, double *A, int arith) {
    if (d < 1 || d > 128) return -1;
    for (int64_t i = 0; i < n; i++) {
        double k = pair_any(arith, x + i * d, 1, x + i * d, 1, g + i * d, g + i * d, d, l, tr);
        if (w) k = (k * w[i]) * w[i];
        A[i] = k;
    }
    for (int64_t t = 0; t < m; t++) {
        if (t > 0) {
            int64_t j = idx[t - 1];
            for (int64_t i = 0; i < n; i++) {
                double k = pair_any(arith, x + i * d, 1, x + j * d, 1, g + i * d, g + j * d, d, l, tr);
                if (w) k = (k * w[i]) * w[j];
                A[i] = A[i] + 2.0 * k;
            }
        }
        int64_t best = 0;
        for (int64_t i = 1; i < n; i++)
            if (better(A[i], i, A[best], best)) best = i;
        idx[t] = (uint32_t)best;
    }
    return 0;
}

/*
 * sr_greedy with the candidate rows split over `nthreads` POSIX threads: every step each thread
 * updates its contiguous row block and finds its block's first minimum; thread 0 then reduces the
 * block results in block order with the same `better` rule, so the result is the one sequential
 * scan's (lowest global index among equal values, first NaN) for any thread count.  Same
 * arithmetic per row as sr_greedy, so A is bit-identical too.  Lets the tests check every index of
 * the full-size configs (n = 2e6, m = 1000) in seconds.
 */
#include <pthread.h>

typedef struct {
    const double *x, *g, *w;
    int64_t n, m;
    int d, nthreads;
    double l, tr;
    int arith;
    uint32_t *idx;
    double *A;
    double *bv;
    int64_t *bi;
    pthread_barrier_t bar;
    double *gap;   /* sr_greedy_mt_ties: per step, (smallest sum > the winner's) - (the winner's) */
    double *rv;    /* per thread: its smallest sum above the step's winning value */
    double *wv;    /* sr_greedy_mt_ties: per step, the winner's running sum */
} mt_ctx;

typedef struct { mt_ctx *c; int tid; } mt_arg;

/* rows i and j equal bit for bit in x, g (and w): identical pair values in any arithmetic, hence equal
 * running sums at every step; np.argmin always prefers the lower index, so neither path can tell them
 * apart (the near-tie rule below does not count such a tie) */
static int same_row(const mt_ctx *c, int64_t i, int64_t j) {
    const int d = c->d;
    if (memcmp(c->x + i * d, c->x + j * d, sizeof(double) * d) != 0) return 0;
    if (memcmp(c->g + i * d, c->g + j * d, sizeof(double) * d) != 0) return 0;
    return !c->w || memcmp(c->w + i, c->w + j, sizeof(double)) == 0;
}

static void *mt_worker(void *p) {
    mt_arg *a = (mt_arg *)p;
    mt_ctx *c = a->c;
    const int d = c->d;
    const int64_t r0 = c->n * a->tid / c->nthreads, r1 = c->n * (a->tid + 1) / c->nthreads;
    for (int64_t i = r0; i < r1; i++) {
        const double *xi = c->x + i * d, *gi = c->g + i * d;
        double k = pair_any(c->arith, xi, 1, xi, 1, gi, gi, d, c->l, c->tr);
        if (c->w) k = (k * c->w[i]) * c->w[i];
        c->A[i] = k;
    }
    for (int64_t t = 0; t < c->m; t++) {
        if (t > 0) {
            int64_t j = c->idx[t - 1];
            const double *xj = c->x + j * d, *gj = c->g + j * d;
            for (int64_t i = r0; i < r1; i++) {
                double k = pair_any(c->arith, c->x + i * d, 1, xj, 1, c->g + i * d, gj, d, c->l, c->tr);
                if (c->w) k = (k * c->w[i]) * c->w[j];
                c->A[i] = c->A[i] + 2.0 * k;
            }
        }
        int64_t best = -1;
        for (int64_t i = r0; i < r1; i++)
            if (best < 0 || better(c->A[i], i, c->A[best], best)) best = i;
        c->bi[a->tid] = best;
        c->bv[a->tid] = best >= 0 ? c->A[best] : 0.0;
        pthread_barrier_wait(&c->bar);
        if (a->tid == 0) {
            int64_t gb = -1;
            double gv = 0.0;
            for (int q = 0; q < c->nthreads; q++) {
                if (c->bi[q] < 0) continue;
                if (gb < 0 || better(c->bv[q], c->bi[q], gv, gb)) { gb = c->bi[q]; gv = c->bv[q]; }
            }
            c->idx[t] = (uint32_t)gb;
            c->bv[0] = gv;
        }
        pthread_barrier_wait(&c->bar);
        if (c->gap) {   /* the runner-up: smallest sum of any row other than the winner and its bitwise
                           duplicates (an exact tie with any other row counts) */
            const double gv = c->bv[0];
            const int64_t wi = c->idx[t];
            double r = INFINITY;
            for (int64_t i = r0; i < r1; i++)
                if (i != wi && c->A[i] < r && !(c->A[i] == gv && same_row(c, i, wi))) r = c->A[i];
            c->rv[a->tid] = r;
            pthread_barrier_wait(&c->bar);
            if (a->tid == 0) {
                double rr = INFINITY;
                for (int q = 0; q < c->nthreads; q++) rr = c->rv[q] < rr ? c->rv[q] : rr;
                c->gap[t] = rr - gv;
                if (c->wv) c->wv[t] = gv;
            }
            pthread_barrier_wait(&c->bar);
        }
    }
    return NULL;
}

static int greedy_mt(const double *x, const double *g, const double *w, int64_t n, int d,
                     double l, double tr, int64_t m, uint32_t *idx, double *A, int nthreads, int arith,
                     double *gap, double *wv) {
    if (d < 1 || d > 128 || n < 1) return -1;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    if (nthreads > n) nthreads = (int)n;
    mt_ctx c = {x, g, w, n, m, d, nthreads, l, tr, arith, idx, A, NULL, NULL};
    c.gap = gap;
    c.wv = wv;
    c.rv = (double *)malloc(sizeof(double) * nthreads);
    c.bv = (double *)malloc(sizeof(double) * nthreads);
    c.bi = (int64_t *)malloc(sizeof(int64_t) * nthreads);
    pthread_t *th = (pthread_t *)malloc(sizeof(pthread_t) * nthreads);
    mt_arg *args = (mt_arg *)malloc(sizeof(mt_arg) * nthreads);
    int rc = 0;
    if (!c.bv || !c.bi || !th || !args || pthread_barrier_init(&c.bar, NULL, (unsigned)nthreads) != 0) {
        rc = -2;
    } else {
        int started = 0;
        for (int q = 1; q < nthreads; q++) {
            args[q].c = &c;
            args[q].tid = q;
            if (pthread_create(&th[q], NULL, mt_worker, &args[q]) != 0) { rc = -3; break; }
            started++;
        }
        if (rc == 0) {
            args[0].c = &c;
            args[0].tid = 0;
            mt_worker(&args[0]);
        }
        /* a failed pthread_create leaves the started workers blocked on the barrier: abort */
        if (rc != 0) abort();
        for (int q = 1; q <= started; q++) pthread_join(th[q], NULL);
        pthread_barrier_destroy(&c.bar);
    }
    free(c.rv);
    free(c.bv);
    free(c.bi);
    free(th);
    free(args);
    return rc;
}

int sr_greedy_mt(const double *x, const double *g, const double *w, int64_t n, int d,
                 double l, double tr, int64_t m, uint32_t *idx, double *A, int nthreads, int arith) {
    return greedy_mt(x, g, w, n, d, l, tr, m, idx, A, nthreads, arith, NULL, NULL);
}

/*
 * Near-tie guard of the compact arithmetic (the kernels' rule, persistent_kernel.hpp tie_check): step t
 * (the argmin that gives idx[t]) is flagged when the smallest running sum of any OTHER row -- an exact tie
 * included -- lies within thr(t) of the winner's, where rows equal to the winner bit for bit (x, g, w: a
 * repeated MCMC row, adjacent or not) do not count: their sums equal the winner's in every arithmetic and
 * NumPy resolves them by the lower index exactly as the kernels do.  Any other exact tie counts: two
 * different rows with equal sums tie only by accident of rounding.  thr(t) bounds how far two rows' sums may move
 * between the compact arithmetic, the exact one and NumPy's evaluation -- diagnostics.py's band (8 ulps
 * per term of the magnitudes a pair value is built from, plus an ulp of the sum per step) for both rows,
 * times 2 -- with ulp(v) <= |v| 2^-52 and the magnitudes bounded by
 *   pair terms of row i against the column j:  scale <= (3 l + tr + sqrt(l) (gmax + |g_j|) + gmax |g_j|) wmax w_j
 *     (3 l^2 S / qf^2.5 <= 3 l; l |sum dg delta| / qf^1.5 <= sqrt(l) |dg|; |g_i . g_j| / sqrt(qf) <= gmax |g_j|)
 *     <= (c1 + |g_j|^2) wmax w_j,  c1 = 3 l + tr + sqrt(l) gmax + l / 2 + gmax^2 / 2   (a b <= (a^2 + b^2) / 2)
 *   the diagonal:                               Dmax = (tr + gmax^2) wmax^2
 *   a running sum at step s:                    |A_i(s)| <= Dmax + 2 sqrt(Dmax Q(s)) <= 2 Dmax + Q(s)
 * where Q(s) = sum of the winners' sums before step s = the Stein quadratic form of the selected multiset
 * (A_i(s) = |phi_i|^2 + 2 <phi_i, Phi_S>, Q = |Phi_S|^2: the kernel is positive semi-definite), gmax^2 =
 * max_i |g_i|^2 and wmax^2 = max_i w_i^2 (1 without weights).  Recurrence (one lane per block of the
 * kernels evaluates it with these operations in this order; no square root per step):
 *   thr(0) = 2^-50 (8 Dmax);  for s >= 1 with j = idx[s-1], v = its sum at step s-1:
 *     Q += v;  E += 16 (c1 + |g_j|^2) wmax w_j + (2 Dmax + max(Q, 0));  thr(s) = 2^-50 (8 Dmax + E)
 */
typedef struct {
    double c1, wmax, dmax, Q, E, thr;
} tie_state;

static void tie_init(tie_state *ts, double l, double tr, double g2max, double w2max) {
    const double gm = sqrt(g2max), sl = sqrt(l);
    ts->c1 = (((3.0 * l + tr) + sl * gm) + 0.5 * l) + 0.5 * g2max;
    ts->wmax = sqrt(w2max);
    ts->dmax = (tr + g2max) * w2max;
    ts->Q = 0.0;
    ts->E = 0.0;
    ts->thr = 0x1p-50 * (8.0 * ts->dmax);
}

/* one step: v = the previous winner's sum, gj its score row, wj its weight (1 without weights) */
static void tie_step(tie_state *ts, double v, const double *gj, int d, double wj) {
    ts->Q = ts->Q + v;
    double gj2 = gj[0] * gj[0];
    for (int k = 1; k < d; k++) gj2 = gj2 + gj[k] * gj[k];
    const double scale = (ts->c1 + gj2) * (ts->wmax * wj);
    ts->E = ts->E + (16.0 * scale + (2.0 * ts->dmax + fmax(ts->Q, 0.0)));
    ts->thr = 0x1p-50 * (8.0 * ts->dmax + ts->E);
}

/* the bounds' inputs as the kernels compute them: max_i of g_i0 g_i0 + g_i1 g_i1 + ... (sequential) and of
 * w_i w_i (1 without weights); a NaN counts as +inf */
void sr_tie_bounds(const double *g, const double *w, int64_t n, int d, double *g2max, double *w2max) {
    double gm = 0.0, wm = w ? 0.0 : 1.0;
    for (int64_t i = 0; i < n; i++) {
        double s = g[i * d] * g[i * d];
        for (int k = 1; k < d; k++) s = s + g[i * d + k] * g[i * d + k];
        if (isnan(s)) s = INFINITY;
        gm = s > gm ? s : gm;
        if (w) {
            double v = w[i] * w[i];
            if (isnan(v)) v = INFINITY;
            wm = v > wm ? v : wm;
        }
    }
    *g2max = gm;
    *w2max = wm;
}

/* sr_greedy_mt plus the near-tie model per step: gap[t] = (smallest sum of any other row) - (the
 * winner's) (NaN when a NaN won), thr[t] = the guard's threshold (recurrence above) and wv[t] = the
 * winner's sum (wv may be NULL); the guard flags step t when gap[t] <= thr[t] */
int sr_greedy_mt_ties(const double *x, const double *g, const double *w, int64_t n, int d,
                      double l, double tr, int64_t m, uint32_t *idx, double *A, int nthreads, int arith,
                      double *gap, double *thr, double *wv) {
    double *v = wv ? wv : (double *)malloc(sizeof(double) * (m > 0 ? m : 1));
    if (!v) return -2;
    int rc = greedy_mt(x, g, w, n, d, l, tr, m, idx, A, nthreads, arith, gap, v);
    if (rc == 0) {
        double g2max, w2max;
        sr_tie_bounds(g, w, n, d, &g2max, &w2max);
        tie_state ts;
        tie_init(&ts, l, tr, g2max, w2max);
        for (int64_t t = 0; t < m; t++) {
            if (t > 0) {
                const int64_t j = idx[t - 1];
                tie_step(&ts, v[t - 1], g + j * d, d, w ? w[j] : 1.0);
            }
            thr[t] = ts.thr;
        }
    }
    if (!wv) free(v);
    return rc;
}

/* the bit model's powers for a vector of qf values (tests: against Decimal-exact powers) */
void sr_pow_15_25(const double *q, int64_t n, double *p15, double *p25) {
    for (int64_t i = 0; i < n; i++) {
        double s;
        pow_15_25(q[i], &p15[i], &p25[i], &s);
    }
}

/* pair values out[p] = k(i1[p], i2[p]) with weights fl(fl(k*w_i1)*w_i2) */
int sr_pairs(const double *x, const double *g, const double *w, int64_t n, int d, double l, double tr,
             const int64_t *i1, const int64_t *i2, int64_t L, double *out, int arith) {
    if (d < 1 || d > 128) return -1;
    (void)n;
    for (int64_t p = 0; p < L; p++) {
        int64_t a = i1[p], b = i2[p];
        double k = pair_any(arith, x + a * d, 1, x + b * d, 1, g + a * d, g + b * d, d, l, tr);
        if (w) k = (k * w[a]) * w[b];
        out[p] = k;
    }
    return 0;
}
