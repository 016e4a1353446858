// Pair-list, cumulative-KSD and Gram-matrix kernels (K5) for gfx950.
//
// * pairs:     out[p] = k(i1[p], i2[p]) -- the integrand protocol integrand(ind1, ind2) of the
//              reference (stein_thinning.thinning._make_stein_integrand / _make_stein_gf_integrand;
//              used at code/src/utils/ksd.py:9-16, JAX_Stein_Thinning.ipynb cells 17, 30).
// * ksd:       column sums of the strictly lower triangle (K6, below; stein_thinning.stein.ksd,
//              called at code/src/utils/ksd.py:27; report.tex:311-313), then
//              ps_i = sum_{a<=i} (2 csum_a + k_aa), ks_i = sqrt(ps_i) / (i+1).
// * kmat:      K[r, c] = integrand(min(r,c), max(r,c)) (stein_thinning.stein.kmat,
//              code/tests/test_ksd.py:20, Gaussian_mixture.ipynb cell 94).
// All operate on a compact SoA problem (leading dimension ld); fp64 VALU bound, no MFMA.
#include <type_traits>

#include "stein_math.hpp"
#include "stein_internal.hpp"

namespace st {

constexpr int kTile = 64;      // rows per tile (one row per lane)
constexpr int kChunk = 16;     // columns staged in LDS per pass

__global__ __launch_bounds__(256) void pairs_kernel(PairArgs p, const int64_t* __restrict__ i1,
                                                    const int64_t* __restrict__ i2, int64_t L,
                                                    double* __restrict__ out) {
    const double l2 = p.l * p.l;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < L;
         q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a = i1[q], b = i2[q];
        double kv = pair_value_rt(p.x + a, p.g + a, p.ld, p.x + b, p.g + b, p.ld, p.d, p.l, l2, p.tr);
        if (p.w) kv = (kv * p.w[a]) * p.w[b];
        out[q] = kv;
    }
}

// Stage columns [c0, c0+kChunk) of the compact problem into LDS: s[k][c], k < 2d+1.
__device__ __forceinline__ void stage_chunk(const PairArgs& p, int64_t m, int64_t c0,
                                            double (*s)[kChunk]) {
    const int d = p.d;
    const int total = (2 * d + 1) * kChunk;
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
        const int k = e / kChunk, c = e % kChunk;
        const int64_t j = c0 + c;
        double v = 0.0;
        if (j < m) {
            if (k < d) v = p.x[(int64_t)k * p.ld + j];
            else if (k < 2 * d) v = p.g[(int64_t)(k - d) * p.ld + j];
            else v = p.w ? p.w[j] : 1.0;
        }
        s[k][c] = v;
    }
}

// kmat: grid (ntiles, ntiles); lane <-> row r of the tile, columns staged; out is (k, k) row-major
// and symmetric by construction (weights applied in (min, max) order), so the lane-contiguous
// store out[c * k + r] is coalesced.
__global__ __launch_bounds__(256) void kmat_kernel(PairArgs p, int64_t k, double* __restrict__ out) {
    const int64_t bi = blockIdx.y, bj = blockIdx.x;
    __shared__ double s[2 * kMaxDim + 1][kChunk];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t r = bi * kTile + lane;
    const double l2 = p.l * p.l;
    const int d = p.d;
    const double wr = (p.w && r < k) ? p.w[r] : 1.0;
    const int64_t cend = (bj * kTile + kTile < k) ? bj * kTile + kTile : k;
    for (int64_t c0 = bj * kTile; c0 < cend; c0 += kChunk) {
        __syncthreads();
        stage_chunk(p, k, c0, s);
        __syncthreads();
        if (r < k) {
            for (int c = wave; c < kChunk; c += 4) {
                const int64_t cc = c0 + c;
                if (cc >= k) continue;
                double kv = pair_value_rt(p.x + r, p.g + r, p.ld, &s[0][c], &s[d][c], kChunk, d,
                                          p.l, l2, p.tr);
                if (p.w) {
                    const double wc = s[2 * d][c];
                    kv = (r <= cc) ? (kv * wr) * wc : (kv * wc) * wr;
                }
                out[cc * k + r] = kv;
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// K6 -- full-sample KSD at scale: column sums of the strictly lower triangle over a row range
//   csum[i] = sum_{a in [a0, a1), a < i} k(x_i, x_a)   ((k w_i) w_a for gradient-free),
// i.e. the reference's 2*np.sum(k0[:i]) term of stein_thinning.stein.ksd (restated in
// oracle/stein_numpy.py ksd; report.tex:311-313) split over row ranges.  A row-sharded multi-GPU
// run computes csum over its rows and all-reduces the n-length vector (RCCL) before ksd_finish.
// One thread per column i (its row in registers); rows a staged kRows at a time in LDS and read
// as block-uniform broadcasts; 4 blocks (16 waves) per CU; block b takes column block NB-1-b so
// the heavy (late) columns are dispatched first.  Per pair: the compact arithmetic (st_tune key 11,
// the default; stein_math.hpp pair_compact_ct) when the block's columns and the staged rows are all
// in range; in other tiles the same setting decides per pair (pair_value_sel), so a row shard's
// bounds never change a pair's bits; the exact setting takes pair_value_ct (the range-guarded fast
// form when the tile admits it); per column: a sequential sum in increasing a.
// ------------------------------------------------------------------------------------------
constexpr int kColBlock = 256;
constexpr int kColsumUnroll = 2;   // rows per iteration of the column-sum sweep

struct ColsumArgs {
    const double* x;
    const double* g;
    const double* w;
    int64_t n, ld;
    double l, tr;
    int64_t a0, a1;
    double* csum;
    int compact;
};

template <int D, bool GF>
__global__ __launch_bounds__(kColBlock, 4) void ksd_colsum_kernel(ColsumArgs p) {
    constexpr int R = kColBlock;
    __shared__ double sx[D][R];
    __shared__ double sg[D][R];
    __shared__ double sw[GF ? R : 1];
    const int tid = threadIdx.x;
    const int64_t nb = (p.n + R - 1) / R;
    const int64_t c0 = (nb - 1 - (int64_t)blockIdx.x) * R;
    const int64_t i = c0 + tid;
    const int64_t ld = p.ld;
    double xi[D], gi[D];
    const bool live = i < p.n;
    int cok = fast_range_ok(p.l) & (int)(p.l > 0.0) & (int)(p.tr > 0.0) & (int)(p.tr <= 0x1p64);
#pragma unroll
    for (int k = 0; k < D; ++k) {
        xi[k] = live ? p.x[k * ld + i] : 0.0;
        gi[k] = live ? p.g[k * ld + i] : 0.0;
        cok &= fast_range_ok(xi[k]) & fast_range_ok(gi[k]);
    }
    const double wi = (GF && live) ? p.w[i] : 1.0;
    const double l = p.l, l2 = p.l * p.l, m3l2 = -3.0 * l2, tr = p.tr;
    const bool col_ok = cok != 0;   // this column (and l, tr) in range: the per-pair rule's column half
    const int col_fast = __syncthreads_and(cok);
    const int64_t a_stop = p.a1 < c0 + R ? p.a1 : c0 + R;   // rows a < i <= c0 + R - 1
    double acc = 0.0;
    for (int64_t ac = p.a0; ac < a_stop; ac += R) {
        const int64_t a = ac + tid;
        int rok = 1;
        __syncthreads();
        if (a < a_stop) {
#pragma unroll
            for (int k = 0; k < D; ++k) {
                const double xv = p.x[k * ld + a], gv = p.g[k * ld + a];
                sx[k][tid] = xv;
                sg[k][tid] = gv;
                rok &= fast_range_ok(xv) & fast_range_ok(gv);
            }
            if constexpr (GF) sw[tid] = p.w[a];
        }
        const int fast = __syncthreads_and(rok) & col_fast;
        const int cnt = (int)((a_stop - ac) < R ? (a_stop - ac) : R);
        // every row of a tile that ends at or before the block's first column precedes all its
        // columns: no per-pair triangle predicate (only the diagonal tile keeps it)
        const bool below = ac + cnt <= c0;
        // AR: 0 exact general, 1 exact range-guarded (same bits), 2 compact, 3 compact per pair
        // (stein_math.hpp pair_value_sel: compact iff the column and the row are in range, else exact
        // general) -- a tile with some row or column out of range under the compact setting, so a
        // pair's bits never depend on which tile (or which rank's row shard) it falls in
        auto sweep = [&](auto ar_tag, auto below_tag) {
            constexpr int AR = decltype(ar_tag)::value;
            constexpr bool BELOW = decltype(below_tag)::value;
            asm volatile(";; colsum variant" ::);
            auto pair_at = [&](int e) -> double {
                double xa[D], ga[D];
#pragma unroll
                for (int k = 0; k < D; ++k) { xa[k] = sx[k][e]; ga[k] = sg[k][e]; }
                double kv;
                if constexpr (AR == 2) kv = pair_compact_ct<D>(xi, gi, xa, ga, l, m3l2, tr);
                else if constexpr (AR == 3)
                    kv = pair_value_sel<D>(col_ok && row_in_range<D>(xa, ga), xi, gi, xa, ga, l, l2, m3l2, tr);
                else kv = pair_value_ct<D, AR == 1>(xi, gi, xa, ga, l, l2, tr);
                if constexpr (GF) kv = (kv * wi) * sw[e];
                return kv;
            };
            // kColsumUnroll rows per iteration: independent pair chains for the fp64 pipe, summed
            // into acc in row order (same bits as one row at a time)
            int e = 0;
            for (; e + kColsumUnroll <= cnt; e += kColsumUnroll) {
                double kv[kColsumUnroll];
#pragma unroll
                for (int u = 0; u < kColsumUnroll; ++u) kv[u] = pair_at(e + u);
#pragma unroll
                for (int u = 0; u < kColsumUnroll; ++u) {
                    if constexpr (BELOW) acc = acc + kv[u];
                    else acc = (ac + e + u < i) ? acc + kv[u] : acc;
                }
            }
            for (; e < cnt; ++e) {
                const double kv = pair_at(e);
                if constexpr (BELOW) acc = acc + kv;
                else acc = (ac + e < i) ? acc + kv : acc;
            }
        };
        using C0 = std::integral_constant<int, 0>;
        using C1 = std::integral_constant<int, 1>;
        using C2 = std::integral_constant<int, 2>;
        using C3 = std::integral_constant<int, 3>;
        if (fast && p.compact) {
            if (below) sweep(C2{}, std::true_type{});
            else sweep(C2{}, std::false_type{});
        } else if (p.compact) {
            if (below) sweep(C3{}, std::true_type{});
            else sweep(C3{}, std::false_type{});
        } else if (fast) {
            if (below) sweep(C1{}, std::true_type{});
            else sweep(C1{}, std::false_type{});
        } else {
            if (below) sweep(C0{}, std::true_type{});
            else sweep(C0{}, std::false_type{});
        }
    }
    if (live) p.csum[i] = acc;
}

// d > 8: the column's coordinates are re-read (L1/L2) per pair; rows staged kRowsRt at a time.
constexpr int kRowsRt = 32;
template <bool GF>
__global__ __launch_bounds__(kColBlock) void ksd_colsum_rt_kernel(ColsumArgs p, int d) {
    __shared__ double srow[2 * kMaxDim][kRowsRt];
    __shared__ double sw[kRowsRt];
    const int tid = threadIdx.x;
    const int64_t nb = (p.n + kColBlock - 1) / kColBlock;
    const int64_t c0 = (nb - 1 - (int64_t)blockIdx.x) * kColBlock;
    const int64_t i = c0 + tid;
    const int64_t ld = p.ld;
    const bool live = i < p.n;
    const int64_t ic = live ? i : 0;
    const double wi = (GF && live) ? p.w[i] : 1.0;
    const double l = p.l, l2 = p.l * p.l, tr = p.tr;
    const int64_t a_stop = p.a1 < c0 + kColBlock ? p.a1 : c0 + kColBlock;
    double acc = 0.0;
    for (int64_t ac = p.a0; ac < a_stop; ac += kRowsRt) {
        const int cnt = (int)((a_stop - ac) < kRowsRt ? (a_stop - ac) : kRowsRt);
        __syncthreads();
        for (int e = tid; e < 2 * d * kRowsRt; e += kColBlock) {
            const int k = e / kRowsRt, r = e % kRowsRt;
            if (r < cnt) srow[k][r] = k < d ? p.x[(int64_t)k * ld + ac + r] : p.g[(int64_t)(k - d) * ld + ac + r];
        }
        if (GF && tid < cnt) sw[tid] = p.w[ac + tid];
        __syncthreads();
        for (int e = 0; e < cnt; ++e) {
            double kv = pair_value_rt(p.x + ic, p.g + ic, ld, &srow[0][e], &srow[d][e], kRowsRt, d,
                                      l, l2, tr);
            if constexpr (GF) kv = (kv * wi) * sw[e];
            acc = (ac + e < i) ? acc + kv : acc;
        }
    }
    if (live) p.csum[i] = acc;
}

// ks_i = sqrt(S_i) / (i+1), S_i = sum_{a <= i} (2 csum_a + k(a, a)); single block: contiguous
// chunk per thread, exclusive scan of the 1024 chunk totals, second pass writes ks.
__global__ __launch_bounds__(1024) void ksd_finish_kernel(ColsumArgs p, int d, double* __restrict__ ks) {
    __shared__ double s_tot[1024];
    const int tid = threadIdx.x;
    const int64_t m = p.n;
    const int64_t per = (m + blockDim.x - 1) / blockDim.x;
    const int64_t b = tid * per, e = (b + per < m) ? b + per : m;
    double run = 0.0;
    for (int64_t i = b; i < e; ++i) {
        double kd = diag_value_rt(p.g + i, p.ld, d, p.tr);
        if (p.w) kd = (kd * p.w[i]) * p.w[i];
        const double r = 2.0 * p.csum[i] + kd;
        run += r;
        ks[i] = r;
    }
    s_tot[tid] = run;
    __syncthreads();
    if (tid == 0) {
        double acc = 0.0;
        for (int t = 0; t < (int)blockDim.x; ++t) {
            const double v = s_tot[t];
            s_tot[t] = acc;
            acc += v;
        }
    }
    __syncthreads();
    double ps = s_tot[tid];
    for (int64_t i = b; i < e; ++i) {
        ps += ks[i];
        ks[i] = __builtin_sqrt(ps) / (double)(i + 1);
    }
}

// ------------------------------------------------------------------------------------------
// K7 -- energy distance (dcor.energy_distance, used by the reference's fit_quality,
// Comparison.ipynb cell 19 / Gradient_free_Student_t.ipynb; Gaussian_mixture.ipynb cells 63-71):
//   out[i] = sum_{b in [b0, b1), (!tri or b < i)} || A_i - B_b ||_2
// Euclidean distance as scipy's cdist: sqrt of the sequential sum over k of (a_k - b_k)^2.
// Same structure as K6: one A point per thread, B points staged in LDS, block-uniform reads.
// ------------------------------------------------------------------------------------------
struct DistArgs {
    const double* a;
    int64_t lda, na;
    const double* b;
    int64_t ldb;
    int64_t b0, b1;
    int tri;
    double* out;       // K == 1: the sums; K > 1: partial sums [K][na] (reduced by dist_reduce_kernel)
    int64_t chunk;     // B points per blockIdx.y chunk (multiple of the staging tile)
};

// sqrt(ss) for ss = 0 or ss in [2^-224, 2^124] (the block-uniform fast range): the compiler's sqrt
// sequence without its scaling (ss >= 2^-767) and class fix-up (only 0 and inf) -- the same bits as
// __builtin_sqrt there -- with no branch (a conditional sqrt was compiled as an exec-mask branch).
// ss = 0: rsq(0) = inf makes the sequence a quiet NaN, and fmin (IEEE minNum: the non-NaN operand)
// returns ss * 2^200 = 0; ss > 0: ss * 2^200 = sqrt(ss)^2 * 2^200 >= sqrt(ss) since sqrt(ss) >=
// 2^-112 > 2^-200 (and ss * 2^200 <= 2^324 is finite), so fmin returns the sqrt.  Two instructions instead of SEL's four
// (fmax, compare, two 32-bit selects)
template <bool SEL>
__device__ __forceinline__ double fast_dist(double ss) {
    double h;
    if constexpr (SEL) {
        const double r = fast_sqrt(__builtin_fmax(ss, 0x1p-224), h);
        return ss == 0.0 ? 0.0 : r;
    } else {
        return __builtin_fmin(fast_sqrt(ss, h), ss * 0x1p200);
    }
}

// B range of this block: chunk blockIdx.y of [b0, b1), cut at the block's last column for the triangle
__device__ __forceinline__ void dist_range(const DistArgs& p, int64_t c0, int64_t cols, int64_t& lo, int64_t& hi) {
    lo = p.b0 + (int64_t)blockIdx.y * p.chunk;
    hi = lo + p.chunk < p.b1 ? lo + p.chunk : p.b1;
    if (p.tri && c0 + cols < hi) hi = c0 + cols;
}

// U: independent partial sums per thread in full below-diagonal tiles (U pairs in flight, U sqrt
// chains interleaved; the partials are added at the end -- a different but deterministic order, the
// energy curve is checked to a tolerance, not bitwise); MINB: blocks per CU the compiler budgets for
// SEL: the round-2 zero-distance form (fmax, compare, select) instead of the fmin form below
template <int D, int U, int MINB, bool SEL = false>
__global__ __launch_bounds__(kColBlock, MINB) void dist_colsum_kernel(DistArgs p) {
    constexpr int R = kColBlock;
    __shared__ double sb[D][R];
    const int tid = threadIdx.x;
    const int64_t nb = (p.na + R - 1) / R;
    const int64_t c0 = (nb - 1 - (int64_t)blockIdx.x) * R;
    const int64_t i = c0 + tid;
    const bool live = i < p.na;
    double ai[D];
    int aok = 1;
#pragma unroll
    for (int k = 0; k < D; ++k) {
        ai[k] = live ? p.a[k * p.lda + i] : 0.0;
        aok &= fast_range_ok(ai[k]);
    }
    int64_t lo, b_stop;
    dist_range(p, c0, R, lo, b_stop);
    double acc = 0.0;
    for (int64_t bc = lo; bc < b_stop; bc += R) {
        __syncthreads();
        const int64_t bb = bc + tid;
        int tok = aok;
        if (bb < b_stop) {
#pragma unroll
            for (int k = 0; k < D; ++k) {
                const double v = p.b[k * p.ldb + bb];
                sb[k][tid] = v;
                tok &= fast_range_ok(v);
            }
        }
        // block-uniform: every coordinate of the tile and the block's columns is 0 or in
        // [2^-60, 2^60] (squared distances 0 or in [2^-224, 2^124]), and the whole tile lies below
        // the block's first column (no triangle predicate per pair)
        const bool fast = __syncthreads_and(tok) != 0;
        const int cnt = (int)((b_stop - bc) < R ? (b_stop - bc) : R);
        const bool below = !p.tri || bc + cnt <= c0;
        auto pair_dist = [&](int e, auto fast_tag) -> double {
            constexpr bool FAST = decltype(fast_tag)::value;
            double ss = 0.0;
#pragma unroll
            for (int k = 0; k < D; ++k) {
                const double dk = ai[k] - sb[k][e];
                ss += dk * dk;
            }
            if constexpr (FAST) return fast_dist<SEL>(ss);
            else {
                return __builtin_sqrt(ss);
            }
        };
        auto tile = [&](auto fast_tag, auto below_tag) {
            constexpr bool FAST = decltype(fast_tag)::value, BELOW = decltype(below_tag)::value;
            if constexpr (BELOW && U > 1) {
                double part[U];
#pragma unroll
                for (int u = 0; u < U; ++u) part[u] = 0.0;
                int e = 0;
                for (; e + U <= cnt; e += U) {
#pragma unroll
                    for (int u = 0; u < U; ++u) part[u] += pair_dist(e + u, fast_tag);
                }
                for (; e < cnt; ++e) part[0] += pair_dist(e, fast_tag);
#pragma unroll
                for (int u = 1; u < U; ++u) part[0] += part[u];
                acc = acc + part[0];
                return;
            }
            for (int e = 0; e < cnt; ++e) {
                double ss = 0.0;
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    const double dk = ai[k] - sb[k][e];
                    ss += dk * dk;
                }
                double dist;
                if constexpr (FAST) {
                    dist = fast_dist<SEL>(ss);
                } else {
                    dist = __builtin_sqrt(ss);
                }
                if constexpr (BELOW) acc = acc + dist;
                else acc = (!p.tri || bc + e < i) ? acc + dist : acc;
            }
        };
        if (fast) {
            if (below) tile(std::true_type{}, std::true_type{});
            else tile(std::true_type{}, std::false_type{});
        } else {
            if (below) tile(std::false_type{}, std::true_type{});
            else tile(std::false_type{}, std::false_type{});
        }
    }
    if (live) p.out[(int64_t)blockIdx.y * p.na + i] = acc;
}

__global__ __launch_bounds__(kColBlock) void dist_colsum_rt_kernel(DistArgs p, int d) {
    constexpr int R = kRowsRt;
    __shared__ double sb[kMaxDim][R];
    const int tid = threadIdx.x;
    const int64_t nb = (p.na + kColBlock - 1) / kColBlock;
    const int64_t c0 = (nb - 1 - (int64_t)blockIdx.x) * kColBlock;
    const int64_t i = c0 + tid;
    const bool live = i < p.na;
    const int64_t ic = live ? i : 0;
    int64_t lo, b_stop;
    dist_range(p, c0, kColBlock, lo, b_stop);
    double acc = 0.0;
    for (int64_t bc = lo; bc < b_stop; bc += R) {
        const int cnt = (int)((b_stop - bc) < R ? (b_stop - bc) : R);
        __syncthreads();
        for (int e = tid; e < d * R; e += kColBlock) {
            const int k = e / R, r = e % R;
            if (r < cnt) sb[k][r] = p.b[(int64_t)k * p.ldb + bc + r];
        }
        __syncthreads();
        for (int e = 0; e < cnt; ++e) {
            double ss = 0.0;
            for (int k = 0; k < d; ++k) {
                const double dk = p.a[(int64_t)k * p.lda + ic] - sb[k][e];
                ss += dk * dk;
            }
            const double dist = __builtin_sqrt(ss);
            acc = (!p.tri || bc + e < i) ? acc + dist : acc;
        }
    }
    if (live) p.out[(int64_t)blockIdx.y * p.na + i] = acc;
}

// out[i] = sum over the K chunk partials, in chunk order (deterministic)
__global__ void dist_reduce_kernel(const double* part, int64_t na, int K, double* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= na) return;
    double acc = part[i];
    for (int k = 1; k < K; ++k) acc += part[(int64_t)k * na + i];
    out[i] = acc;
}

// st_tune key 13: energy kernel variant (0 / -1 auto; 1: one partial sum, 4 blocks per CU -- round 2;
// 2: U = 2, 4 blocks; 3: U = 1, 8 blocks; 4: U = 2, 8 blocks; 5: U = 4, 4 blocks;
// 6: variant 1 with the round-2 zero-distance select, SEL)
static int g_dist_variant = 0;
int dist_tune(int value) {
    if (value < -1 || value > 6) return -1;
    g_dist_variant = value < 0 ? 0 : value;
    return 0;
}

template <int D>
static void launch_dist_ct(const DistArgs& p, dim3 grid, hipStream_t s) {
    switch (g_dist_variant) {
        case 2: dist_colsum_kernel<D, 2, 4><<<grid, kColBlock, 0, s>>>(p); break;
        case 3: dist_colsum_kernel<D, 1, 8><<<grid, kColBlock, 0, s>>>(p); break;
        case 4: dist_colsum_kernel<D, 2, 8><<<grid, kColBlock, 0, s>>>(p); break;
        case 5: dist_colsum_kernel<D, 4, 4><<<grid, kColBlock, 0, s>>>(p); break;
        case 6: dist_colsum_kernel<D, 1, 4, true><<<grid, kColBlock, 0, s>>>(p); break;
        default: dist_colsum_kernel<D, 1, 4><<<grid, kColBlock, 0, s>>>(p); break;
    }
}

// B chunks per launch: enough (block, chunk) work units that the chip's 1024 resident blocks take
// many rounds of them, so the last round's imbalance is a small share of the launch, without chunks
// shorter than four staging tiles (1024 points).  Round 3 aimed at 2 048 units: the 2e5-point
// validation triangle then had ~1 170 equal full-chunk units for 1 024 slots -- two rounds, the
// second 14 % full (PMC: ~3 waves per SIMD on average, profiles/r04_energy_stall.json).  Same box,
// alternating (profiles/r04_energy_units_ab.log): 2 048 -> 22.5 ms per uncached curve, 8 192 -> 19.1,
// 16 384 -> 17.5, 32 768 -> 16.9 (0.148 -> 0.198 of fp64 peak); st_tune key 14 sets the target (grid
// blocks over both dimensions).
static int64_t g_dist_units = 32768;
int dist_units_tune(int value) {
    if (value != -1 && (value < 256 || value > (1 << 22))) return -1;
    g_dist_units = value < 0 ? 32768 : value;
    return 0;
}
int64_t distance_chunks(int64_t na, int64_t b_begin, int64_t b_end) {
    const int64_t ablocks = (na + kColBlock - 1) / kColBlock;
    const int64_t range = b_end - b_begin;
    if (ablocks <= 0 || range <= 0) return 1;
    int64_t K = (g_dist_units + ablocks - 1) / ablocks;
    const int64_t kmax = (range + 4 * kColBlock - 1) / (4 * kColBlock);
    if (K > kmax) K = kmax;
    if (K > 65535) K = 65535;
    return K < 1 ? 1 : K;
}

hipError_t launch_distance_colsum(const double* a, int64_t lda, int64_t na, const double* b,
                                  int64_t ldb, int64_t b0, int64_t b1, int d, int tri,
                                  double* out, double* ws, int64_t ws_doubles, hipStream_t s) {
    int64_t K = distance_chunks(na, b0, b1);
    if (!ws || ws_doubles < K * na) K = 1;   // no workspace: one chunk, sums straight into out
    const int64_t range = b1 - b0;
    int64_t chunk = K > 1 ? (range + K - 1) / K : (range > 0 ? range : 1);
    if (K > 1) chunk = (chunk + kColBlock - 1) / kColBlock * kColBlock;   // whole staging tiles
    DistArgs p{a, lda, na, b, ldb, b0, b1, tri, K > 1 ? ws : out, chunk};
    const dim3 grid((unsigned)((na + kColBlock - 1) / kColBlock), (unsigned)K);
    switch (d) {
        case 1: launch_dist_ct<1>(p, grid, s); break;
        case 2: launch_dist_ct<2>(p, grid, s); break;
        case 3: launch_dist_ct<3>(p, grid, s); break;
        case 4: launch_dist_ct<4>(p, grid, s); break;
        case 5: launch_dist_ct<5>(p, grid, s); break;
        case 6: launch_dist_ct<6>(p, grid, s); break;
        case 7: launch_dist_ct<7>(p, grid, s); break;
        case 8: launch_dist_ct<8>(p, grid, s); break;
        default: dist_colsum_rt_kernel<<<grid, kColBlock, 0, s>>>(p, d); break;
    }
    if (K > 1) dist_reduce_kernel<<<(unsigned)((na + 255) / 256), 256, 0, s>>>(ws, na, (int)K, out);
    return hipGetLastError();
}

template <int D>
static void launch_colsum_ct(const ColsumArgs& a, unsigned grid, hipStream_t s) {
    if (a.w) ksd_colsum_kernel<D, true><<<grid, kColBlock, 0, s>>>(a);
    else ksd_colsum_kernel<D, false><<<grid, kColBlock, 0, s>>>(a);
}

hipError_t launch_ksd_colsum(const PairArgs& p, int64_t n, int64_t a0, int64_t a1, double* csum,
                             hipStream_t s) {
    ColsumArgs a{p.x, p.g, p.w, n, p.ld, p.l, p.tr, a0, a1, csum, arith_compact()};
    // columns at or below a0 get no rows: zero them, then launch only the blocks above a0
    const int64_t first_block = (a0 + 1) / kColBlock;          // block containing column a0 + 1
    const int64_t nb = (n + kColBlock - 1) / kColBlock;
    if (first_block * kColBlock > 0) {
        hipError_t e = hipMemsetAsync(csum, 0, (size_t)(first_block * kColBlock < n ? first_block * kColBlock : n) * 8, s);
        if (e != hipSuccess) return e;
    }
    if (nb <= first_block || a1 <= a0) {
        if (nb > first_block) return hipMemsetAsync(csum, 0, (size_t)n * 8, s);
        return hipSuccess;
    }
    const unsigned grid = (unsigned)(nb - first_block);   // block b -> column block nb-1-b
    switch (p.d) {
        case 1: launch_colsum_ct<1>(a, grid, s); break;
        case 2: launch_colsum_ct<2>(a, grid, s); break;
        case 3: launch_colsum_ct<3>(a, grid, s); break;
        case 4: launch_colsum_ct<4>(a, grid, s); break;
        case 5: launch_colsum_ct<5>(a, grid, s); break;
        case 6: launch_colsum_ct<6>(a, grid, s); break;
        case 7: launch_colsum_ct<7>(a, grid, s); break;
        case 8: launch_colsum_ct<8>(a, grid, s); break;
        default:
            if (a.w) ksd_colsum_rt_kernel<true><<<grid, kColBlock, 0, s>>>(a, p.d);
            else ksd_colsum_rt_kernel<false><<<grid, kColBlock, 0, s>>>(a, p.d);
            break;
    }
    return hipGetLastError();
}

hipError_t launch_ksd_finish(const PairArgs& p, int64_t n, const double* csum, double* ks,
                             hipStream_t s) {
    ColsumArgs a{p.x, p.g, p.w, n, p.ld, p.l, p.tr, 0, 0, const_cast<double*>(csum)};
    ksd_finish_kernel<<<1, 1024, 0, s>>>(a, p.d, ks);
    return hipGetLastError();
}

__global__ void layout_soa_kernel(const double* __restrict__ rowmajor, int64_t n, int d, int64_t ld,
                                  double* __restrict__ soa) {
    const int64_t total = n * d;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e / d;
        const int k = (int)(e - i * d);
        soa[(int64_t)k * ld + i] = rowmajor[e];
    }
}

// the same with the per-dimension scaling of _validate_and_standardize applied on the way: x / scl
// (divide) or g * scl -- one IEEE operation per element, the bits of the host's st_standardize_host
__global__ void layout_soa_scaled_kernel(const double* __restrict__ rowmajor, int64_t n, int d, int64_t ld,
                                         const double* __restrict__ scale, int divide,
                                         double* __restrict__ soa) {
    const int64_t total = n * d;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e / d;
        const int k = (int)(e - i * d);
        const double v = rowmajor[e], c = scale[k];
        soa[(int64_t)k * ld + i] = divide ? v / c : v * c;
    }
}

static int grid_for(int64_t work, int block) {
    int64_t b = (work + block - 1) / block;
    if (b > 2048) b = 2048;
    if (b < 1) b = 1;
    return (int)b;
}

hipError_t launch_pairs(const PairArgs& p, const int64_t* i1, const int64_t* i2, int64_t L,
                        double* out, hipStream_t s) {
    pairs_kernel<<<grid_for(L, 256), 256, 0, s>>>(p, i1, i2, L, out);
    return hipGetLastError();
}

hipError_t launch_kmat(const PairArgs& p, const int64_t* idx, int64_t k, double* out,
                       hipStream_t s) {
    (void)idx;
    const int64_t nt = (k + kTile - 1) / kTile;
    dim3 grid((unsigned)nt, (unsigned)nt);
    kmat_kernel<<<grid, 256, 0, s>>>(p, k, out);
    return hipGetLastError();
}

hipError_t launch_layout_soa(const double* rowmajor, int64_t n, int d, int64_t ld, double* soa,
                             hipStream_t s) {
    layout_soa_kernel<<<grid_for(n * d, 256), 256, 0, s>>>(rowmajor, n, d, ld, soa);
    return hipGetLastError();
}

hipError_t launch_layout_soa_scaled(const double* rowmajor, int64_t n, int d, int64_t ld, const double* scale,
                                    int divide, double* soa, hipStream_t s) {
    layout_soa_scaled_kernel<<<grid_for(n * d, 256), 256, 0, s>>>(rowmajor, n, d, ld, scale, divide, soa);
    return hipGetLastError();
}

}  // namespace st
