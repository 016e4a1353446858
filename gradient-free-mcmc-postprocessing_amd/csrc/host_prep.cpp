// Host-side input preparation of stein_thinning.thinning._validate_and_standardize (restated at
// JAX_Stein_Thinning.ipynb cells 15-18, json ~212, 476), bit-identical to the
// NumPy expressions it replaces:
//     NaN / inf checks (np.isnan(...).any(), np.isinf(...).any()), then
//     loc = np.mean(x, axis=0); scl = np.mean(np.abs(x - loc), axis=0); x / scl; g * scl
// NumPy reduces a C-contiguous (n, d) array along axis 0 row by row (sequential per column) for
// d >= 2, and with its pairwise summation over 8192-element buffer chunks when d == 1 (the column
// is contiguous; NumPy's default bufsize -- the shim falls back to NumPy if it was changed); the
// division of the sum by n is one IEEE division.  One pass over x and g for the checks + column sums, one for
// the absolute deviations, one (row-parallel) for the scaling -- instead of NumPy's seven passes and
// four temporaries.  Pure host code, no HIP calls.
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <initializer_list>

#include <algorithm>
#include <thread>
#include <vector>

#include <emmintrin.h>

#include "../../include/stein_thinning_hip.h"

namespace {

// numpy/core/src/umath/loops_utils.h.src pairwise_sum (PW_BLOCKSIZE 128), stride 1
double pairwise_sum(const double* a, int64_t n) {
    if (n < 8) {
        double res = -0.0;   // NumPy starts at -0.0 so that a sum of -0.0 stays -0.0
        for (int64_t i = 0; i < n; ++i) res += a[i];
        return res;
    }
    if (n <= 128) {
        double r[8];
        for (int k = 0; k < 8; ++k) r[k] = a[k];
        int64_t i;
        for (i = 8; i < n - (n % 8); i += 8)
            for (int k = 0; k < 8; ++k) r[k] += a[i + k];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; ++i) res += a[i];
        return res;
    }
    int64_t n2 = n / 2;
    n2 -= n2 % 8;
    return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
}

// np.add.reduce over one contiguous column: the ufunc loop runs on buffer-sized chunks (NumPy's
// default bufsize, 8192 elements), each a pairwise sum added to the accumulator (start: 0)
constexpr int64_t kNumpyBufsize = 8192;
double numpy_column_sum(const double* a, int64_t n) {
    double acc = 0.0;
    for (int64_t c = 0; c < n; c += kNumpyBufsize)
        acc += pairwise_sum(a + c, n - c < kNumpyBufsize ? n - c : kNumpyBufsize);
    return acc;
}

int hardware_threads() {
    const unsigned h = std::thread::hardware_concurrency();
    return h == 0 ? 1 : (int)std::min(h, 16u);
}

// d = 2 .. 8: both column passes over x by ONE thread, every column's sequential sum in registers
// (one stream of the array instead of one per column thread, each of which had to fetch every cache
// line), with x's NaN / inf flags taken in the first pass; g is scanned by the other threads meanwhile.
template <int D>
void column_stats(const double* x, int64_t n, double* loc, double* scl, int& nan, int& inf) {
    double acc[D];
    int fn = 0, fi = 0;
#pragma unroll
    for (int j = 0; j < D; ++j) {
        acc[j] = x[j];
        fn |= (int)(x[j] != x[j]);
        fi |= (int)(fabs(x[j]) == INFINITY);
    }
    for (int64_t i = 1; i < n; ++i) {
        const double* row = x + i * D;
        __builtin_prefetch(row + 64 * D);
#pragma unroll
        for (int j = 0; j < D; ++j) {
            acc[j] += row[j];
            fn |= (int)(row[j] != row[j]);
            fi |= (int)(fabs(row[j]) == INFINITY);
        }
    }
    nan = fn;
    inf = fi;
    if (fn | fi) return;
    const double dn = (double)n;
    double l[D];
#pragma unroll
    for (int j = 0; j < D; ++j) { l[j] = acc[j] / dn; acc[j] = fabs(x[j] - l[j]); }
    for (int64_t i = 1; i < n; ++i) {
        const double* row = x + i * D;
        __builtin_prefetch(row + 64 * D);
#pragma unroll
        for (int j = 0; j < D; ++j) acc[j] += fabs(row[j] - l[j]);
    }
#pragma unroll
    for (int j = 0; j < D; ++j) { loc[j] = l[j]; scl[j] = acc[j] / dn; }
}

using StatsFn = void (*)(const double*, int64_t, double*, double*, int&, int&);
StatsFn stats_for(int d) {
    switch (d) {
        case 2: return column_stats<2>;
        case 3: return column_stats<3>;
        case 4: return column_stats<4>;
        case 5: return column_stats<5>;
        case 6: return column_stats<6>;
        case 7: return column_stats<7>;
        case 8: return column_stats<8>;
        default: return nullptr;
    }
}

// loc / scl of a NaN / inf-free x outside the d = 2 .. 8 single pass: d == 1 the pairwise column sum,
// d > 8 row-by-row accumulation (NumPy's axis-0 order: sequential per column) with the columns split
// over up to hw threads (contiguous column groups)
template <typename Par>
void stats_general(const double* sample, int64_t n, int d, int hw, double* loc, double* scl, Par&& parallel) {
    const double dn = (double)n;
    if (d == 1) {
        loc[0] = numpy_column_sum(sample, n) / dn;
        std::vector<double> dev((size_t)n);
        for (int64_t i = 0; i < n; ++i) dev[i] = fabs(sample[i] - loc[0]);
        scl[0] = numpy_column_sum(dev.data(), n) / dn;
        return;
    }
    const int tc = (int)std::max<int64_t>(1, std::min<int64_t>({(int64_t)hw, (int64_t)d, n / 65536}));
    parallel(tc, [&](int t, int T) {
        const int j0 = d * t / T, j1 = d * (t + 1) / T, w = j1 - j0;
        std::vector<double> acc(sample + j0, sample + j1);
        for (int64_t i = 1; i < n; ++i) {
            const double* row = sample + i * d + j0;
            for (int j = 0; j < w; ++j) acc[j] += row[j];
        }
        for (int j = 0; j < w; ++j) loc[j0 + j] = acc[j] / dn;
        for (int j = 0; j < w; ++j) acc[j] = fabs(sample[j0 + j] - loc[j0 + j]);
        for (int64_t i = 1; i < n; ++i) {
            const double* row = sample + i * d + j0;
            for (int j = 0; j < w; ++j) acc[j] += fabs(row[j] - loc[j0 + j]);
        }
        for (int j = 0; j < w; ++j) scl[j0 + j] = acc[j] / dn;
    });
}

// run fn(t, T) on T threads (T = 1: inline)
struct Parallel {
    template <typename Fn>
    void operator()(int T, Fn&& fn) const {
        if (T <= 1) { fn(0, 1); return; }
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) th.emplace_back([&fn, t, T] { fn(t, T); });
        for (auto& x : th) x.join();
    }
};

}  // namespace

namespace st {
// for st_standardize_download (prep_upload.cpp): x's NaN / inf flags, then loc / scl, any n >= 1, d >= 1
void column_stats_any(const double* x, int64_t n, int d, double* loc, double* scl, int& nan, int& inf) {
    if (StatsFn f = stats_for(d)) { f(x, n, loc, scl, nan, inf); return; }
    int fn = 0, fi = 0;
    for (int64_t e = 0; e < n * (int64_t)d; ++e) {
        fn |= (int)(x[e] != x[e]);
        fi |= (int)(fabs(x[e]) == INFINITY);
    }
    nan = fn;
    inf = fi;
    if (fn | fi) return;
    stats_general(x, n, d, hardware_threads(), loc, scl, Parallel{});
}
// for st_standardize_upload (prep_upload.cpp): the d = 2 .. 8 single-thread column pass over x
bool column_stats_fast(const double* x, int64_t n, int d, double* loc, double* scl, int& nan, int& inf) {
    StatsFn f = stats_for(d);
    if (!f) return false;
    f(x, n, loc, scl, nan, inf);
    return true;
}
int host_threads() { return hardware_threads(); }
}  // namespace st

extern "C" int st_standardize_host(const double* sample, const double* gradient, int64_t n,
                                   int32_t d, int32_t standardize, double* sample_out,
                                   double* gradient_out, double* loc_out, double* scl_out,
                                   int32_t* status) {
    // status: 0 ok, 1 NaN in sample/gradient, 2 inf, 3 a zero scale ("too few unique samples")
    if (!sample || !gradient || !sample_out || !gradient_out || !status || n < 1 || d < 1)
        return ST_ERR_INVALID;
    *status = 0;
    const int64_t total = n * (int64_t)d;
    const int hw = hardware_threads();
    const Parallel parallel;
    std::vector<double> loc(d, 0.0), scl(d, 0.0);
    StatsFn fast = standardize && n >= 65536 ? stats_for(d) : nullptr;
    if (fast) {
        // thread 0: x's flags, column sums and absolute deviations; the others: g's flags
        const int tg = std::max(1, hw - 1);
        std::vector<int> nanf(tg + 1, 0), inff(tg + 1, 0);
        parallel(tg + 1, [&](int t, int) {
            if (t == 0) {
                fast(sample, n, loc.data(), scl.data(), nanf[0], inff[0]);
                return;
            }
            bool nan = false, inf = false;
            for (int64_t e = total * (t - 1) / tg; e < total * t / tg; ++e) {
                const double gv = gradient[e];
                nan |= gv != gv;
                inf |= fabs(gv) == INFINITY;
            }
            nanf[t] = nan;
            inff[t] = inf;
        });
        for (int t = 0; t <= tg; ++t) if (nanf[t]) { *status = 1; return ST_OK; }
        for (int t = 0; t <= tg; ++t) if (inff[t]) { *status = 2; return ST_OK; }
    }
    // pass 1: NaN / inf flags (NaN reported first, as the NumPy checks run in that order)
    const int tn = (int)std::max<int64_t>(1, std::min<int64_t>(hw, total / (1 << 18)));
    std::vector<int> nanf(tn, 0), inff(tn, 0);
    if (!fast) parallel(tn, [&](int t, int T) {
        bool nan = false, inf = false;
        for (int64_t e = total * t / T; e < total * (t + 1) / T; ++e) {
            const double xv = sample[e], gv = gradient[e];
            nan |= (int)(xv != xv) | (int)(gv != gv);
            inf |= (int)(fabs(xv) == INFINITY) | (int)(fabs(gv) == INFINITY);
        }
        nanf[t] = nan;
        inff[t] = inf;
    });
    for (int t = 0; t < tn; ++t) if (nanf[t]) { *status = 1; return ST_OK; }
    for (int t = 0; t < tn; ++t) if (inff[t]) { *status = 2; return ST_OK; }
    if (!standardize) {
        if (sample_out != sample) memcpy(sample_out, sample, (size_t)total * 8);
        if (gradient_out != gradient) memcpy(gradient_out, gradient, (size_t)total * 8);
        return ST_OK;
    }
    if (!fast) stats_general(sample, n, d, hw, loc.data(), scl.data(), parallel);   // else: done above
    for (int j = 0; j < d; ++j)
        if (scl[j] == 0.0) { *status = 3; return ST_OK; }
    if (loc_out) memcpy(loc_out, loc.data(), (size_t)d * 8);
    if (scl_out) memcpy(scl_out, scl.data(), (size_t)d * 8);
    // pass 3: x / scl, g * scl -- elementwise, row blocks in parallel.  Large 16-B-aligned outputs
    // (the page-locked upload buffers) are written with non-temporal stores, two elements per
    // instruction (IEEE division / multiplication either way: the same bits): no read-for-ownership
    // of lines that are only written, and nothing the upload reads back evicted from the caches
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(hw, n / 65536));
    const bool nt_ok = n >= 65536 && d <= 64 && ((uintptr_t)sample_out % 16 == 0) &&
                       ((uintptr_t)gradient_out % 16 == 0) && ((uintptr_t)sample % 8 == 0) &&
                       ((uintptr_t)gradient % 8 == 0);
    if (nt_ok) {
        std::vector<double> rep(2 * (size_t)d + 2);   // scl repeated: rep[k .. k+1] = scl[k % d], scl[(k+1) % d]
        for (size_t k = 0; k < rep.size(); ++k) rep[k] = scl[k % d];
        parallel(nt, [&](int t, int T) {
            int64_t e0 = total * t / T;
            const int64_t e1 = total * (t + 1) / T;
            e0 += e0 & 1;                                // even start: 16-B aligned output
            auto scalar = [&](int64_t e) {
                sample_out[e] = sample[e] / scl[e % d];
                gradient_out[e] = gradient[e] * scl[e % d];
            };
            int64_t e = e0;
            int k = (int)(e % d);
            for (; e + 1 < e1; e += 2) {
                const __m128d sv = _mm_loadu_pd(rep.data() + k);
                _mm_stream_pd(sample_out + e, _mm_div_pd(_mm_loadu_pd(sample + e), sv));
                _mm_stream_pd(gradient_out + e, _mm_mul_pd(_mm_loadu_pd(gradient + e), sv));
                k += 2;
                while (k >= d) k -= d;   // (d = 1: twice)
            }
            for (; e < e1; ++e) scalar(e);
            // the element this thread's range skipped to start even belongs to the previous thread
            if (t > 0 && ((total * t / T) & 1)) scalar(total * t / T);
            _mm_sfence();
        });
        return ST_OK;
    }
    parallel(nt, [&](int t, int T) {
        for (int64_t i = n * t / T; i < n * (t + 1) / T; ++i)
            for (int j = 0; j < d; ++j) {
                sample_out[i * d + j] = sample[i * d + j] / scl[j];
                gradient_out[i * d + j] = gradient[i * d + j] * scl[j];
            }
    });
    return ST_OK;
}
