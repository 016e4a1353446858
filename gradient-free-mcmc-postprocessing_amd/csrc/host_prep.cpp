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

}  // namespace

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
    // run fn(t, T) on T threads (T = 1: inline)
    auto parallel = [](int T, auto&& fn) {
        if (T <= 1) { fn(0, 1); return; }
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) th.emplace_back([&fn, t, T] { fn(t, T); });
        for (auto& x : th) x.join();
    };
    // pass 1: NaN / inf flags (NaN reported first, as the NumPy checks run in that order)
    const int tn = (int)std::max<int64_t>(1, std::min<int64_t>(hw, total / (1 << 18)));
    std::vector<int> nanf(tn, 0), inff(tn, 0);
    parallel(tn, [&](int t, int T) {
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
    std::vector<double> loc(d, 0.0), scl(d, 0.0);
    const double dn = (double)n;
    if (d == 1) {
        loc[0] = numpy_column_sum(sample, n) / dn;
        std::vector<double> dev((size_t)n);
        for (int64_t i = 0; i < n; ++i) dev[i] = fabs(sample[i] - loc[0]);
        scl[0] = numpy_column_sum(dev.data(), n) / dn;
    } else {
        // row-by-row accumulation acc[j] += x[i, j] (NumPy's axis-0 reduction order): sequential
        // per column, so the columns are split over threads (contiguous column groups)
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
    for (int j = 0; j < d; ++j)
        if (scl[j] == 0.0) { *status = 3; return ST_OK; }
    if (loc_out) memcpy(loc_out, loc.data(), (size_t)d * 8);
    if (scl_out) memcpy(scl_out, scl.data(), (size_t)d * 8);
    // pass 3: x / scl, g * scl -- elementwise, row blocks in parallel
    const int nt = (int)std::max<int64_t>(1, std::min<int64_t>(hw, n / 65536));
    parallel(nt, [&](int t, int T) {
        for (int64_t i = n * t / T; i < n * (t + 1) / T; ++i)
            for (int j = 0; j < d; ++j) {
                sample_out[i * d + j] = sample[i * d + j] / scl[j];
                gradient_out[i * d + j] = gradient[i * d + j] * scl[j];
            }
    });
    return ST_OK;
}
