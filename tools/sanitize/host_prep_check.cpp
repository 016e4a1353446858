// Host-code sanitizer driver (ASan + UBSan, or TSan): st_standardize_host over random shapes, the
// multi-threaded sizes, aliased outputs, NaN / inf / zero-scale inputs and invalid arguments,
// checked against a direct restatement (sequential column sums for d >= 2: exact; d = 1: NumPy's
// pairwise order against the sequential sums, 1e-11 relative; bit identity with NumPy itself is
// tests/test_shim_host.py's).  Built and run by scripts/sanitize_host.sh; any sanitizer report
// aborts (-fno-sanitize-recover=all), a wrong value exits 1.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <random>
#include <vector>

#include "../../include/stein_thinning_hip.h"

namespace st {   // host_prep.cpp: x's flags and loc / scl alone (st_standardize_download's general path)
void column_stats_any(const double* x, int64_t n, int d, double* loc, double* scl, int& nan, int& inf);
}

static int fails = 0;
#define CHECK(c, ...) do { if (!(c)) { printf("FAIL %s:%d: ", __FILE__, __LINE__); printf(__VA_ARGS__); printf("\n"); ++fails; } } while (0)

static void reference(const std::vector<double>& x, const std::vector<double>& g, int64_t n, int d,
                      std::vector<double>& xo, std::vector<double>& go, bool& zero) {
    std::vector<double> loc(d, 0.0), scl(d, 0.0);
    for (int j = 0; j < d; ++j) {
        double s = 0.0;
        for (int64_t i = 0; i < n; ++i) s += x[i * d + j];
        loc[j] = s / (double)n;
        double a = 0.0;
        for (int64_t i = 0; i < n; ++i) a += fabs(x[i * d + j] - loc[j]);
        scl[j] = a / (double)n;
    }
    zero = false;
    for (int j = 0; j < d; ++j) zero |= scl[j] == 0.0;
    xo.resize(x.size());
    go.resize(g.size());
    for (int64_t i = 0; i < n; ++i)
        for (int j = 0; j < d; ++j) { xo[i * d + j] = x[i * d + j] / scl[j]; go[i * d + j] = g[i * d + j] * scl[j]; }
}

static void run_case(int64_t n, int d, int kind, bool alias, std::mt19937_64& rng) {
    std::normal_distribution<double> nd(0.0, 1.0);
    std::vector<double> x((size_t)(n * d)), g((size_t)(n * d));
    for (auto& v : x) v = nd(rng) * 3.0 + 1.5;
    for (auto& v : g) v = nd(rng);
    if (n > 1) for (int j = 0; j < d; ++j) x[(n / 2) * d + j] = x[j];   // a duplicated row
    if (kind == 1) x[(size_t)((n * d) / 3)] = NAN;
    if (kind == 2) g[(size_t)((n * d) / 2)] = -INFINITY;
    if (kind == 3) for (int64_t i = 0; i < n; ++i) x[i * d + (d - 1)] = 4.25;   // constant column
    std::vector<double> xo, go;
    bool zero = false;
    if (kind == 0) reference(x, g, n, d, xo, go, zero);
    std::vector<double> xs = x, gs = g, loc(d), scl(d);
    std::vector<double> xout(alias ? 0 : x.size()), gout(alias ? 0 : g.size());
    int32_t status = -1;
    const int rc = st_standardize_host(x.data(), g.data(), n, d, 1, alias ? xs.data() : xout.data(),
                                       alias ? gs.data() : gout.data(), loc.data(), scl.data(), &status);
    CHECK(rc == ST_OK, "rc %d (n %lld d %d)", rc, (long long)n, d);
    const int want = kind == 0 ? (zero ? 3 : 0) : kind;
    CHECK(status == want, "status %d want %d (n %lld d %d kind %d)", status, want, (long long)n, d, kind);
    {   // the x-only statistics give the same flags (x's) and the same loc / scl bits
        std::vector<double> l2(d), s2(d);
        int fn = 0, fi = 0;
        st::column_stats_any(x.data(), n, d, l2.data(), s2.data(), fn, fi);
        CHECK(fn == (kind == 1) && fi == 0, "column_stats_any flags %d %d (kind %d)", fn, fi, kind);
        if (kind == 0 && status == 0)
            for (int j = 0; j < d; ++j)
                CHECK(l2[j] == loc[j] && s2[j] == scl[j], "column_stats_any loc/scl[%d] (n %lld d %d)", j,
                      (long long)n, d);
    }
    if (kind != 0 || status != 0) return;
    const std::vector<double>& gx = alias ? xs : xout;
    const std::vector<double>& gg = alias ? gs : gout;
    const double tol = d == 1 ? 1e-11 : 0.0;   // d = 1: NumPy's pairwise order vs the sequential restatement
    for (size_t e = 0; e < x.size(); ++e) {
        CHECK(fabs(gx[e] - xo[e]) <= tol * fabs(xo[e]), "x[%zu] %.17g vs %.17g (n %lld d %d)", e, gx[e], xo[e], (long long)n, d);
        CHECK(fabs(gg[e] - go[e]) <= tol * fabs(go[e]), "g[%zu] %.17g vs %.17g (n %lld d %d)", e, gg[e], go[e], (long long)n, d);
        if (fails > 20) return;
    }
}

int main() {
    std::mt19937_64 rng(12345);
    const int64_t ns[] = {1, 2, 7, 129, 8193, 70001, 300003};
    const int ds[] = {1, 2, 3, 50, 128};
    for (int64_t n : ns)
        for (int d : ds) {
            if (n * d > 8000000) continue;
            for (int kind = 0; kind < 4; ++kind)
                for (int alias = 0; alias < 2; ++alias) run_case(n, d, kind, alias != 0, rng);
        }
    // standardize = 0 copies through; invalid arguments are rejected without touching memory
    std::vector<double> x(12, 1.0), g(12, 2.0), xo(12), go(12);
    int32_t st = -1;
    CHECK(st_standardize_host(x.data(), g.data(), 4, 3, 0, xo.data(), go.data(), nullptr, nullptr, &st) == ST_OK && st == 0 &&
              xo[11] == 1.0 && go[0] == 2.0, "standardize = 0");
    CHECK(st_standardize_host(nullptr, g.data(), 4, 3, 1, xo.data(), go.data(), nullptr, nullptr, &st) == ST_ERR_INVALID, "NULL sample");
    CHECK(st_standardize_host(x.data(), g.data(), 0, 3, 1, xo.data(), go.data(), nullptr, nullptr, &st) == ST_ERR_INVALID, "n = 0");
    CHECK(st_standardize_host(x.data(), g.data(), 4, 0, 1, xo.data(), go.data(), nullptr, nullptr, &st) == ST_ERR_INVALID, "d = 0");
    CHECK(st_standardize_host(x.data(), g.data(), 4, 3, 1, xo.data(), go.data(), nullptr, nullptr, nullptr) == ST_ERR_INVALID, "NULL status");
    printf("%s: %d failure(s)\n", fails ? "FAILED" : "ok", fails);
    return fails ? 1 : 0;
}
