// Host input preparation with the upload running underneath it (the drop-in thin's path, round 4).
//
// _validate_and_standardize (JAX_Stein_Thinning.ipynb cells 15-18) needs two sequential passes over
// the sample's columns -- NumPy's axis-0 reductions are one dependency chain of n adds per column,
// which bit-exactness keeps on one core (host_prep.cpp) -- and only then can x / scl, g * scl be
// formed.  st_standardize_host does the scaling on the host and the arrays go up afterwards.  Here
// thread 0 runs the column passes while the other threads copy the RAW x and g into page-locked
// staging buffers (with g's NaN / inf scan fused in) and queue each copied chunk's DMA to the device
// at once, so the upload is finished, or nearly, when the statistics are; the caller then applies
// the scaling on the device (st_layout_soa_scaled: one IEEE division / multiplication per element,
// the same bits as the host's).  Returns ST_ERR_UNSUPPORTED outside the d = 2 .. 8, n >= 65536 case
// the single-thread column pass covers; the caller then takes the st_standardize_host route.
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include <emmintrin.h>

#include "../../include/stein_thinning_hip.h"

namespace st {
bool column_stats_fast(const double* x, int64_t n, int d, double* loc, double* scl, int& nan, int& inf);
void column_stats_any(const double* x, int64_t n, int d, double* loc, double* scl, int& nan, int& inf);
int host_threads();
int report_error(int code, const char* msg);   // capi.hip: sets st_last_error()
}  // namespace st

namespace {

constexpr int64_t kChunk = 1 << 19;   // elements per DMA (4 MB)

// copy src[e0, e1) into stage (16-B aligned base) with non-temporal stores; optionally flag NaN / inf
void copy_scan(const double* src, double* stage, int64_t e0, int64_t e1, bool scan, bool& nan, bool& inf) {
    int64_t e = e0;
    if ((e & 1) && e < e1) {   // to an even element: 16-B aligned stores
        const double v = src[e];
        stage[e] = v;
        nan |= scan && v != v;
        inf |= scan && fabs(v) == INFINITY;
        ++e;
    }
    const __m128d vinf = _mm_set1_pd(INFINITY);
    const __m128d absmask = _mm_castsi128_pd(_mm_set1_epi64x(0x7FFFFFFFFFFFFFFFll));
    __m128d anynan = _mm_setzero_pd(), anyinf = _mm_setzero_pd();
    for (; e + 1 < e1; e += 2) {
        const __m128d v = _mm_loadu_pd(src + e);
        _mm_stream_pd(stage + e, v);
        if (scan) {
            anynan = _mm_or_pd(anynan, _mm_cmpunord_pd(v, v));
            anyinf = _mm_or_pd(anyinf, _mm_cmpeq_pd(_mm_and_pd(v, absmask), vinf));
        }
    }
    nan |= _mm_movemask_pd(anynan) != 0;
    inf |= _mm_movemask_pd(anyinf) != 0;
    for (; e < e1; ++e) {
        const double v = src[e];
        stage[e] = v;
        nan |= scan && v != v;
        inf |= scan && fabs(v) == INFINITY;
    }
}

}  // namespace

extern "C" int st_standardize_upload(const double* sample, const double* gradient, int64_t n, int32_t d,
                                     double* stage_x, double* stage_g, double* dev_x, double* dev_g,
                                     double* loc_out, double* scl_out, int32_t* status, void* stream) {
    if (!sample || !gradient || !stage_x || !stage_g || !dev_x || !dev_g || !loc_out || !scl_out || !status)
        return st::report_error(ST_ERR_INVALID, "st_standardize_upload: NULL pointer");
    if ((uintptr_t)stage_x % 16 || (uintptr_t)stage_g % 16)
        return st::report_error(ST_ERR_INVALID, "st_standardize_upload: staging buffers must be 16-byte aligned");
    if (d < 2 || d > 8 || n < 65536)
        return st::report_error(ST_ERR_UNSUPPORTED, "st_standardize_upload: d = 2 .. 8 and n >= 65536 only");
    *status = 0;
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t total = n * (int64_t)d;
    const int tc = std::max(1, st::host_threads() - 1);   // copy threads; thread 0 runs the column pass
    std::vector<char> gnan(tc, 0), ginf(tc, 0);
    std::atomic<int> dma_err{0};
    int xnan = 0, xinf = 0;
    double loc[8], scl[8];
    std::vector<std::thread> th;
    th.emplace_back([&] { st::column_stats_fast(sample, n, d, loc, scl, xnan, xinf); });
    for (int t = 0; t < tc; ++t) {
        th.emplace_back([&, t] {
            const int64_t e0 = total * t / tc, e1 = total * (t + 1) / tc;
            bool nan = false, inf = false;
            for (int pass = 0; pass < 2; ++pass) {   // this thread's part of x, then of g
                const double* src = pass ? gradient : sample;
                double* stage = pass ? stage_g : stage_x;
                double* dev = pass ? dev_g : dev_x;
                for (int64_t c = e0; c < e1; c += kChunk) {
                    const int64_t ce = std::min(c + kChunk, e1);
                    copy_scan(src, stage, c, ce, pass == 1, nan, inf);
                    _mm_sfence();   // the staged chunk is in memory before the DMA reads it
                    if (hipMemcpyAsync(dev + c, stage + c, (size_t)(ce - c) * 8, hipMemcpyHostToDevice, s) !=
                        hipSuccess)
                        dma_err.store(1);
                }
            }
            gnan[t] = nan;
            ginf[t] = inf;
        });
    }
    for (auto& x : th) x.join();
    if (dma_err.load()) {
        (void)hipStreamSynchronize(s);
        return st::report_error(ST_ERR_HIP, "st_standardize_upload: a host-to-device copy could not be queued");
    }
    // NaN reported before inf, as the NumPy checks run in that order
    bool nan = xnan != 0, inf = xinf != 0;
    for (int t = 0; t < tc; ++t) { nan |= gnan[t] != 0; inf |= ginf[t] != 0; }
    if (nan || inf) {
        *status = nan ? 1 : 2;
    } else {
        for (int j = 0; j < d; ++j)
            if (scl[j] == 0.0) *status = 3;
    }
    if (*status) {   // the caller drops the buffers: let the queued copies finish reading them first
        (void)hipStreamSynchronize(s);
        return ST_OK;
    }
    memcpy(loc_out, loc, (size_t)d * 8);
    memcpy(scl_out, scl, (size_t)d * 8);
    return ST_OK;
}

namespace {
// st_standardize_download's two column passes over the page-locked copy, the first one chunk by chunk
// as the copies land (event c = rows [c kRows, (c + 1) kRows) are on the host): the sequential sums of
// st_standardize_host's column_stats, x's NaN / inf flags, then the absolute deviations from loc
template <int D>
int download_stats(const double* x, int64_t n, int64_t kRows, const std::vector<hipEvent_t>& ev, double* loc,
                   double* scl, int& nan, int& inf) {
    double acc[D];
    int fn = 0, fi = 0;
    for (size_t c = 0; c < ev.size(); ++c) {
        if (hipEventSynchronize(ev[c]) != hipSuccess) return ST_ERR_HIP;
        const int64_t r0 = (int64_t)c * kRows, r1 = std::min(n, r0 + kRows);
        int64_t i = r0;
        if (c == 0) {
#pragma unroll
            for (int j = 0; j < D; ++j) {
                acc[j] = x[j];
                fn |= (int)(x[j] != x[j]);
                fi |= (int)(fabs(x[j]) == INFINITY);
            }
            i = 1;
        }
        for (; i < r1; ++i) {
            const double* row = x + i * D;
            __builtin_prefetch(row + 64 * D);
#pragma unroll
            for (int j = 0; j < D; ++j) {
                acc[j] += row[j];
                fn |= (int)(row[j] != row[j]);
                fi |= (int)(fabs(row[j]) == INFINITY);
            }
        }
    }
    nan = fn;
    inf = fi;
    if (fn | fi) return ST_OK;
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
    return ST_OK;
}
}  // namespace

// The reverse direction for samples that already live on the device (the drop-in thin called with ROCm
// tensors): only x has to visit the host -- the column sums are one dependency chain of n adds per
// column, which a CPU core runs ~8x faster than a GPU lane -- and g never leaves the device (its NaN /
// inf flags are the caller's device reduction).  x comes back in 64 K-row chunks on `stream`, each
// summed as it lands (NumPy's axis-0 order: acc[j] += x[i, j], row after row), then the absolute
// deviations from loc in a second pass over the page-locked copy; the caller scales on the device
// (st_layout_soa_scaled from the original device arrays).  *status: 0 ok, 1 NaN in x, 2 inf in x, 3 a
// zero scale (x's flags only).  Other shapes (d = 1 or d > 8, n < 65536): one copy, then the host
// routine's column passes (d = 1: NumPy's pairwise sums over its default 8192-element buffer).
extern "C" int st_standardize_download(const double* dev_x, int64_t n, int32_t d, double* stage_x, double* loc_out,
                                       double* scl_out, int32_t* status, void* stream) {
    if (!dev_x || !stage_x || !loc_out || !scl_out || !status)
        return st::report_error(ST_ERR_INVALID, "st_standardize_download: NULL pointer");
    if (n < 1 || d < 1) return st::report_error(ST_ERR_INVALID, "st_standardize_download: empty input");
    *status = 0;
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (d < 2 || d > 8 || n < 65536) {   // one copy, then the host routine's column passes on x alone
        if (hipMemcpyAsync(stage_x, dev_x, (size_t)n * d * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return st::report_error(ST_ERR_HIP, "st_standardize_download: a device-to-host copy failed");
        std::vector<double> l((size_t)d), c((size_t)d);
        int fn = 0, fi = 0;
        st::column_stats_any(stage_x, n, d, l.data(), c.data(), fn, fi);
        if (fn || fi) {
            *status = fn ? 1 : 2;
            return ST_OK;
        }
        for (int j = 0; j < d; ++j) {
            if (c[j] == 0.0) *status = 3;
            loc_out[j] = l[j];
            scl_out[j] = c[j];
        }
        return ST_OK;
    }
    constexpr int64_t kRows = 1 << 16;
    const int64_t chunks = (n + kRows - 1) / kRows;
    std::vector<hipEvent_t> ev((size_t)chunks, nullptr);
    int rc = ST_OK;
    for (int64_t c = 0; c < chunks && rc == ST_OK; ++c) {
        const int64_t r0 = c * kRows, r1 = std::min(n, r0 + kRows);
        if (hipEventCreateWithFlags(&ev[c], hipEventDisableTiming) != hipSuccess ||
            hipMemcpyAsync(stage_x + r0 * d, dev_x + r0 * d, (size_t)(r1 - r0) * d * 8, hipMemcpyDeviceToHost, s) !=
                hipSuccess ||
            hipEventRecord(ev[c], s) != hipSuccess)
            rc = ST_ERR_HIP;
    }
    int fn = 0, fi = 0;
    if (rc == ST_OK) {
        switch (d) {   // compile-time d: each column's chain in a register, the row loop unrolled
            case 2: rc = download_stats<2>(stage_x, n, kRows, ev, loc_out, scl_out, fn, fi); break;
            case 3: rc = download_stats<3>(stage_x, n, kRows, ev, loc_out, scl_out, fn, fi); break;
            case 4: rc = download_stats<4>(stage_x, n, kRows, ev, loc_out, scl_out, fn, fi); break;
            case 5: rc = download_stats<5>(stage_x, n, kRows, ev, loc_out, scl_out, fn, fi); break;
            case 6: rc = download_stats<6>(stage_x, n, kRows, ev, loc_out, scl_out, fn, fi); break;
            case 7: rc = download_stats<7>(stage_x, n, kRows, ev, loc_out, scl_out, fn, fi); break;
            default: rc = download_stats<8>(stage_x, n, kRows, ev, loc_out, scl_out, fn, fi); break;
        }
    }
    for (auto e : ev)
        if (e) (void)hipEventDestroy(e);
    if (rc != ST_OK) {
        (void)hipStreamSynchronize(s);
        return st::report_error(rc, "st_standardize_download: a device-to-host copy failed");
    }
    if (fn || fi) {
        *status = fn ? 1 : 2;
        return ST_OK;
    }
    for (int j = 0; j < d; ++j)
        if (scl_out[j] == 0.0) *status = 3;
    return ST_OK;
}
