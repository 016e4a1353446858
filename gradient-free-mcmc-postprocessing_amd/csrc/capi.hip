// C ABI (include/stein_thinning_hip.h): argument validation, workspace carving, launch sequencing.
// No allocation, no synchronisation: every entry point only enqueues work on the caller's stream.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include "../../include/stein_thinning_hip.h"
#include "stein_internal.hpp"

namespace {

thread_local char g_err[512] = "";

int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
    return code;
}

int hip_check(hipError_t e, const char* what) {
    if (e == hipSuccess) return ST_OK;
    return fail(ST_ERR_HIP, "%s: %s", what, hipGetErrorString(e));
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

int check_problem(const double* x, const double* g, const double* w, int64_t n, int32_t d,
                  int64_t ld) {
    if (!x || !g) return fail(ST_ERR_INVALID, "sample/gradient pointer is NULL");
    if (n < 1) return fail(ST_ERR_INVALID, "n must be >= 1 (got %lld)", (long long)n);
    if (d < 1) return fail(ST_ERR_INVALID, "d must be >= 1 (got %d)", d);
    if (d > st::kMaxDim)
        return fail(ST_ERR_UNSUPPORTED, "d = %d exceeds the supported maximum %d", d, st::kMaxDim);
    if (ld < n + (n & 1) || (ld & 1))
        return fail(ST_ERR_INVALID, "ld must be even and >= n + (n & 1) (n=%lld, ld=%lld)",
                    (long long)n, (long long)ld);
    if (!aligned16(x) || !aligned16(g) || (w && !aligned16(w)))
        return fail(ST_ERR_INVALID, "device arrays must be 16-byte aligned");
    return ST_OK;
}

// workspace layout: [ticket: 16 B][part_val: kMaxBlocks f64][part_idx: kMaxBlocks i64][cands: 2 x stride f64]
struct GreedyWs {
    unsigned* ticket;
    double* part_val;
    int64_t* part_idx;
    double* cands;
};

int64_t greedy_ws_bytes(int32_t d) {
    return 16 + (int64_t)st::kMaxBlocks * 16 + 2 * st::cand_stride(d) * 8;
}

GreedyWs carve(void* ws, int32_t d) {
    char* p = static_cast<char*>(ws);
    GreedyWs w;
    w.ticket = reinterpret_cast<unsigned*>(p);
    w.part_val = reinterpret_cast<double*>(p + 16);
    w.part_idx = reinterpret_cast<int64_t*>(p + 16 + (int64_t)st::kMaxBlocks * 8);
    w.cands = reinterpret_cast<double*>(p + 16 + (int64_t)st::kMaxBlocks * 16);
    (void)d;
    return w;
}

st::GreedyArgs make_args(const double* x, const double* g, const double* w, int64_t n, int32_t d,
                         int64_t ld, double l, double tr, double* A, const GreedyWs& ws) {
    st::GreedyArgs a{};
    a.x = x; a.g = g; a.w = w; a.A = A;
    a.n = n; a.ld = ld; a.d = d; a.l = l; a.tr = tr;
    a.row_offset = 0;
    a.nranks = 1;
    a.cand_stride = st::cand_stride(d);
    a.part_val = ws.part_val; a.part_idx = ws.part_idx; a.ticket = ws.ticket;
    return a;
}

}  // namespace

extern "C" {

int st_abi_version(void) { return ST_ABI_VERSION; }

const char* st_last_error(void) { return g_err; }

int64_t st_greedy_workspace_bytes(int64_t n, int32_t d, int32_t nranks) {
    (void)n; (void)nranks;
    if (d < 1 || d > st::kMaxDim) return -1;
    return greedy_ws_bytes(d);
}

int64_t st_candidate_stride(int32_t d) {
    if (d < 1 || d > st::kMaxDim) return -1;
    return st::cand_stride(d);
}

int st_greedy(const double* x_soa, const double* g_soa, const double* weights, int64_t n,
              int32_t d, int64_t ld, double linv_scale, double linv_trace, int64_t n_points,
              uint32_t* idx_out, double* a_work, void* workspace, int64_t workspace_bytes,
              void* stream) {
    int rc = check_problem(x_soa, g_soa, weights, n, d, ld);
    if (rc) return rc;
    if (n_points < 1) return fail(ST_ERR_INVALID, "n_points must be >= 1");
    if (!idx_out || !a_work || !workspace) return fail(ST_ERR_INVALID, "NULL output/workspace");
    if (!aligned16(a_work) || !aligned16(workspace))
        return fail(ST_ERR_INVALID, "a_work/workspace must be 16-byte aligned");
    if (workspace_bytes < greedy_ws_bytes(d))
        return fail(ST_ERR_INVALID, "workspace too small (%lld < %lld)", (long long)workspace_bytes,
                    (long long)greedy_ws_bytes(d));
    hipStream_t s = static_cast<hipStream_t>(stream);
    GreedyWs ws = carve(workspace, d);
    rc = hip_check(hipMemsetAsync(ws.ticket, 0, 16, s), "hipMemsetAsync(ticket)");
    if (rc) return rc;
    st::GreedyArgs a = make_args(x_soa, g_soa, weights, n, d, ld, linv_scale, linv_trace, a_work, ws);
    a.idx_out = idx_out;
    const int64_t stride = a.cand_stride;
    for (int64_t t = 0; t < n_points; ++t) {
        a.t = t;
        a.cands_in = ws.cands + ((t + 1) & 1) * stride;
        a.cand_out = ws.cands + (t & 1) * stride;
        rc = hip_check(st::launch_greedy_step(a, t == 0, s), "greedy step launch");
        if (rc) return rc;
    }
    return hip_check(st::launch_greedy_finalize(ws.cands + ((n_points - 1) & 1) * stride, 1,
                                                stride, idx_out, n_points - 1, s),
                     "greedy finalize launch");
}

int st_greedy_step(const double* x_soa, const double* g_soa, const double* weights, int64_t n,
                   int32_t d, int64_t ld, double linv_scale, double linv_trace, int64_t row_offset,
                   int64_t t, int32_t nranks, const double* cands_in, double* cand_out,
                   uint32_t* idx_out, double* a_work, void* workspace, int64_t workspace_bytes,
                   void* stream) {
    int rc = check_problem(x_soa, g_soa, weights, n, d, ld);
    if (rc) return rc;
    if (t < 0) return fail(ST_ERR_INVALID, "t must be >= 0");
    if (nranks < 1 || nranks > 64) return fail(ST_ERR_INVALID, "nranks must be in [1, 64]");
    if (t > 0 && !cands_in) return fail(ST_ERR_INVALID, "cands_in is NULL for t > 0");
    if (!cand_out || !a_work || !workspace) return fail(ST_ERR_INVALID, "NULL output/workspace");
    if (t > 0 && !idx_out) return fail(ST_ERR_INVALID, "idx_out is NULL");
    if (row_offset < 0) return fail(ST_ERR_INVALID, "row_offset must be >= 0");
    if (!aligned16(a_work) || !aligned16(workspace))
        return fail(ST_ERR_INVALID, "a_work/workspace must be 16-byte aligned");
    if (workspace_bytes < greedy_ws_bytes(d)) return fail(ST_ERR_INVALID, "workspace too small");
    hipStream_t s = static_cast<hipStream_t>(stream);
    GreedyWs ws = carve(workspace, d);
    if (t == 0) {
        rc = hip_check(hipMemsetAsync(ws.ticket, 0, 16, s), "hipMemsetAsync(ticket)");
        if (rc) return rc;
    }
    st::GreedyArgs a = make_args(x_soa, g_soa, weights, n, d, ld, linv_scale, linv_trace, a_work, ws);
    a.row_offset = row_offset;
    a.nranks = nranks;
    a.t = t;
    a.cands_in = cands_in;
    a.cand_out = cand_out;
    a.idx_out = idx_out;
    return hip_check(st::launch_greedy_step(a, t == 0, s), "greedy step launch");
}

int st_greedy_finalize(const double* cands_in, int32_t nranks, int32_t d, uint32_t* idx_out,
                       int64_t t, void* stream) {
    if (!cands_in || !idx_out) return fail(ST_ERR_INVALID, "NULL pointer");
    if (nranks < 1 || nranks > 64) return fail(ST_ERR_INVALID, "nranks must be in [1, 64]");
    if (d < 1 || d > st::kMaxDim) return fail(ST_ERR_UNSUPPORTED, "unsupported d");
    if (t < 0) return fail(ST_ERR_INVALID, "t must be >= 0");
    return hip_check(st::launch_greedy_finalize(cands_in, nranks, st::cand_stride(d), idx_out, t,
                                                static_cast<hipStream_t>(stream)),
                     "greedy finalize launch");
}

int st_kernel_pairs(const double* x_soa, const double* g_soa, const double* weights, int64_t ld,
                    int32_t d, double linv_scale, double linv_trace, const int64_t* i1,
                    const int64_t* i2, int64_t n_pairs, double* out, void* stream) {
    if (n_pairs == 0) return ST_OK;
    if (!x_soa || !g_soa) return fail(ST_ERR_INVALID, "sample/gradient pointer is NULL");
    if (d < 1 || d > st::kMaxDim) return fail(ST_ERR_UNSUPPORTED, "unsupported d = %d", d);
    if (ld < 1) return fail(ST_ERR_INVALID, "ld must be >= 1");
    if (n_pairs < 0 || !i1 || !i2 || !out) return fail(ST_ERR_INVALID, "bad pair list");
    st::PairArgs p{x_soa, g_soa, weights, ld, d, linv_scale, linv_trace};
    return hip_check(st::launch_pairs(p, i1, i2, n_pairs, out, static_cast<hipStream_t>(stream)),
                     "pairs launch");
}

int64_t st_ksd_workspace_bytes(int64_t m, int64_t ld) {
    if (m < 1 || ld < m) return -1;
    const int64_t ntiles = (m + 63) / 64;
    return ntiles * ld * 8;
}

int st_ksd_cumulative(const double* x_soa, const double* g_soa, const double* weights, int64_t m,
                      int64_t ld, int32_t d, double linv_scale, double linv_trace, double* ks_out,
                      void* workspace, int64_t workspace_bytes, void* stream) {
    int rc = check_problem(x_soa, g_soa, weights, m, d, ld);
    if (rc) return rc;
    if (!ks_out || !workspace) return fail(ST_ERR_INVALID, "NULL output/workspace");
    if (workspace_bytes < st_ksd_workspace_bytes(m, ld))
        return fail(ST_ERR_INVALID, "workspace too small");
    hipStream_t s = static_cast<hipStream_t>(stream);
    const int64_t ntiles = (m + 63) / 64;
    if (ntiles > 65535) return fail(ST_ERR_UNSUPPORTED, "m too large for the tiled KSD grid");
    st::PairArgs p{x_soa, g_soa, weights, ld, d, linv_scale, linv_trace};
    double* part = static_cast<double*>(workspace);
    rc = hip_check(st::launch_ksd_rows(p, nullptr, m, part, ntiles, s), "ksd rows launch");
    if (rc) return rc;
    return hip_check(st::launch_ksd_scan(part, m, ld, ks_out, s), "ksd scan launch");
}

int st_kmat(const double* x_soa, const double* g_soa, const double* weights, int64_t k, int64_t ld,
            int32_t d, double linv_scale, double linv_trace, double* kmat_out, void* stream) {
    int rc = check_problem(x_soa, g_soa, weights, k, d, ld);
    if (rc) return rc;
    if (!kmat_out) return fail(ST_ERR_INVALID, "NULL output");
    if ((k + 63) / 64 > 65535) return fail(ST_ERR_UNSUPPORTED, "k too large for the tiled grid");
    st::PairArgs p{x_soa, g_soa, weights, ld, d, linv_scale, linv_trace};
    return hip_check(st::launch_kmat(p, nullptr, k, kmat_out, static_cast<hipStream_t>(stream)),
                     "kmat launch");
}

int st_layout_soa(const double* rowmajor, int64_t n, int32_t d, int64_t ld, double* soa,
                  void* stream) {
    if (!rowmajor || !soa) return fail(ST_ERR_INVALID, "NULL pointer");
    if (n < 1 || d < 1 || ld < n) return fail(ST_ERR_INVALID, "bad sizes");
    return hip_check(st::launch_layout_soa(rowmajor, n, d, ld, soa, static_cast<hipStream_t>(stream)),
                     "layout launch");
}

}  // extern "C"
