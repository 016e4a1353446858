// C ABI (include/stein_thinning_hip.h): argument validation, workspace carving, launch sequencing.
// No allocation, no synchronisation: every entry point only enqueues work on the caller's stream.
#include <math.h>
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

}  // namespace

namespace st {
// st_last_error text for entry points defined in other translation units (prep_upload.cpp)
int report_error(int code, const char* msg) { return fail(code, "%s", msg); }
}  // namespace st

namespace {

int check_problem(const double* x, const double* g, const double* w, int64_t n, int32_t d,
                  int64_t ld) {
    if (!x || !g) return fail(ST_ERR_INVALID, "sample/gradient pointer is NULL");
    if (n < 1) return fail(ST_ERR_INVALID, "n must be >= 1 (got %lld)", (long long)n);
    if (d < 1) return fail(ST_ERR_INVALID, "d must be >= 1 (got %d)", d);
    if (d > st::kMaxDim)
        return fail(ST_ERR_UNSUPPORTED, "d = %d exceeds the supported maximum %d", d, st::kMaxDim);
    if (ld < n || (ld & 7))
        return fail(ST_ERR_INVALID, "ld must be a multiple of 8 and >= n (n=%lld, ld=%lld)",
                    (long long)n, (long long)ld);
    if (!aligned16(x) || !aligned16(g) || (w && !aligned16(w)))
        return fail(ST_ERR_INVALID, "device arrays must be 16-byte aligned");
    return ST_OK;
}

// workspace layout: [control block (persistent kernel counters/status)][two ping-pong banks of
// per-block candidate records, kMaxBlocks x stride doubles each]
int64_t greedy_ws_bytes(int32_t d) {
    const int64_t steps = st::kWsControlBytes + 2 * (int64_t)st::kMaxBlocks * st::cand_stride(d) * 8;
    const int64_t persist = st::persistent_ws_max_bytes();
    return steps > persist ? steps : persist;
}

double* bank(void* ws, int32_t d, int b) {
    return reinterpret_cast<double*>(static_cast<char*>(ws) + st::kWsControlBytes) +
           (int64_t)b * st::kMaxBlocks * st::cand_stride(d);
}

st::GreedyArgs make_args(const double* x, const double* g, const double* w, int64_t n, int32_t d,
                         int64_t ld, double l, double tr, double* A) {
    st::GreedyArgs a{};
    a.x = x; a.g = g; a.w = w; a.A = A;
    a.n = n; a.ld = ld; a.d = d; a.l = l; a.tr = tr;
    a.row_offset = 0;
    a.rec_stride = st::cand_stride(d);
    a.compact = st::arith_compact();
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

int st_tune(int32_t key, int32_t value) {
    int rc;
    if (key == 7) rc = st::proxy_tune(value);
    else if (key == 13) rc = st::dist_tune(value);
    else if (key == 14) rc = st::dist_units_tune(value);
    else if (key == 17) rc = st::lv_tune(value);
    else if (key == 18) rc = st::lv_pieces_tune(value);
    else rc = ((key >= 3 && key <= 5) || key == 8 || key == 9 || key == 10 || key == 12 || key == 15 || key == 16 ||
               key == 19 || key == 23)
                  ? st::persistent_tune(key, value)
                  : st::tune(key, value);
    if (rc != 0) return fail(ST_ERR_INVALID, "bad tuning key/value %d=%d", key, value);
    return ST_OK;
}

int32_t st_tune_get(int32_t key) {
    const bool persist = (key >= 3 && key <= 5) || key == 8 || key == 9 || key == 10 || key == 12 || key == 15 ||
                         key == 16 || key == 19 || key == 23;
    return persist ? st::persistent_tune_get(key) : st::tune_get(key);
}

int64_t st_candidate_stride(int32_t d) {
    if (d < 1 || d > st::kMaxDim) return -1;
    return st::cand_stride(d);
}

int st_greedy_steps(const double* x_soa, const double* g_soa, const double* weights, int64_t n,
                    int32_t d, int64_t ld, double linv_scale, double linv_trace, int64_t t_begin,
                    int64_t t_end, int64_t n_points, uint32_t* idx_out, double* a_work,
                    void* workspace, int64_t workspace_bytes, void* stream) {
    int rc = check_problem(x_soa, g_soa, weights, n, d, ld);
    if (rc) return rc;
    if (n_points < 1) return fail(ST_ERR_INVALID, "n_points must be >= 1");
    if (t_begin < 0 || t_end < t_begin || t_end > n_points)
        return fail(ST_ERR_INVALID, "need 0 <= t_begin <= t_end <= n_points");
    if (!idx_out || !a_work || !workspace) return fail(ST_ERR_INVALID, "NULL output/workspace");
    if (!aligned16(a_work) || !aligned16(workspace))
        return fail(ST_ERR_INVALID, "a_work/workspace must be 16-byte aligned");
    if (workspace_bytes < greedy_ws_bytes(d))
        return fail(ST_ERR_INVALID, "workspace too small (%lld < %lld)", (long long)workspace_bytes,
                    (long long)greedy_ws_bytes(d));
    hipStream_t s = static_cast<hipStream_t>(stream);
    st::GreedyArgs a = make_args(x_soa, g_soa, weights, n, d, ld, linv_scale, linv_trace, a_work);
    a.idx_out = idx_out;
    const int blocks = st::greedy_blocks(n, d);
    if (t_begin == 0) {   // a run starts: no near-tie word of an earlier run may survive (step kernels: unguarded)
        rc = hip_check(hipMemsetAsync(static_cast<char*>(workspace) + st::kWsTieOff, 0,
                                      (size_t)(st::kWsBoundsOff + 40 - st::kWsTieOff), s),
                       "near-tie words reset");
        if (rc) return rc;
    }
    for (int64_t t = t_begin; t < t_end; ++t) {
        a.t = t;
        a.recs_in = bank(workspace, d, (int)((t + 1) & 1));
        a.nrecs_in = blocks;
        a.recs_out = bank(workspace, d, (int)(t & 1));
        rc = hip_check(st::launch_greedy_step(a, t == 0, blocks, s), "greedy step launch");
        if (rc) return rc;
    }
    if (t_end < n_points || t_end == t_begin) return ST_OK;
    return hip_check(st::launch_greedy_finalize(bank(workspace, d, (int)((n_points - 1) & 1)), blocks,
                                                a.rec_stride, idx_out, n_points - 1, s),
                     "greedy finalize launch");
}

int st_greedy(const double* x_soa, const double* g_soa, const double* weights, int64_t n,
              int32_t d, int64_t ld, double linv_scale, double linv_trace, int64_t n_points,
              uint32_t* idx_out, double* a_work, void* workspace, int64_t workspace_bytes,
              void* stream) {
    if (n_points < 1) return fail(ST_ERR_INVALID, "n_points must be >= 1");
    int rc = check_problem(x_soa, g_soa, weights, n, d, ld);
    if (rc) return rc;
    if (!idx_out || !a_work || !workspace) return fail(ST_ERR_INVALID, "NULL output/workspace");
    if (!aligned16(a_work) || !aligned16(workspace))
        return fail(ST_ERR_INVALID, "a_work/workspace must be 16-byte aligned");
    if (workspace_bytes < greedy_ws_bytes(d))
        return fail(ST_ERR_INVALID, "workspace too small (%lld < %lld)", (long long)workspace_bytes,
                    (long long)greedy_ws_bytes(d));
    int used = 0;
    const hipError_t pe = st::launch_greedy_persistent(
        x_soa, g_soa, weights, a_work, n, d, ld, linv_scale, linv_trace, n_points, idx_out, workspace,
        workspace_bytes, static_cast<hipStream_t>(stream), &used);
    if (used) return ST_OK;
    if (pe != hipErrorNotSupported) (void)hipGetLastError();   // clear a failed launch
    return st_greedy_steps(x_soa, g_soa, weights, n, d, ld, linv_scale, linv_trace, 0, n_points,
                           n_points, idx_out, a_work, workspace, workspace_bytes, stream);
}

int st_greedy_near_tie(const void* workspace, int64_t workspace_bytes, int64_t* step_out, void* stream) {
    if (!workspace || !step_out) return fail(ST_ERR_INVALID, "NULL workspace/output");
    if (workspace_bytes < st::kWsControlBytes) return fail(ST_ERR_INVALID, "workspace too small");
    hipStream_t s = static_cast<hipStream_t>(stream);
    uint32_t w[12];   // status [0], [1] ... tie words [8 .. 11]
    int rc = hip_check(hipMemcpyAsync(w, static_cast<const char*>(workspace) + st::kWsStatusOff, sizeof(w),
                                      hipMemcpyDeviceToHost, s), "near-tie read-back");
    if (rc) return rc;
    rc = hip_check(hipStreamSynchronize(s), "near-tie read-back sync");
    if (rc) return rc;
    constexpr int kTie = (int)((st::kWsTieOff - st::kWsStatusOff) / 4);
    if (w[kTie + 3] != 1u) {
        *step_out = -2;
        return ST_OK;
    }
    // the step kernels' word when they ran; else the gated general kernel's after a compact-only hand-off
    // words hold ~step (atomic max over blocks = the first flagged step), 0 = none
    const uint32_t tv = w[kTie + 2] ? w[kTie + 2] : (w[0] == 2u ? w[kTie + 1] : w[kTie]);
    *step_out = tv ? (int64_t)(uint32_t)~tv : -1;
    return ST_OK;
}

int st_greedy_batch(int32_t count, const double* const* x_soa, const double* const* g_soa,
                    const double* const* weights, const int64_t* n, int32_t d, const int64_t* ld,
                    const double* linv_scale, const double* linv_trace, int64_t n_points,
                    uint32_t* const* idx_out, double* const* a_work, void* const* workspace,
                    const int64_t* workspace_bytes, void* stream) {
    if (count < 1 || count > st::kMaxBatchProblems)
        return fail(ST_ERR_INVALID, "count must be in [1, %d]", st::kMaxBatchProblems);
    if (!x_soa || !g_soa || !n || !ld || !linv_scale || !linv_trace || !idx_out || !a_work || !workspace ||
        !workspace_bytes)
        return fail(ST_ERR_INVALID, "NULL argument array");
    if (n_points < 1) return fail(ST_ERR_INVALID, "n_points must be >= 1");
    st::BatchProblem pr[st::kMaxBatchProblems];
    for (int q = 0; q < count; ++q) {
        const double* w = weights ? weights[q] : nullptr;
        if ((w == nullptr) != (!weights || weights[0] == nullptr))
            return fail(ST_ERR_INVALID, "problem %d: weights must be given for every problem or none", q);
        int rc = check_problem(x_soa[q], g_soa[q], w, n[q], d, ld[q]);
        if (rc) return rc;
        if (!idx_out[q] || !a_work[q] || !workspace[q])
            return fail(ST_ERR_INVALID, "problem %d: NULL output/workspace", q);
        if (!aligned16(a_work[q]) || !aligned16(workspace[q]))
            return fail(ST_ERR_INVALID, "problem %d: a_work/workspace must be 16-byte aligned", q);
        if (workspace_bytes[q] < greedy_ws_bytes(d))
            return fail(ST_ERR_INVALID, "problem %d: workspace too small (%lld < %lld)", q,
                        (long long)workspace_bytes[q], (long long)greedy_ws_bytes(d));
        pr[q] = st::BatchProblem{x_soa[q], g_soa[q], w, a_work[q], n[q], ld[q], linv_scale[q], linv_trace[q],
                                 idx_out[q], workspace[q], workspace_bytes[q]};
    }
    int used = 0;
    const hipError_t e = st::launch_greedy_persistent_batch(count, pr, d, n_points, static_cast<hipStream_t>(stream),
                                                            &used);
    if (used) return ST_OK;
    if (e == hipErrorNotSupported)
        return fail(ST_ERR_UNSUPPORTED, "batch launch does not apply (d = 2 / 4, every problem planned onto the same "
                    "kernel -- threads per block, register rows -- at #CU / count blocks); run st_greedy per problem");
    (void)hipGetLastError();
    return hip_check(e, "batch persistent launch");
}

int64_t st_mailbox_bytes(int32_t nranks) {
    if (nranks < 1 || nranks > st::kMailboxRanks) return -1;
    return st::kMailboxBytes;
}

int st_mailbox_alloc(int64_t bytes, void** mailbox) {
    if (!mailbox || bytes < st::kMailboxBytes) return fail(ST_ERR_INVALID, "bad mailbox request");
    *mailbox = nullptr;
    // uncached device memory: peers' xGMI stores land in HBM and local polls never hit a stale
    // L2 line
    void* p = nullptr;
    int rc = hip_check(hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached),
                       "hipExtMallocWithFlags(uncached)");
    if (rc) return rc;
    rc = hip_check(hipMemset(p, 0, (size_t)bytes), "mailbox memset");
    if (rc) { (void)hipFree(p); return rc; }
    *mailbox = p;
    return ST_OK;
}

int st_mailbox_free(void* mailbox) {
    if (!mailbox) return ST_OK;
    return hip_check(hipFree(mailbox), "hipFree(mailbox)");
}

int st_ipc_get_handle(void* dev_ptr, void* handle_out) {
    if (!dev_ptr || !handle_out) return fail(ST_ERR_INVALID, "NULL pointer");
    hipIpcMemHandle_t h;
    int rc = hip_check(hipIpcGetMemHandle(&h, dev_ptr), "hipIpcGetMemHandle");
    if (rc) return rc;
    memcpy(handle_out, &h, sizeof(h));
    return ST_OK;
}

int st_ipc_handle_bytes(void) { return (int)sizeof(hipIpcMemHandle_t); }

int st_ipc_open_handle(const void* handle, void** dev_ptr) {
    if (!handle || !dev_ptr) return fail(ST_ERR_INVALID, "NULL pointer");
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    *dev_ptr = nullptr;
    return hip_check(hipIpcOpenMemHandle(dev_ptr, h, hipIpcMemLazyEnablePeerAccess),
                     "hipIpcOpenMemHandle");
}

int st_ipc_close_handle(void* dev_ptr) {
    if (!dev_ptr) return ST_OK;
    return hip_check(hipIpcCloseMemHandle(dev_ptr), "hipIpcCloseMemHandle");
}

static int check_peers(void* const* peer_mailboxes, int32_t nranks, int32_t rank) {
    if (nranks < 2 || nranks > st::kMailboxRanks)
        return fail(ST_ERR_INVALID, "nranks must be in [2, %d]", st::kMailboxRanks);
    if (rank < 0 || rank >= nranks) return fail(ST_ERR_INVALID, "rank out of range");
    if (!peer_mailboxes) return fail(ST_ERR_INVALID, "NULL peer mailbox table");
    for (int r = 0; r < nranks; ++r)
        if (!peer_mailboxes[r] || !aligned16(peer_mailboxes[r]))
            return fail(ST_ERR_INVALID, "peer mailbox %d is NULL or misaligned", r);
    return ST_OK;
}

int st_mailbox_handshake(void* const* peer_mailboxes, int32_t nranks, int32_t rank,
                         uint64_t token, int32_t* ok_device, void* stream) {
    int rc = check_peers(peer_mailboxes, nranks, rank);
    if (rc) return rc;
    if (!ok_device) return fail(ST_ERR_INVALID, "NULL ok flag");
    if (token >> 63) return fail(ST_ERR_INVALID, "token must be < 2^63");
    st::MailboxPeers peers{};
    for (int r = 0; r < nranks; ++r) peers.p[r] = static_cast<uint64_t*>(peer_mailboxes[r]);
    return hip_check(st::launch_mailbox_handshake(peers, peers.p[rank], rank, nranks,
                                                  token | (1ull << 63), ok_device,
                                                  static_cast<hipStream_t>(stream)),
                     "handshake launch");
}

int st_greedy_sharded(const double* x_soa, const double* g_soa, const double* weights, int64_t n,
                      int32_t d, int64_t ld, double linv_scale, double linv_trace,
                      int64_t row_begin, int64_t row_end, int32_t rank, int32_t nranks,
                      void* const* peer_mailboxes, uint64_t seq_base, int64_t n_points,
                      uint32_t* idx_out, double* a_work, void* workspace,
                      int64_t workspace_bytes, void* stream) {
    if (n_points < 1) return fail(ST_ERR_INVALID, "n_points must be >= 1");
    int rc = check_problem(x_soa, g_soa, weights, n, d, ld);
    if (rc) return rc;
    rc = check_peers(peer_mailboxes, nranks, rank);
    if (rc) return rc;
    if (row_begin < 0 || row_end <= row_begin || row_end > n)
        return fail(ST_ERR_INVALID, "need 0 <= row_begin < row_end <= n");
    if (!idx_out || !a_work || !workspace) return fail(ST_ERR_INVALID, "NULL output/workspace");
    if (!aligned16(a_work) || !aligned16(workspace))
        return fail(ST_ERR_INVALID, "a_work/workspace must be 16-byte aligned");
    if (workspace_bytes < greedy_ws_bytes(d))
        return fail(ST_ERR_INVALID, "workspace too small (%lld < %lld)", (long long)workspace_bytes,
                    (long long)greedy_ws_bytes(d));
    st::RankSpec rs{};
    rs.row_begin = row_begin;
    rs.row_end = row_end;
    rs.rank = rank;
    rs.nranks = nranks;
    rs.seq_base = seq_base;
    rs.inbox = static_cast<uint64_t*>(peer_mailboxes[rank]);
    for (int r = 0; r < nranks; ++r) rs.peer[r] = static_cast<uint64_t*>(peer_mailboxes[r]);
    int used = 0;
    const hipError_t e = st::launch_greedy_persistent(
        x_soa, g_soa, weights, a_work, n, d, ld, linv_scale, linv_trace, n_points, idx_out, workspace,
        workspace_bytes, static_cast<hipStream_t>(stream), &used, &rs);
    if (used) return ST_OK;
    if (e == hipErrorNotSupported)
        return fail(ST_ERR_UNSUPPORTED, "multi-rank persistent kernel: d = %d not supported (d = 2, 4; d = 50 "
                    "with at most 256 rows per CU)", d);
    (void)hipGetLastError();
    return hip_check(e, "multi-rank persistent launch");
}

int st_greedy_sharded_supported(int64_t n, int32_t d, int32_t has_weights, int64_t row_begin,
                                int64_t row_end, int32_t rank, int32_t nranks, int64_t n_points) {
    if (d < 1 || d > st::kMaxDim || n < 1 || n_points < 1)
        return fail(ST_ERR_INVALID, "bad problem (n = %lld, d = %d)", (long long)n, d);
    if (nranks < 2 || nranks > st::kMailboxRanks || rank < 0 || rank >= nranks)
        return fail(ST_ERR_INVALID, "bad rank %d of %d", rank, nranks);
    if (row_begin < 0 || row_end <= row_begin || row_end > n)
        return fail(ST_ERR_INVALID, "need 0 <= row_begin < row_end <= n");
    // the same decision st_greedy_sharded takes, without touching any buffer: placeholders for the
    // pointers, a non-null inbox, the workspace size the caller allocates (st_greedy_workspace_bytes)
    static uint64_t dummy_box[2];
    st::RankSpec rs{};
    rs.row_begin = row_begin;
    rs.row_end = row_end;
    rs.rank = rank;
    rs.nranks = nranks;
    rs.inbox = dummy_box;
    static double dummy_w;
    int used = 0;
    const hipError_t e = st::launch_greedy_persistent(
        nullptr, nullptr, has_weights ? &dummy_w : nullptr, nullptr, n, d, 0, 1.0, 1.0, n_points, nullptr,
        nullptr, greedy_ws_bytes(d), nullptr, &used, &rs, true);
    if (e == hipErrorInvalidValue) return fail(ST_ERR_INVALID, "invalid shard");
    return used ? 1 : 0;
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
    st::GreedyArgs a = make_args(x_soa, g_soa, weights, n, d, ld, linv_scale, linv_trace, a_work);
    a.row_offset = row_offset;
    a.t = t;
    a.recs_in = cands_in;
    a.nrecs_in = nranks;
    a.recs_out = bank(workspace, d, 0);
    a.idx_out = idx_out;
    const int blocks = st::greedy_blocks(n, d);
    rc = hip_check(st::launch_greedy_step(a, t == 0, blocks, s), "greedy step launch");
    if (rc) return rc;
    return hip_check(st::launch_greedy_publish(a.recs_out, blocks, a.rec_stride, d, cand_out, s),
                     "greedy publish launch");
}

int st_greedy_step_exchange(const double* x_soa, const double* g_soa, const double* weights,
                            int64_t n, int32_t d, int64_t ld, double linv_scale, double linv_trace,
                            int64_t row_offset, int64_t t, int32_t rank, int32_t nranks,
                            void* const* peer_mailboxes, double* cands, uint32_t* idx_out,
                            double* a_work, void* workspace, int64_t workspace_bytes,
                            uint32_t* status_device, void* stream) {
    int rc = check_problem(x_soa, g_soa, weights, n, d, ld);
    if (rc) return rc;
    rc = check_peers(peer_mailboxes, nranks, rank);
    if (rc) return rc;
    if (t < 0) return fail(ST_ERR_INVALID, "t must be >= 0");
    if (!cands || !a_work || !workspace || !status_device) return fail(ST_ERR_INVALID, "NULL output/workspace");
    if (t > 0 && !idx_out) return fail(ST_ERR_INVALID, "idx_out is NULL");
    if (row_offset < 0) return fail(ST_ERR_INVALID, "row_offset must be >= 0");
    if (!aligned16(a_work) || !aligned16(workspace))
        return fail(ST_ERR_INVALID, "a_work/workspace must be 16-byte aligned");
    if (workspace_bytes < greedy_ws_bytes(d)) return fail(ST_ERR_INVALID, "workspace too small");
    hipStream_t s = static_cast<hipStream_t>(stream);
    st::GreedyArgs a = make_args(x_soa, g_soa, weights, n, d, ld, linv_scale, linv_trace, a_work);
    a.row_offset = row_offset;
    a.t = t;
    a.recs_in = cands;
    a.nrecs_in = nranks;
    a.recs_out = bank(workspace, d, 0);
    a.idx_out = idx_out;
    const int blocks = st::greedy_blocks(n, d);
    rc = hip_check(st::launch_greedy_step(a, t == 0, blocks, s), "greedy step launch");
    if (rc) return rc;
    st::MailboxPeers peers{};
    for (int r = 0; r < nranks; ++r) peers.p[r] = static_cast<uint64_t*>(peer_mailboxes[r]);
    return hip_check(st::launch_greedy_rank_exchange(a.recs_out, blocks, a.rec_stride, d, peers, rank,
                                                     nranks, t, cands, status_device, s),
                     "rank exchange launch");
}

int64_t st_kde_workspace_bytes(int64_t m, int32_t d) {
    if (m < 0 || d < 1 || d > st::kMaxDim) return -1;
    return st::kde_workspace_bytes(m, d);
}

int st_kde_logpdf_grad(const double* p_soa, int64_t ldp, int64_t n, const double* log_weights,
                       double log_weight_uniform, const double* q_soa, int64_t ldq, int64_t m, int32_t d,
                       double log_norm, const double* whiten, double* log_q_out, double* grad_out,
                       void* workspace, int64_t workspace_bytes, void* stream) {
    if (m == 0) return ST_OK;
    if (!p_soa || !q_soa || !whiten || !log_q_out || !grad_out) return fail(ST_ERR_INVALID, "NULL pointer");
    if (d < 1 || d > st::kMaxDim) return fail(ST_ERR_UNSUPPORTED, "unsupported d = %d", d);
    if (n < 1 || m < 0 || ldp < n || ldq < m) return fail(ST_ERR_INVALID, "bad sizes (need n >= 1, ld >= count)");
    if ((m + 255) / 256 > 0x7FFFFFFFll) return fail(ST_ERR_UNSUPPORTED, "m too large");
    if (workspace_bytes < st::kde_workspace_bytes(m, d) || (st::kde_workspace_bytes(m, d) > 0 && !workspace))
        return fail(ST_ERR_INVALID, "workspace too small (%lld < %lld)", (long long)workspace_bytes,
                    (long long)st::kde_workspace_bytes(m, d));
    return hip_check(st::launch_kde(p_soa, ldp, n, log_weights, log_weight_uniform, q_soa, ldq, m, d, log_norm,
                                    whiten, log_q_out, grad_out, static_cast<double*>(workspace),
                                    static_cast<hipStream_t>(stream)),
                     "kde launch");
}

int st_proxy_logpdf_grad(const double* x, int64_t n, int32_t d, const double* loc,
                         const double* whiten, const double* precision, double df, double c_log,
                         double* log_q_out, double* grad_out, void* stream) {
    if (n < 0) return fail(ST_ERR_INVALID, "n must be >= 0");
    if (d < 1) return fail(ST_ERR_INVALID, "d must be >= 1");
    if (d > st::kMaxDim) return fail(ST_ERR_UNSUPPORTED, "d = %d exceeds %d", d, st::kMaxDim);
    if (!(df >= 0.0) || df == INFINITY) return fail(ST_ERR_INVALID, "df must be 0 (Gaussian) or finite > 0");
    if (n == 0) return ST_OK;
    if (!x || !loc || !whiten || !precision || !log_q_out || !grad_out)
        return fail(ST_ERR_INVALID, "NULL pointer");
    st::ProxyArgs a{x, loc, whiten, precision, n, d, df, c_log, log_q_out, grad_out};
    return hip_check(st::launch_proxy(a, static_cast<hipStream_t>(stream)), "proxy launch");
}

// accepted RK45 steps recorded per point by the two-phase gradient (typical: ~32 at the reference's
// tolerances); a point that takes more is recomputed by the single-phase kernel
constexpr int kLvStepCap = 64;

static int lv_common(st::LvArgs& a, const double* theta, int64_t n, const double* t_eval, int32_t t_n,
                     const double* y_obs, const double* span_u0_tol, int64_t max_steps, double* out,
                     int32_t* status) {
    if (n < 0) return fail(ST_ERR_INVALID, "n must be >= 0");
    if (t_n < 1) return fail(ST_ERR_INVALID, "t_n must be >= 1");
    if (!span_u0_tol) return fail(ST_ERR_INVALID, "NULL solver settings");
    if (max_steps < 1) return fail(ST_ERR_INVALID, "max_steps must be >= 1");
    if (n > 0 && (!theta || !t_eval || !y_obs || !out || !status)) return fail(ST_ERR_INVALID, "NULL pointer");
    const double t0 = span_u0_tol[0], t1 = span_u0_tol[1];
    if (!(t1 > t0)) return fail(ST_ERR_INVALID, "need t1 > t0 (forward integration)");
    if (!(span_u0_tol[4] > 0) || !(span_u0_tol[5] > 0)) return fail(ST_ERR_INVALID, "rtol and atol must be > 0");
    a.theta = theta;
    a.n = n;
    a.t_eval = t_eval;
    a.t_n = t_n;
    a.y_obs = y_obs;
    a.t0 = t0;
    a.t1 = t1;
    a.u0[0] = span_u0_tol[2];
    a.u0[1] = span_u0_tol[3];
    a.rtol = span_u0_tol[4];
    a.atol = span_u0_tol[5];
    a.max_steps = max_steps;
    a.out = out;
    a.status = status;
    return ST_OK;
}

int st_lv_grad_log_posterior(const double* theta, int64_t n, const double* t_eval, int32_t t_n,
                             const double* y_obs, const double* span_u0_tol, const double* cov_inv,
                             int64_t max_steps, double* grad_out, int32_t* status, void* stream) {
    st::LvArgs a{};
    int rc = lv_common(a, theta, n, t_eval, t_n, y_obs, span_u0_tol, max_steps, grad_out, status);
    if (rc) return rc;
    if (!cov_inv) return fail(ST_ERR_INVALID, "NULL cov_inv");
    for (int q = 0; q < 4; ++q) a.cinv[q] = cov_inv[q];
    if (n == 0) return ST_OK;
    return hip_check(st::launch_lv(a, true, static_cast<hipStream_t>(stream)), "lv gradient launch");
}

int64_t st_lv_grad_workspace_bytes(int64_t n, int32_t t_n) {
    if (n < 0 || t_n < 1) return -1;
    return st::lv_grad_workspace_bytes(n, kLvStepCap);
}

int st_lv_grad_log_posterior_ws(const double* theta, int64_t n, const double* t_eval, int32_t t_n,
                                const double* y_obs, const double* span_u0_tol, const double* cov_inv,
                                int64_t max_steps, double* grad_out, int32_t* status, void* workspace,
                                int64_t workspace_bytes, void* stream) {
    st::LvArgs a{};
    int rc = lv_common(a, theta, n, t_eval, t_n, y_obs, span_u0_tol, max_steps, grad_out, status);
    if (rc) return rc;
    if (!cov_inv) return fail(ST_ERR_INVALID, "NULL cov_inv");
    if (n > 0 && !workspace) return fail(ST_ERR_INVALID, "NULL workspace");
    if (workspace_bytes < st::lv_grad_workspace_bytes(n, kLvStepCap)) return fail(ST_ERR_INVALID, "workspace too small");
    for (int q = 0; q < 4; ++q) a.cinv[q] = cov_inv[q];
    a.step_cap = kLvStepCap;
    a.steps = static_cast<double*>(workspace);
    a.nsteps = reinterpret_cast<int32_t*>(static_cast<char*>(workspace) + n * (int64_t)kLvStepCap * 56 * 8);
    if (n == 0) return ST_OK;
    return hip_check(st::launch_lv(a, true, static_cast<hipStream_t>(stream)), "lv gradient launch");
}

int64_t st_lv_log_density_workspace_bytes(int64_t n, int32_t t_n) {
    if (n < 0 || t_n < 1) return -1;
    return n * (int64_t)t_n * 8;
}

int st_lv_log_target_density(const double* log_theta, const double* theta, int64_t n,
                             const double* t_eval, int32_t t_n, const double* y_obs,
                             const double* span_u0_tol, const double* whiten, double c_log,
                             double norm_logc, int64_t max_steps, double* out, int32_t* status,
                             void* workspace, int64_t workspace_bytes, void* stream) {
    st::LvArgs a{};
    int rc = lv_common(a, theta, n, t_eval, t_n, y_obs, span_u0_tol, max_steps, out, status);
    if (rc) return rc;
    if (!whiten) return fail(ST_ERR_INVALID, "NULL whiten");
    if (n > 0 && (!log_theta || !workspace)) return fail(ST_ERR_INVALID, "NULL log_theta / workspace");
    if (workspace_bytes < n * (int64_t)t_n * 8) return fail(ST_ERR_INVALID, "workspace too small");
    for (int q = 0; q < 4; ++q) a.U[q] = whiten[q];
    a.log_theta = log_theta;
    a.c_log = c_log;
    a.norm_logc = norm_logc;
    a.work = static_cast<double*>(workspace);
    if (n == 0) return ST_OK;
    return hip_check(st::launch_lv(a, false, static_cast<hipStream_t>(stream)), "lv log density launch");
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
    return ld * 8;   // the column-sum vector
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
    st::PairArgs p{x_soa, g_soa, weights, ld, d, linv_scale, linv_trace};
    double* csum = static_cast<double*>(workspace);
    rc = hip_check(st::launch_ksd_colsum(p, m, 0, m, csum, s), "ksd column-sum launch");
    if (rc) return rc;
    return hip_check(st::launch_ksd_finish(p, m, csum, ks_out, s), "ksd finish launch");
}

int st_ksd_colsum(const double* x_soa, const double* g_soa, const double* weights, int64_t n,
                  int64_t ld, int32_t d, double linv_scale, double linv_trace, int64_t row_begin,
                  int64_t row_end, double* csum_out, void* stream) {
    int rc = check_problem(x_soa, g_soa, weights, n, d, ld);
    if (rc) return rc;
    if (!csum_out) return fail(ST_ERR_INVALID, "NULL output");
    if (row_begin < 0 || row_end < row_begin || row_end > n)
        return fail(ST_ERR_INVALID, "need 0 <= row_begin <= row_end <= n");
    st::PairArgs p{x_soa, g_soa, weights, ld, d, linv_scale, linv_trace};
    return hip_check(st::launch_ksd_colsum(p, n, row_begin, row_end, csum_out,
                                           static_cast<hipStream_t>(stream)),
                     "ksd column-sum launch");
}

int st_ksd_finish(const double* x_soa, const double* g_soa, const double* weights, int64_t n,
                  int64_t ld, int32_t d, double linv_scale, double linv_trace, const double* csum,
                  double* ks_out, void* stream) {
    int rc = check_problem(x_soa, g_soa, weights, n, d, ld);
    if (rc) return rc;
    if (!csum || !ks_out) return fail(ST_ERR_INVALID, "NULL pointer");
    st::PairArgs p{x_soa, g_soa, weights, ld, d, linv_scale, linv_trace};
    return hip_check(st::launch_ksd_finish(p, n, csum, ks_out, static_cast<hipStream_t>(stream)),
                     "ksd finish launch");
}

int64_t st_distance_workspace_bytes(int64_t na, int64_t b_begin, int64_t b_end) {
    if (na < 0 || b_begin < 0 || b_end < b_begin) return -1;
    const int64_t K = st::distance_chunks(na, b_begin, b_end);
    return K > 1 ? K * na * (int64_t)sizeof(double) : 0;
}

int st_distance_colsum(const double* a_soa, int64_t lda, int64_t na, const double* b_soa,
                       int64_t ldb, int64_t nb, int32_t d, int64_t b_begin, int64_t b_end,
                       int32_t triangle, double* out, void* stream) {
    return st_distance_colsum_ws(a_soa, lda, na, b_soa, ldb, nb, d, b_begin, b_end, triangle, out,
                                 nullptr, 0, stream);
}

int st_distance_colsum_ws(const double* a_soa, int64_t lda, int64_t na, const double* b_soa,
                          int64_t ldb, int64_t nb, int32_t d, int64_t b_begin, int64_t b_end,
                          int32_t triangle, double* out, void* workspace, int64_t workspace_bytes,
                          void* stream) {
    if (na == 0) return ST_OK;
    if (!a_soa || !b_soa || !out) return fail(ST_ERR_INVALID, "NULL pointer");
    if (d < 1 || d > st::kMaxDim) return fail(ST_ERR_UNSUPPORTED, "unsupported d = %d", d);
    if (na < 0 || nb < 0 || lda < na || ldb < nb || (lda & 7) || (ldb & 7))
        return fail(ST_ERR_INVALID, "bad sizes (ld must be a multiple of 8 and >= the row count)");
    if (b_begin < 0 || b_end < b_begin || b_end > nb)
        return fail(ST_ERR_INVALID, "need 0 <= b_begin <= b_end <= nb");
    if (triangle && (a_soa != b_soa || lda != ldb))
        return fail(ST_ERR_INVALID, "triangle=1 needs A and B to be the same array");
    if ((na + 255) / 256 > 0x7FFFFFFFll) return fail(ST_ERR_UNSUPPORTED, "na too large");
    if (workspace && !aligned16(workspace)) return fail(ST_ERR_INVALID, "workspace must be 16-byte aligned");
    return hip_check(st::launch_distance_colsum(a_soa, lda, na, b_soa, ldb, b_begin, b_end, d,
                                                triangle ? 1 : 0, out, static_cast<double*>(workspace),
                                                workspace ? workspace_bytes / 8 : 0,
                                                static_cast<hipStream_t>(stream)),
                     "distance column-sum launch");
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

int st_layout_soa_scaled(const double* rowmajor, int64_t n, int32_t d, int64_t ld, const double* scale,
                         int32_t divide, double* soa, void* stream) {
    if (!rowmajor || !soa || !scale) return fail(ST_ERR_INVALID, "NULL pointer");
    if (n < 1 || d < 1 || ld < n) return fail(ST_ERR_INVALID, "bad sizes");
    return hip_check(st::launch_layout_soa_scaled(rowmajor, n, d, ld, scale, divide ? 1 : 0, soa,
                                                  static_cast<hipStream_t>(stream)),
                     "scaled layout launch");
}

int st_pdist(const double* rows, int64_t k, int32_t d, double* out, void* stream) {
    if (!rows || !out) return fail(ST_ERR_INVALID, "NULL pointer");
    if (k < 2 || k > 65535 || d < 1 || d > st::kMaxDim)
        return fail(ST_ERR_INVALID, "need 2 <= k <= 65535 rows and 1 <= d <= %d", st::kMaxDim);
    return hip_check(st::launch_pdist(rows, k, d, out, static_cast<hipStream_t>(stream)), "pdist launch");
}

// workspace of st_run_starts / st_run_compact: [0, 8) the run count (int64), then the per-tile
// counts and offsets (int32 each)
int64_t st_run_workspace_bytes(int64_t n) {
    if (n < 1) return 16;
    return (8 + 8 * st::run_tiles(n) + 15) / 16 * 16;
}

int st_run_starts(const double* x_soa, const double* g_soa, const double* weights, int64_t n, int32_t d,
                  int64_t ld, uint8_t* starts_out, void* workspace, int64_t workspace_bytes, void* stream) {
    int rc = check_problem(x_soa, g_soa, weights, n, d, ld);
    if (rc) return rc;
    if (n > 0x7FFFFFFFll) return fail(ST_ERR_UNSUPPORTED, "n >= 2^31 rows");
    if (!starts_out || !workspace) return fail(ST_ERR_INVALID, "NULL output/workspace");
    if (!aligned16(workspace)) return fail(ST_ERR_INVALID, "workspace must be 16-byte aligned");
    if (workspace_bytes < st_run_workspace_bytes(n))
        return fail(ST_ERR_INVALID, "workspace too small (%lld < %lld)", (long long)workspace_bytes,
                    (long long)st_run_workspace_bytes(n));
    int64_t* count = static_cast<int64_t*>(workspace);
    int32_t* tile_count = reinterpret_cast<int32_t*>(count + 1);
    int32_t* tile_off = tile_count + st::run_tiles(n);
    return hip_check(st::launch_run_starts(x_soa, g_soa, weights, n, d, ld, starts_out, tile_count, tile_off,
                                           count, static_cast<hipStream_t>(stream)),
                     "run-start launch");
}

int st_run_compact(const double* x_soa, const double* g_soa, const double* weights, int64_t n, int32_t d,
                   int64_t ld, const uint8_t* starts, const void* workspace, int64_t count, int64_t ld_out,
                   double* x_out, double* g_out, double* w_out, int32_t* rows_out, void* stream) {
    int rc = check_problem(x_soa, g_soa, weights, n, d, ld);
    if (rc) return rc;
    if (n > 0x7FFFFFFFll) return fail(ST_ERR_UNSUPPORTED, "n >= 2^31 rows");
    if (!starts || !workspace || !x_out || !g_out || !rows_out || (weights && !w_out))
        return fail(ST_ERR_INVALID, "NULL input/output");
    if (count < 1 || count > n || ld_out < count || (ld_out & 7))
        return fail(ST_ERR_INVALID, "need 1 <= count <= n and ld_out >= count, a multiple of 8");
    const int32_t* tile_off = reinterpret_cast<const int32_t*>(static_cast<const int64_t*>(workspace) + 1) +
                              st::run_tiles(n);
    return hip_check(st::launch_run_compact(x_soa, g_soa, weights, n, d, ld, starts, tile_off, count, ld_out,
                                            x_out, g_out, weights ? w_out : nullptr, rows_out,
                                            static_cast<hipStream_t>(stream)),
                     "run-compact launch");
}

}  // extern "C"
