// C-ABI argument validation under host ASan + UBSan (scripts/sanitize_host.sh abi): every entry point
// of include/stein_thinning_hip.h called with NULL pointers, negative / inconsistent sizes, bad
// ranks, misaligned workspaces and out-of-range tuning keys must return an error status (never
// crash, never touch the pointers) and leave a message in st_last_error(); the size helpers must
// answer edge values.  These paths return before any HIP call, so the driver runs without a GPU.
#include <stdio.h>
#include <string.h>

#include "../../include/stein_thinning_hip.h"

static int fails = 0;
#define EXPECT_ERR(call) do { const int rc_ = (call); \
    if (rc_ >= 0) { printf("FAIL line %d: %s returned %d\n", __LINE__, #call, rc_); ++fails; } \
    else if (!st_last_error() || !st_last_error()[0]) { printf("FAIL line %d: no message\n", __LINE__); ++fails; } } while (0)
#define EXPECT(c) do { if (!(c)) { printf("FAIL line %d: %s\n", __LINE__, #c); ++fails; } } while (0)

int main() {
    alignas(16) static double buf[4096];
    double* p = buf;
    double* mis = reinterpret_cast<double*>(reinterpret_cast<char*>(buf) + 8);   // 8-B aligned only
    uint32_t idx[16];
    void* box = buf;
    void* peers[8] = {box, box, box, box, box, box, box, box};
    int32_t ok = 0;
    uint32_t ustatus = 0;
    EXPECT(st_abi_version() == ST_ABI_VERSION);
    EXPECT(st_greedy_workspace_bytes(10, 0, 1) < 0 && st_greedy_workspace_bytes(10, 129, 1) < 0);
    EXPECT(st_greedy_workspace_bytes(10, 4, 1) > 0);
    EXPECT(st_candidate_stride(0) < 0 && st_candidate_stride(4) > 0);
    EXPECT(st_mailbox_bytes(0) < 0 && st_mailbox_bytes(9) < 0 && st_mailbox_bytes(8) > 0);
    EXPECT(st_ksd_workspace_bytes(-1, 64) < 0 || st_ksd_workspace_bytes(-1, 64) >= 0);   // defined for any input
    EXPECT(st_distance_workspace_bytes(-1, 0, 10) < 0 && st_distance_workspace_bytes(10, 5, 4) < 0);
    EXPECT(st_distance_workspace_bytes(1000, 0, 200000) > 0);
    EXPECT(st_lv_log_density_workspace_bytes(-5, 10) <= 0 || st_lv_log_density_workspace_bytes(-5, 10) > 0);
    EXPECT_ERR(st_tune(99, 0));
    EXPECT_ERR(st_tune(3, 1000));
    EXPECT_ERR(st_tune(4, 300));
    EXPECT_ERR(st_tune(5, 0));
    EXPECT_ERR(st_tune(7, 99));
    EXPECT_ERR(st_tune(9, 24));
    // greedy: NULL data, n < 1, d out of range, ld < n, n_points < 1, misaligned / short workspace
    EXPECT_ERR(st_greedy(nullptr, p, nullptr, 10, 4, 64, 1.0, 4.0, 5, idx, p, p, 32768, nullptr));
    EXPECT_ERR(st_greedy(p, p, nullptr, 0, 4, 64, 1.0, 4.0, 5, idx, p, p, 32768, nullptr));
    EXPECT_ERR(st_greedy(p, p, nullptr, 10, 0, 64, 1.0, 4.0, 5, idx, p, p, 32768, nullptr));
    EXPECT_ERR(st_greedy(p, p, nullptr, 10, 200, 64, 1.0, 4.0, 5, idx, p, p, 32768, nullptr));
    EXPECT_ERR(st_greedy(p, p, nullptr, 100, 4, 64, 1.0, 4.0, 5, idx, p, p, 32768, nullptr));
    EXPECT_ERR(st_greedy(p, p, nullptr, 10, 4, 64, 1.0, 4.0, 0, idx, p, p, 32768, nullptr));
    EXPECT_ERR(st_greedy(p, p, nullptr, 10, 4, 64, 1.0, 4.0, 5, idx, mis, p, 32768, nullptr));
    EXPECT_ERR(st_greedy(p, p, nullptr, 10, 4, 64, 1.0, 4.0, 5, idx, p, p, 8, nullptr));
    EXPECT_ERR(st_greedy(p, p, nullptr, 10, 4, 64, 1.0, 4.0, 5, nullptr, p, p, 32768, nullptr));
    EXPECT_ERR(st_greedy_steps(p, p, nullptr, 10, 4, 64, 1.0, 4.0, 3, 2, 5, idx, p, p, 32768, nullptr));
    EXPECT_ERR(st_greedy_steps(p, p, nullptr, 10, 4, 64, 1.0, 4.0, 0, 6, 5, idx, p, p, 32768, nullptr));
    // sharded: bad rank layout, NULL peers, row range outside [0, n)
    EXPECT_ERR(st_greedy_sharded(p, p, nullptr, 10, 4, 64, 1.0, 4.0, 0, 5, 0, 1, peers, 0, 5, idx, p, p, 32768, nullptr));
    EXPECT_ERR(st_greedy_sharded(p, p, nullptr, 10, 4, 64, 1.0, 4.0, 0, 5, 2, 2, peers, 0, 5, idx, p, p, 32768, nullptr));
    EXPECT_ERR(st_greedy_sharded(p, p, nullptr, 10, 4, 64, 1.0, 4.0, 0, 5, 0, 2, nullptr, 0, 5, idx, p, p, 32768, nullptr));
    EXPECT_ERR(st_greedy_sharded(p, p, nullptr, 10, 4, 64, 1.0, 4.0, 5, 11, 0, 2, peers, 0, 5, idx, p, p, 32768, nullptr));
    EXPECT_ERR(st_greedy_sharded_supported(10, 4, 0, 5, 4, 0, 2, 5));
    EXPECT_ERR(st_greedy_sharded_supported(10, 4, 0, 0, 5, 3, 2, 5));
    EXPECT_ERR(st_greedy_sharded_supported(10, 0, 0, 0, 5, 0, 2, 5));
    EXPECT_ERR(st_mailbox_alloc(8, &box));
    EXPECT_ERR(st_mailbox_alloc(1 << 20, nullptr));
    EXPECT_ERR(st_ipc_get_handle(nullptr, buf));
    EXPECT_ERR(st_ipc_open_handle(nullptr, &box));
    EXPECT_ERR(st_mailbox_handshake(peers, 1, 0, 1, &ok, nullptr));
    EXPECT_ERR(st_mailbox_handshake(peers, 2, 2, 1, &ok, nullptr));
    EXPECT_ERR(st_mailbox_handshake(peers, 2, 0, 1ull << 63, &ok, nullptr));
    // step / exchange / finalize
    EXPECT_ERR(st_greedy_step(p, p, nullptr, 10, 4, 64, 1.0, 4.0, 0, 0, 0, p, p, idx, p, p, 32768, nullptr));
    EXPECT_ERR(st_greedy_step_exchange(p, p, nullptr, 10, 4, 64, 1.0, 4.0, 0, 0, 0, 1, peers, p, idx, p, p, 32768,
                                       &ustatus, nullptr));
    EXPECT_ERR(st_greedy_finalize(nullptr, 1, 4, idx, 0, nullptr));
    // pairs / KSD / kmat / layout
    int64_t i1[4] = {0, 1, 2, 3};
    EXPECT_ERR(st_kernel_pairs(p, p, nullptr, 64, 4, 1.0, 4.0, nullptr, i1, 4, p, nullptr));
    EXPECT_ERR(st_kernel_pairs(p, p, nullptr, 64, 0, 1.0, 4.0, i1, i1, 4, p, nullptr));
    EXPECT_ERR(st_ksd_cumulative(p, p, nullptr, 100, 64, 4, 1.0, 4.0, p, p, 32768, nullptr));
    EXPECT_ERR(st_ksd_colsum(p, p, nullptr, 10, 64, 4, 1.0, 4.0, 5, 3, p, nullptr));
    EXPECT_ERR(st_ksd_finish(p, p, nullptr, 10, 64, 4, 1.0, 4.0, nullptr, p, nullptr));
    EXPECT_ERR(st_kmat(p, p, nullptr, 100, 64, 4, 1.0, 4.0, p, nullptr));
    EXPECT_ERR(st_layout_soa(nullptr, 10, 4, 64, p, nullptr));
    EXPECT_ERR(st_layout_soa(p, 10, 4, 5, p, nullptr));
    // round 5: the device-tensor download, the near-tie flag read-back, the tuning read-back
    int32_t st5 = 0;
    int64_t step5 = 0;
    EXPECT_ERR(st_standardize_download(nullptr, 100, 4, p, p, p, &st5, nullptr));
    EXPECT_ERR(st_standardize_download(p, 0, 4, p, p, p, &st5, nullptr));
    EXPECT_ERR(st_standardize_download(p, 100, 4, p, p, p, nullptr, nullptr));
    EXPECT_ERR(st_greedy_near_tie(nullptr, 4096, &step5, nullptr));
    EXPECT_ERR(st_greedy_near_tie(p, 64, &step5, nullptr));
    EXPECT(st_tune_get(20) == 0 || st_tune_get(20) == 1);
    EXPECT(st_tune_get(12345) < 0);
    // energy distance
    EXPECT_ERR(st_distance_colsum(nullptr, 64, 10, p, 64, 10, 4, 0, 10, 0, p, nullptr));
    EXPECT_ERR(st_distance_colsum(p, 64, 10, p, 64, 10, 4, 5, 11, 0, p, nullptr));
    EXPECT_ERR(st_distance_colsum(p, 63, 10, p, 64, 10, 4, 0, 10, 0, p, nullptr));
    EXPECT_ERR(st_distance_colsum(p, 64, 10, p + 64, 64, 10, 4, 0, 10, 1, p, nullptr));
    EXPECT_ERR(st_distance_colsum_ws(p, 64, 10, p, 64, 10, 4, 0, 10, 0, p, mis, 64, nullptr));
    // proxy / LV
    EXPECT_ERR(st_proxy_logpdf_grad(nullptr, 10, 4, p, p, p, 0.0, 0.0, p, p, nullptr));
    EXPECT_ERR(st_proxy_logpdf_grad(p, 10, 0, p, p, p, 0.0, 0.0, p, p, nullptr));
    EXPECT_ERR(st_proxy_logpdf_grad(p, 10, 4, p, p, p, -1.0, 0.0, p, p, nullptr));
    EXPECT_ERR(st_lv_grad_log_posterior(nullptr, 10, p, 5, p, p, p, 100, p, nullptr, nullptr));
    printf("%s: %d failure(s)\n", fails ? "FAILED" : "ok", fails);
    return fails ? 1 : 0;
}
