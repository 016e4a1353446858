// Internal (non-ABI) declarations shared by the HIP translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace st {

constexpr int kMaxDim = 128;     // NumPy pairwise_sum modelled without recursion up to 128 lanes
constexpr int kMaxCtDim = 8;     // compile-time-d kernels for d <= 8
constexpr int kMaxBlocks = 1024; // greedy step grid cap (4 x 256-thread blocks per CU)
constexpr int kCandHeader = 2;   // candidate record: {val, gidx(bits)} then x[d], g[d], w
constexpr int64_t kWsControlBytes = 8 * 128 + 128;   // persistent kernel: arrival counters + status
// control block words (byte offsets into the greedy workspace):
constexpr int64_t kWsStatusOff = 8 * 128;   // u32 status: [0] persistent kernel, [1] the general kernel behind
                                            // a compact-only run
constexpr int64_t kWsTieOff = kWsStatusOff + 32;     // u32 near-tie words (first flagged step + 1, 0 = none):
                                                     // [0] persistent kernel, [1] gated general kernel, [2] step
                                                     // kernels; [3] = 1: the run is guarded (bounds computed)
constexpr int64_t kWsBoundsOff = kWsStatusOff + 64;  // near-tie bounds: max_i |g_i|^2, max_i w_i^2 (f64 bits),
                                                     // then the persistent run's final Q, E, thr (tests)
static_assert(kWsBoundsOff + 40 <= kWsControlBytes, "control block layout");
// peer mailbox (u64 words), one per rank, uncached device memory:
//   [0, 32)        persistent kernel: 2 banks x kMailboxRanks slots x 2 tagged granules
//   [32, 40)       handshake words (one per rank)
//   [40]           exchange counter of the step-kernel path (written by this rank only)
//   [64, ...)      step-kernel path: 2 banks x kMailboxRanks record slots, each a flag word then
//                  the candidate record (cand_stride(d) doubles) at word 8
constexpr int kMailboxRanks = 8;
constexpr int kMailboxHandshake = 2 * kMailboxRanks * 2;
constexpr int kMailboxXchgCount = kMailboxHandshake + kMailboxRanks;
constexpr int kMailboxRecBase = 64;
constexpr int kMailboxRecSlotWords = 272;   // 8 header words + cand_stride(kMaxDim) = 260, 64-B multiple
constexpr int64_t kMailboxBytes = (int64_t)(kMailboxRecBase + 2 * kMailboxRanks * kMailboxRecSlotWords) * 8;
static_assert(kMailboxXchgCount < kMailboxRecBase, "mailbox layout");

struct MailboxPeers {
    uint64_t* p[kMailboxRanks];
};

// row block and peers of one rank of a multi-GPU persistent run (nranks == 1: one device)
struct RankSpec {
    int64_t row_begin, row_end;
    int rank, nranks;
    uint64_t seq_base;
    uint64_t* inbox;
    uint64_t* peer[kMailboxRanks];
};

inline int64_t cand_stride(int d) { return ((kCandHeader + 2 * d + 1) + 1) & ~int64_t(1); }
static_assert(8 + ((kCandHeader + 2 * kMaxDim + 1) + 1) / 2 * 2 <= kMailboxRecSlotWords, "record slot");

struct GreedyArgs {
    const double* x;      // SoA (d, ld) standardised sample shard
    const double* g;      // SoA (d, ld) standardised gradient (or gradient_q) shard
    const double* w;      // (ld) gradient-free weights, or nullptr for the Langevin kernel
    double* A;            // (ld) running sums, in place
    int64_t n;            // rows in this shard
    int64_t ld;           // leading dimension (multiple of 8, >= n)
    int d;
    double l;             // isotropic preconditioner Gamma^-1 = l * I
    double tr;            // np.trace(Gamma^-1), computed on the host exactly as the reference
    int64_t row_offset;   // global index of shard row 0
    const double* recs_in;  // K candidate records of the previous step (unused for the diagonal)
    int nrecs_in;
    int64_t rec_stride;   // doubles per record
    double* recs_out;     // one record per block of this launch
    uint32_t* idx_out;    // device index array; launch t writes idx[t-1]
    int64_t t;            // step being computed (0 = diagonal)
    int compact;          // 1: the compact arithmetic for pairs in range (d <= 8; stein_math.hpp)
};

int greedy_blocks(int64_t n, int d);
// near-tie guard of the compact arithmetic (st_tune key 20: 1 = on, the default; 0 = off)
int tie_guard();
// st_tune key 11: arithmetic of the d <= 8 greedy kernels (1 = compact, the default; 0 = exact)
int arith_compact();
int tune(int key, int value);
int persistent_tune(int key, int value);
int persistent_tune_get(int key);
int tune_get(int key);
int64_t persistent_ws_bytes(int d, int G, int rec_stride, int nrep);
int64_t persistent_ws_max_bytes();
hipError_t launch_greedy_persistent(const double* x, const double* g, const double* w, double* A,
                                    int64_t n, int d, int64_t ld, double l, double tr, int64_t m,
                                    uint32_t* idx_out, void* ws, int64_t ws_bytes, hipStream_t s,
                                    int* used, const RankSpec* ranks = nullptr, bool plan_only = false);
// one thin of a batch launch (st_greedy_batch): the st_greedy arguments of one problem
struct BatchProblem {
    const double* x;
    const double* g;
    const double* w;
    double* A;
    int64_t n, ld;
    double l, tr;
    uint32_t* idx_out;
    void* ws;
    int64_t ws_bytes;
};
constexpr int kMaxBatchProblems = 8;
hipError_t launch_greedy_persistent_batch(int count, const BatchProblem* problems, int d, int64_t m,
                                          hipStream_t s, int* used);
hipError_t launch_mailbox_handshake(const MailboxPeers& peers, uint64_t* inbox, int rank,
                                    int nranks, uint64_t token, int* ok, hipStream_t s);
hipError_t launch_greedy_step(const GreedyArgs& a, bool diag, int blocks, hipStream_t s);
hipError_t launch_greedy_publish(const double* recs, int K, int64_t stride, int d, double* out,
                                 hipStream_t s);
hipError_t launch_greedy_finalize(const double* recs, int K, int64_t stride, uint32_t* idx_out,
                                  int64_t t, hipStream_t s);
struct ProxyArgs {
    const double* x;     // row-major (n, d) raw sample
    const double* loc;   // (d)
    const double* U;     // (d, d) row-major, scipy _PSD factor: maha = |(x - loc) @ U|^2
    const double* P;     // (d, d) row-major, np.linalg.inv(cov / shape)
    int64_t n;
    int d;
    double df;           // 0: Gaussian; > 0: Student-t degrees of freedom
    double c_log;        // Gaussian: rank*log(2 pi) + log_pdet; t: A - B - C - D
    double* log_q;       // (n)
    double* grad;        // row-major (n, d)
};
int64_t proxy_lds_bytes(int d);
int64_t kde_workspace_bytes(int64_t m, int d);
hipError_t launch_kde(const double* p, int64_t ldp, int64_t n, const double* logw, double logw0,
                      const double* q, int64_t ldq, int64_t m, int d, double log_norm, const double* L,
                      double* log_q, double* grad, double* ws, hipStream_t s);
hipError_t launch_proxy(const ProxyArgs& a, hipStream_t s);
int proxy_tune(int value);   // st_tune key 7
int dist_tune(int value);    // st_tune key 13 (energy kernel variant)

struct LvArgs {
    const double* theta;      // (n, 4) row-major ODE parameters
    const double* log_theta;  // (n, 4) row-major, log density only
    int64_t n;
    const double* t_eval;     // (t_n) ascending observation times
    int t_n;
    const double* y_obs;      // (t_n, 2) row-major observations
    double t0, t1;            // integration span
    double u0[2];             // initial state
    double rtol, atol;
    double cinv[4];           // inv(C) row-major (gradient)
    double U[4];              // scipy _PSD(C).U row-major (log density)
    double c_log;             // rank * log(2 pi) + log_pdet of C
    double norm_logc;         // scipy.stats.norm's log(sqrt(2 pi))
    int64_t max_steps;
    double* out;              // gradient: (n, 4); log density: (n)
    double* work;             // log density: (t_n, n) per-time terms
    int32_t* status;          // (n): 0 ok, 1 step size too small, 2 step limit reached
    double* steps;            // gradient, two-phase: (n, step_cap, 56) step table, or nullptr
    int32_t* nsteps;          // (n) recorded steps per point
    int step_cap;
};
hipError_t launch_lv(const LvArgs& a, bool gradient, hipStream_t s);
int64_t lv_grad_workspace_bytes(int64_t n, int step_cap);

hipError_t launch_greedy_rank_exchange(const double* recs, int K, int64_t stride, int d,
                                       const MailboxPeers& peers, int rank, int nranks, int64_t t,
                                       double* recv, unsigned* status, hipStream_t s);

struct PairArgs {
    const double* x;
    const double* g;
    const double* w;
    int64_t ld;
    int d;
    double l;
    double tr;
};

hipError_t launch_pairs(const PairArgs& p, const int64_t* i1, const int64_t* i2, int64_t L,
                        double* out, hipStream_t s);
hipError_t launch_kmat(const PairArgs& p, const int64_t* idx, int64_t k, double* out,
                       hipStream_t s);
hipError_t launch_ksd_colsum(const PairArgs& p, int64_t n, int64_t a0, int64_t a1, double* csum,
                             hipStream_t s);
hipError_t launch_ksd_finish(const PairArgs& p, int64_t n, const double* csum, double* ks,
                             hipStream_t s);
int64_t distance_chunks(int64_t na, int64_t b_begin, int64_t b_end);
int dist_units_tune(int value);   // st_tune key 14
int lv_tune(int value);           // st_tune key 17
int lv_pieces_tune(int value);    // st_tune key 18
hipError_t launch_distance_colsum(const double* a, int64_t lda, int64_t na, const double* b,
                                  int64_t ldb, int64_t b0, int64_t b1, int d, int tri,
                                  double* out, double* ws, int64_t ws_doubles, hipStream_t s);
hipError_t launch_layout_soa(const double* rowmajor, int64_t n, int d, int64_t ld, double* soa,
                             hipStream_t s);
hipError_t launch_layout_soa_scaled(const double* rowmajor, int64_t n, int d, int64_t ld, const double* scale,
                                    int divide, double* soa, hipStream_t s);
// 'med' preconditioner distances (precon.hip)
hipError_t launch_pdist(const double* rows, int64_t k, int d, double* out, hipStream_t s);
// repeated-row compaction (dedup.hip)
int64_t run_tiles(int64_t n);
hipError_t launch_run_starts(const double* x, const double* g, const double* w, int64_t n, int d, int64_t ld,
                             uint8_t* starts, int32_t* tile_count, int32_t* tile_off, int64_t* count,
                             hipStream_t s);
hipError_t launch_run_compact(const double* x, const double* g, const double* w, int64_t n, int d, int64_t ld,
                              const uint8_t* starts, const int32_t* tile_off, int64_t count, int64_t ld_out,
                              double* xo, double* go, double* wo, int32_t* rows_out, hipStream_t s);

}  // namespace st
