// Greedy Stein-thinning step kernels for gfx950 (K1 diagonal, K2 fused step, K3 finalize).
//
// Replaces the reference's hot loop (stein_thinning.thinning._greedy_search, restated at
// JAX_Stein_Thinning.ipynb cell 22, json ~281-295; Algorithm 3, report.tex:413-426):
//     A = integrand(:, :); idx[0] = argmin(A)
//     for t in 1..m-1:  A += 2 * integrand(:, [idx[t-1]]);  idx[t] = argmin(A)
//
// One launch per greedy step, no inter-workgroup synchronisation inside a launch:
//   head   -- every block reduces the K candidate records of the previous launch (np.argmin order:
//             NaN first, then lowest value, then lowest global index) and stages the winner's row
//             (x_j, g_j, w_j) in LDS; block 0 writes idx[t-1].  For one GPU the K records are the
//             previous launch's per-block records; for R ranks they are the R rank records the
//             RCCL all-gather delivered (greedy_publish reduces a rank's block records first).
//   stream -- the candidate columns of this shard (SoA, coalesced 16-B loads, CPT adjacent
//             candidates per lane, optional register prefetch of the next tile), k(x_i, x_j),
//             A_i += 2 k in place; per-lane MINLOC.
//   tail   -- block MINLOC and ONE record {A_min, global index, x row, g row, w} per block.
// The kernel boundary is the only hand-off (no tickets, no last-block epilogue).
#include "stein_math.hpp"
#include "stein_internal.hpp"

namespace st {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

// wave_minloc (stein_math.hpp): needs every lane of the wave active -- true at each call site.

// Block-wide MINLOC; result valid in every thread.
__device__ __forceinline__ void block_minloc(double& v, int64_t& i, double* s_v, int64_t* s_i) {
    wave_minloc(v, i);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) { s_v[wave] = v; s_i[wave] = i; }
    __syncthreads();
    v = s_v[0]; i = s_i[0];
#pragma unroll
    for (int w = 1; w < kWaves; ++w)
        if (better(s_v[w], s_i[w], v, i)) { v = s_v[w]; i = s_i[w]; }
    __syncthreads();
}

__device__ __forceinline__ int64_t rec_gidx(const double* r) {
    return (int64_t)__double_as_longlong(r[1]);
}

// Head: reduce K records; stage the winner row (2d+1 doubles) in s_row; return its global index.
// ROWREG (d <= 8): each thread pre-loads the row of its best record with the header (no dependent
// global round trip); otherwise the winner row is fetched after the reduction.
template <bool ROWREG, int DR>
__device__ __forceinline__ int64_t pick_winner(const double* __restrict__ recs, int K,
                                               int64_t stride, int d, double* s_row,
                                               double* s_v, int64_t* s_i, int* s_slot) {
    double v = INFINITY;
    int64_t gi = INT64_MAX;
    int slot = -1;
    double row[ROWREG ? 2 * DR + 1 : 1];
    for (int r = threadIdx.x; r < K; r += kBlock) {
        const double* rec = recs + (int64_t)r * stride;
        const double rv = rec[0];
        const int64_t ri = rec_gidx(rec);
        double rrow[ROWREG ? 2 * DR + 1 : 1];
        if constexpr (ROWREG) {
#pragma unroll
            for (int k = 0; k < 2 * DR + 1; ++k) rrow[k] = rec[kCandHeader + k];
        }
        if (better(rv, ri, v, gi)) {
            v = rv; gi = ri; slot = r;
            if constexpr (ROWREG) {
#pragma unroll
                for (int k = 0; k < 2 * DR + 1; ++k) row[k] = rrow[k];
            }
        }
    }
    double bv = v;
    int64_t bi = gi;
    block_minloc(bv, bi, s_v, s_i);
    if (slot >= 0 && gi == bi) {   // global indices are unique across records
        if constexpr (ROWREG) {
#pragma unroll
            for (int k = 0; k < 2 * DR + 1; ++k) s_row[k] = row[k];
        } else {
            *s_slot = slot;
        }
    }
    __syncthreads();
    if constexpr (!ROWREG) {
        const double* rec = recs + (int64_t)(*s_slot) * stride + kCandHeader;
        for (int k = threadIdx.x; k < 2 * d + 1; k += kBlock) s_row[k] = rec[k];
        __syncthreads();
    }
    return bi;
}

// Tail: block MINLOC and this block's record.
__device__ __forceinline__ void write_block_record(const GreedyArgs& a, double v, int64_t li,
                                                   double* s_v, int64_t* s_i) {
    block_minloc(v, li, s_v, s_i);
    double* out = a.recs_out + (int64_t)blockIdx.x * a.rec_stride;
    const int d = a.d;
    if (threadIdx.x == 0) {
        out[0] = v;
        out[1] = __longlong_as_double((long long)(li == INT64_MAX ? INT64_MAX : a.row_offset + li));
    }
    if (li != INT64_MAX) {
        for (int k = threadIdx.x; k < 2 * d + 1; k += kBlock) {
            double val;
            if (k < d) val = a.x[(int64_t)k * a.ld + li];
            else if (k < 2 * d) val = a.g[(int64_t)(k - d) * a.ld + li];
            else val = a.w ? a.w[li] : 1.0;
            out[kCandHeader + k] = val;
        }
    }
}

// ------------------------------------------------------------------------------------------
// K1/K2: compile-time d.  DIAG: A_i = k(x_i, x_i) [w_i^2]; else A_i += 2 k(x_i, x_j) [w_i w_j].
// CPT adjacent candidates per lane (16-B loads of the SoA columns for CPT >= 2), grid-stride;
// PF: the next tile is loaded into registers before the current one is evaluated.
// ------------------------------------------------------------------------------------------
template <int D, bool GF, bool DIAG, int CPT>
struct Tile {
    double x[DIAG ? 1 : D][CPT];
    double g[D][CPT];
    double w[GF ? CPT : 1];
    double a[DIAG ? 1 : CPT];
};

template <int D, bool GF, bool DIAG, int CPT>
__device__ __forceinline__ void load_tile(const GreedyArgs& a, int64_t i0, Tile<D, GF, DIAG, CPT>& t) {
    const int64_t ld = a.ld;
    if constexpr (CPT == 1) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            if constexpr (!DIAG) t.x[k][0] = a.x[k * ld + i0];
            t.g[k][0] = a.g[k * ld + i0];
        }
        if constexpr (GF) t.w[0] = a.w[i0];
        if constexpr (!DIAG) t.a[0] = a.A[i0];
    } else {
#pragma unroll
        for (int k = 0; k < D; ++k) {
#pragma unroll
            for (int c = 0; c < CPT; c += 2) {
                if constexpr (!DIAG) {
                    const double2 xv = *reinterpret_cast<const double2*>(a.x + k * ld + i0 + c);
                    t.x[k][c] = xv.x; t.x[k][c + 1] = xv.y;
                }
                const double2 gv = *reinterpret_cast<const double2*>(a.g + k * ld + i0 + c);
                t.g[k][c] = gv.x; t.g[k][c + 1] = gv.y;
            }
        }
#pragma unroll
        for (int c = 0; c < CPT; c += 2) {
            if constexpr (GF) {
                const double2 wv = *reinterpret_cast<const double2*>(a.w + i0 + c);
                t.w[c] = wv.x; t.w[c + 1] = wv.y;
            }
            if constexpr (!DIAG) {
                const double2 av = *reinterpret_cast<const double2*>(a.A + i0 + c);
                t.a[c] = av.x; t.a[c + 1] = av.y;
            }
        }
    }
}

// jok: the compact arithmetic is on and l, tr and the selected row are in range (pair_value_sel's
// rule: a candidate row in range too -> compact, otherwise exact)
template <int D, bool GF, bool DIAG, int CPT>
__device__ __forceinline__ void eval_tile(const GreedyArgs& a, int64_t i0,
                                          const Tile<D, GF, DIAG, CPT>& t, const double (&xj)[D],
                                          const double (&gj)[D], double wj, double l, double l2,
                                          double m3l2, double tr, int jok, double& best_v,
                                          int64_t& best_i) {
    double out[CPT];
#pragma unroll
    for (int c = 0; c < CPT; ++c) {
        double gi[D];
#pragma unroll
        for (int k = 0; k < D; ++k) gi[k] = t.g[k][c];
        double kv;
        if constexpr (DIAG) {
            int cok = jok;
#pragma unroll
            for (int k = 0; k < D; ++k) cok &= fast_range_ok(t.g[k][c]);
            if (cok) {   // the diagonal's row check needs its x too (the DIAG tile carries only g)
#pragma unroll
                for (int k = 0; k < D; ++k) cok &= fast_range_ok(a.x[(int64_t)k * a.ld + i0 + c]);
            }
            kv = diag_value_sel<D>(cok, gi, tr);
            if constexpr (GF) kv = (kv * t.w[c]) * t.w[c];
            out[c] = kv;
        } else {
            double xi[D];
#pragma unroll
            for (int k = 0; k < D; ++k) xi[k] = t.x[k][c];
            kv = pair_value_sel<D>(jok && row_in_range<D>(xi, gi), xi, gi, xj, gj, l, l2, m3l2, tr);
            if constexpr (GF) kv = (kv * t.w[c]) * wj;
            out[c] = t.a[c] + 2.0 * kv;
        }
    }
    if constexpr (CPT == 1) {
        a.A[i0] = out[0];
    } else {
#pragma unroll
        for (int c = 0; c < CPT; c += 2)
            *reinterpret_cast<double2*>(a.A + i0 + c) = make_double2(out[c], out[c + 1]);
    }
#pragma unroll
    for (int c = 0; c < CPT; ++c)
        if (i0 + c < a.n && better(out[c], i0 + c, best_v, best_i)) { best_v = out[c]; best_i = i0 + c; }
}

template <int D, bool GF, bool DIAG, int CPT, bool PF>
__global__ __launch_bounds__(kBlock) void greedy_step_ct(GreedyArgs a) {
    __shared__ double s_row[2 * D + 1];
    __shared__ double s_v[kWaves];
    __shared__ int64_t s_i[kWaves];
    __shared__ int s_slot;

    const int64_t nunits = (a.n + CPT - 1) / CPT;
    const int64_t ustride = (int64_t)gridDim.x * kBlock;
    int64_t u = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    using T = Tile<D, GF, DIAG, CPT>;
    T cur;
    if (PF && u < nunits) load_tile<D, GF, DIAG, CPT>(a, u * CPT, cur);   // in flight during the head

    double xj[D], gj[D];
    double wj = 1.0;
    if constexpr (!DIAG) {
        const int64_t gw = pick_winner<true, D>(a.recs_in, a.nrecs_in, a.rec_stride, D, s_row,
                                                s_v, s_i, &s_slot);
        if (blockIdx.x == 0 && threadIdx.x == 0 && a.idx_out) a.idx_out[a.t - 1] = (uint32_t)gw;
#pragma unroll
        for (int k = 0; k < D; ++k) { xj[k] = s_row[k]; gj[k] = s_row[D + k]; }
        if constexpr (GF) wj = s_row[2 * D];
    } else {
#pragma unroll
        for (int k = 0; k < D; ++k) { xj[k] = 0.0; gj[k] = 0.0; }
    }

    const double l = a.l, l2 = a.l * a.l, m3l2 = -3.0 * l2, tr = a.tr;
    int jok = a.compact & scale_in_range(l, tr);
    if constexpr (!DIAG) jok &= row_in_range<D>(xj, gj);
    double best_v = INFINITY;
    int64_t best_i = INT64_MAX;
    if constexpr (PF) {
        while (u < nunits) {
            const int64_t un = u + ustride;
            T nxt;
            if (un < nunits) load_tile<D, GF, DIAG, CPT>(a, un * CPT, nxt);
            eval_tile<D, GF, DIAG, CPT>(a, u * CPT, cur, xj, gj, wj, l, l2, m3l2, tr, jok, best_v, best_i);
            cur = nxt;
            u = un;
        }
    } else {
        for (; u < nunits; u += ustride) {
            load_tile<D, GF, DIAG, CPT>(a, u * CPT, cur);
            eval_tile<D, GF, DIAG, CPT>(a, u * CPT, cur, xj, gj, wj, l, l2, m3l2, tr, jok, best_v, best_i);
        }
    }
    write_block_record(a, best_v, best_i, s_v, s_i);
}

// ------------------------------------------------------------------------------------------
// Runtime-d variant (any 1 <= d <= 128): one candidate per lane per iteration, selected row in LDS.
// ------------------------------------------------------------------------------------------
template <bool GF, bool DIAG, bool NTL>
__global__ __launch_bounds__(kBlock, 4) void greedy_step_rt(GreedyArgs a) {
    __shared__ double s_row[2 * kMaxDim + 1];
    __shared__ double s_v[kWaves];
    __shared__ int64_t s_i[kWaves];
    __shared__ int s_slot;
    const int d = a.d;
    double wj = 1.0;
    if constexpr (!DIAG) {
        const int64_t gw = pick_winner<false, 1>(a.recs_in, a.nrecs_in, a.rec_stride, d, s_row,
                                                 s_v, s_i, &s_slot);
        if (blockIdx.x == 0 && threadIdx.x == 0 && a.idx_out) a.idx_out[a.t - 1] = (uint32_t)gw;
        if constexpr (GF) wj = s_row[2 * d];
    }
    const int64_t n = a.n, ld = a.ld;
    const double l = a.l, l2 = a.l * a.l, tr = a.tr;
    double best_v = INFINITY;
    int64_t best_i = INT64_MAX;
    for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * kBlock) {
        double kv;
        if constexpr (DIAG) {
            kv = diag_value_rt(a.g + i, ld, d, tr);
            if constexpr (GF) kv = (kv * a.w[i]) * a.w[i];
            a.A[i] = kv;
        } else {
            const double ai = a.A[i];
            const double wi = GF ? a.w[i] : 1.0;
            kv = d >= 8 ? pair_value_rt8<NTL>(a.x + i, a.g + i, ld, s_row, s_row + d, d, l, l2, tr)
                        : pair_value_rt(a.x + i, a.g + i, ld, s_row, s_row + d, 1, d, l, l2, tr);
            if constexpr (GF) kv = (kv * wi) * wj;
            kv = ai + 2.0 * kv;
            a.A[i] = kv;
        }
        if (better(kv, i, best_v, best_i)) { best_v = kv; best_i = i; }
    }
    write_block_record(a, best_v, best_i, s_v, s_i);
}

// R > 1 ranks: reduce this rank's K block records to ONE rank record (the all-gather payload).
__global__ __launch_bounds__(kBlock) void greedy_publish(const double* __restrict__ recs, int K,
                                                        int64_t stride, int d,
                                                        double* __restrict__ out) {
    __shared__ double s_v[kWaves];
    __shared__ int64_t s_i[kWaves];
    __shared__ int s_slot;
    double v = INFINITY;
    int64_t gi = INT64_MAX;
    int slot = -1;
    for (int r = threadIdx.x; r < K; r += kBlock) {
        const double rv = recs[(int64_t)r * stride];
        const int64_t ri = rec_gidx(recs + (int64_t)r * stride);
        if (better(rv, ri, v, gi)) { v = rv; gi = ri; slot = r; }
    }
    double bv = v;
    int64_t bi = gi;
    block_minloc(bv, bi, s_v, s_i);
    if (slot >= 0 && gi == bi) s_slot = slot;
    __syncthreads();
    const double* src = recs + (int64_t)s_slot * stride;
    for (int k = threadIdx.x; k < 2 * d + 1 + kCandHeader; k += kBlock) out[k] = src[k];
}

// R > 1 ranks without RCCL: reduce this rank's K block records to the rank record (as
// greedy_publish) and exchange the rank records through the peers' mailboxes (IPC-mapped uncached
// device memory, system-scope stores over xGMI): every thread pushes words of the record into slot
// `rank` of every peer, the block drains its stores, one flag word per peer follows; then lanes
// r < nranks poll the flags of their own mailbox and the block copies the R records into recv
// (rank order = np.argmin order of the concatenation, as the all-gather delivers).  Flags carry a
// per-rank exchange counter kept in the own mailbox (the same on every rank: all ranks run the
// same exchanges), so a graph replay never matches a stale flag; banks alternate with it, so a
// slot is rewritten only after every rank has consumed it.  Bounded waits set status[0] = 1.
__global__ __launch_bounds__(kBlock) void greedy_rank_exchange(const double* __restrict__ recs, int K,
                                                              int64_t stride, int d,
                                                              MailboxPeers peers, int rank,
                                                              int nranks, int64_t t,
                                                              double* __restrict__ recv,
                                                              unsigned* status) {
    __shared__ double s_v[kWaves];
    __shared__ int64_t s_i[kWaves];
    __shared__ int s_slot;
    __shared__ int s_ok;
    // an earlier exchange of this run timed out: finish the run without waiting again
    if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) return;
    double v = INFINITY;
    int64_t gi = INT64_MAX;
    int slot = -1;
    for (int r = threadIdx.x; r < K; r += kBlock) {
        const double rv = recs[(int64_t)r * stride];
        const int64_t ri = rec_gidx(recs + (int64_t)r * stride);
        if (better(rv, ri, v, gi)) { v = rv; gi = ri; slot = r; }
    }
    double bv = v;
    int64_t bi = gi;
    block_minloc(bv, bi, s_v, s_i);
    if (slot >= 0 && gi == bi) s_slot = slot;
    __syncthreads();
    const double* src = recs + (int64_t)s_slot * stride;
    uint64_t* inbox = peers.p[rank];
    const uint64_t count = __hip_atomic_load(inbox + kMailboxXchgCount, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t flag = count + 1;   // never 0 (the zeroed mailbox) and never reused
    const int64_t bank = (int64_t)(count & 1) * kMailboxRanks;
    auto slot_of = [&](uint64_t* mb, int r) { return mb + kMailboxRecBase + (bank + r) * kMailboxRecSlotWords; };
    for (int64_t k = threadIdx.x; k < stride; k += kBlock) {
        const uint64_t w = (uint64_t)__double_as_longlong(src[k]);
        for (int p = 0; p < nranks; ++p)
            __hip_atomic_store(slot_of(peers.p[p], rank) + 8 + k, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every word of the record has landed
    __syncthreads();
    if (threadIdx.x == 0)
        for (int p = 0; p < nranks; ++p)
            __hip_atomic_store(slot_of(peers.p[p], rank), flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        bool got = lane >= nranks;
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        const uint64_t limit = t == 0 ? 1000000000ull : 200000000ull;   // 10 s at a run's start, else 2 s
        int ok = 1;
        for (unsigned it = 0;; ++it) {
            if (!got)
                got = __hip_atomic_load(slot_of(inbox, lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == flag;
            if (__all(got)) break;
            __builtin_amdgcn_s_sleep(1);
            if ((it & 15) == 15 && __any(__builtin_amdgcn_s_memrealtime() - t0 > limit)) { ok = 0; break; }
        }
        if (lane == 0) s_ok = ok;
    }
    __syncthreads();
    if (!s_ok) {
        if (threadIdx.x == 0) __hip_atomic_store(status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    for (int64_t e = threadIdx.x; e < (int64_t)nranks * stride; e += kBlock) {
        const int r = (int)(e / stride);
        const int64_t k = e - (int64_t)r * stride;
        recv[e] = __longlong_as_double((long long)__hip_atomic_load(slot_of(inbox, r) + 8 + k, __ATOMIC_RELAXED,
                                                                    __HIP_MEMORY_SCOPE_SYSTEM));
    }
    // every flag of this exchange has been seen: advance the counter (own mailbox, this rank only)
    if (threadIdx.x == 0)
        __hip_atomic_store(inbox + kMailboxXchgCount, count + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// K3: idx[t] from the K records of the last launch (or the last all-gather).
__global__ __launch_bounds__(kBlock) void greedy_finalize(const double* __restrict__ recs, int K,
                                                         int64_t stride, uint32_t* idx_out,
                                                         int64_t t) {
    __shared__ double s_v[kWaves];
    __shared__ int64_t s_i[kWaves];
    double v = INFINITY;
    int64_t gi = INT64_MAX;
    for (int r = threadIdx.x; r < K; r += kBlock) {
        const double rv = recs[(int64_t)r * stride];
        const int64_t ri = rec_gidx(recs + (int64_t)r * stride);
        if (better(rv, ri, v, gi)) { v = rv; gi = ri; }
    }
    block_minloc(v, gi, s_v, s_i);
    if (threadIdx.x == 0) idx_out[t] = (uint32_t)gi;
}

// ------------------------------------------------------------------------------------------
// host-side launchers; tuning state set by st_tune (defaults: measured best on MI355X)
// ------------------------------------------------------------------------------------------
// Defaults measured on MI355X (tools/probe.hip sweeps, DESIGN.md "Tuning"): 256 blocks (one per
// CU); d = 2/4 shards of >= 1e6 rows: one candidate per lane with register prefetch, smaller
// shards: two candidates per lane without prefetch.  st_tune overrides (-1 = automatic).
static int g_max_blocks = 256;
static int g_cpt = -1;
static int g_pf = -1;
static int g_rt_max_blocks = kMaxBlocks;
static int g_arith = 1;   // st_tune key 11 (process-wide)
// st_tune key 22: the calling host thread's own arithmetic (-1: none, the process-wide key 11 applies) --
// stein_thinning.arithmetic_override, so that threads thinning side by side (thin_chains: one per GPU)
// never change each other's launches
static thread_local int t_arith = -1;
static int g_tie_guard = 1;   // st_tune key 20
constexpr int64_t kLargeShard = 1000000;

int arith_compact() { return t_arith >= 0 ? t_arith : g_arith; }
int tie_guard() { return g_tie_guard; }

int tune_get(int key) {
    switch (key) {
        case 0: return g_max_blocks;
        case 1: return g_cpt;
        case 2: return g_pf;
        case 6: return g_rt_max_blocks;
        case 11: return g_arith;
        case 20: return g_tie_guard;
        case 22: return t_arith;
        default: return INT32_MIN;
    }
}

int tune(int key, int value) {
    switch (key) {
        case 11: if (value < -1 || value > 1) return -1; g_arith = value < 0 ? 1 : value; return 0;
        case 20: if (value < -1 || value > 1) return -1; g_tie_guard = value < 0 ? 1 : value; return 0;
        case 22: if (value < -1 || value > 1) return -1; t_arith = value; return 0;
        case 6: if (value < 1 || value > kMaxBlocks) return -1; g_rt_max_blocks = value; return 0;
        case 0: if (value < 1 || value > kMaxBlocks) return -1; g_max_blocks = value; return 0;
        case 1: if (value != -1 && value != 1 && value != 2 && value != 4) return -1; g_cpt = value; return 0;
        case 2: if (value < -1 || value > 1) return -1; g_pf = value; return 0;
        default: return -1;
    }
}

// kernel variant (candidates per lane, prefetch) launched for an (n, d) shard
static void variant_for(int64_t n, int d, int& cpt, int& pf) {
    if (d == 2 || d == 4) {
        const bool large = n >= kLargeShard;
        cpt = g_cpt > 0 ? g_cpt : (large ? 1 : 2);
        pf = g_pf >= 0 ? g_pf : (large ? 1 : 0);
    } else {
        cpt = d <= kMaxCtDim ? 2 : 1;
        pf = g_pf > 0 ? 1 : 0;
    }
}

int greedy_blocks(int64_t n, int d) {
    int cpt, pf;
    variant_for(n, d, cpt, pf);
    const int64_t per_block = (int64_t)cpt * kBlock;
    int64_t b = (n + per_block - 1) / per_block;
    // d > 8: one candidate per lane and a long dependent chain per candidate -- latency is hidden
    // by waves, not by registers: up to 4 blocks (16 waves) per CU
    const int cap = d > kMaxCtDim ? g_rt_max_blocks : g_max_blocks;
    if (b > cap) b = cap;
    if (b < 1) b = 1;
    return (int)b;
}

template <int D, int CPT, bool PF>
static void launch_ct3(const GreedyArgs& a, bool diag, int blocks, hipStream_t s) {
    const bool gf = a.w != nullptr;
    if (diag) {
        if (gf) greedy_step_ct<D, true, true, CPT, PF><<<blocks, kBlock, 0, s>>>(a);
        else greedy_step_ct<D, false, true, CPT, PF><<<blocks, kBlock, 0, s>>>(a);
    } else {
        if (gf) greedy_step_ct<D, true, false, CPT, PF><<<blocks, kBlock, 0, s>>>(a);
        else greedy_step_ct<D, false, false, CPT, PF><<<blocks, kBlock, 0, s>>>(a);
    }
}

template <int D>
static void launch_ct(const GreedyArgs& a, bool diag, int blocks, hipStream_t s) {
    int cpt, pf;
    variant_for(a.n, D, cpt, pf);
    if constexpr (D == 2 || D == 4) {   // full variant set
        switch (cpt * 2 + pf) {
            case 2: launch_ct3<D, 1, false>(a, diag, blocks, s); break;
            case 3: launch_ct3<D, 1, true>(a, diag, blocks, s); break;
            case 4: launch_ct3<D, 2, false>(a, diag, blocks, s); break;
            case 5: launch_ct3<D, 2, true>(a, diag, blocks, s); break;
            case 8: launch_ct3<D, 4, false>(a, diag, blocks, s); break;
            default: launch_ct3<D, 4, true>(a, diag, blocks, s); break;
        }
    } else {
        if (pf) launch_ct3<D, 2, true>(a, diag, blocks, s);
        else launch_ct3<D, 2, false>(a, diag, blocks, s);
    }
}

// bytes a step streams above which its column loads are non-temporal: 3/4 of the 256 MB MALL
constexpr double kStreamNtBytes = 192e6;

hipError_t launch_greedy_step(const GreedyArgs& a, bool diag, int blocks, hipStream_t s) {
    switch (a.d) {
        case 1: launch_ct<1>(a, diag, blocks, s); return hipGetLastError();
        case 2: launch_ct<2>(a, diag, blocks, s); return hipGetLastError();
        case 3: launch_ct<3>(a, diag, blocks, s); return hipGetLastError();
        case 4: launch_ct<4>(a, diag, blocks, s); return hipGetLastError();
        case 5: launch_ct<5>(a, diag, blocks, s); return hipGetLastError();
        case 6: launch_ct<6>(a, diag, blocks, s); return hipGetLastError();
        case 7: launch_ct<7>(a, diag, blocks, s); return hipGetLastError();
        case 8: launch_ct<8>(a, diag, blocks, s); return hipGetLastError();
        default: break;
    }
    const bool gf = a.w != nullptr;
    if (diag) {
        if (gf) greedy_step_rt<true, true, false><<<blocks, kBlock, 0, s>>>(a);
        else greedy_step_rt<false, true, false><<<blocks, kBlock, 0, s>>>(a);
        return hipGetLastError();
    }
    // non-temporal column loads once a step's columns outgrow the memory-side cache (stein_math.hpp
    // stream_load): config 5 (412 MB per step) 77.0 -> 70.0 us per step
    // (profiles/r02_step_rt_nt_ab.log); smaller shards keep default loads and re-hit the MALL
    const bool ntl = (double)a.n * (16.0 * a.d + 24.0) > kStreamNtBytes;
    if (gf) {
        if (ntl) greedy_step_rt<true, false, true><<<blocks, kBlock, 0, s>>>(a);
        else greedy_step_rt<true, false, false><<<blocks, kBlock, 0, s>>>(a);
    } else {
        if (ntl) greedy_step_rt<false, false, true><<<blocks, kBlock, 0, s>>>(a);
        else greedy_step_rt<false, false, false><<<blocks, kBlock, 0, s>>>(a);
    }
    return hipGetLastError();
}

hipError_t launch_greedy_publish(const double* recs, int K, int64_t stride, int d, double* out,
                                 hipStream_t s) {
    greedy_publish<<<1, kBlock, 0, s>>>(recs, K, stride, d, out);
    return hipGetLastError();
}

hipError_t launch_greedy_rank_exchange(const double* recs, int K, int64_t stride, int d,
                                       const MailboxPeers& peers, int rank, int nranks, int64_t t,
                                       double* recv, unsigned* status, hipStream_t s) {
    greedy_rank_exchange<<<1, kBlock, 0, s>>>(recs, K, stride, d, peers, rank, nranks, t, recv, status);
    return hipGetLastError();
}

hipError_t launch_greedy_finalize(const double* recs, int K, int64_t stride, uint32_t* idx_out,
                                  int64_t t, hipStream_t s) {
    greedy_finalize<<<1, kBlock, 0, s>>>(recs, K, stride, idx_out, t);
    return hipGetLastError();
}

}  // namespace st
