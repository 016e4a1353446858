// Persistent, on-chip-resident greedy kernel (K4) for gfx950.
//
// One launch runs the whole greedy loop of the reference's _greedy_search
// (JAX_Stein_Thinning.ipynb cell 22, json ~281-295; report.tex:413-426) for one device:
//   * G <= #CU blocks of 256 threads, one per CU.  Block b owns rows [b*R, (b+1)*R).
//   * Its rows live on chip for the whole run: RT rows per thread in VGPRs/AGPRs (x, g, A[, w]),
//     RL rows in LDS (SoA), the remainder streamed from HBM each step (coalesced, like K2).
//   * Per step: every block evaluates k(x_i, x_j) for its rows, A_i += 2k, block MINLOC, and
//     publishes ONE record {A_min, index} as two data-tagged 8-byte granules (8-bit step tag;
//     MI355X_MICROARCH.md recipe R2, "the data IS the flag": no fence, no counter).  One wave per
//     block sweeps all G records until every tag matches, reduces them (np.argmin order) and the
//     block reads the winner's row from the read-only x / g / w arrays -> next step.  Block 0
//     writes idx.  Two record banks alternate by step parity.
//   * Every spin is bounded by a wall-clock timeout (s_memrealtime); a timeout sets status[0] and
//     every block leaves the step loop, so the grid always drains.
// Multi-rank (one process per GPU, nranks > 1): every rank runs this kernel over its row block
// [row_begin, row_end) of the full (replicated, read-only) arrays.  After the block-level sweep,
// block 0 pushes the rank's winner {A_min, global index} as a 16-bit-tagged two-granule record
// into slot `rank` of every peer's mailbox (IPC-mapped uncached device memory, system-scope
// stores over xGMI); one wave per block polls the R slots of its own mailbox, loads each arriving
// candidate's row from the replicated inputs, and picks the global winner in np.argmin order.
// No host round trip and no collective launch per step.
// Arithmetic per pair: K2's (stein_math.hpp) or, when the block's rows and the winner lie in the
// guarded range, its division/sqrt-light form that returns the same bits (finish_pair_fast):
// results are bit-identical to st_greedy's launch-per-step path and to the C bit model.
#pragma once
#include <algorithm>
#include <type_traits>

#include "stein_math.hpp"
#include "stein_internal.hpp"

namespace st {

namespace {

constexpr int kMaxPWaves = 8;                // up to 512-thread blocks
constexpr int kMaxGrid = 512;               // up to two blocks per CU on MI355X (256 CUs)
constexpr int kMaxRanks = kMailboxRanks;    // GPUs of one node
constexpr uint64_t kTimeoutTicks = 200000000ull;   // s_memrealtime runs at 100 MHz: 2 s
constexpr uint64_t kFirstRankTimeoutTicks = 1000000000ull;   // 10 s: peers' launch skew at step 0
// one device, step 0: every block of the grid publishes its diagonal minimum microseconds after it
// starts, so a record still missing after 100 ms means the grid is not co-resident (another
// kernel holds CUs: the plain launch below cannot reserve them).  The run aborts early and the
// host re-runs the thin on the launch-per-step path (DeviceProblem.greedy).
constexpr uint64_t kFirstStepTimeoutTicks = 10000000ull;
// wide variant (D > 8, instantiated for D = 50): one row per thread in registers and no LDS or
// streamed rows -- only when a block's rows fit (R <= 256: shards up to 256 x #CU rows, e.g. one
// rank of an 8-GPU config-5 run); the winner row is read from LDS inside the pair loop
constexpr int kWideD = 50;

__device__ __forceinline__ void p_wave_minloc(double& v, int64_t& i) { wave_minloc(v, i); }

struct Scratch {          // small per-block scratch at the start of the dynamic LDS region
    double row[2 * kWideD + 2];   // winner row {x[d], g[d], w}
    double vblk;          // this block's last published minimum (NaN iff some row's A is NaN)
    uint64_t wk[kMaxPWaves]; // per-wave minima as value_key (publish) and
    int64_t i[kMaxPWaves];   // their rows: valid until the next publish (the guard's rescans combine them)
    int64_t win;          // the step's winner, from the picking wave to the block
    int abort;
    int rowfast;          // wide d: the winner row lies in the fast range (set by the fetching wave)
    int ctr[2];           // 512-thread blocks: per-step chunk counters (dynamic LDS / streamed rows)
};

// near-tie guard state (GUARD kernels only: after Scratch in the dynamic LDS), by step parity: per wave,
// the rescan's smallest sum of the block's rows other than the block's minimum row and its bitwise
// duplicates ("other"); the step's winner (row and sum; tie_check reads its score row and weight from the
// inputs) and this block's published minimum and its row; the threshold recurrence
// LDS rows a guarded plan keeps at most (the repeat bits of GuardScratch::lrep; persistent.hip caps RL)
constexpr int kGuardLdsRows = 4096;
struct GuardScratch {
    double rs_o[2][kMaxPWaves];
    uint32_t win_i[2], blk_i[2];
    double win_v[2], blk_v[2];
    double tg[6];         // recurrence state (stein_ref.c tie_state): c1, wmax, Dmax, Q, E, thr
    double bnd[kMaxPWaves][2];   // per wave: max_i |g_i|^2, max_i w_i^2 over its rows (staging)
    // 512-thread kernels: wave 0's per-lane rescan of its register rows (step t - 1, written at the start
    // of step t) -- the lane's "other" and the mask of its register rows whose sum equals the block's
    // minimum -- finished (duplicate test) and reduced by wave 1 after publishing step t, off the critical path
    double w0_o[64];
    uint32_t w0_m[64];
    // LDS rows that repeat their predecessor row bit for bit (x, g, w): bit e of the LDS rows (staging)
    uint32_t lrep[kGuardLdsRows / 32];
    int tied;             // a step was flagged (this block's word was written)
};

// 256-thread GUARD kernels (no dynamic chunks): every thread's "other" of a step and the mask of its
// register rows still to be tested for being duplicates of the block's minimum row (wave 0's threads; the
// other waves test theirs while rescanning), by parity, after GuardScratch in the dynamic LDS.  Only the
// winner's block, or a block whose minimum equals the winner's sum, needs its "other" (tie_check), so
// only such a block reduces these -- the other blocks run no wave reduction for the guard at all
struct GuardLanes {
    double o[2][256];
    uint32_t m[2][256];
};

// Per-thread argmin scan: every thread visits its rows in increasing index order, so a candidate
// replaces the running best only if strictly smaller, or NaN over non-NaN (np.argmin order
// restricted to increasing indices: ties and later NaNs keep the earlier row).  The running best
// starts at the thread's first row.  Branch-free; 32-bit row indices (n < 2^32 - 1).
__device__ __forceinline__ void scan_take(double a, uint32_t ia, double& b, uint32_t& ib) {
    const bool take = (a < b) | (__builtin_isnan(a) & !__builtin_isnan(b));
    b = take ? a : b;
    ib = take ? ia : ib;
}

// The same when no A of the block can be NaN (fast variant: see greedy_persistent): plain '<'.
template <bool NANFREE>
__device__ __forceinline__ void scan_take_v(double a, uint32_t ia, double& b, uint32_t& ib) {
    if constexpr (NANFREE) {
        const bool take = a < b;
        b = take ? a : b;
        ib = take ? ia : ib;
    } else {
        scan_take(a, ia, b, ib);
    }
}

// Order-free form for rows visited out of index order: ties go to the lower index, NaN beats
// non-NaN and the lower-indexed NaN wins (np.argmin).  NANFREE: no A of the block is NaN.
template <bool NANFREE>
__device__ __forceinline__ void scan_take_idx(double a, uint32_t ia, double& b, uint32_t& ib) {
    bool take;
    if constexpr (NANFREE) {
        take = (a < b) | ((a == b) & (ia < ib));
    } else {
        const bool na = __builtin_isnan(a), nb = __builtin_isnan(b);
        take = (a < b) | ((a == b) & (ia < ib)) | (na & !nb) | (na & nb & (ia < ib));
    }
    b = take ? a : b;
    ib = take ? ia : ib;
}

// one f64 through a buffer descriptor: byte offsets voff (per lane) + soff (uniform, an SGPR)
__device__ __forceinline__ double buf_load_f64(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
    return __longlong_as_double((long long)(((uint64_t)v.y << 32) | v.x));
}

// value known to be identical in every lane: move it to SGPRs
__device__ __forceinline__ double uniform(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

// Wide d: pair_value_ct's arithmetic (same operations, same order -> same bits) for a row whose x
// is in registers and whose g is in LDS (gi[k * gs]) against the winner row in LDS, eight
// coordinates per stage with a scheduling barrier between stages, so LDS values are read just
// before use instead of being hoisted into VGPRs next to the register row.
template <int D, bool FAST>
__device__ __forceinline__ double pair_value_wide(const double (&xi)[D], const double* gi, int gs,
                                                  const double* xj, const double* gj, double l,
                                                  double l2, double tr) {
    static_assert(D >= 8, "wide variant");
    constexpr int full = D - (D % 8);
    double qs = 0.0, t1s = 0.0, t2s = 0.0, t3s = 0.0;
    double r[8];
#pragma unroll
    for (int k0 = 0; k0 < D; k0 += 8) {
        double bx[8], bg[8], ag[8];
#pragma unroll
        for (int j = 0; j < 8; ++j)
            if (k0 + j < D) { bx[j] = xj[k0 + j]; bg[j] = gj[k0 + j]; ag[j] = gi[(k0 + j) * gs]; }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int k = k0 + j;
            if (k < D) {
                const double dl = xi[k] - bx[j];
                const double gd = ag[j] - bg[j];
                const double q = (l * dl) * dl;
                const double u = (l2 * dl) * dl;
                const double v = (l * gd) * dl;
                if (k == 0) {
                    qs = q; t1s = u; t2s = v;
                } else {
                    qs = qs + q; t1s = t1s + u; t2s = t2s + v;
                }
                const double p = ag[j] * bg[j];
                if (k < 8) {
                    r[k] = p;
                } else if (k < full) {
                    r[k % 8] += p;
                } else {
                    if (k == full) t3s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
                    t3s += p;
                }
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (full == D) t3s = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    if constexpr (FAST) return finish_pair_fast(qs, t1s, t2s, t3s, tr);
    else return finish_pair(qs, t1s, t2s, t3s, tr);
}

// Pair arithmetic of one sweep variant (block-uniform choice per step):
//   AR 0: exact, general (NaN / overflow semantics of NumPy)   AR 1: exact, range-guarded (same bits)
//   AR 2: compact (every pair of the block-step in range)     AR 3: per pair, compact iff jok (l, tr and
//         the winner in range) and this row in range, else exact general (pair_value_sel's rule)
template <int D, int AR>
__device__ __forceinline__ double pair_ar(const double (&xi)[D], const double (&gi)[D], const double* xj,
                                          const double* gj, double l, double l2, double m3l2, double tr,
                                          int jok) {
    if constexpr (AR == 2) return pair_compact_ct<D>(xi, gi, xj, gj, l, m3l2, tr);
    else if constexpr (AR == 3)
        return pair_value_sel<D>(jok && row_in_range<D>(xi, gi), xi, gi, xj, gj, l, l2, m3l2, tr);
    else return pair_value_ct<D, AR == 1>(xi, gi, xj, gj, l, l2, tr);
}

}  // namespace

struct PersistArgs {
    const double* x;      // SoA (d, ld), full sample (replicated on every rank)
    const double* g;
    const double* w;
    double* A;            // (ld) running sums; rows [row_begin, row_end) are this rank's
    int64_t n, ld;        // n = total rows
    double l, tr;
    int64_t m;            // n_points
    uint32_t* idx_out;
    uint64_t* gran;       // 2 banks x G records x 2 granules
    unsigned* status;     // [0]: 0 ok, 1 timeout, 2 (compact-only kernel) a pair needs the exact arithmetic
    const unsigned* gate; // general kernel after a compact-only one: run only if *gate == 2
    int64_t rows_per_block;
    int RL;               // LDS-resident rows per block
    int stream_a_lds;     // 512-thread kernels: the streamed rows' running sums are kept in LDS
    int poll_delay;       // s_memrealtime ticks added before aligning a step's first poll (st_tune key 16)
    int lds_two_chains;   // 512-thread kernels: two LDS chunks as two independent chains (st_tune key 19)
    uint64_t* stamps;     // diagnostic build only (ST_PERSIST_STAMPS): [G][kStampSteps][kStampPhases]
    int rec_stride;               // record pitch in granules (2 = packed; wider spreads the polled
                                  // records over more memory channels)
    int nrep;                     // record replicas: every block stores its record into each of
                                  // them, block b sweeps replica b % nrep (fewer readers per line)
    int64_t rep_stride;           // granules between replicas (and between banks' replica sets)
    int64_t row_begin, row_end;   // this rank's rows (global indices); one device: [0, n)
    int rank, nranks;
    uint64_t seq_base;            // exchange sequence number of step 0 (mailbox banks / tags)
    uint64_t* inbox;              // this rank's mailbox (nranks > 1)
    uint64_t* peer[kMaxRanks];    // every rank's mailbox as mapped in this process
    // near-tie guard of the compact arithmetic (the GUARD kernels; nullptr = off): the problem's
    // [max_i |g_i|^2, max_i w_i^2] -- every block merges its rows' maxima during staging (u64 atomic max on
    // the bit patterns); a multi-rank run's host has merged all n rows' beforehand -- and the word
    // receiving the first flagged step as ~step through an atomic max (0: none); tie[3] = 1 marks a
    // guarded run
    const double* tie_bounds;
    unsigned* tie;
};

// Diagnostic build (-DST_PERSIST_STAMPS, tools/probe only; never the product library): lane 0 of
// every block records s_memrealtime (100 MHz, chip-wide clock) at each phase of steps
// [kStampFirst, kStampFirst + kStampSteps).
[[maybe_unused]] constexpr int kStampFirst = 20, kStampSteps = 32, kStampPhases = 32;
#ifdef ST_PERSIST_STAMPS
#define ST_STAMP(a, t, ph)                                                                         \
    do {                                                                                            \
        if ((a).stamps && threadIdx.x == 0 && (t) >= kStampFirst && (t) < kStampFirst + kStampSteps) \
            (a).stamps[((int64_t)blockIdx.x * kStampSteps + ((t) - kStampFirst)) * kStampPhases + (ph)] = \
                __builtin_amdgcn_s_memrealtime();                                                    \
    } while (0)
// value-ordered stamp: taken only after `val` has been computed (an opaque use pins the order)
#define ST_STAMP_AFTER(a, t, ph, val)                                                              \
    do {                                                                                            \
        asm volatile("" ::"v"(val));                                                                \
        ST_STAMP(a, t, ph);                                                                         \
    } while (0)
// per-wave stamp: lane 0 of every wave writes phase ph + wave
#define ST_STAMP_WAVE(a, t, ph)                                                                    \
    do {                                                                                            \
        if ((a).stamps && (threadIdx.x & 63) == 0 && (t) >= kStampFirst && (t) < kStampFirst + kStampSteps) \
            (a).stamps[((int64_t)blockIdx.x * kStampSteps + ((t) - kStampFirst)) * kStampPhases + (ph) + \
                       (threadIdx.x >> 6)] = __builtin_amdgcn_s_memrealtime();                         \
    } while (0)
#else
#define ST_STAMP_WAVE(a, t, ph) do { } while (0)
#define ST_STAMP(a, t, ph) do { } while (0)
#define ST_STAMP_AFTER(a, t, ph, val) do { } while (0)
#endif

// Exchange = self-validating granules (MI355X_MICROARCH.md R2: "the data IS the flag"): each block
// publishes {A_min, index} for step t as ONE 16-byte record of two 8-byte granules, each written
// by one aligned 8-B agent-scope store and each carrying the 8-bit tag (t+1) mod 256 in its top
// byte:   g0 = tag:8 | value bits 63..8         g1 = tag:8 | pad:16 | value bits 7..0 | index:32
// A consumer accepts a record only when both tags match.  Banks alternate by step parity, so a
// slot's stale content is exactly two steps old (tag t-1): an 8-bit tag cannot alias it.
constexpr int kRecGranules = 2;
// bytes between consecutive blocks' records: 256 spreads the 256 polled records of a step over
// more memory channels than 16-B packing (-0.3 us per step, profiles/r01_sweep_pitch.log)
constexpr int kDefaultRecPitch = 256;
// replicas of the record array (st_tune key 10): every block stores its record into each replica
// (16-B sc1 stores by 8 lanes) and block b sweeps replica b % 8, densely packed: 32 readers per
// line instead of 256, 32 lines per poll instead of 256.  Round 2 (16 replicas): config 4 11.6 ->
// 11.1 ms per thin; n = 2.5e5 per device (one rank of 8): 4.80 -> 4.47 us per step
// (profiles/r02_record_replicas.log).  Round 4, the round-4 kernel, same box, two sweeps
// (profiles/r04_replicas_nt_sweep.log): 8 replicas against 16 -- config 2 3.32 vs 3.41 / 3.46 us per
// step, 2.5e5 rows 3.31 / 3.32 vs 3.34, config 4 6.82 / 6.84 vs 6.89 (4 replicas within 0.01 of 8, 32
// slower); the flat-sweep probe without pair arithmetic agrees (1.80 vs 2.15 us per step,
// profiles/r04_flat_sweep_probe.log)
constexpr int kDefaultRecReplicas = 8;
constexpr int64_t kNt512MinRows = 1280;

__device__ __forceinline__ uint64_t step_tag(int64_t t) { return (uint64_t)((t + 1) & 0xFF) << 56; }

// Block records carry the minimum as an order-preserving 64-bit KEY instead of its raw bits, so the
// sweeping wave compares records with integer compares (no NaN classification per record):
//   NaN -> 0 (np.argmin: NaN is the minimum), x >= +0 -> bits | 2^63, x < 0 -> ~bits,
// with -0 taken as +0 (they compare equal).  Unsigned key order = np.argmin's value order; equal
// keys tie on the lower index as before.  key_value inverts it (key 0 -> a NaN).
__device__ __forceinline__ uint64_t value_key(double v) {
    const uint64_t b = (uint64_t)__double_as_longlong(v == 0.0 ? 0.0 : v);
    const uint64_t k = (b >> 63) ? ~b : (b | 0x8000000000000000ull);
    return __builtin_isnan(v) ? 0ull : k;
}
__device__ __forceinline__ double key_value(uint64_t k) {
    return __longlong_as_double((long long)((k >> 63) ? (k ^ 0x8000000000000000ull) : ~k));
}

// the block's wave minima in np.argmin order, as (value_key, index) with integer compares (no NaN
// classification: value_key already orders NaN first and -0 with +0); one lane, NT / 64 - 1 steps
template <int NT>
__device__ __forceinline__ void combine_waves(const Scratch* sc, uint64_t& k, uint32_t& li) {
    k = sc->wk[0];
    li = sc->i[0] == INT64_MAX ? 0xFFFFFFFFu : (uint32_t)sc->i[0];
#pragma unroll
    for (int w = 1; w < NT / 64; ++w) {
        const uint64_t ok = sc->wk[w];
        const uint32_t oi = sc->i[w] == INT64_MAX ? 0xFFFFFFFFu : (uint32_t)sc->i[w];
        const bool tk = (ok < k) | ((ok == k) & (oi < li));
        k = tk ? ok : k;
        li = tk ? oi : li;
    }
}

template <int NT, bool GUARD = false>
__device__ __forceinline__ void publish(const PersistArgs& a, Scratch* sc, double v, uint32_t row,
                                        int64_t t, int64_t r1, unsigned bid, GuardScratch* gsc = nullptr) {
    // padding rows (>= r1) carry +inf and the "no row" sentinel index, so they lose every tie --
    // their indices may be real rows of the next rank
    int64_t li = (int64_t)row < r1 ? (int64_t)row : INT64_MAX;
    ST_STAMP_WAVE(a, t, 12);
    p_wave_minloc(v, li);
    ST_STAMP_AFTER(a, t, 10, v);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) { sc->wk[wave] = value_key(v); sc->i[wave] = li; }
    __syncthreads();
    ST_STAMP(a, t, 11);
    if (a.nrep == 1) {
        if (threadIdx.x == 0) {   // ONE lane combines the wave minima and stores the two granules
            uint64_t k;
            uint32_t ib;
            combine_waves<NT>(sc, k, ib);
            const double vb = key_value(k);
            sc->vblk = vb;   // read by every thread after wait_and_pick's barrier
            uint64_t* gr = a.gran + (t & 1) * a.rep_stride + (int64_t)bid * a.rec_stride;
            const uint64_t tag = step_tag(t);
            __hip_atomic_store(gr + 0, tag | (k >> 8), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(gr + 1, tag | ((k & 0xFFull) << 32) | ib, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            if constexpr (GUARD) {   // this block's minimum of step t and its row (after the record: off its path)
                gsc->blk_v[t & 1] = vb;
                gsc->blk_i[t & 1] = ib;
            }
        }
    } else if (threadIdx.x < 64) {
        // replicated records: wave 0 combines (every lane the same values from LDS) and lane r
        // stores the record into replica r as ONE 16-B sc1 store (both granules tagged: a torn
        // store fails the reader's tag check like two 8-B stores would)
        uint64_t k;
        uint32_t ib;
        combine_waves<NT>(sc, k, ib);
        if (threadIdx.x == 0) sc->vblk = key_value(k);
        if ((int)threadIdx.x < a.nrep) {
            const uint64_t tag = step_tag(t);
            const uint64_t g0 = tag | (k >> 8), g1 = tag | ((k & 0xFFull) << 32) | ib;
            const int64_t off = (((t & 1) * a.nrep + threadIdx.x) * a.rep_stride +
                                 (int64_t)bid * a.rec_stride) * 8;
            const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(a.gran, 0, 0x7FFFFFFF, 0x00020000);
            typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{(unsigned)g0, (unsigned)(g0 >> 32), (unsigned)g1,
                                                         (unsigned)(g1 >> 32)},
                                                   rsrc, (int)off, 0, 16 /* sc1 */);
        }
        if constexpr (GUARD) {   // this block's minimum of step t and its row (after the record: off its path)
            if (threadIdx.x == 0) {
                gsc->blk_v[t & 1] = key_value(k);
                gsc->blk_i[t & 1] = ib;
            }
        }
    }
}

// Polls are issued on a chip-wide grid of ST_POLL_SYNC ticks of s_memrealtime (100 MHz: 450 ns).
// Every block then sees the last record of a step at about the same moment and starts the next
// step together, instead of each at its own poll phase (the spread of next-step starts was about
// one poll period, ~1.1 us, and the latest starter bounds the next exchange).  Same-box, three
// rounds (profiles/r03_poll_sync.log): n = 2e6 7.06 -> 6.83 us per step, n = 1e6 5.06 -> 4.97,
// n = 2.5e5 (the 8-GPU shard size) 3.30 -> 3.17; grids of 300 / 380 / 520 / 600 / 800 / 1100 /
// 1300 ns, and leaving the first poll of a step unaligned, were measured beside it (coarser grids
// quantise the step: 1.3 us made n = 2.5e5 3.9 us per step).
#ifndef ST_POLL_SYNC
#define ST_POLL_SYNC 45
#endif
// near-tie guard layout experiment (measurement builds only; the default is the product's)
#ifndef ST_GUARD_RW0
#define ST_GUARD_RW0 2
#endif
#ifndef ST_LANES_W0_IN_POLL
#define ST_LANES_W0_IN_POLL 1
#endif
// the rescan's streamed / LDS row loops unrolled (measurement builds; 1 = the product)
#ifndef ST_GUARD_UNROLL
#define ST_GUARD_UNROLL 1
#endif
#define ST_PRAGMA_(x) _Pragma(#x)
#define ST_UNROLL_N_(n) ST_PRAGMA_(unroll n)
#if ST_GUARD_UNROLL > 1
#define ST_GUARD_UNROLL_LOOP ST_UNROLL_N_(ST_GUARD_UNROLL)
#else
#define ST_GUARD_UNROLL_LOOP
#endif
// the near-tie bounds' per-block atomic maxima: spread over this many 64-B slots of the workspace's
// control block (block b -> slot b % ST_BOUNDS_SLOTS; the late check of step 0 reduces them), or all into the
// two bounds words (0)
#ifndef ST_BOUNDS_SLOTS
#define ST_BOUNDS_SLOTS 16
#endif
static_assert(ST_BOUNDS_SLOTS * 64 <= kWsStatusOff, "bounds slots: the control block's first 1 KB");
#ifndef ST_POLL_SYNC_FIRST
#define ST_POLL_SYNC_FIRST 1
#endif



// ---- near-tie guard (compact arithmetic) ------------------------------------------------------
// Step t is flagged when the smallest running sum of any row other than the winner and its bitwise
// duplicates -- any other exact tie included -- lies within thr(t) of the winner's (oracle/stein_ref.c
// sr_greedy_mt_ties is the model: the rule, the bound thr(t) and its recurrence).  A row equal to the
// winner bit for bit (x, g, w: a repeated MCMC row, adjacent or not) has the winner's sum at every step in
// every arithmetic and loses the tie to the lower index on both paths, so it does not count.
// Nothing is added to the pair loop or to the exchange's critical path.  After publishing step t the waves
// that do not sweep rescan the block's running sums (already on chip: registers, LDS, and the streamed
// rows' sums in L2) against the block's minimum vmin and its row ibk, both known from the publish: per
// thread the smallest sum != vmin ("other"), and for the rows whose sum == vmin (other than ibk) a bitwise
// comparison with row ibk -- a row that differs is a genuine tie and contributes vmin.  So "other" is the
// smallest sum of the block's rows other than ibk and its duplicates.  The picking wave (wave 0) only
// records its register rows' "other" and the mask of those tied with vmin (while its first poll is in
// flight; 512-thread kernels: right after the pick); the comparison of those rows is done later by the
// wave that reduces them (global loads of both rows), off the critical path.  One step later (during step
// t + 1's exchange) one lane checks step t: in the winner's block (ibk = the winner), the block's "other";
// in a block whose minimum equals the winner's sum exactly, its "other" if its row ibk duplicates the
// winner, else that minimum; in every other block, its minimum -- together exactly the model's rule.  A
// flagged block writes ~t into the tie word with an atomic max (the largest ~t = the first flagged step);
// the same lane advances the threshold recurrence.  Multi-rank runs (nranks > 1): every rank's blocks run
// the same check against the global winner (each rank flags its own rows; the host combines the ranks'
// words with one all-reduce after the run) over bounds the host computed from all n rows beforehand.

// slot s of the near-tie bounds' per-block maxima (ST_BOUNDS_SLOTS): 64 B apart in the first kilobyte of the
// workspace's control block, which st_greedy zeroes with the rest before every launch
__device__ __forceinline__ uint64_t* bounds_slot(const PersistArgs& a, int s) {
    char* base = reinterpret_cast<char*>(const_cast<double*>(a.tie_bounds)) - kWsBoundsOff;
    return reinterpret_cast<uint64_t*>(base + (int64_t)s * 64);
}

// the row (x, g[, w]) of row r from the read-only inputs
template <int D, bool GF>
struct RowBits {
    double v[2 * D + (GF ? 1 : 0)];
    __device__ __forceinline__ void load(const PersistArgs& a, int64_t r) {
#pragma unroll
        for (int k = 0; k < D; ++k) {
            v[k] = a.x[(int64_t)k * a.ld + r];
            v[D + k] = a.g[(int64_t)k * a.ld + r];
        }
        if constexpr (GF) v[2 * D] = a.w[r];
    }
};

__device__ __forceinline__ bool same_bits(double p, double q) {
    return __double_as_longlong(p) == __double_as_longlong(q);
}

template <int D, bool GF>
__device__ __forceinline__ bool rows_equal(const RowBits<D, GF>& p, const RowBits<D, GF>& q) {
    bool eq = true;
#pragma unroll
    for (int k = 0; k < 2 * D + (GF ? 1 : 0); ++k) eq &= same_bits(p.v[k], q.v[k]);
    return eq;
}

// a sum's contribution to "other": everything but the block's minimum value (rows tied with it are
// tested separately)
__device__ __forceinline__ double other_of(double a, double vmin) { return a == vmin ? INFINITY : a; }

__device__ __forceinline__ double wave_max_f64(double m) {
    m = __builtin_fmax(m, dpp_f64<0xB1>(m));
    m = __builtin_fmax(m, dpp_f64<0x4E>(m));
    m = __builtin_fmax(m, dpp_f64<0x124>(m));
    m = __builtin_fmax(m, dpp_f64<0x128>(m));
    const uint64_t mb = (uint64_t)__double_as_longlong(m);
    const double r0 = __longlong_as_double((long long)readlane_u64(mb, 0));
    const double r1 = __longlong_as_double((long long)readlane_u64(mb, 16));
    const double r2 = __longlong_as_double((long long)readlane_u64(mb, 32));
    const double r3 = __longlong_as_double((long long)readlane_u64(mb, 48));
    return __builtin_fmax(__builtin_fmax(r0, r1), __builtin_fmax(r2, r3));
}

__device__ __forceinline__ double wave_min_f64(double m) {
    m = __builtin_fmin(m, dpp_f64<0xB1>(m));
    m = __builtin_fmin(m, dpp_f64<0x4E>(m));
    m = __builtin_fmin(m, dpp_f64<0x124>(m));
    m = __builtin_fmin(m, dpp_f64<0x128>(m));
    const uint64_t mb = (uint64_t)__double_as_longlong(m);
    const double r0 = __longlong_as_double((long long)readlane_u64(mb, 0));
    const double r1 = __longlong_as_double((long long)readlane_u64(mb, 16));
    const double r2 = __longlong_as_double((long long)readlane_u64(mb, 32));
    const double r3 = __longlong_as_double((long long)readlane_u64(mb, 48));
    return __builtin_fmin(__builtin_fmin(r0, r1), __builtin_fmin(r2, r3));
}

// The duplicate test of register rows recorded as a mask (wave 0's rows): thread `owner`'s register rows
// q set in `msk` (rows r0 + q * NT + owner, sum == vmin) are compared with row ibk through global loads; a
// row that differs contributes vmin.  Per lane; the caller keeps it behind a wave-uniform branch.
template <int D, bool GF, int NT>
__device__ __forceinline__ double finish_mask(const PersistArgs& a, double o, uint32_t msk, int owner, int64_t r0,
                                              double vmin, const RowBits<D, GF>& b) {
    while (msk) {
        const int q = __builtin_ctz(msk);
        msk &= msk - 1;
        RowBits<D, GF> r;
        r.load(a, r0 + (int64_t)q * NT + owner);
        if (!rows_equal(r, b)) o = __builtin_fmin(o, vmin);
    }
    return o;
}

// one lane: the check of step t (its rescan and winner are in slot t & 1), then thr(t) -> thr(t + 1)
// (stein_ref.c tie_init / tie_step, the same operations).  Step 0 first reads the problem's bounds,
// which every block merged before publishing step 0 (so this block's sweep of step 0 saw them all), or
// the host wrote before the launch (multi-rank: all n rows)
// the winner's score row and weight of step t for the recurrence, from the read-only inputs
template <int D, bool GF>
struct WinnerG {
    double g[D], w;
    __device__ __forceinline__ void load(const PersistArgs& a, const GuardScratch* sc, int64_t t) {
        const uint32_t gi = sc->win_i[t & 1];
        const int64_t gr = (int64_t)gi < a.n ? (int64_t)gi : 0;   // a completed pick's row is always < n
#pragma unroll
        for (int k = 0; k < D; ++k) g[k] = a.g[(int64_t)k * a.ld + gr];
        w = GF ? a.w[gr] : 1.0;
    }
};

template <int D, bool GF>
__device__ __forceinline__ void tie_check(const PersistArgs& a, GuardScratch* sc, int64_t t, int64_t r0, int64_t r1,
                                          int nwaves, const WinnerG<D, GF>& wg) {
    const int par = (int)(t & 1);
    double* ts = sc->tg;   // c1, wmax, Dmax, Q, E, thr
    if (t == 0) {   // stein_ref.c tie_init
        uint64_t* bw = reinterpret_cast<uint64_t*>(const_cast<double*>(a.tie_bounds));
        uint64_t g2b = __hip_atomic_load(bw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        uint64_t w2b = __hip_atomic_load(bw + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#if ST_BOUNDS_SLOTS
        // the blocks' slots (the words hold the host's all-row bounds of a multi-rank run, else 0): maxima of
        // non-negative doubles as u64, like the atomics (block 0 writes the result into the words at the end)
        for (int s = 0; s < ST_BOUNDS_SLOTS; ++s) {
            const uint64_t* sw = bounds_slot(a, s);
            g2b = std::max(g2b, (uint64_t)__hip_atomic_load(sw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            w2b = std::max(w2b, (uint64_t)__hip_atomic_load(sw + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        }
#endif
        const double g2 = __longlong_as_double((long long)g2b);
        const double w2 = __longlong_as_double((long long)w2b);
        const double l = a.l, tr = a.tr;
        const double gm = __builtin_sqrt(g2), sl = __builtin_sqrt(l);
        ts[0] = (((3.0 * l + tr) + sl * gm) + 0.5 * l) + 0.5 * g2;
        ts[1] = __builtin_sqrt(w2);
        ts[2] = (tr + g2) * w2;
        ts[3] = 0.0;
        ts[4] = 0.0;
        ts[5] = 0x1p-50 * (8.0 * ts[2]);
    }
    const double v = sc->win_v[par];
    const uint32_t gi = sc->win_i[par];
    // a completed pick's row is always < n; so is a block's minimum row unless the block holds no row
    const int64_t gr = (int64_t)gi < a.n ? (int64_t)gi : 0;
    double other = sc->blk_v[par];
    bool rest = (int64_t)gi >= r0 && (int64_t)gi < r1;   // the winner's block: its "other"
    if (!rest && other == v) {   // this block's minimum ties the winner's sum: a duplicate of the winner?
        const uint32_t bi = sc->blk_i[par];
        RowBits<D, GF> p, q;
        p.load(a, gr);
        q.load(a, (int64_t)bi < a.n ? (int64_t)bi : 0);
        rest = rows_equal(p, q);
    }
    if (rest) {
        other = INFINITY;
        for (int w = 0; w < nwaves; ++w) other = __builtin_fmin(other, sc->rs_o[par][w]);
    }
    if (other - v <= ts[5] && !sc->tied) {
        sc->tied = 1;
        __hip_atomic_fetch_max(a.tie, ~(unsigned)t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const double Q = ts[3] + v;
    // the winner's g row and weight, loaded by the caller at the start of its chain (WinnerG): the loads fly
    // while it reduces the rescans (Scratch::row may already hold the next step's winner)
    double gj2 = wg.g[0] * wg.g[0];
#pragma unroll
    for (int k = 1; k < D; ++k) gj2 = gj2 + wg.g[k] * wg.g[k];
    const double wj = GF ? wg.w : 1.0;
    const double scale = (ts[0] + gj2) * (ts[1] * wj);
    const double E = ts[4] + (16.0 * scale + (2.0 * ts[2] + __builtin_fmax(Q, 0.0)));
    ts[3] = Q;
    ts[4] = E;
    ts[5] = 0x1p-50 * (8.0 * ts[2] + E);
}

// tie_check for the 256-thread GUARD kernels (one whole wave): in a block that needs its "other" (the
// winner's block, or one whose minimum equals the winner's sum) the wave finishes the duplicate test of
// wave 0's recorded rows and reduces the block's per-thread "other" of step t (GuardLanes) into rs slot 0;
// the other blocks only compare their published minimum; then lane 0 runs tie_check on that one slot
template <int D, bool GF, int NT>
__device__ __forceinline__ void tie_check_lanes(const PersistArgs& a, GuardScratch* sc, const GuardLanes* gl,
                                                int64_t t, int64_t r0, int64_t r1) {
    static_assert(NT <= 256, "GuardLanes holds 256 threads");
    const int par = (int)(t & 1);
    WinnerG<D, GF> wg;   // issued first: lands while the lanes reduce
    if ((threadIdx.x & 63) == 0) wg.load(a, sc, t);
    const uint32_t gi = sc->win_i[par];
    const double vmin = sc->blk_v[par];
    if (((int64_t)gi >= r0 && (int64_t)gi < r1) || vmin == sc->win_v[par]) {   // block-uniform
        const int lane = (int)(threadIdx.x & 63);
        double o = INFINITY;
        uint32_t any = 0;
#pragma unroll
        for (int k = lane; k < NT; k += 64) {
            o = __builtin_fmin(o, gl->o[par][k]);
            any |= gl->m[par][k];
        }
        if (__any(any != 0)) {
            const uint32_t bi = sc->blk_i[par];
            RowBits<D, GF> b;
            b.load(a, (int64_t)bi < a.n ? (int64_t)bi : 0);
#pragma unroll
            for (int k = lane; k < NT; k += 64) o = finish_mask<D, GF, NT>(a, o, gl->m[par][k], k, r0, vmin, b);
        }
        o = wave_min_f64(o);
        if (lane == 0) sc->rs_o[par][0] = o;
    }
    if ((threadIdx.x & 63) == 0) tie_check<D, GF>(a, sc, t, r0, r1, 1, wg);
}

// wave 0 sweeps the G records of step t until every tag matches (bounded) and reduces them
// (np.argmin order).  Lane L owns records L, L+64, L+128, L+192 and re-polls only those it has not
// seen yet.  Whenever its best-so-far changes it loads that candidate's row (x, g[, w]) from the
// read-only inputs, so the winner's row is normally in registers when the slowest block has
// published -- except in the iteration that completes the sweep: loads issued there would hold up
// the in-order vmcnt wait in front of the row's use.  After the wave MINLOC the winning lane
// writes the row to sc->row.  Returns the winner's index, or -1 if the sweep timed out (grid-wide
// abort).
// guard: the near-tie bookkeeping of this step -- the winner's row and sum in slot t & 1 --
// and, with rescan_here, rescan0() (wave 0's register rows, while the first poll is in flight; the
// 512-thread kernels rescan them at the start of the next step instead, away from the sweep's registers)
struct NoRescan {
    __device__ __forceinline__ void operator()() const {}
};
template <int D, bool GF, int MAXG, bool GUARD = false, typename RS = NoRescan>
__device__ __forceinline__ int64_t wait_and_pick(const PersistArgs& a, Scratch* sc, int64_t t, unsigned bid,
                                                 const int G, GuardScratch* gsc = nullptr, bool guard = false,
                                                 bool rescan_here = false, const RS& rescan0 = RS{}) {
    static_assert(MAXG % 64 == 0 && MAXG <= kMaxGrid && MAXG / 64 <= 32, "records per lane");
    constexpr bool kWide = D > kMaxCtDim;
    // wide rows are not prefetched into registers (2d + 1 doubles per lane): the wave loads the
    // winner's row into LDS after the pick
    constexpr int kRow = kWide ? 1 : 2 * D + (GF ? 1 : 0);
    ST_STAMP(a, t + 1, 0);
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        // nrep is a power of two (the plan's): a mask, not an integer division on the exchange's path
        const uint64_t* bank = a.gran + ((t & 1) * a.nrep + ((int)bid & (a.nrep - 1))) * a.rep_stride;
        const uint64_t want = step_tag(t);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        const uint64_t wait_limit = (t == 0 && a.nranks == 1) ? kFirstStepTimeoutTicks : kTimeoutTicks;
        uint32_t need = 0;
#pragma unroll
        for (int c = 0; c < MAXG / 64; ++c) need |= (lane + 64 * c < G) ? (1u << c) : 0u;
        uint32_t seen = 0;
        // the lane's best record so far as (key, index): value_key order, ties on the lower index;
        // "none" = the key of +inf with the no-row index (a padding block's record ties with it)
        constexpr uint64_t kNoKey = 0xFFF0000000000000ull;
        uint64_t bk = kNoKey;
        uint32_t bi = 0xFFFFFFFFu;
        auto lane_best = [&](double& v, int64_t& i) {
            v = key_value(bk);
            i = bi == 0xFFFFFFFFu ? INT64_MAX : (int64_t)bi;
        };
        int64_t row_of = INT64_MAX;        // index whose row is in rowv
        double rowv[kRow];
#pragma unroll
        for (int k = 0; k < kRow; ++k) rowv[k] = 0.0;
        auto load_row = [&](int64_t r) {
            if constexpr (kWide) {
                (void)r;
            } else {
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    rowv[k] = a.x[(int64_t)k * a.ld + r];
                    rowv[D + k] = a.g[(int64_t)k * a.ld + r];
                }
                if constexpr (GF) rowv[2 * D] = a.w[r];
            }
        };
        int ok_all = 1;
        unsigned it = 0;   // polls taken
        // one 16-B sc1 buffer load per record (both granules; a torn pair fails its tag check)
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t*>(bank), 0,
                                                            G * a.rec_stride * 8, 0x00020000);
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        // all four loads unconditionally (records past G read as zeros: the descriptor's range
        // check), so they issue back to back and a poll costs ONE round trip, not four; a record
        // already seen is re-read at an out-of-range offset (zeros, no memory access), so later
        // polls only load what is still missing
        const uint32_t oob = (uint32_t)G * a.rec_stride * 8;
        auto issue = [&](u32x4 (&qs)[MAXG / 64]) {
#pragma unroll
            for (int c = 0; c < MAXG / 64; ++c) {
                const uint32_t off = (uint32_t)(lane + 64 * c) * a.rec_stride * 8;
                qs[c] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, ((need & ~seen) >> c) & 1u ? off : oob,
                                                              0, 16 /* sc1 */);
            }
        };
        // branch-free: per record the two tag bytes, the key's two halves and one (key, index)
        // compare -- integer work only (records carry value_key, see publish); a record already seen
        // (or past G) is skipped by its mask bit, whatever the zeros it was re-read as
        const uint32_t want8 = (uint32_t)(want >> 56);
        auto take = [&](const u32x4 (&qs)[MAXG / 64]) {
            const uint32_t open = need & ~seen;
#pragma unroll
            for (int c = 0; c < MAXG / 64; ++c) {
                const u32x4 q = qs[c];
                const bool ok = (bool)((open >> c) & 1u) & ((q.y >> 24) == want8) & ((q.w >> 24) == want8);
                const uint64_t k = ((uint64_t)((q.y << 8) | (q.x >> 24)) << 32) | ((q.x << 8) | (q.w & 0xFFu));
                const uint32_t ib = q.z;
                const bool tk = ok & ((k < bk) | ((k == bk) & (ib < bi)));
                bk = tk ? k : bk;
                bi = tk ? ib : bi;
                seen |= ok ? (1u << c) : 0u;
            }
        };
        // after a poll: speculative row of the best so far; every 16 polls the bounded-wait check
        auto between = [&]() -> bool {
            if (bi != 0xFFFFFFFFu && (int64_t)bi != row_of) {
                load_row((int64_t)bi);
                row_of = (int64_t)bi;
            }
            if ((it & 15) == 15) {
                const bool late = __builtin_amdgcn_s_memrealtime() - t0 > wait_limit;
                const bool other = __hip_atomic_load(a.status, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT) != 0;
                if (__any(late || other)) { ok_all = 0; return false; }
            }
            ++it;
            return true;
        };
        // one poll in flight (two staggered polls were measured slower at every stagger, with
        // and without replicas: profiles/r02_poll_stagger_rejected.log)
        // While a poll is in flight the wave reduces what the earlier polls brought (wv, wi: the
        // wave's best so far, uniform), so after the last poll only lanes whose best changed in it
        // need combining -- usually none (the last records seldom hold the winner).
        double wv = INFINITY;
        int64_t wi = INT64_MAX;
#ifdef ST_PERSIST_STAMPS
        // speculation study (diagnostic build only): the wave's best record after the first poll,
        // how many records that poll saw, and the poll after which the best stopped changing
        int64_t spec_first = -1, spec_prev = -2;
        unsigned spec_seen0 = 0, spec_settle = 0;
        uint64_t proc_ticks = 0;   // sum over polls of (records processed) - (poll data landed)
#endif
        for (;;) {
            u32x4 qs[MAXG / 64];
#if ST_POLL_SYNC > 0
            if (ST_POLL_SYNC_FIRST || it > 0) {   // polls on a chip-wide grid of ST_POLL_SYNC ticks
                const uint64_t now = __builtin_amdgcn_s_memrealtime() + (it == 0 ? (uint64_t)a.poll_delay : 0);
                const uint64_t slot = (now + ST_POLL_SYNC - 1) / ST_POLL_SYNC * ST_POLL_SYNC;
                while (__builtin_amdgcn_s_memrealtime() < slot) __builtin_amdgcn_s_sleep(1);
            }
#endif
            issue(qs);
            if constexpr (GUARD) {
                if (it == 0 && rescan_here) rescan0();   // the near-tie rescan of wave 0's rows, loads in flight
            }
            if (it > 0) {   // no memory access: runs while the loads above are in flight
                double rv;
                int64_t ri;
                lane_best(rv, ri);
                p_wave_minloc(rv, ri);
                wv = rv;
                wi = ri;
            }
#ifdef ST_PERSIST_STAMPS
            __builtin_amdgcn_s_waitcnt(0);   // diagnostic only: the poll's data has landed here
            const uint64_t tp0 = __builtin_amdgcn_s_memrealtime();
#endif
            take(qs);
#ifdef ST_PERSIST_STAMPS
            {
                const int allseen = __all(seen == need) ? 1 : 0;
                asm volatile("" ::"v"(allseen));
                proc_ticks += __builtin_amdgcn_s_memrealtime() - tp0;
            }
            {
                double sv;
                int64_t si;
                lane_best(sv, si);
                p_wave_minloc(sv, si);
                if (it == 0) {
                    spec_first = si;
#pragma unroll
                    for (int c = 0; c < MAXG / 64; ++c)
                        spec_seen0 += (unsigned)__builtin_popcountll(__builtin_amdgcn_ballot_w64((seen >> c) & 1u));
                }
                if (si != spec_prev) { spec_prev = si; spec_settle = it + 1; }
            }
#endif
            // (loading every lane's best row here when the first poll completes the sweep, before the
            // wave minloc, was measured +0.9 us per step: profiles/r04_single_poll_rowload_rejected.log)
            if (__all(seen == need)) break;
            if (!between()) break;
            __builtin_amdgcn_s_sleep(1);
        }
        ST_STAMP(a, t + 1, 1);
#ifdef ST_PERSIST_STAMPS
        if (a.stamps && lane == 0 && t + 1 >= kStampFirst && t + 1 < kStampFirst + kStampSteps) {
            uint64_t* sq = a.stamps + ((int64_t)blockIdx.x * kStampSteps + (t + 1 - kStampFirst)) * kStampPhases;
            sq[9] = it + 1;
            sq[20] = spec_seen0;
            sq[21] = spec_settle;
            sq[22] = (uint64_t)spec_first;
            sq[23] = proc_ticks;
        }
#endif
        double v;
        int64_t gi;
        lane_best(v, gi);
        int64_t my = gi;
        {   // lanes whose best beats the pre-reduced (wv, wi): none -> (wv, wi); one -> that lane's
            // (it beats every other lane's best too); several, or no earlier reduction -> full minloc
            const uint64_t bt = __builtin_amdgcn_ballot_w64(better(v, gi, wv, wi));
            if (bt == 0) {
                v = wv;
                gi = wi;
            } else if (__builtin_popcountll(bt) == 1) {
                const int L = __builtin_ctzll(bt);
                v = __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(v), L));
                gi = (int64_t)readlane_u64((uint64_t)gi, L);
            } else {
                p_wave_minloc(v, gi);
            }
        }
        ST_STAMP(a, t + 1, 7);
        if (a.nranks > 1 && ok_all) {
            // ---- rank level: push this rank's winner to every peer, gather the R winners ----
            const uint64_t seq = a.seq_base + (uint64_t)t;
            const uint64_t rtag = ((seq + 1) & 0xFFFFull) << 48;
            const int64_t mbank = (int64_t)(seq & 1) * kMaxRanks * 2;
            const uint32_t lib = gi == INT64_MAX ? 0xFFFFFFFFu : (uint32_t)gi;
            if (bid == 0 && lane == 0) {
                const uint64_t vb = (uint64_t)__double_as_longlong(v);
                const uint64_t g0 = rtag | (vb >> 16);
                const uint64_t g1 = rtag | ((vb & 0xFFFFull) << 32) | lib;
                for (int r = 0; r < a.nranks; ++r) {
                    if (r == a.rank) continue;   // every block of this rank already has it
                    uint64_t* dst = a.peer[r] + mbank + 2 * a.rank;
                    __hip_atomic_store(dst + 0, g0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(dst + 1, g1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
            // lane r < nranks owns rank r's record; lane `rank` holds the local winner already
            double rv = INFINITY;
            int64_t ri = INT64_MAX;
            bool got = lane >= a.nranks;
            if (lane == a.rank) {
                rv = v;
                ri = gi;
                got = true;
                if (ri != INT64_MAX && ri != row_of) { load_row(ri); row_of = ri; }
            }
            const uint64_t* slot = a.inbox + mbank + 2 * lane;
            const uint64_t want16 = rtag;
            const uint64_t limit = t == 0 ? kFirstRankTimeoutTicks : kTimeoutTicks;
            const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
            for (unsigned it = 0;; ++it) {
                if (!got) {
                    const uint64_t g0 = __hip_atomic_load(slot + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    const uint64_t g1 = __hip_atomic_load(slot + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    if (((g0 & 0xFFFF000000000000ull) == want16) & ((g1 & 0xFFFF000000000000ull) == want16)) {
                        got = true;
                        rv = __longlong_as_double(
                            (long long)(((g0 & 0x0000FFFFFFFFFFFFull) << 16) | ((g1 >> 32) & 0xFFFFull)));
                        const uint32_t ib = (uint32_t)g1;
                        ri = ib == 0xFFFFFFFFu ? INT64_MAX : (int64_t)ib;
                        if (ri != INT64_MAX && ri < a.n) { load_row(ri); row_of = ri; }
                    }
                }
                if (__all(got)) break;
                __builtin_amdgcn_s_sleep(1);
                if ((it & 15) == 15) {
                    const bool late = __builtin_amdgcn_s_memrealtime() - t1 > limit;
                    const bool other = __hip_atomic_load(a.status, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT) != 0;
                    if (__any(late || other)) { ok_all = 0; break; }
                }
            }
            my = ri;
            v = rv;
            gi = ri;
            p_wave_minloc(v, gi);
            // a record's index is never past n (a peer's padding sentinel is INT64_MAX)
            if (gi != INT64_MAX && gi >= a.n) ok_all = 0;
        }
        // record indices are distinct across blocks (and ranks), so exactly one lane holds the winner
        if (ok_all && my == gi && gi != INT64_MAX) {
#ifdef ST_PERSIST_STAMPS
            if (a.stamps && t + 1 >= kStampFirst && t + 1 < kStampFirst + kStampSteps)
                a.stamps[((int64_t)blockIdx.x * kStampSteps + (t + 1 - kStampFirst)) * kStampPhases + 8] =
                    row_of != gi ? 2 : 1;
#endif
            if constexpr (!kWide) {
                if (row_of != gi) load_row(gi);
#pragma unroll
                for (int k = 0; k < kRow; ++k) sc->row[k] = rowv[k];
            }
        }
        if constexpr (kWide) {   // the winner is wave-uniform now: 64 lanes fetch its 2d (+1) values
            int fast = 1;
            if (ok_all && gi != INT64_MAX) {
                constexpr int kWRow = 2 * D + (GF ? 1 : 0);
                for (int k = lane; k < kWRow; k += 64) {
                    const double v = k < D ? a.x[(int64_t)k * a.ld + gi]
                                           : (k < 2 * D ? a.g[(int64_t)(k - D) * a.ld + gi] : a.w[gi]);
                    sc->row[k] = v;
                    if (k < 2 * D) fast &= fast_range_ok(v);
                }
            }
            fast = __all(fast);
            if (lane == 0) sc->rowfast = fast;
        }
        if (lane == 0) {
            // (max: a compact-only kernel's "needs the exact arithmetic" (2) is not overwritten)
            if (!ok_all) __hip_atomic_fetch_max(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sc->abort = !ok_all;
            sc->win = gi;
            if constexpr (GUARD) {
                if (guard) {
                    gsc->win_i[t & 1] = gi == INT64_MAX ? 0xFFFFFFFFu : (uint32_t)gi;
                    gsc->win_v[t & 1] = v;
                }
            }
        }
    }
    __syncthreads();
    ST_STAMP(a, t + 1, 2);
    if (sc->abort) return -1;
    return sc->win;
}

// BPC = blocks per CU: 2 puts two 256-thread blocks on each CU (two waves per SIMD, RT <= 8
// register rows each, every block its own record): the fp64 pipe issues from two waves.
// CMP: the compact arithmetic for pairs in range (stein_math.hpp pair_compact_ct; st_tune key 11).
// GEN = false (with CMP): the compact-only kernel -- no exact / mixed sweep compiled in, which frees
// the registers those paths need for more register rows.  A step that would need them (a block row
// or the winner out of range, a NaN running sum) sets status 2 and every block leaves; the general
// kernel, enqueued right behind it with gate = that status word, then runs the whole thin (and
// returns at once when the compact-only run completed).  One device only.
//
// KA = BatchArgs: the batch launch (st_greedy_batch) -- independent thins in ONE launch, problem q
// on the blocks [blk_begin[q], blk_begin[q + 1]), each group running exactly as a plain launch of
// that many blocks would: its own records, status word and indices; the groups never read each
// other's memory.  The thins then run side by side whatever hardware queues streams would map to.
// (The body stays in the kernel itself: moved into a device function, the compact-only kernel
// spilled 22 VGPRs instead of 8.)
constexpr int kMaxBatch = kMaxBatchProblems;
struct BatchArgs {
    PersistArgs p[kMaxBatch];
    int blk_begin[kMaxBatch + 1];
    int count;
};
static_assert(sizeof(BatchArgs) <= 4096, "kernel arguments are limited to 4 KB");

//
// GUARD (compact kernels, one device; compiled in persistent_guard.hip): the near-tie guard above
// tie_check.  GUARD = false instantiations carry none of it.
template <int D, bool GF, int RT, int NT, int BPC, bool CMP, bool GEN = true, typename KA = PersistArgs,
          bool GUARD = false>
__global__ __launch_bounds__(NT, BPC) void greedy_persistent(KA ka) {
    constexpr bool kBatch = std::is_same<KA, BatchArgs>::value;
    int grp = 0;   // the block's group
    if constexpr (kBatch)
        for (int k = 1; k < ka.count; ++k) grp += (int)blockIdx.x >= ka.blk_begin[k];
    const PersistArgs& a = [&]() -> const PersistArgs& {
        if constexpr (kBatch) return ka.p[grp]; else return ka;
    }();
    // the block's place in its group and the group's size (plain launch: the builtins)
    auto bid = [&]() -> unsigned {
        if constexpr (kBatch) return blockIdx.x - (unsigned)ka.blk_begin[grp]; else return blockIdx.x;
    };
    auto G = [&]() -> int {
        if constexpr (kBatch) return ka.blk_begin[grp + 1] - ka.blk_begin[grp]; else return (int)gridDim.x;
    };
    static_assert(!CMP || D <= kMaxCtDim, "compact arithmetic: d <= 8 only");
    static_assert(GEN || CMP, "the compact-only kernel is a compact kernel");
    if (a.gate && *a.gate != 2u) return;   // general kernel behind a compact-only run that finished
    constexpr int kPBlock = NT;
    constexpr int kMaxG = 256 * BPC;     // records swept per step
    constexpr bool kTwoWaves = NT >= 512 || BPC > 1;   // two waves per SIMD
    constexpr bool kWide = D > kMaxCtDim;              // register rows only (host guarantees it)
    // one 512-thread block per CU: the LDS and streamed rows are dealt to the waves in 64-row
    // chunks from a block counter, so the waves the SIMD arbiter favours take more of them and
    // all eight finish together (a static split leaves the younger wave of each SIMD running
    // alone for ~3 us of every step: profiles/r01_stamps_nt512_rt8_rt6_n2e6.log)
    constexpr bool kDyn = NT >= 512 && BPC == 1 && !kWide;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    Scratch* sc = reinterpret_cast<Scratch*>(lds);
    const int RL = a.RL;
    // LDS rows, chunk-major: 64-row chunks of kLF fields (x[D], g[D], A[, w]) x 64 doubles, so a
    // row's fields lie 64 doubles apart -- one address per row, the fields at immediate offsets
    // (ds_read2st64_b64 pairs them) instead of a runtime-stride address per coordinate
    constexpr int kLF = 2 * D + 1 + (GF ? 1 : 0);
    GuardScratch* const gsc = reinterpret_cast<GuardScratch*>(lds + (sizeof(Scratch) + 15) / 16 * 2);
    // the per-thread slots of the 256-thread guarded kernels (GuardLanes), after GuardScratch
    constexpr bool kLanes = GUARD && !kDyn && !kWide;
    // wave 0 rescans its register rows while its first poll is in flight (the 256-thread kernels), or right
    // after the pick (512 threads; ST_LANES_W0_IN_POLL = 0: the 256-thread kernels too -- measurement builds)
    constexpr bool kW0InPoll = !kDyn && ST_LANES_W0_IN_POLL;
    GuardLanes* const gl = reinterpret_cast<GuardLanes*>(lds + (sizeof(Scratch) + 15) / 16 * 2 +
                                                         (sizeof(GuardScratch) + 15) / 16 * 2);
    double* const srow0 = lds + (sizeof(Scratch) + 15) / 16 * 2 + (GUARD ? (sizeof(GuardScratch) + 15) / 16 * 2 : 0) +
                          (kLanes ? (sizeof(GuardLanes) + 15) / 16 * 2 : 0);
    auto lrow = [&](int e) -> double* { return srow0 + (e >> 6) * (kLF * 64) + (e & 63); };
    constexpr int fX = 0, fG = D * 64, fA = 2 * D * 64, fW = (2 * D + 1) * 64;   // field offsets
    // 512-thread kernels with st_tune key 15 = 1: the streamed rows' running sums live in LDS too,
    // after the LDS rows (one double per streamed row, whole 64-row chunks), so a streamed row is
    // read-only L2 traffic -- no per-step load and store of A (measured slower: see key 15)
    double* const sA = srow0 + (int64_t)(RL >> 6) * (kLF * 64);
    const int tid = threadIdx.x;
    const int64_t ld = a.ld;
    const int64_t r0 = a.row_begin + (int64_t)bid() * a.rows_per_block;
    const int64_t r1 = (r0 + a.rows_per_block < a.row_end) ? r0 + a.rows_per_block : a.row_end;
    const int64_t lds_base = r0 + (int64_t)RT * kPBlock;
    const int64_t str_base = lds_base + RL;
    const double l = a.l, l2 = a.l * a.l, m3l2 = -3.0 * l2, tr = a.tr;
    const int lok = CMP ? scale_in_range(l, tr) : 0;   // compact: the per-problem part of the rule
    // near-tie guard (GUARD kernels, launched only with a.tie_bounds set; module comment above tie_check).
    // Compile-time, and its wave conditions on the wave index in an SGPR (scalar branches): runtime
    // flags and per-lane masks here cost SGPRs that spill into VGPR lanes on the exchange's path
    constexpr bool guard = GUARD && CMP && !kWide;
    const int wid = __builtin_amdgcn_readfirstlane((int)tid >> 6);
    if constexpr (guard) {
        if (tid == 0) {
            gsc->tied = 0;
            if (bid() == 0) a.tie[3] = 1u;   // a guarded run (st_greedy_near_tie)
        }
    }

    // ---- stage the block's rows on chip ----------------------------------------------------
    // and decide whether every row of the block admits the range-guarded fast pair arithmetic
    // (stein_math.hpp fast_range_ok; padding rows are zeros)
    // wide d: x in registers, g in LDS (sgw[k][NT], where the LDS rows would start: RL = 0)
    double xr[RT > 0 ? RT : 1][D], gr[RT > 0 ? RT : 1][kWide ? 1 : D], ar[RT > 0 ? RT : 1];
    double* sgw = srow0;
    double wr[(GF && RT > 0) ? RT : 1];
    int rok = scale_in_range(l, tr);
#pragma unroll
    for (int q = 0; q < RT; ++q) {
        const int64_t row = r0 + (int64_t)q * kPBlock + tid;
        const bool ok = row < r1;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            xr[q][k] = ok ? a.x[k * ld + row] : 0.0;
            const double gv = ok ? a.g[k * ld + row] : 0.0;
            if constexpr (kWide) sgw[k * kPBlock + tid] = gv;
            else gr[q][k] = gv;
            rok &= fast_range_ok(xr[q][k]) & fast_range_ok(gv);
        }
        if constexpr (GF) wr[q] = ok ? a.w[row] : 0.0;
    }
    if constexpr (!kWide) {
        for (int e = tid; e < RL; e += kPBlock) {
            const int64_t row = lds_base + e;
            const bool ok = row < r1;
#pragma unroll
            for (int k = 0; k < D; ++k) {
                const double xv = ok ? a.x[k * ld + row] : 0.0, gv = ok ? a.g[k * ld + row] : 0.0;
                lrow(e)[fX + k * 64] = xv;
                lrow(e)[fG + k * 64] = gv;
                rok &= fast_range_ok(xv) & fast_range_ok(gv);
            }
            if constexpr (GF) lrow(e)[fW] = ok ? a.w[row] : 0.0;
        }
        for (int64_t row = str_base + tid; row < r1; row += kPBlock) {
#pragma unroll
            for (int k = 0; k < D; ++k) rok &= fast_range_ok(a.x[k * ld + row]) & fast_range_ok(a.g[k * ld + row]);
        }
    }
    if constexpr (GUARD && !kWide) {
        // the problem's bounds for the guard's threshold (stein_ref.c sr_tie_bounds): max_i of
        // g_i0 g_i0 + g_i1 g_i1 + ... and of w_i w_i over this block's rows, a NaN as +inf, merged into the
        // block's bounds slot (bounds_slot) with u64 atomic maxima that complete before any record of this
        // block is published (the fence) -- so a block that has seen every step-0 record sees the final bounds
        {
            double gm = 0.0, wm = GF ? 0.0 : 1.0;
            auto take_row = [&](double s2, double wv) {
                gm = __builtin_fmax(gm, __builtin_isnan(s2) ? INFINITY : s2);
                if constexpr (GF) wm = __builtin_fmax(wm, __builtin_isnan(wv * wv) ? INFINITY : wv * wv);
            };
#pragma unroll
            for (int q = 0; q < RT; ++q) {
                if (r0 + (int64_t)q * kPBlock + tid < r1) {
                    double s2 = gr[q][0] * gr[q][0];
#pragma unroll
                    for (int k = 1; k < D; ++k) s2 = s2 + gr[q][k] * gr[q][k];
                    take_row(s2, GF ? wr[q] : 1.0);
                }
            }
            for (int e = tid; e < RL; e += kPBlock) {
                if (lds_base + e < r1) {
                    double s2 = lrow(e)[fG] * lrow(e)[fG];
#pragma unroll
                    for (int k = 1; k < D; ++k) s2 = s2 + lrow(e)[fG + k * 64] * lrow(e)[fG + k * 64];
                    take_row(s2, GF ? lrow(e)[fW] : 1.0);
                }
            }
            for (int64_t row = str_base + tid; row < r1; row += kPBlock) {
                double s2 = a.g[row] * a.g[row];
#pragma unroll
                for (int k = 1; k < D; ++k) s2 = s2 + a.g[k * ld + row] * a.g[k * ld + row];
                take_row(s2, GF ? a.w[row] : 1.0);
            }
            gm = wave_max_f64(gm);
            wm = wave_max_f64(wm);
            if ((tid & 63) == 0) {
                gsc->bnd[tid >> 6][0] = gm;
                gsc->bnd[tid >> 6][1] = wm;
            }
        }
    }
    if (tid == 0) { sc->ctr[0] = 0; sc->ctr[1] = 0; }
    const int block_fast = __syncthreads_and(rok);
    if constexpr (GUARD && !kWide) {
        // one atomic pair per block; their latency overlaps step 0's diagonal, and the release fence
        // in front of publish(0) orders them before this block's step-0 record (written by wave 0)
        if (tid == 0) {
            double gm = gsc->bnd[0][0], wm = gsc->bnd[0][1];
            for (int w = 1; w < NT / 64; ++w) {
                gm = __builtin_fmax(gm, gsc->bnd[w][0]);
                wm = __builtin_fmax(wm, gsc->bnd[w][1]);
            }
            uint64_t* bw = reinterpret_cast<uint64_t*>(const_cast<double*>(a.tie_bounds));
#if ST_BOUNDS_SLOTS
            bw = bounds_slot(a, (int)(bid() % ST_BOUNDS_SLOTS));
#endif
            __hip_atomic_fetch_max(bw, (uint64_t)__double_as_longlong(gm), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_max(bw + 1, (uint64_t)__double_as_longlong(wm), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    }

    // near-tie guard: the block's rows that repeat their predecessor row bit for bit (x, g, w) -- a rejected
    // MCMC proposal.  Such a row has its run's first row's sum at every step, so a tie it shows with the
    // block's minimum is either with a duplicate of that minimum or a repeat of a tie its run's first row
    // already counts: the rescans skip it (no duplicate test).  Register rows: bit q of rrep; LDS rows: bit e
    // of GuardScratch::lrep; streamed rows are tested when they tie (rescan_rest)
    uint32_t rrep = 0;
    if constexpr (guard) {
#pragma unroll
        for (int q = 0; q < RT; ++q) {
            const int64_t row = r0 + (int64_t)q * kPBlock + tid;
            if (row < r1 && row > 0) {
                bool same = true;
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    same &= same_bits(a.x[k * ld + row - 1], xr[q][k]);
                    same &= same_bits(a.g[k * ld + row - 1], gr[q][k]);
                }
                if constexpr (GF) same &= same_bits(a.w[row - 1], wr[q]);
                rrep |= same ? 1u << q : 0u;
            }
        }
        for (int e = tid; e < RL; e += kPBlock) {   // RL: whole 64-row chunks, so whole waves
            const int64_t row = lds_base + e;
            bool same = false;
            if (row < r1 && row > 0) {
                same = true;
#pragma unroll
                for (int k = 0; k < D; ++k) {
                    same &= same_bits(a.x[k * ld + row - 1], lrow(e)[fX + k * 64]);
                    same &= same_bits(a.g[k * ld + row - 1], lrow(e)[fG + k * 64]);
                }
                if constexpr (GF) same &= same_bits(a.w[row - 1], lrow(e)[fW]);
            }
            const uint64_t bal = __ballot(same);
            if ((tid & 63) == 0) {
                gsc->lrep[(e >> 5)] = (uint32_t)bal;
                gsc->lrep[(e >> 5) + 1] = (uint32_t)(bal >> 32);
            }
        }
        // (visible to the rescans: they run after publish(0)'s barrier)
    }

    // ---- step 0: diagonal --------------------------------------------------------------------
    // running best of this thread: starts at its first row (register row 0, which precedes all its
    // other rows); an out-of-range row contributes +inf with its (>= n) index and never wins
    double bv = INFINITY;
    uint32_t bi = (uint32_t)(r0 + tid);
#pragma unroll
    for (int q = 0; q < RT; ++q) {
        const int64_t row = r0 + (int64_t)q * kPBlock + tid;
        double kv;
        if constexpr (kWide) {
            double gt[D];
#pragma unroll
            for (int k = 0; k < D; ++k) gt[k] = sgw[k * kPBlock + tid];
            kv = diag_value_ct<D>(gt, tr);
        } else if constexpr (CMP) {
            kv = diag_value_sel<D>(lok && row_in_range<D>(xr[q], gr[q]), gr[q], tr);
        } else {
            kv = diag_value_ct<D>(gr[q], tr);
        }
        if constexpr (GF) kv = (kv * wr[q]) * wr[q];
        ar[q] = row < r1 ? kv : INFINITY;   // padding rows hold +inf for the whole run
        if (q == 0) { bv = ar[q]; bi = (uint32_t)row; } else scan_take(ar[q], (uint32_t)row, bv, bi);
    }
    if constexpr (!kWide) {
        for (int e = tid; e < RL; e += kPBlock) {
            const int64_t row = lds_base + e;
            double gi[D], xi[D];
#pragma unroll
            for (int k = 0; k < D; ++k) { gi[k] = lrow(e)[fG + k * 64]; xi[k] = lrow(e)[fX + k * 64]; }
            double kv = CMP ? diag_value_sel<D>(lok && row_in_range<D>(xi, gi), gi, tr) : diag_value_ct<D>(gi, tr);
            if constexpr (GF) kv = (kv * lrow(e)[fW]) * lrow(e)[fW];
            kv = row < r1 ? kv : INFINITY;
            lrow(e)[fA] = kv;
            scan_take(kv, (uint32_t)row, bv, bi);
        }
        for (int64_t row = str_base + tid; row < r1; row += kPBlock) {
            double gi[D], xi[D];
#pragma unroll
            for (int k = 0; k < D; ++k) { gi[k] = a.g[k * ld + row]; xi[k] = a.x[k * ld + row]; }
            double kv = CMP ? diag_value_sel<D>(lok && row_in_range<D>(xi, gi), gi, tr) : diag_value_ct<D>(gi, tr);
            if constexpr (GF) kv = (kv * a.w[row]) * a.w[row];
            if (kDyn && a.stream_a_lds) sA[row - str_base] = kv;
            else a.A[row] = kv;
            scan_take(kv, (uint32_t)row, bv, bi);
        }
    }
    if constexpr (GUARD) {
        if (wid == 0) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");   // the bounds (above)
    }
    publish<NT, GUARD>(a, sc, bv, bi, 0, r1, bid(), gsc);

    // near-tie guard: the rescans of the block's running sums after each publish (module comment above
    // tie_check).  Wave 0: its register rows (inside wait_and_pick, while its first poll is in flight; the
    // 512-thread kernels at the start of the next step), the duplicate test of its tied rows left to the
    // wave that reduces them; the other waves: their register rows and, dealt statically over their
    // threads, the LDS and streamed rows, duplicate test included.
    constexpr int kNW = NT / 64;
    // register rows: "other" and the mask of the rows whose sum equals vmin (other than ibk).  No row test:
    // padding rows hold +inf, which changes neither (a tie at +inf would contribute +inf: ignored)
    auto rescan_regs = [&](double vmin, uint32_t ibk, double& o, uint32_t& msk) {
        const uint32_t row0 = (uint32_t)(r0 + tid);
        const bool fin = vmin < INFINITY;
#pragma unroll
        for (int q = 0; q < RT; ++q) {
            o = __builtin_fmin(o, other_of(ar[q], vmin));
            msk |= ((ar[q] == vmin) & fin & (row0 + (uint32_t)(q * kPBlock) != ibk) & !((rrep >> q) & 1u)) ? 1u << q
                                                                                                      : 0u;
        }
    };
    // the LDS and streamed rows' rescan is dealt over waves kRW0 .. kNW - 1: with three or more waves wave 1
    // keeps only its register rows, so its chain after the publish -- reduce_w0 / tie_check, then its rows --
    // issues no global load unless a tie needs the duplicate test
    constexpr int kRW0 = kNW >= 3 ? ST_GUARD_RW0 : 1;
    auto rescan_rest = [&](int64_t tt) {   // waves 1 .. kNW - 1, right after publish(tt)
        // the block's minimum and its row, combined from the wave minima publish(tt) left in Scratch (wave 0
        // writes blk_v / blk_i only after publish's barrier)
        uint64_t kmin;
        uint32_t ibk;
        combine_waves<NT>(sc, kmin, ibk);
        const double vmin = key_value(kmin);
        const bool fin = vmin < INFINITY;
        double o = INFINITY;
        uint32_t msk = 0, smsk = 0;   // tied register rows; tied streamed rows by this thread's visit number
        bool tie = false;             // a tied LDS row, or a tied streamed row past visit 31
        const int rt0 = tid - 64 * kRW0, rstep = kPBlock - 64 * kRW0;
        if constexpr (!kWide) {
            if (wid >= kRW0) {
                int j = 0;
                ST_GUARD_UNROLL_LOOP
                for (int64_t row = str_base + rt0; row < r1; row += rstep, ++j) {
                    const double av = (kDyn && a.stream_a_lds) ? sA[row - str_base] : a.A[row];
                    o = __builtin_fmin(o, other_of(av, vmin));
                    const bool tj = av == vmin && fin && (uint32_t)row != ibk;
                    if (j < 32) smsk |= tj ? 1u << j : 0u;
                    else tie |= tj;
                }
                ST_GUARD_UNROLL_LOOP
                for (int e = rt0; e < RL; e += rstep) {
                    const double av = lrow(e)[fA];
                    if (lds_base + e < r1) {
                        o = __builtin_fmin(o, other_of(av, vmin));
                        tie |= av == vmin && fin && (uint32_t)(lds_base + e) != ibk &&
                               !((gsc->lrep[e >> 5] >> (e & 31)) & 1u);
                    }
                }
            }
        }
        rescan_regs(vmin, ibk, o, msk);
        if (__any(msk != 0 || smsk != 0 || tie)) {   // rows tied with the block's minimum: duplicates of row ibk?
            RowBits<D, GF> b;
            b.load(a, (int64_t)ibk < a.n ? (int64_t)ibk : 0);
            if constexpr (!kWide) {
                if (wid >= kRW0) {
                    int j = 0;
                    for (int64_t row = str_base + rt0; row < r1; row += rstep, ++j) {
                        bool tj;
                        if (j < 32) {
                            tj = (smsk >> j) & 1u;
                        } else {
                            const double av = (kDyn && a.stream_a_lds) ? sA[row - str_base] : a.A[row];
                            tj = av == vmin && fin && (uint32_t)row != ibk;
                        }
                        if (tj) {   // (a repeat of its predecessor row counts nothing new: see rrep)
                            RowBits<D, GF> r, p;
                            r.load(a, row);
                            p.load(a, row > 0 ? row - 1 : row);
                            if (!(row > 0 && rows_equal(r, p)) && !rows_equal(r, b)) o = __builtin_fmin(o, vmin);
                        }
                    }
                    for (int e = rt0; e < RL; e += rstep) {
                        const int64_t row = lds_base + e;
                        const double* rp = lrow(e);
                        if (row < r1 && rp[fA] == vmin && fin && (uint32_t)row != ibk &&
                            !((gsc->lrep[e >> 5] >> (e & 31)) & 1u)) {
                            bool same = true;
#pragma unroll
                            for (int k = 0; k < D; ++k) {
                                same &= same_bits(rp[fX + k * 64], b.v[k]);
                                same &= same_bits(rp[fG + k * 64], b.v[D + k]);
                            }
                            if constexpr (GF) same &= same_bits(rp[fW], b.v[2 * D]);
                            if (!same) o = __builtin_fmin(o, vmin);
                        }
                    }
                }
            }
#pragma unroll
            for (int q = 0; q < RT; ++q) {
                if ((msk >> q) & 1u) {
                    bool same = true;
#pragma unroll
                    for (int k = 0; k < D; ++k) {
                        same &= same_bits(xr[q][k], b.v[k]);
                        same &= same_bits(gr[q][k], b.v[D + k]);
                    }
                    if constexpr (GF) same &= same_bits(wr[q], b.v[2 * D]);
                    if (!same) o = __builtin_fmin(o, vmin);
                }
            }
        }
        const int par = (int)(tt & 1);
        if constexpr (kLanes) {   // per thread, reduced only where tie_check needs it (tie_check_lanes)
            gl->o[par][tid] = o;
            gl->m[par][tid] = 0u;
        } else {
            o = wave_min_f64(o);
            if ((tid & 63) == 0) gsc->rs_o[par][wid] = o;
        }
        ST_STAMP_WAVE(a, tt, 24);   // diagnostic build: this wave's rescan of step tt done (phase 24 + wave)
    };
    // wave 0's own rescan leaves its lanes' "other" and tied-row masks in LDS; the duplicate test and the
    // reduction follow after the next publish (wave 1: reduce_w0; the 256-thread kernels: tie_check_lanes)
    int64_t t = 1;   // the step loop's counter (rescan_w0 files by the parity of step t - 1)
    auto rescan_w0 = [&]() {   // the sums of step t - 1; blk_v / blk_i were written by this wave's lane 0
        const int par = (int)((t - 1) & 1);
        double o = INFINITY;
        uint32_t msk = 0;
        rescan_regs(gsc->blk_v[par], gsc->blk_i[par], o, msk);
        if constexpr (kLanes) {   // inside wait_and_pick(t - 1)
            gl->o[par][tid] = o;
            gl->m[par][tid] = msk;
        } else {
            gsc->w0_o[tid] = o;
            gsc->w0_m[tid] = msk;
        }
    };
    auto reduce_w0 = [&](int64_t tt) {   // wave 1: wave 0's lanes of step tt
        const int par = (int)(tt & 1);
        const int lane = tid - 64;
        double o = gsc->w0_o[lane];
        const uint32_t msk = gsc->w0_m[lane];
        if (__any(msk != 0)) {
            const uint32_t ibk = gsc->blk_i[par];
            RowBits<D, GF> b;
            b.load(a, (int64_t)ibk < a.n ? (int64_t)ibk : 0);
            o = finish_mask<D, GF, NT>(a, o, msk, lane, r0, gsc->blk_v[par], b);
        }
        o = wave_min_f64(o);
        if (lane == 0) gsc->rs_o[par][0] = o;
    };
    if constexpr (guard) {
        if (wid >= 1) rescan_rest(0);
    }

    // ---- steps 1 .. m-1 ----------------------------------------------------------------------
    for (; t < a.m; ++t) {
        const int64_t win = wait_and_pick<D, GF, kMaxG, GUARD>(a, sc, t - 1, bid(), G(), gsc, guard,
                                                               guard && kW0InPoll, rescan_w0);
        if (win < 0) break;
        if constexpr (guard && !kW0InPoll) {   // wave 0's register rows of step t - 1: per lane into LDS (wave 1
            if (wid == 0) rescan_w0();         // reduces them after publish(t))
        }
        if (bid() == 0 && tid == 0) a.idx_out[t - 1] = (uint32_t)win;
        // chunk counter of the NEXT step (its last use, step t - 1, ended before publish's barrier)
        if (kDyn && tid == 0) sc->ctr[(t + 1) & 1] = 0;
        // small d: the winner row in SGPRs (VALU fp64 ops take one scalar operand); wide d: read
        // from LDS inside the pair loop (block-uniform broadcast reads)
        double xj_r[kWide ? 1 : D], gj_r[kWide ? 1 : D];
        const double* xj = kWide ? sc->row : xj_r;
        const double* gj = kWide ? sc->row + D : gj_r;
        // fast variant: range-guarded arithmetic (block rows and winner row in range) and a
        // NaN-free scan -- valid while no A of this block is NaN: the block's last minimum is NaN
        // iff one is, and fast steps keep finite sums finite (|2k| < 2^191 per step)
        int wfast = (block_fast != 0) & (int)!__builtin_isnan(sc->vblk);
        int jok = lok;   // compact, mixed sweep: l, tr and the winner row in range
        if constexpr (kWide) {
            wfast &= sc->rowfast;   // checked by the wave that fetched the row (no 2d reloads here)
        } else {
            int rowok = 1;
#pragma unroll
            for (int k = 0; k < D; ++k) {
                xj_r[k] = uniform(sc->row[k]);
                gj_r[k] = uniform(sc->row[D + k]);
                rowok &= fast_range_ok(xj[k]) & fast_range_ok(gj[k]);
            }
            wfast &= rowok;
            jok &= rowok;
        }
        const double wj = GF ? uniform(sc->row[2 * D]) : 1.0;
        // one block-uniform choice per step: range-guarded fast arithmetic or the general one
        auto sweep_rows = [&](auto ar_tag) {
            constexpr int AR = decltype(ar_tag)::value;
            constexpr bool FAST = AR == 1 || AR == 2;   // in range, NaN-free block: fma update, '<' scan
            // opaque marker: keeps LLVM from if-converting the two variants into
            // compute-both-and-select (both are pure arithmetic over the register rows)
            asm volatile(";; sweep_rows variant" ::);
            if constexpr (kWide) {   // register rows only (x in VGPRs, g in LDS)
                uint32_t bq = 0;
#pragma unroll
                for (int q = 0; q < RT; ++q) {
                    const int64_t row = r0 + (int64_t)q * kPBlock + tid;
                    double kv = pair_value_wide<D, FAST>(xr[q], sgw + tid, kPBlock, xj, gj, l, l2, tr);
                    if constexpr (GF) kv = (kv * wr[q]) * wj;
                    if constexpr (FAST) ar[q] = add_twice<true>(ar[q], kv);
                    else ar[q] = row < r1 ? add_twice<false>(ar[q], kv) : INFINITY;
                    if (q == 0) { bv = ar[q]; bq = 0; } else scan_take_v<FAST>(ar[q], (uint32_t)q, bv, bq);
                }
                bi = (uint32_t)(r0 + tid) + bq * (uint32_t)kPBlock;
                ST_STAMP_AFTER(a, t, 5, bv);
            } else {
            // streamed rows go two at a time; the first pair's loads are issued now and land while
            // the on-chip rows compute.  Addresses of rows past r1 are clamped to r0 (a valid row
            // of this block): their loads are harmless and their results are dropped.
            struct SRow { double x[D], g[D], a, w; };
            auto fetch = [&](int64_t row, SRow& r) {
                const int64_t rr = row < r1 ? row : r0;
#pragma unroll
                for (int k = 0; k < D; ++k) { r.x[k] = a.x[k * ld + rr]; r.g[k] = a.g[k * ld + rr]; }
                r.a = a.A[rr];
                r.w = GF ? a.w[rr] : 1.0;
            };
            // (with two waves per SIMD the registers are too tight to carry the prefetched pair
            // through the on-chip rows: the 512-thread variant issues it after them)
            constexpr bool kEarlyStream = !kTwoWaves && !kDyn;
            int64_t srow = str_base + tid;
            // opaque per step: otherwise LICM hoists the ~20 64-bit load addresses of the first
            // streamed pair out of the step loop and they end up spilled to scratch
            asm volatile("" : "+v"(srow));
            SRow c0, c1;
            if (kEarlyStream && srow < r1) { fetch(srow, c0); fetch(srow + kPBlock, c1); }
            // register rows: track the slot q (a constant) and convert it to the row once
            uint32_t bq = 0;
#pragma unroll
            for (int q = 0; q < RT; ++q) {
                const int64_t row = r0 + (int64_t)q * kPBlock + tid;
                double kv = pair_ar<D, AR>(xr[q], gr[q], xj, gj, l, l2, m3l2, tr, jok);
                if constexpr (GF) kv = (kv * wr[q]) * wj;
                // padding rows (zeros) keep A = +inf: in the fast range k is finite, so
                // inf + 2k = inf needs no mask; the general path masks the update instead
                if constexpr (FAST) ar[q] = add_twice<true>(ar[q], kv);
                else ar[q] = row < r1 ? add_twice<false>(ar[q], kv) : INFINITY;
                (void)row;
                if (q == 0) { bv = ar[q]; bq = 0; } else scan_take_v<FAST>(ar[q], (uint32_t)q, bv, bq);
                // two waves per SIMD hide latency by themselves: cap the scheduler's interleaving
                // of independent rows (it costs registers the 512-thread variant does not have)
                if constexpr (kTwoWaves) {
                    if ((q & 1) == 1) __builtin_amdgcn_sched_barrier(0);
                }
            }
            bi = (uint32_t)(r0 + tid) + bq * (uint32_t)kPBlock;
            ST_STAMP_AFTER(a, t, 5, bv);
            // LDS rows, UL per iteration: independent dependency chains for the scheduler
            // (one wave per SIMD: a single chain leaves the fp64 pipe idle between dependent ops).
            // RL is a multiple of 64, so the trip counts are wave-uniform.
            auto lds_pair = [&](int e) -> double {
                const int64_t row = lds_base + e;
                double xi[D], gi[D];
                double* const rp = lrow(e);
#pragma unroll
                for (int k = 0; k < D; ++k) { xi[k] = rp[fX + k * 64]; gi[k] = rp[fG + k * 64]; }
                double kv = pair_ar<D, AR>(xi, gi, xj, gj, l, l2, m3l2, tr, jok);
                if constexpr (GF) kv = (kv * rp[fW]) * wj;
                double av;
                if constexpr (FAST) av = add_twice<true>(rp[fA], kv);
                else av = row < r1 ? add_twice<false>(rp[fA], kv) : INFINITY;
                rp[fA] = av;
                return av;
            };
            // streamed rows: two per iteration, the next two rows' loads in flight meanwhile
            auto stream_pair = [&](const SRow& r) -> double {
                double kv = pair_ar<D, AR>(r.x, r.g, xj, gj, l, l2, m3l2, tr, jok);
                if constexpr (GF) kv = (kv * r.w) * wj;
                return add_twice<FAST>(r.a, kv);
            };
            if constexpr (kDyn) {
                // chunk c < nS: streamed rows [str_base + 64c, +64); c >= nS: LDS rows
                // [64(c - nS), +64).  Streamed chunks go first: the waves the arbiter favours reach
                // them while the others still compute register rows, which hides the HBM latency.
                // A thread's chunk rows are not visited in index order, so their scan compares
                // indices on ties (scan_take_idx); all of them follow the register rows.
                const int lane = tid & 63;
                const int nL = RL >> 6;
                const int64_t ns = r1 - str_base;
                const int nS = ns > 0 ? (int)((ns + 63) >> 6) : 0;
                const int nC = nS + nL;
                int* ctr = &sc->ctr[t & 1];
                auto grab = [&]() -> int {
                    int c = 0;
                    if (lane == 0)
                        c = __hip_atomic_fetch_add(ctr, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    return __builtin_amdgcn_readfirstlane(c);
                };
                // streamed rows through descriptors based at str_base: ONE 32-bit lane offset per
                // row, the column offsets k * ld * 8 as SGPR operands (no 64-bit address per
                // coordinate; the host keeps (d - 1) * ld * 8 + rows * 8 below 2^31).  Rows past r1
                // read row str_base (their results are dropped).
                const auto xrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(a.x + str_base), 0,
                                                                   0x7FFFFFFF, 0x00020000);
                const auto grs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(a.g + str_base), 0,
                                                                   0x7FFFFFFF, 0x00020000);
                const auto wrs = __builtin_amdgcn_make_buffer_rsrc(
                    const_cast<double*>(GF ? a.w + str_base : a.x), 0, 0x7FFFFFFF, 0x00020000);
                // SAL: the streamed rows' sums in LDS (sA; the host's choice whenever they fit next to
                // the LDS rows) -- else in HBM through a descriptor that ends at r1.  Branch-free
                // tail handling either way, so the two streamed chunks of an iteration stay in one
                // basic block with all their loads issued up front: rows past r1 (the last chunk's
                // tail) keep their garbage sum in the chunk's unused LDS slots or store past the
                // descriptor's range (dropped), and scan as +inf with the largest index
                auto chunk_loop = [&](auto sal_tag) {
                    constexpr bool SAL = decltype(sal_tag)::value;
                    const auto arsrc = __builtin_amdgcn_make_buffer_rsrc(
                        a.A + str_base, 0, (!SAL && ns > 0) ? (int)(ns * 8) : 0, 0x00020000);
                    auto fetch = [&](int64_t row, SRow& r) {
                        const int off = row < r1 ? (int)((row - str_base) * 8) : 0;
#pragma unroll
                        for (int k = 0; k < D; ++k) {
                            r.x[k] = buf_load_f64(xrs, off, (int)(k * ld * 8));
                            r.g[k] = buf_load_f64(grs, off, (int)(k * ld * 8));
                        }
                        if constexpr (SAL) r.a = sA[row - str_base];
                        else r.a = buf_load_f64(arsrc, off, 0);
                        r.w = GF ? buf_load_f64(wrs, off, 0) : 1.0;
                    };
                    auto take_stream = [&](int64_t row, double av) {
                        const bool in = row < r1;
                        if constexpr (SAL) {
                            sA[row - str_base] = av;
                        } else {
                            typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                            const uint64_t ab = (uint64_t)__double_as_longlong(av);
                            __builtin_amdgcn_raw_buffer_store_b64(u32x2{(unsigned)ab, (unsigned)(ab >> 32)}, arsrc,
                                                                  in ? (int)((row - str_base) * 8) : (int)(ns * 8), 0, 0);
                        }
                        scan_take_idx<FAST>(in ? av : INFINITY, in ? (uint32_t)row : 0xFFFFFFFFu, bv, bi);
                    };
                    auto one_chunk = [&](int c) {
                        if (c < nS) {
                            const int64_t s0 = str_base + ((int64_t)c << 6) + lane;
                            SRow ra;
                            fetch(s0, ra);
                            take_stream(s0, stream_pair(ra));
                        } else {
                            const int e0 = ((c - nS) << 6) + lane;
                            scan_take_idx<FAST>(lds_pair(e0), (uint32_t)(lds_base + e0), bv, bi);
                        }
                    };
                    for (int c = grab(); c < nC; c = grab()) {
                        if (c + 1 < nS) {            // two streamed chunks: both loads in flight
                            const int64_t s0 = str_base + ((int64_t)c << 6) + lane, s1 = s0 + 64;
                            SRow ra, rb;
                            fetch(s0, ra);
                            fetch(s1, rb);
                            const double av0 = stream_pair(ra), av1 = stream_pair(rb);
                            take_stream(s0, av0);
                            take_stream(s1, av1);
                        } else if (c >= nS && c + 1 < nC) {   // two LDS chunks: two chains
                            const int e0 = ((c - nS) << 6) + lane, e1 = e0 + 64;
                            double av0, av1;
                            if (a.lds_two_chains) {
                                // both rows' fields (running sums included) read up front, then two
                                // independent chains with no LDS access between them, then both
                                // stores: the scheduler can interleave the chains (lds_pair's store
                                // of the first row's sum kept the second row's reads behind it)
                                double* const rp0 = lrow(e0);
                                double* const rp1 = lrow(e1);
                                SRow ra, rb;
#pragma unroll
                                for (int k = 0; k < D; ++k) {
                                    ra.x[k] = rp0[fX + k * 64]; ra.g[k] = rp0[fG + k * 64];
                                    rb.x[k] = rp1[fX + k * 64]; rb.g[k] = rp1[fG + k * 64];
                                }
                                ra.a = rp0[fA];
                                rb.a = rp1[fA];
                                ra.w = GF ? rp0[fW] : 1.0;
                                rb.w = GF ? rp1[fW] : 1.0;
                                av0 = stream_pair(ra);
                                av1 = stream_pair(rb);
                                if constexpr (!FAST) {
                                    av0 = lds_base + e0 < r1 ? av0 : INFINITY;
                                    av1 = lds_base + e1 < r1 ? av1 : INFINITY;
                                }
                                rp0[fA] = av0;
                                rp1[fA] = av1;
                            } else {
                                av0 = lds_pair(e0);
                                av1 = lds_pair(e1);
                            }
                            scan_take_idx<FAST>(av0, (uint32_t)(lds_base + e0), bv, bi);
                            scan_take_idx<FAST>(av1, (uint32_t)(lds_base + e1), bv, bi);
                        } else {                     // the stream/LDS seam or the last chunk
                            one_chunk(c);
                            if (c + 1 < nC) one_chunk(c + 1);
                        }
                    }
                };
                if (a.stream_a_lds) chunk_loop(std::true_type{});
                else chunk_loop(std::false_type{});
                ST_STAMP_AFTER(a, t, 6, bv);
            } else {
                // (two waves per SIMD: two chains per wave are enough and leave room for the rows)
                constexpr int UL = kTwoWaves ? 2 : 4;
                int e = tid;
                for (; e + (UL - 1) * kPBlock < RL; e += UL * kPBlock) {
                    double av[UL];
#pragma unroll
                    for (int u = 0; u < UL; ++u) av[u] = lds_pair(e + u * kPBlock);
#pragma unroll
                    for (int u = 0; u < UL; ++u)
                        scan_take_v<FAST>(av[u], (uint32_t)(lds_base + e + u * kPBlock), bv, bi);
                }
                for (; e < RL; e += kPBlock) scan_take_v<FAST>(lds_pair(e), (uint32_t)(lds_base + e), bv, bi);
                ST_STAMP_AFTER(a, t, 6, bv);
                if constexpr (kTwoWaves) {
                    // two waves per SIMD: one row at a time, no prefetch registers (the other wave
                    // computes while this one waits for its loads)
                    for (; srow < r1; srow += kPBlock) {
                        SRow r;
                        fetch(srow, r);
                        const double av = stream_pair(r);
                        a.A[srow] = av;
                        scan_take_v<FAST>(av, (uint32_t)srow, bv, bi);
                    }
                }
                while (!kTwoWaves && srow < r1) {
                    const int64_t nrow = srow + 2 * kPBlock;
                    SRow n0, n1;
                    fetch(nrow, n0);
                    fetch(nrow + kPBlock, n1);
                    const double av0 = stream_pair(c0);
                    const double av1 = stream_pair(c1);
                    const bool ok1 = srow + kPBlock < r1;
                    a.A[srow] = av0;
                    if (ok1) a.A[srow + kPBlock] = av1;
                    scan_take_v<FAST>(av0, (uint32_t)srow, bv, bi);
                    scan_take_v<FAST>(ok1 ? av1 : INFINITY, (uint32_t)(srow + kPBlock), bv, bi);
                    c0 = n0;
                    c1 = n1;
                    srow = nrow;
                }
            }   // !kDyn
            }   // !kWide
        };
        // the flag is block-uniform (same LDS row, same block flag): make that explicit so the
        // branch is scalar and the two variants stay separate code paths
        if (__builtin_amdgcn_readfirstlane(wfast)) {
            sweep_rows(std::integral_constant<int, CMP ? 2 : 1>{});
        } else if constexpr (!GEN) {   // compact-only: hand the thin to the general kernel
            if (tid == 0) __hip_atomic_fetch_max(a.status, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            break;
        } else {
            sweep_rows(std::integral_constant<int, CMP ? 3 : 0>{});
        }
        ST_STAMP(a, t, 3);
        publish<NT, GUARD>(a, sc, bv, bi, t, r1, bid(), gsc);
        ST_STAMP(a, t, 4);
        if constexpr (guard) {
            if (wid >= 1) {   // off the critical path: these waves only wait for the sweep now
                if (wid == 1) {
                    if constexpr (kLanes) {
                        tie_check_lanes<D, GF, NT>(a, gsc, gl, t - 1, r0, r1);
                    } else {
                        WinnerG<D, GF> wg;   // issued first: lands while wave 0's lanes are reduced
                        if (tid == 64) wg.load(a, gsc, t - 1);
                        reduce_w0(t - 1);   // wave 0's lanes of step t - 1
                        if (tid == 64) tie_check<D, GF>(a, gsc, t - 1, r0, r1, kNW, wg);
                    }
                }
                rescan_rest(t);
            }
        }
    }
    int64_t done = t;   // idx[0 .. done-1) are written
    if (t == a.m) {
        const int64_t win = wait_and_pick<D, GF, kMaxG, GUARD>(a, sc, a.m - 1, bid(), G(), gsc, guard,
                                                               guard && kW0InPoll, rescan_w0);
        if (win >= 0) {
            if (bid() == 0 && tid == 0) a.idx_out[a.m - 1] = (uint32_t)win;
            done = a.m + 1;
        }
    }
    if constexpr (guard) {
        if (!kW0InPoll && done == a.m + 1) {
            if (wid == 0) rescan_w0();
            __syncthreads();
        }
        if (wid == 1 && done == a.m + 1) {
            if constexpr (kLanes) tie_check_lanes<D, GF, NT>(a, gsc, gl, a.m - 1, r0, r1);
            else reduce_w0(a.m - 1);
        }
        if (tid == 64 && done == a.m + 1) {
            if constexpr (!kLanes) {
                WinnerG<D, GF> wg;
                wg.load(a, gsc, a.m - 1);
                tie_check<D, GF>(a, gsc, a.m - 1, r0, r1, kNW, wg);
            }
            if (bid() == 0) {   // block 0's final recurrence state (Q, E, thr(m)) after the bounds (tests)
#if ST_BOUNDS_SLOTS
                uint64_t* bw = reinterpret_cast<uint64_t*>(const_cast<double*>(a.tie_bounds));
                uint64_t g2b = bw[0], w2b = bw[1];
                for (int s = 0; s < ST_BOUNDS_SLOTS; ++s) {
                    const uint64_t* sw = bounds_slot(a, s);
                    g2b = std::max(g2b, (uint64_t)__hip_atomic_load(sw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                    w2b = std::max(w2b, (uint64_t)__hip_atomic_load(sw + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                }
                bw[0] = g2b;   // the bounds the threshold was built from (st_greedy's workspace words)
                bw[1] = w2b;
#endif
                double* st_out = const_cast<double*>(a.tie_bounds) + 2;
                st_out[0] = gsc->tg[3];
                st_out[1] = gsc->tg[4];
                st_out[2] = gsc->tg[5];
            }
        }
    }
    // timeout: poison the unwritten indices (UINT32_MAX) so the host detects the failure
    if (done <= a.m && bid() == 0)
        for (int64_t q = (done > 0 ? done - 1 : 0) + tid; q < a.m; q += kPBlock) a.idx_out[q] = 0xFFFFFFFFu;

    // ---- write the on-chip running sums back (A_out contract of st_greedy) --------------------
#pragma unroll
    for (int q = 0; q < RT; ++q) {
        const int64_t row = r0 + (int64_t)q * kPBlock + tid;
        if (row < r1) a.A[row] = ar[q];
    }
    for (int e = tid; e < RL; e += kPBlock) {
        const int64_t row = lds_base + e;
        if (row < r1) a.A[row] = lrow(e)[fA];
    }
    if (kDyn && a.stream_a_lds)
        for (int64_t row = str_base + tid; row < r1; row += kPBlock) a.A[row] = sA[row - str_base];
}

}  // namespace st
