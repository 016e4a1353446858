// Persistent greedy kernel (K4): host side -- planning, workspace, launches (st_greedy / st_greedy_batch /
// st_greedy_sharded).  The kernel and its device helpers are in persistent_kernel.hpp; the near-tie
// guarded instantiations (GUARD = true) are compiled in persistent_guard.hip, next to this file's.
#include "persistent_kernel.hpp"

namespace st {

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
// granules between replicas: one replica = G records rec_stride granules apart; with several
// replicas each starts on a fresh 512-B boundary plus 256 B, so their lines fall on other channels
// the GUARD instantiations (persistent_guard.hip): the kernel for a plan, or nullptr
const void* guarded_persistent_fn(int d, bool gf, int rt, int nt, int bpc, bool gen, bool batch);
// the small-shard instantiations (persistent_small.hip: 256 threads, 1 / 2 register rows), or nullptr
const void* small_persistent_fn(int d, bool gf, int rt, bool cmp, bool batch, bool guard);

int64_t persistent_rep_stride(int G, int rec_stride, int nrep) {
    const int64_t one = (int64_t)G * rec_stride;
    return nrep == 1 ? one : (one + 63) / 64 * 64 + 32;
}

// one kernel's record region: 2 banks x nrep replicas x G records
static int64_t persistent_region_bytes(int G, int rec_stride, int nrep) {
    return 2 * (int64_t)nrep * persistent_rep_stride(G, rec_stride, nrep) * 8;
}

int64_t persistent_ws_bytes(int d, int G, int rec_stride, int nrep) {
    // [control: status (and reserved) words][record region][record region of the general kernel
    // behind a compact-only run, when the workspace holds it]
    (void)d;
    return kWsControlBytes + persistent_region_bytes(G, rec_stride, nrep);
}

// workspace the persistent launcher can use at most: two record regions (compact-only kernel and
// the general kernel gated behind it) at the widest grid, the most replicas st_tune key 10 allows and
// packed records
int64_t persistent_ws_max_bytes() {
    return kWsControlBytes + 2 * persistent_region_bytes(kMaxGrid, kRecGranules, 32);
}

static int g_persist_rt = -1;   // st_tune key 3: -1 auto, 0 = off
static int g_persist_nt = -1;   // st_tune key 4: threads per block, -1 auto (256)
static int g_persist_grid = -1; // st_tune key 5: grid cap (blocks), -1 auto (one per CU)
// st_tune key 23: the calling host thread's own grid cap (-1: none; greedy_concurrent's streams), so that
// threads thinning side by side never change each other's grids
static thread_local int t_persist_grid = -1;
static int grid_cap() { return t_persist_grid > 0 ? t_persist_grid : g_persist_grid; }
static int g_persist_pitch = -1; // st_tune key 9: record pitch in bytes (16 .. 4096, power of 2), -1 auto
static int g_persist_nrep = -1;  // st_tune key 10: record replicas (1 .. 32, power of 2), -1 auto
static int g_persist_cmp = -1;   // st_tune key 12: compact-only kernel register rows (8, 9), 0 off, -1 auto
// st_tune key 15: the 512-thread kernels keep the streamed rows' running sums in LDS (1) or in HBM (0,
// the default).  Measured (round 4, same box, config 4, profiles/r04_streamed_sums_lds_rejected.log):
// PMC WRITE_SIZE 1.08 GB -> 0.15 GB per thin, but 6.82 -> 6.94-7.01 ms: the 8 B per streamed row take
// LDS from ~120 LDS rows, which then stream (~1.1 ns instead of ~0.36 ns per row-step), and the A
// load / store it saves was not on the critical path (L2-resident, stores fire-and-forget).
// -1 (auto): on under the near-tie guard, whose rescans read every streamed row's sum after each publish --
// from LDS instead of L2 the guarded all-row config-4 thin takes 9.96 instead of 10.71-10.79 ms (round 6,
// same box, profiles/r06_guard_knobs.log)
static int g_persist_sal = -1;
// st_tune key 16: ticks (10 ns) added to a step's first poll time before it is aligned to the poll
// grid: -1 auto = 10 for the one-device compact-only kernel, 0 otherwise.  A block whose first poll
// would fall just before the last records land takes the next grid slot instead of an early,
// incomplete poll.  Round 4, same box, two sweeps (profiles/r04_first_poll_delay.log): n = 2e6
// (compact-only kernel) 7.10 / 7.21 (0) -> 6.80 / 6.88 us per step (10), 5: 6.82 / 6.91, 15: 6.83 /
// 6.86, 20 and 25 slower; n = 1e6 and 4e5 (general 512-thread kernel) and 2e5 / 2.5e5 (256-thread
// kernels): every delay slower or equal.
static int g_persist_delay = -1;
// st_tune key 19: 512-thread kernels, two LDS chunks as two independent dependency chains (fields read
// up front, sums stored after both) -- 1 / -1 automatic; 0 = one lds_pair after the other (round 4's
// earlier form, whose LDS store of the first sum held the second row's reads and chain behind it).
// Same box, alternating (profiles/r04_lds_two_chains.log): config 4 6.91-6.94 (0) -> 6.80-6.81 (1) ms
// per thin.  The two pair evaluations interleaved statement by statement in the source as well were
// measured and dropped: the extra live registers spilled inside the step loop (75 VGPRs of scratch)
// and every variant ran at 8.6-8.7 ms (profiles/r04_lds_interleaved_rejected.log)
static int g_persist_lds2 = -1;
// automatic register rows of the compact-only kernel: 9 (28 B of scratch at d = 4; 8 under the near-tie
// guard).  Same-box, d = 4, m = 1000 (profiles/r03_compact_only_rt.log): n = 2e6: 7.81 (general kernel) /
// 7.76 (8) / 7.05 (9) us per step.  (Round 6 pruned the 10-row plan -- 17.8 against 18.5 us per step at
// n = 3e6 only, no BASELINE config -- with the other families that won nothing on a BASELINE config or the
// LV call: DESIGN.md section 4, "Plans".)
static uint64_t* g_stamps = nullptr;
#ifdef ST_PERSIST_STAMPS
extern "C" int st_debug_set_stamps(uint64_t* buf) { g_stamps = buf; return 0; }
#endif
// the current value of a persistent-kernel st_tune key (st_tune_get); INT32_MIN for other keys
int persistent_tune_get(int key) {
    switch (key) {
        case 3: return g_persist_rt;
        case 4: return g_persist_nt;
        case 5: return g_persist_grid;
        case 23: return t_persist_grid;
        case 9: return g_persist_pitch;
        case 10: return g_persist_nrep;
        case 12: return g_persist_cmp;
        case 15: return g_persist_sal;
        case 16: return g_persist_delay;
        case 19: return g_persist_lds2;
        default: return INT32_MIN;
    }
}

int persistent_tune(int key, int value) {
    if (key == 3) {
        if (value != -1 && value != 0 && value != 1 && value != 2 && value != 4 && value != 8 && value != 16) return -1;
        g_persist_rt = value;
        return 0;
    }
    if (key == 4) {
        if (value != -1 && value != 256 && value != 512) return -1;
        g_persist_nt = value;
        return 0;
    }
    if (key == 5) {
        if (value < -1 || value == 0 || value > kMaxGrid) return -1;
        g_persist_grid = value;
        return 0;
    }
    if (key == 23) {
        if (value < -1 || value == 0 || value > kMaxGrid) return -1;
        t_persist_grid = value;
        return 0;
    }
    if (key == 8) {   // blocks per CU: one (two-block plans pruned in round 6)
        return value == -1 || value == 1 ? 0 : -1;
    }
    if (key == 9) {
        if (value != -1 && (value < 16 || value > 4096 || (value & (value - 1)))) return -1;
        g_persist_pitch = value;
        return 0;
    }
    if (key == 10) {
        if (value != -1 && (value < 1 || value > 32 || (value & (value - 1)))) return -1;
        g_persist_nrep = value;
        return 0;
    }
    if (key == 12) {
        if (value != -1 && value != 0 && value != 8 && value != 9) return -1;
        g_persist_cmp = value;
        return 0;
    }
    if (key == 16) {
        if (value < -1 || value > 450) return -1;
        g_persist_delay = value;
        return 0;
    }
    if (key == 15) {
        if (value < -1 || value > 1) return -1;
        g_persist_sal = value;
        return 0;
    }
    if (key == 19) {
        if (value < -1 || value > 1) return -1;
        g_persist_lds2 = value;
        return 0;
    }
    return -1;
}

// b != nullptr: the batch kernel over b's problems (G = every group's blocks together); it is
// instantiated for the one-block-per-CU kernels (256 and 512 threads) with the compact arithmetic only
template <int D, bool GF, int RT, int NT, int BPC = 1, bool GEN = true>
static hipError_t launch_p(const PersistArgs& a, int G, size_t lds, hipStream_t s, bool dry,
                           const BatchArgs* b = nullptr) {
    // the compact instantiation for d <= 8 when st_tune key 11 selects it (the default); GEN = false:
    // the compact-only kernel (launch_greedy_persistent enqueues the general one behind it); a guarded
    // plan (tie_bounds set: compact, one device) takes the GUARD instantiation of persistent_guard.hip
    const void* fn;
    const bool guarded = b ? b->p[0].tie_bounds != nullptr : a.tie_bounds != nullptr;
    if constexpr (RT < 4 && D <= kMaxCtDim) {   // small shards: compiled in persistent_small.hip
        static_assert(NT == 256 && BPC == 1 && GEN, "small-shard plans only");
        fn = small_persistent_fn(D, GF, RT, arith_compact(), b != nullptr, guarded);
        if (!fn) return hipErrorNotSupported;
    } else if (guarded) {
        if constexpr (D <= kMaxCtDim) {
            fn = guarded_persistent_fn(D, GF, RT, NT, BPC, GEN, b != nullptr);
            if (!fn) return hipErrorNotSupported;
        } else {
            return hipErrorNotSupported;
        }
    } else if constexpr (!GEN && RT < 8) {   // the mid-size compact-only plan is a guarded plan only
        return hipErrorNotSupported;
    } else if (b) {
        if constexpr (BPC == 1 && D <= kMaxCtDim) {
            if (!arith_compact()) return hipErrorNotSupported;
            fn = reinterpret_cast<const void*>(greedy_persistent<D, GF, RT, NT, BPC, true, GEN, BatchArgs>);
        } else {
            return hipErrorNotSupported;
        }
    } else if constexpr (!GEN) {
        fn = reinterpret_cast<const void*>(greedy_persistent<D, GF, RT, NT, BPC, true, false>);
    } else if constexpr (D <= kMaxCtDim) {
        fn = arith_compact() ? reinterpret_cast<const void*>(greedy_persistent<D, GF, RT, NT, BPC, true>)
                             : reinterpret_cast<const void*>(greedy_persistent<D, GF, RT, NT, BPC, false>);
    } else {
        fn = reinterpret_cast<const void*>(greedy_persistent<D, GF, RT, NT, BPC, false>);
    }
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    // co-residency of the whole grid (every block spins on the others' records): checked here
    // against the occupancy query -- what hipLaunchCooperativeKernel would check at launch -- and
    // then a PLAIN launch of the same one-block-per-CU grid (same residency, MI355X_MICROARCH.md
    // coop-launch row).  The cooperative path also made the HIP runtime create a cooperative queue
    // whose exit-time teardown crashes when rocprofv3's tool has finalised HSA first
    // (profiles/r02_exit_crash_bisect.log); a rank that cannot make progress times out, it never hangs.
    // The occupancy query cannot see kernels of other streams / processes: a grid that is not
    // co-resident aborts at step 0 after kFirstStepTimeoutTicks and the host re-runs the thin on
    // the launch-per-step kernels (DeviceProblem.greedy; tests/test_gpu_fallback.py provokes it).
    int dev = 0, cus = 0, per_cu = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
    if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, NT, lds)) != hipSuccess)
        return e;
    if ((int64_t)per_cu * cus < G) return hipErrorNotSupported;
    if (dry) return hipSuccess;
    PersistArgs args = a;
    BatchArgs bargs;
    if (b) bargs = *b;
    void* kargs[] = {b ? static_cast<void*>(&bargs) : static_cast<void*>(&args)};
    return hipLaunchKernel(fn, dim3(G), dim3(NT), kargs, lds, s);
}

// compact-only kernels: 512-thread blocks, 8 / 9 register rows per thread (4 under the near-tie guard)
template <int D, bool GF>
static hipError_t launch_p_cmp(const PersistArgs& a, int rt, int G, size_t lds, hipStream_t s, bool dry,
                               const BatchArgs* b) {
    if (rt == 9) return launch_p<D, GF, 9, 512, 1, false>(a, G, lds, s, dry, b);
    if (rt == 4) return launch_p<D, GF, 4, 512, 1, false>(a, G, lds, s, dry, b);
    return launch_p<D, GF, 8, 512, 1, false>(a, G, lds, s, dry, b);
}

// the plans ("Plans"): 512-thread blocks with 4 / 8 register rows, 256-thread blocks with
// 1 / 2 (persistent_small.hip) / 4
template <int D, bool GF>
static hipError_t launch_p_rt(const PersistArgs& a, int rt, int nt, int G, size_t lds, hipStream_t s,
                               bool dry, const BatchArgs* b) {
    if (nt == 512) {
        if (rt <= 4) return launch_p<D, GF, 4, 512>(a, G, lds, s, dry, b);
        return launch_p<D, GF, 8, 512>(a, G, lds, s, dry, b);
    }
    switch (rt) {
        case 1: return launch_p<D, GF, 1, 256>(a, G, lds, s, dry, b);
        case 2: return launch_p<D, GF, 2, 256>(a, G, lds, s, dry, b);
        default: return launch_p<D, GF, 4, 256>(a, G, lds, s, dry, b);
    }
}

static hipError_t launch_cmp(const PersistArgs& a, int d, bool gf, int rt, int G, size_t lds, hipStream_t s,
                             bool dry, const BatchArgs* b = nullptr) {
    if (d == 2) return gf ? launch_p_cmp<2, true>(a, rt, G, lds, s, dry, b) : launch_p_cmp<2, false>(a, rt, G, lds, s, dry, b);
    return gf ? launch_p_cmp<4, true>(a, rt, G, lds, s, dry, b) : launch_p_cmp<4, false>(a, rt, G, lds, s, dry, b);
}

static hipError_t launch_kind(const PersistArgs& a, int d, bool wide, bool gf, int rt, int nt, int G,
                              size_t lds, hipStream_t s, bool dry, const BatchArgs* b = nullptr) {
    if (wide) {
        if (b) return hipErrorNotSupported;
        return gf ? launch_p<kWideD, true, 1, 256>(a, G, lds, s, dry) : launch_p<kWideD, false, 1, 256>(a, G, lds, s, dry);
    }
    if (d == 2) return gf ? launch_p_rt<2, true>(a, rt, nt, G, lds, s, dry, b) : launch_p_rt<2, false>(a, rt, nt, G, lds, s, dry, b);
    return gf ? launch_p_rt<4, true>(a, rt, nt, G, lds, s, dry, b) : launch_p_rt<4, false>(a, rt, nt, G, lds, s, dry, b);
}

namespace {
// one thin's launch decision: the kernel instantiation(s), grid, LDS and arguments
struct Plan {
    PersistArgs a, ac;     // general kernel / compact-only kernel (use_cmp)
    bool wide, gf, use_cmp, own_region;
    int d, rt, nt, G, rt_c;
    size_t lds, lds_c;
    int64_t region;        // bytes of one record region
    char* ws;
};
}  // namespace

// Everything up to the launches; hipErrorNotSupported when the persistent path does not apply.
// plan_only: the eligibility query (every pointer may be a placeholder); *used = 1 if it applies.
static hipError_t plan_persistent(const double* x, const double* g, const double* w, double* A, int64_t n,
                                  int d, int64_t ld, double l, double tr, int64_t m, uint32_t* idx_out,
                                  void* ws, int64_t ws_bytes, hipStream_t s, int* used, const RankSpec* rs,
                                  bool plan_only, int grid_cap, Plan& P, int rt_force = 0,
                                  int cmp_force = 0, bool batch = false) {
    const RankSpec one{0, n, 0, 1, 0, nullptr, {}};
    if (!rs) rs = &one;
    // 32-bit row indices, padding rows included (< n + one block's register rows)
    const bool wide = d == kWideD;
    if (g_persist_rt == 0 || (d != 2 && d != 4 && !wide) || m < 1 || m >= 0xFFFFFFFFll || n >= 0x7FFFFFFFll)
        return hipErrorNotSupported;
    if (rs->nranks < 1 || rs->nranks > kMaxRanks || rs->rank < 0 || rs->rank >= rs->nranks ||
        rs->row_begin < 0 || rs->row_end <= rs->row_begin || rs->row_end > n ||
        (rs->nranks > 1 && !rs->inbox))
        return hipErrorInvalidValue;
    const int64_t n_shard = rs->row_end - rs->row_begin;
    int dev = 0, cus = 0, lds_max = 0, lds_optin = 0;
    if (hipGetDevice(&dev) != hipSuccess) return hipErrorNotSupported;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return hipErrorNotSupported;
    if (hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess)
        return hipErrorNotSupported;
    if (hipDeviceGetAttribute(&lds_optin, hipDeviceAttributeSharedMemPerBlockOptin, dev) == hipSuccess &&
        lds_optin > lds_max)
        lds_max = lds_optin;
    if (lds_max > 163840) lds_max = 163840;
    int nt = wide ? 256 : (g_persist_nt > 0 ? g_persist_nt : 256);
    int G = cus > kMaxGrid ? kMaxGrid : cus;   // one block per CU
    if (grid_cap > 0 && G > grid_cap) G = grid_cap;
    const int64_t min_rows = 256;   // fewer blocks for small n: exchange cost grows with G
    if (n_shard < (int64_t)G * min_rows) G = (int)((n_shard + min_rows - 1) / min_rows);
    if (G < 1) G = 1;
    // record pitch: the widest requested / default that the workspace holds (>= 16 B)
    int nrep = g_persist_nrep > 0 ? g_persist_nrep : kDefaultRecReplicas;
    if (nrep > G) nrep = G;
    while (nrep & (nrep - 1)) nrep &= nrep - 1;
    int pitch = (g_persist_pitch > 0 ? g_persist_pitch : (nrep > 1 ? 16 : kDefaultRecPitch)) / 8;
    while (nrep > 1 && persistent_ws_bytes(d, G, pitch, nrep) > ws_bytes) nrep /= 2;
    while (pitch > kRecGranules && persistent_ws_bytes(d, G, pitch, nrep) > ws_bytes) pitch /= 2;
    if (persistent_ws_bytes(d, G, pitch, nrep) > ws_bytes) return hipErrorNotSupported;
    const int64_t R = (n_shard + G - 1) / G;
    if (wide && R > 256) return hipErrorNotSupported;   // wide: one register row per thread only
    // the 512-thread kernels address streamed rows with 32-bit buffer offsets (column k at
    // k * ld * 8 bytes from the block's first streamed row): only a launch that streams rows needs
    // them below 2^31 (the 256-thread and wide kernels use 64-bit addresses)
    auto offsets_ok = [&](int nt_, int rt_, int64_t rl_) {
        return nt_ != 512 || R <= (int64_t)rt_ * nt_ + rl_ || (int64_t)(d - 1) * ld * 8 + (R + 64) * 8 < 0x7FFFFFFFll;
    };
    // auto: 512-thread blocks (two waves per SIMD, dynamic chunks) once a block has more rows than
    // one wave per SIMD keeps in registers comfortably (measured crossover 1e3 .. 2e3 rows per CU,
    // scripts/sweep_nt_crossover.sh)
    if (!wide && g_persist_nt <= 0 && R > kNt512MinRows) nt = 512;
    // register rows per thread: 512-thread blocks 8, or 4 when 8 would leave register slots empty;
    // 256-thread blocks 4 (st_tune key 3 may ask for fewer, or for 4 on 512 threads)
    const int rt_max = nt == 512 ? 8 : 4;
    int rt = rt_force > 0 ? rt_force : (g_persist_rt > 0 ? g_persist_rt : rt_max);
    const bool small_ok = nt == 256 && !wide;   // 1 / 2 register rows: persistent_small.hip
    if (rt != 4 && rt != 8 && !(small_ok && (rt == 1 || rt == 2))) rt = rt_max;
    if (rt > rt_max) rt = rt_max;
    if (rt == 8 && (int64_t)rt * nt > R) rt = 4;   // no empty register rows
    // the near-tie guard's general kernel: 4 register rows (with 8 its guard state spills ~0.7 KB per lane
    // inside the step loop; it runs where the compact-only kernel does not -- a rank of a multi-rank thin)
    if (rt == 8 && nt == 512 && tie_guard() && arith_compact() && g_persist_rt <= 0 && rt_force <= 0) rt = 4;
    // small shards: the fewest register rows that hold the block's rows (padding rows compute like real
    // ones; 1 / 2 rows per thread at <= 256 / 512 rows per block)
    if (small_ok && g_persist_rt <= 0 && rt_force <= 0 && R <= 2 * 256) rt = R <= 256 ? 1 : 2;
    if (wide) rt = 1;
    const bool gf = w != nullptr;
    const size_t row_bytes = (size_t)(2 * d + 1 + (gf ? 1 : 0)) * sizeof(double);
    // near-tie guard: the compact arithmetic, d = 2 / 4 (st_tune key 20), one device or every rank of a
    // multi-rank run -- the GUARD kernels, whose LDS holds the guard's scratch after Scratch
    const bool guard = tie_guard() && arith_compact() && !wide && !plan_only;
    // (the 256-thread guarded kernels also hold every thread's step record, GuardLanes)
    const size_t head = (sizeof(Scratch) + 15) / 16 * 16 + (guard ? (sizeof(GuardScratch) + 15) / 16 * 16 : 0) +
                        (guard && nt != 512 ? (sizeof(GuardLanes) + 15) / 16 * 16 : 0);
    const size_t budget = (size_t)(lds_max > 0 ? lds_max : 65536) - 1024;   // static + slack
    // LDS rows (whole 64-row chunks) for rows past the register rows; the 512-thread (dynamic-chunk)
    // kernels also keep every streamed row's running sum in LDS (8 B per row, whole chunks)
    // (st_tune key 15 = 1, or -1 under the near-tie guard; when the streamed sums alone would not fit -- more than ~20 000
    // streamed rows per block -- they stay in HBM: sal = 0)
    auto lds_rows = [&](int nt_, int rt_, int64_t& rl, size_t& bytes, int& sal) {
        const int64_t need_ = R - (int64_t)rt_ * nt_;
        sal = (g_persist_sal == 1 || (g_persist_sal < 0 && guard)) && nt_ == 512 && need_ > 0 &&
              head + (size_t)(need_ + 63) / 64 * 64 * sizeof(double) <= budget;
        rl = need_ > 0 ? need_ / 64 * 64 : 0;
        if (guard && rl > kGuardLdsRows) rl = kGuardLdsRows;   // the guard's repeat bits (GuardScratch::lrep)
        auto total = [&](int64_t l) {
            const int64_t st = need_ - l > 0 ? (need_ - l + 63) / 64 * 64 : 0;
            return head + (size_t)l * row_bytes + (sal ? (size_t)st * sizeof(double) : 0);
        };
        while (rl > 0 && total(rl) > budget) rl -= 64;
        bytes = total(rl);
    };
    int64_t RL = 0;
    size_t lds_rows_bytes = head;
    int sal = 0;
    if (!wide) lds_rows(nt, rt, RL, lds_rows_bytes, sal);
    // wide: the rows' g lives in LDS (d x 256 doubles: 100 KB at d = 50)
    const size_t lds = wide ? head + (size_t)d * 256 * sizeof(double) : lds_rows_bytes;
    if (wide && lds > (size_t)(lds_max > 0 ? lds_max : 65536)) return hipErrorNotSupported;
    if (!wide && !offsets_ok(nt, rt, RL)) return hipErrorNotSupported;

    char* p = static_cast<char*>(ws);
    PersistArgs a{};
    if (plan_only) {   // eligibility query (st_greedy_sharded_supported): everything but the launch
        hipError_t e = launch_kind(a, d, wide, gf, rt, nt, G, lds, s, true);
        if (e == hipSuccess) *used = 1;
        return e;
    }
    a.x = x; a.g = g; a.w = w; a.A = A;
    a.n = n; a.ld = ld; a.l = l; a.tr = tr; a.m = m;
    a.idx_out = idx_out;
    a.status = reinterpret_cast<unsigned*>(p + kWsStatusOff);
    if (guard) {
        a.tie_bounds = reinterpret_cast<const double*>(p + kWsBoundsOff);
        a.tie = reinterpret_cast<unsigned*>(p + kWsTieOff);
    }
    a.gran = reinterpret_cast<uint64_t*>(p + kWsControlBytes);
    a.rows_per_block = R;
    a.RL = (int)RL;
    a.stream_a_lds = sal;
    a.poll_delay = g_persist_delay >= 0 ? g_persist_delay : 0;
    a.lds_two_chains = g_persist_lds2 >= 0 ? g_persist_lds2 : 1;
    a.rec_stride = pitch;
    a.nrep = nrep;
    a.rep_stride = persistent_rep_stride(G, pitch, nrep);
    a.stamps = g_stamps;
    a.row_begin = rs->row_begin;
    a.row_end = rs->row_end;
    a.rank = rs->rank;
    a.nranks = rs->nranks;
    a.seq_base = rs->seq_base;
    a.inbox = rs->inbox;
    for (int r = 0; r < kMaxRanks; ++r) a.peer[r] = r < rs->nranks ? rs->peer[r] : nullptr;
    // one device, 512-thread blocks with at least 8 register rows' worth of rows per block: the
    // compact-only kernel (more register rows per thread, fewer streamed rows) runs the thin first and
    // the general kernel, enqueued behind it, runs only if a step needed the exact arithmetic (its
    // gate is the compact-only kernel's status word, its own status the next word)
    PersistArgs ac = a;
    bool use_cmp = false;
    int rt_c = 0;
    size_t lds_c = 0;
    // Mid-size blocks (1 280 .. 4 095 rows): unguarded, the general kernel (round 5's compact-only 4 / 6-row
    // plans gained 1.5 % on the LV call and were pruned in round 6 with the other families below the 3 % bar);
    // guarded, the compact-only kernel of 4 register rows -- the guarded general kernel of 4 rows spills, and
    // the LV call's all-row thin takes 44.6 ms on it against 40.7 ms (profiles/r06_plans_ab.log)
    const bool mid_guard = guard && !batch && cmp_force <= 0 && R >= 1280 && R < 8 * 512;
    if (rs->nranks == 1 && arith_compact() && nt == 512 && !wide && g_persist_cmp != 0 &&
        (R >= 8 * 512 || mid_guard)) {
        if (cmp_force > 0)
            rt_c = cmp_force;   // a batch's common register rows (launch_greedy_persistent_batch)
        else if (mid_guard)
            rt_c = 4;
        else
            rt_c = g_persist_cmp > 0 ? g_persist_cmp : 9;
        // guarded: 8 register rows -- the guard's rescans take the registers a ninth row needs (9 rows spill
        // inside the step loop; st_tune key 12 = 9 still selects 9)
        if (guard && rt_c > 8 && g_persist_cmp <= 0 && cmp_force <= 0) rt_c = 8;
        int64_t RLc = 0;
        int salc = 0;
        lds_rows(512, rt_c, RLc, lds_c, salc);
        ac.RL = (int)RLc;
        ac.stream_a_lds = salc;
        // (the first-poll delay pays only at the headline's 2e6 rows: r04_first_poll_delay.log, r05_knobs_recheck.log)
        ac.poll_delay = g_persist_delay >= 0 ? g_persist_delay : (R >= 8 * 512 ? 10 : 0);
        use_cmp = offsets_ok(512, rt_c, RLc) &&
                  launch_cmp(ac, d, gf, rt_c, G, lds_c, s, true) == hipSuccess;   // residency check only
    }
    // The gated general kernel must never see a record of the compact-only run: its tags are 8-bit
    // (they wrap every 256 steps) and the compact-only kernel may stop at any step.  It gets a
    // record region of its own when the workspace holds one (st_greedy_workspace_bytes does), else
    // the shared region is zeroed again between the two launches.
    const int64_t region = persistent_region_bytes(G, pitch, nrep);
    P.a = a;
    P.ac = ac;
    P.wide = wide; P.gf = gf; P.use_cmp = use_cmp;
    P.own_region = use_cmp && kWsControlBytes + 2 * region <= ws_bytes;
    P.d = d; P.rt = rt; P.nt = nt; P.G = G; P.rt_c = rt_c;
    P.lds = lds; P.lds_c = lds_c;
    P.region = region;
    P.ws = p;
    return hipSuccess;
}

// zero status, the near-tie words and bounds and every granule tag (a stale tag from a previous run must
// never match); with the compact-only kernel, point the general kernel's gate / status / tie word /
// records past the compact run's
static hipError_t prepare_ws(Plan& P, hipStream_t s) {
    hipError_t e = hipMemsetAsync(P.ws, 0, (size_t)(kWsControlBytes + (P.own_region ? 2 : 1) * P.region), s);
    if (e != hipSuccess || !P.use_cmp) return e;
    P.a.gate = P.ac.status;
    P.a.status = P.ac.status + 1;
    if (P.a.tie) P.a.tie = P.ac.tie + 1;
    if (P.own_region) P.a.gran = reinterpret_cast<uint64_t*>(P.ws + kWsControlBytes + P.region);
    return hipSuccess;
}

// The near-tie guard's bounds over ALL n rows (stein_ref.c sr_tie_bounds; the staging's operations): a
// multi-rank run's blocks cover only their rank's rows, so every row's maxima are merged into the workspace's
// bounds slots before the launch -- the blocks' own merges then change nothing, and every rank's threshold
// recurrence is the single-device one
template <int D, bool GF>
__global__ __launch_bounds__(256) void tie_bounds_kernel(const double* g, const double* w, int64_t n, int64_t ld,
                                                          double* bounds) {
    double gm = 0.0, wm = GF ? 0.0 : 1.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        double s2 = g[i] * g[i];
#pragma unroll
        for (int k = 1; k < D; ++k) s2 = s2 + g[k * ld + i] * g[k * ld + i];
        gm = __builtin_fmax(gm, __builtin_isnan(s2) ? INFINITY : s2);
        if constexpr (GF) wm = __builtin_fmax(wm, __builtin_isnan(w[i] * w[i]) ? INFINITY : w[i] * w[i]);
    }
    gm = wave_max_f64(gm);
    wm = wave_max_f64(wm);
    // one atomic pair per block, into the block's bounds slot (the persistent blocks' own slots; the late check
    // of step 0 takes the maximum over the slots and the words): no single contended address
    __shared__ double wave_m[4][2];
    if ((threadIdx.x & 63) == 0) { wave_m[threadIdx.x >> 6][0] = gm; wave_m[threadIdx.x >> 6][1] = wm; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < 4; ++w) { gm = __builtin_fmax(gm, wave_m[w][0]); wm = __builtin_fmax(wm, wave_m[w][1]); }
        uint64_t* bw = reinterpret_cast<uint64_t*>(bounds);
#if ST_BOUNDS_SLOTS
        bw = reinterpret_cast<uint64_t*>(reinterpret_cast<char*>(bounds) - kWsBoundsOff +
                                         (int64_t)(blockIdx.x % ST_BOUNDS_SLOTS) * 64);
#endif
        __hip_atomic_fetch_max(bw, (uint64_t)__double_as_longlong(gm), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_max(bw + 1, (uint64_t)__double_as_longlong(wm), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

static hipError_t launch_tie_bounds(const PersistArgs& a, int d, hipStream_t s) {
    const int64_t want = (a.n + 255) / 256;
    const int blocks = (int)(want < 1024 ? want : 1024);
    double* bounds = const_cast<double*>(a.tie_bounds);
    if (d == 2) {
        if (a.w) tie_bounds_kernel<2, true><<<blocks, 256, 0, s>>>(a.g, a.w, a.n, a.ld, bounds);
        else tie_bounds_kernel<2, false><<<blocks, 256, 0, s>>>(a.g, a.w, a.n, a.ld, bounds);
    } else {
        if (a.w) tie_bounds_kernel<4, true><<<blocks, 256, 0, s>>>(a.g, a.w, a.n, a.ld, bounds);
        else tie_bounds_kernel<4, false><<<blocks, 256, 0, s>>>(a.g, a.w, a.n, a.ld, bounds);
    }
    return hipGetLastError();
}

// Returns hipErrorNotSupported when the persistent path does not apply (caller falls back).
hipError_t launch_greedy_persistent(const double* x, const double* g, const double* w, double* A,
                                    int64_t n, int d, int64_t ld, double l, double tr, int64_t m,
                                    uint32_t* idx_out, void* ws, int64_t ws_bytes, hipStream_t s,
                                    int* used, const RankSpec* rs, bool plan_only) {
    *used = 0;
    Plan P;
    hipError_t e = plan_persistent(x, g, w, A, n, d, ld, l, tr, m, idx_out, ws, ws_bytes, s, used, rs, plan_only,
                                   grid_cap(), P);
    if (e != hipSuccess || plan_only) return e;
    if ((e = prepare_ws(P, s)) != hipSuccess) return e;
    if (P.a.tie_bounds && P.a.nranks > 1 && (e = launch_tie_bounds(P.a, P.d, s)) != hipSuccess) return e;
    if (P.use_cmp) {
        if ((e = launch_cmp(P.ac, P.d, P.gf, P.rt_c, P.G, P.lds_c, s, false)) != hipSuccess) return e;
        // the shared record region is zeroed again between the two launches (see above)
        if (!P.own_region && (e = hipMemsetAsync(P.ws + kWsControlBytes, 0, (size_t)P.region, s)) != hipSuccess)
            return e;
    }
    e = launch_kind(P.a, P.d, P.wide, P.gf, P.rt, P.nt, P.G, P.lds, s, false);
    if (e == hipSuccess) *used = 1;
    return e;
}

// Independent single-device thins in one launch (st_greedy_batch): each planned as a plain launch
// capped at #CU / count blocks; all plans must pick the same kernel (d, weights, threads per block,
// register rows), else hipErrorNotSupported (the caller runs them one by one).  The gated general kernel
// behind a compact-only batch is a batch launch too: a group whose compact run completed returns at
// once.
hipError_t launch_greedy_persistent_batch(int count, const BatchProblem* pr, int d, int64_t m, hipStream_t s,
                                          int* used) {
    *used = 0;
    if (count < 1 || count > kMaxBatch || g_persist_rt == 0) return hipErrorNotSupported;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return hipErrorNotSupported;
    int cap = cus / count;
    if (grid_cap() > 0 && cap > grid_cap()) cap = grid_cap();
    if (cap < 1) return hipErrorNotSupported;
    Plan P[kMaxBatch];
    BatchArgs bc{}, bg{};
    bc.count = bg.count = count;
    size_t lds = 0, lds_c = 0;
    // plans that differ only in the small-shard register rows (256 threads, 1 / 2 / 4 rows per thread)
    // or in the compact-only kernel's register rows are planned again with the largest of them: one
    // kernel for the batch
    int rt_force = 0, cmp_force = 0;
    for (int attempt = 0; attempt < 2; ++attempt) {
        bool rt_only = true;
        int rt_max_seen = 0, rtc_max_seen = 0;
        for (int q = 0; q < count; ++q) {
            int u = 0;
            hipError_t e = plan_persistent(pr[q].x, pr[q].g, pr[q].w, pr[q].A, pr[q].n, d, pr[q].ld, pr[q].l,
                                           pr[q].tr, m, pr[q].idx_out, pr[q].ws, pr[q].ws_bytes, s, &u, nullptr, false,
                                           cap, P[q], rt_force, cmp_force, true);
            if (e != hipSuccess) return e;
            const Plan& p0 = P[0];
            if (P[q].wide || P[q].nt != p0.nt || P[q].gf != p0.gf || P[q].use_cmp != p0.use_cmp)
                return hipErrorNotSupported;
            rt_max_seen = std::max(rt_max_seen, P[q].rt);
            rtc_max_seen = std::max(rtc_max_seen, P[q].rt_c);
            if (P[q].rt != p0.rt && !(P[q].nt == 256 && P[q].rt <= 4 && p0.rt <= 4)) rt_only = false;
        }
        bool same_rt = true, same_c = true;
        for (int q = 1; q < count; ++q) {
            same_rt &= P[q].rt == P[0].rt;
            same_c &= P[q].rt_c == P[0].rt_c;
        }
        if (same_rt && same_c) break;
        if (!rt_only || attempt == 1) return hipErrorNotSupported;
        if (!same_rt) rt_force = rt_max_seen;
        if (!same_c) cmp_force = rtc_max_seen;
    }
    for (int q = 0; q < count; ++q) {
        P[q].a.stamps = P[q].ac.stamps = nullptr;
        bc.blk_begin[q + 1] = bg.blk_begin[q + 1] = bc.blk_begin[q] + P[q].G;
        lds = std::max(lds, P[q].lds);
        lds_c = std::max(lds_c, P[q].lds_c);
    }
    const int G = bc.blk_begin[count];
    const Plan& p0 = P[0];
    // residency and the kernel's existence for this combination, before anything is enqueued
    if (launch_kind(p0.a, d, false, p0.gf, p0.rt, p0.nt, G, lds, s, true, &bg) != hipSuccess ||
        (p0.use_cmp && launch_cmp(p0.ac, d, p0.gf, p0.rt_c, G, lds_c, s, true, &bc) != hipSuccess))
        return hipErrorNotSupported;
    hipError_t e;
    for (int q = 0; q < count; ++q) {
        if ((e = prepare_ws(P[q], s)) != hipSuccess) return e;
        bc.p[q] = P[q].ac;
        bg.p[q] = P[q].a;
    }
    if (p0.use_cmp) {
        if ((e = launch_cmp(p0.ac, d, p0.gf, p0.rt_c, G, lds_c, s, false, &bc)) != hipSuccess) return e;
        for (int q = 0; q < count; ++q)
            if (!P[q].own_region &&
                (e = hipMemsetAsync(P[q].ws + kWsControlBytes, 0, (size_t)P[q].region, s)) != hipSuccess)
                return e;
    }
    e = launch_kind(p0.a, d, false, p0.gf, p0.rt, p0.nt, G, lds, s, false, &bg);
    if (e == hipSuccess) *used = 1;
    return e;
}

// ------------------------------------------------------------------------------------------
// mailbox: [2 banks x kMaxRanks slots x 2 granules][kMaxRanks handshake words], u64
// ------------------------------------------------------------------------------------------
__global__ void mailbox_handshake(MailboxPeers peers, uint64_t* inbox, int rank, int nranks,
                                  uint64_t token, int* ok) {
    const int lane = threadIdx.x;
    if (lane == 0)
        for (int r = 0; r < nranks; ++r)
            __hip_atomic_store(peers.p[r] + kMailboxHandshake + rank, token, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
    bool got = lane >= nranks;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    int good = 1;
    for (unsigned it = 0;; ++it) {
        if (!got)
            got = __hip_atomic_load(inbox + kMailboxHandshake + lane, __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_SYSTEM) == token;
        if (__all(got)) break;
        __builtin_amdgcn_s_sleep(2);
        if ((it & 15) == 15 && __any(__builtin_amdgcn_s_memrealtime() - t0 > kFirstRankTimeoutTicks)) {
            good = 0;
            break;
        }
    }
    if (lane == 0) ok[0] = good;
}

hipError_t launch_mailbox_handshake(const MailboxPeers& peers, uint64_t* inbox, int rank,
                                    int nranks, uint64_t token, int* ok, hipStream_t s) {
    hipLaunchKernelGGL(mailbox_handshake, dim3(1), dim3(64), 0, s, peers, inbox, rank, nranks, token, ok);
    return hipGetLastError();
}

}  // namespace st
