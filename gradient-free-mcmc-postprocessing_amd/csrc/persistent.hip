// Persistent, on-chip-resident greedy kernel (K4) for gfx950.
//
// One cooperative launch runs the whole greedy loop of the reference's _greedy_search
// (JAX_Stein_Thinning.ipynb cell 22, json ~281-295; report.tex:413-426) for one device:
//   * G <= #CU blocks of 256 threads, one per CU.  Block b owns rows [b*R, (b+1)*R).
//   * Its rows live on chip for the whole run: RT rows per thread in VGPRs/AGPRs (x, g, A[, w]),
//     RL rows in LDS (SoA), the remainder streamed from HBM each step (coalesced, like K2).
//   * Per step: every block evaluates k(x_i, x_j) for its rows, A_i += 2k, block MINLOC, and
//     publishes ONE record {A_min, index} as three data-tagged 8-byte granules (tag = step + 1;
//     MI355X_MICROARCH.md recipe R2, "the data IS the flag": no fence, no counter).  One wave per
//     block sweeps all G records until every tag matches, reduces them (np.argmin order) and the
//     block reads the winner's row from the read-only x / g / w arrays -> next step.  Block 0
//     writes idx.  Two record banks alternate by step parity.
//   * Every spin is bounded by a wall-clock timeout (s_memrealtime); a timeout sets status[0] and
//     every block leaves the step loop, so the grid always drains.
// Arithmetic per pair: identical to K2 (stein_math.hpp), so results are bit-identical to st_greedy's
// launch-per-step path and to the C bit model.
#include "stein_math.hpp"
#include "stein_internal.hpp"

namespace st {

namespace {

constexpr int kMaxPWaves = 8;                // up to 512-thread blocks
constexpr int kShards = 8;
constexpr int kMaxGrid = 256;               // one block per CU on MI355X (256 CUs)
constexpr uint64_t kTimeoutTicks = 200000000ull;   // s_memrealtime runs at 100 MHz: 2 s

__device__ __forceinline__ void p_wave_minloc(double& v, int64_t& i) { wave_minloc_dpp(v, i); }

struct Scratch {          // small per-block scratch at the start of the dynamic LDS region
    double row[2 * kMaxCtDim + 2];
    double v[kMaxPWaves];
    int64_t i[kMaxPWaves];
    int abort;
    int pad[3];
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

}  // namespace

struct PersistArgs {
    const double* x;
    const double* g;
    const double* w;
    double* A;
    int64_t n, ld;
    double l, tr;
    int64_t m;            // n_points
    uint32_t* idx_out;
    uint64_t* gran;       // 2 banks x G records x 4 granules (3 used)
    unsigned* status;     // [0]: 0 ok, 1 timeout
    int64_t rows_per_block;
    int RL;               // LDS-resident rows per block
    uint64_t* stamps;     // diagnostic build only (ST_PERSIST_STAMPS): [G][kStampSteps][kStampPhases]
};

// Diagnostic build (-DST_PERSIST_STAMPS, tools/probe only; never the product library): lane 0 of
// every block records s_memrealtime (100 MHz, chip-wide clock) at each phase of steps
// [kStampFirst, kStampFirst + kStampSteps).
[[maybe_unused]] constexpr int kStampFirst = 20, kStampSteps = 32, kStampPhases = 6;
#ifdef ST_PERSIST_STAMPS
#define ST_STAMP(a, t, ph)                                                                         \
    do {                                                                                            \
        if ((a).stamps && threadIdx.x == 0 && (t) >= kStampFirst && (t) < kStampFirst + kStampSteps) \
            (a).stamps[((int64_t)blockIdx.x * kStampSteps + ((t) - kStampFirst)) * kStampPhases + (ph)] = \
                __builtin_amdgcn_s_memrealtime();                                                    \
    } while (0)
#else
#define ST_STAMP(a, t, ph) do { } while (0)
#endif

// Exchange = self-validating granules (MI355X_MICROARCH.md R2: "the data IS the flag"): each block
// publishes {A_min, index} for step t as three 8-byte granules {tag = t+1 : 32-bit payload}
// (value low word, value high word, index), each written by ONE aligned 8-B agent-scope store.
// A consumer accepts a record only when all three tags equal t+1; banks alternate by step parity.
template <int NT>
__device__ __forceinline__ void publish(const PersistArgs& a, Scratch* sc, double v, uint32_t row,
                                        int64_t t) {
    int64_t li = (int64_t)row;   // rows >= n (padding) carry +inf and never win
    p_wave_minloc(v, li);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) { sc->v[wave] = v; sc->i[wave] = li; }
    __syncthreads();
    if (threadIdx.x == 0) {   // ONE lane combines the wave minima and stores the three granules
        v = sc->v[0];
        li = sc->i[0];
#pragma unroll
        for (int w = 1; w < NT / 64; ++w) take_if_better(sc->v[w], sc->i[w], v, li);
        uint64_t* gr = a.gran + ((t & 1) * (int64_t)gridDim.x + blockIdx.x) * 4;
        const uint64_t tag = (uint64_t)(uint32_t)(t + 1) << 32;
        const uint64_t vb = (uint64_t)__double_as_longlong(v);
        const uint32_t ib = li == INT64_MAX ? 0xFFFFFFFFu : (uint32_t)li;
        __hip_atomic_store(gr + 0, tag | (vb & 0xFFFFFFFFull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(gr + 1, tag | (vb >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(gr + 2, tag | ib, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// wave 0 sweeps the G records of step t until every tag is t+1 (bounded), reduces them
// (np.argmin order); then the winner's row is read from the read-only x / g / w arrays into
// sc->row.  Returns the winner's index, or -1 if the sweep timed out (grid-wide abort).
template <int D, bool GF>
__device__ __forceinline__ int64_t wait_and_pick(const PersistArgs& a, Scratch* sc, int64_t t) {
    const int G = gridDim.x;
    ST_STAMP(a, t + 1, 0);
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        const uint64_t* bank = a.gran + (t & 1) * (int64_t)G * 4;
        const uint32_t want = (uint32_t)(t + 1);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        double v = INFINITY;
        int64_t gi = INT64_MAX;
        int ok_all = 1;
        for (unsigned it = 0;; ++it) {
            bool ok = true;
            v = INFINITY;
            gi = INT64_MAX;
#pragma unroll
            for (int c = 0; c < kMaxGrid / 64; ++c) {
                const int r = lane + 64 * c;
                if (r < G) {
                    const uint64_t* gr = bank + (int64_t)r * 4;
                    const uint64_t g0 = __hip_atomic_load(gr + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint64_t g1 = __hip_atomic_load(gr + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const uint64_t g2 = __hip_atomic_load(gr + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    ok &= ((uint32_t)(g0 >> 32) == want) & ((uint32_t)(g1 >> 32) == want) &
                          ((uint32_t)(g2 >> 32) == want);
                    const double rv = __longlong_as_double(
                        (long long)((g1 << 32) | (g0 & 0xFFFFFFFFull)));
                    const uint32_t ib = (uint32_t)g2;
                    const int64_t ri = ib == 0xFFFFFFFFu ? INT64_MAX : (int64_t)ib;
                    if (better(rv, ri, v, gi)) { v = rv; gi = ri; }
                }
            }
            if (__all(ok)) break;
            __builtin_amdgcn_s_sleep(1);
            if ((it & 15) == 15) {
                const bool late = __builtin_amdgcn_s_memrealtime() - t0 > kTimeoutTicks;
                const bool other = __hip_atomic_load(a.status, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT) != 0;
                if (__any(late || other)) { ok_all = 0; break; }
            }
        }
        ST_STAMP(a, t + 1, 1);
        p_wave_minloc(v, gi);
        if (lane == 0) {
            if (!ok_all) __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sc->abort = !ok_all;
            sc->i[0] = gi;
        }
    }
    __syncthreads();
    if (sc->abort) return -1;
    const int64_t gi = sc->i[0];
    const int k = threadIdx.x;
    if (k < 2 * D + (GF ? 1 : 0)) {
        double val;
        if (k < D) val = a.x[(int64_t)k * a.ld + gi];
        else if (k < 2 * D) val = a.g[(int64_t)(k - D) * a.ld + gi];
        else val = a.w[gi];
        sc->row[k] = val;
    }
    __syncthreads();
    ST_STAMP(a, t + 1, 2);
    return gi;
}

template <int D, bool GF, int RT, int NT>
__global__ __launch_bounds__(NT, 1) void greedy_persistent(PersistArgs a) {
    constexpr int kPBlock = NT;
    extern __shared__ __attribute__((aligned(16))) double lds[];
    Scratch* sc = reinterpret_cast<Scratch*>(lds);
    const int RL = a.RL;
    double* sx = lds + (sizeof(Scratch) + 15) / 16 * 2;   // [D][RL]
    double* sg = sx + (int64_t)D * RL;                       // [D][RL]
    double* sa = sg + (int64_t)D * RL;                       // [RL]
    double* sw = sa + RL;                                     // [RL] (GF)
    const int tid = threadIdx.x;
    const int64_t ld = a.ld;
    const int64_t r0 = (int64_t)blockIdx.x * a.rows_per_block;
    const int64_t r1 = (r0 + a.rows_per_block < a.n) ? r0 + a.rows_per_block : a.n;
    const int64_t lds_base = r0 + (int64_t)RT * kPBlock;
    const int64_t str_base = lds_base + RL;
    const double l = a.l, l2 = a.l * a.l, tr = a.tr;

    // ---- stage the block's rows on chip ----------------------------------------------------
    double xr[RT > 0 ? RT : 1][D], gr[RT > 0 ? RT : 1][D], ar[RT > 0 ? RT : 1];
    double wr[(GF && RT > 0) ? RT : 1];
#pragma unroll
    for (int q = 0; q < RT; ++q) {
        const int64_t row = r0 + (int64_t)q * kPBlock + tid;
        const bool ok = row < r1;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            xr[q][k] = ok ? a.x[k * ld + row] : 0.0;
            gr[q][k] = ok ? a.g[k * ld + row] : 0.0;
        }
        if constexpr (GF) wr[q] = ok ? a.w[row] : 0.0;
    }
    for (int e = tid; e < RL; e += kPBlock) {
        const int64_t row = lds_base + e;
        const bool ok = row < r1;
#pragma unroll
        for (int k = 0; k < D; ++k) {
            sx[k * RL + e] = ok ? a.x[k * ld + row] : 0.0;
            sg[k * RL + e] = ok ? a.g[k * ld + row] : 0.0;
        }
        if constexpr (GF) sw[e] = ok ? a.w[row] : 0.0;
    }
    __syncthreads();

    // ---- step 0: diagonal --------------------------------------------------------------------
    // running best of this thread: starts at its first row (register row 0, which precedes all its
    // other rows); an out-of-range row contributes +inf with its (>= n) index and never wins
    double bv = INFINITY;
    uint32_t bi = (uint32_t)(r0 + tid);
#pragma unroll
    for (int q = 0; q < RT; ++q) {
        const int64_t row = r0 + (int64_t)q * kPBlock + tid;
        double kv = diag_value_ct<D>(gr[q], tr);
        if constexpr (GF) kv = (kv * wr[q]) * wr[q];
        ar[q] = kv;
        const double cand = row < r1 ? kv : INFINITY;
        if (q == 0) { bv = cand; bi = (uint32_t)row; } else scan_take(cand, (uint32_t)row, bv, bi);
    }
    for (int e = tid; e < RL; e += kPBlock) {
        const int64_t row = lds_base + e;
        double gi[D];
#pragma unroll
        for (int k = 0; k < D; ++k) gi[k] = sg[k * RL + e];
        double kv = diag_value_ct<D>(gi, tr);
        if constexpr (GF) kv = (kv * sw[e]) * sw[e];
        sa[e] = kv;
        scan_take(row < r1 ? kv : INFINITY, (uint32_t)row, bv, bi);
    }
    for (int64_t row = str_base + tid; row < r1; row += kPBlock) {
        double gi[D];
#pragma unroll
        for (int k = 0; k < D; ++k) gi[k] = a.g[k * ld + row];
        double kv = diag_value_ct<D>(gi, tr);
        if constexpr (GF) kv = (kv * a.w[row]) * a.w[row];
        a.A[row] = kv;
        scan_take(kv, (uint32_t)row, bv, bi);
    }
    publish<NT>(a, sc, bv, bi, 0);

    // ---- steps 1 .. m-1 ----------------------------------------------------------------------
    int64_t t = 1;
    for (; t < a.m; ++t) {
        const int64_t win = wait_and_pick<D, GF>(a, sc, t - 1);
        if (win < 0) break;
        if (blockIdx.x == 0 && tid == 0) a.idx_out[t - 1] = (uint32_t)win;
        double xj[D], gj[D];
#pragma unroll
        for (int k = 0; k < D; ++k) { xj[k] = sc->row[k]; gj[k] = sc->row[D + k]; }
        const double wj = GF ? sc->row[2 * D] : 1.0;
        // first streamed row: issue its loads now, they land while the on-chip rows compute
        int64_t srow = str_base + tid;
        bool have = srow < r1;
        double nx[D], ng[D], na = 0.0, nw = 1.0;
        if (have) {
#pragma unroll
            for (int k = 0; k < D; ++k) { nx[k] = a.x[k * ld + srow]; ng[k] = a.g[k * ld + srow]; }
            na = a.A[srow];
            if constexpr (GF) nw = a.w[srow];
        }
#pragma unroll
        for (int q = 0; q < RT; ++q) {
            const int64_t row = r0 + (int64_t)q * kPBlock + tid;
            double kv = pair_value_ct<D>(xr[q], gr[q], xj, gj, l, l2, tr);
            if constexpr (GF) kv = (kv * wr[q]) * wj;
            ar[q] = ar[q] + 2.0 * kv;
            const double cand = row < r1 ? ar[q] : INFINITY;
            if (q == 0) { bv = cand; bi = (uint32_t)row; } else scan_take(cand, (uint32_t)row, bv, bi);
        }
        for (int e = tid; e < RL; e += kPBlock) {
            const int64_t row = lds_base + e;
            double xi[D], gi[D];
#pragma unroll
            for (int k = 0; k < D; ++k) { xi[k] = sx[k * RL + e]; gi[k] = sg[k * RL + e]; }
            double kv = pair_value_ct<D>(xi, gi, xj, gj, l, l2, tr);
            if constexpr (GF) kv = (kv * sw[e]) * wj;
            const double av = sa[e] + 2.0 * kv;
            sa[e] = av;
            scan_take(row < r1 ? av : INFINITY, (uint32_t)row, bv, bi);
        }
        while (have) {   // streamed rows, one row of loads kept in flight ahead of the compute
            double xi[D], gi[D];
#pragma unroll
            for (int k = 0; k < D; ++k) { xi[k] = nx[k]; gi[k] = ng[k]; }
            const double ai = na, wi = nw;
            const int64_t row = srow;
            srow += kPBlock;
            have = srow < r1;
            if (have) {
#pragma unroll
                for (int k = 0; k < D; ++k) { nx[k] = a.x[k * ld + srow]; ng[k] = a.g[k * ld + srow]; }
                na = a.A[srow];
                if constexpr (GF) nw = a.w[srow];
            }
            double kv = pair_value_ct<D>(xi, gi, xj, gj, l, l2, tr);
            if constexpr (GF) kv = (kv * wi) * wj;
            const double av = ai + 2.0 * kv;
            a.A[row] = av;
            scan_take(av, (uint32_t)row, bv, bi);
        }
        ST_STAMP(a, t, 3);
        publish<NT>(a, sc, bv, bi, t);
        ST_STAMP(a, t, 4);
    }
    int64_t done = t;   // idx[0 .. done-1) are written
    if (t == a.m) {
        const int64_t win = wait_and_pick<D, GF>(a, sc, a.m - 1);
        if (win >= 0) {
            if (blockIdx.x == 0 && tid == 0) a.idx_out[a.m - 1] = (uint32_t)win;
            done = a.m + 1;
        }
    }
    // timeout: poison the unwritten indices (UINT32_MAX) so the host detects the failure
    if (done <= a.m && blockIdx.x == 0)
        for (int64_t q = (done > 0 ? done - 1 : 0) + tid; q < a.m; q += kPBlock) a.idx_out[q] = 0xFFFFFFFFu;

    // ---- write the on-chip running sums back (A_out contract of st_greedy) --------------------
#pragma unroll
    for (int q = 0; q < RT; ++q) {
        const int64_t row = r0 + (int64_t)q * kPBlock + tid;
        if (row < r1) a.A[row] = ar[q];
    }
    for (int e = tid; e < RL; e += kPBlock) {
        const int64_t row = lds_base + e;
        if (row < r1) a.A[row] = sa[e];
    }
}

// ------------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------------
int64_t persistent_ws_bytes(int d, int G) {
    // [control: status (and reserved) words][2 banks x G records x 4 granules of 8 B]
    (void)d;
    return kWsControlBytes + 2 * (int64_t)G * 4 * 8;
}

static int g_persist_rt = -1;   // st_tune key 3: -1 auto, 0 = off
static int g_persist_nt = -1;   // st_tune key 4: threads per block, -1 auto (256)
static uint64_t* g_stamps = nullptr;
#ifdef ST_PERSIST_STAMPS
extern "C" int st_debug_set_stamps(uint64_t* buf) { g_stamps = buf; return 0; }
#endif
int persistent_tune(int key, int value) {
    if (key == 3) {
        if (value < -1 || value > 64) return -1;
        g_persist_rt = value;
        return 0;
    }
    if (key == 4) {
        if (value != -1 && value != 256 && value != 512) return -1;
        g_persist_nt = value;
        return 0;
    }
    return -1;
}

template <int D, bool GF, int RT, int NT>
static hipError_t launch_p(const PersistArgs& a, int G, size_t lds, hipStream_t s) {
    auto fn = greedy_persistent<D, GF, RT, NT>;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    PersistArgs args = a;
    void* kargs[] = {&args};
    return hipLaunchCooperativeKernel(reinterpret_cast<const void*>(fn), dim3(G), dim3(NT), kargs,
                                      lds, s);
}

template <int D, bool GF>
static hipError_t launch_p_rt(const PersistArgs& a, int rt, int nt, int G, size_t lds, hipStream_t s) {
    if (nt == 512) {
        if (rt <= 4) return launch_p<D, GF, 4, 512>(a, G, lds, s);
        return launch_p<D, GF, 8, 512>(a, G, lds, s);
    }
    switch (rt) {
        case 4: return launch_p<D, GF, 4, 256>(a, G, lds, s);
        case 8: return launch_p<D, GF, 8, 256>(a, G, lds, s);
        default: return launch_p<D, GF, 16, 256>(a, G, lds, s);
    }
}

// Returns hipErrorNotSupported when the persistent path does not apply (caller falls back).
hipError_t launch_greedy_persistent(const double* x, const double* g, const double* w, double* A,
                                    int64_t n, int d, int64_t ld, double l, double tr, int64_t m,
                                    uint32_t* idx_out, void* ws, int64_t ws_bytes, hipStream_t s,
                                    int* used) {
    *used = 0;
    if (g_persist_rt == 0 || (d != 2 && d != 4) || m < 1 || m >= 0xFFFFFFFFll || n >= 0xFFFFFFFFll)
        return hipErrorNotSupported;
    int dev = 0, cus = 0, lds_max = 0, lds_optin = 0, coop = 0;
    if (hipGetDevice(&dev) != hipSuccess) return hipErrorNotSupported;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return hipErrorNotSupported;
    if (hipDeviceGetAttribute(&coop, hipDeviceAttributeCooperativeLaunch, dev) != hipSuccess || !coop)
        return hipErrorNotSupported;
    if (hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess)
        return hipErrorNotSupported;
    if (hipDeviceGetAttribute(&lds_optin, hipDeviceAttributeSharedMemPerBlockOptin, dev) == hipSuccess &&
        lds_optin > lds_max)
        lds_max = lds_optin;
    if (lds_max > 163840) lds_max = 163840;
    int G = cus > kMaxGrid ? kMaxGrid : cus;
    const int64_t min_rows = 256;   // fewer blocks for small n: exchange cost grows with G
    if (n < (int64_t)G * min_rows) G = (int)((n + min_rows - 1) / min_rows);
    if (G < 1) G = 1;
    if (persistent_ws_bytes(d, G) > ws_bytes) return hipErrorNotSupported;
    const int64_t R = (n + G - 1) / G;
    const int nt = g_persist_nt > 0 ? g_persist_nt : 256;
    const int rt_max = nt == 512 ? 8 : 16;
    int rt = g_persist_rt > 0 ? g_persist_rt : rt_max;
    if (rt != 4 && rt != 8 && rt != 16) rt = rt_max;
    if (rt > rt_max) rt = rt_max;
    while (rt > 4 && (int64_t)rt * nt > R) rt /= 2;   // do not hold empty register rows
    const bool gf = w != nullptr;
    const size_t row_bytes = (size_t)(2 * d + 1 + (gf ? 1 : 0)) * sizeof(double);
    const size_t head = (sizeof(Scratch) + 15) / 16 * 16;
    const size_t budget = (size_t)(lds_max > 0 ? lds_max : 65536) - 1024;   // static + slack
    int64_t RL = (int64_t)((budget - head) / row_bytes);
    const int64_t need = R - (int64_t)rt * nt;
    if (RL > need) RL = need > 0 ? need : 0;
    RL = RL / 64 * 64;
    if (RL < 0) RL = 0;
    const size_t lds = head + (size_t)RL * row_bytes;

    char* p = static_cast<char*>(ws);
    PersistArgs a{};
    a.x = x; a.g = g; a.w = w; a.A = A;
    a.n = n; a.ld = ld; a.l = l; a.tr = tr; a.m = m;
    a.idx_out = idx_out;
    a.status = reinterpret_cast<unsigned*>(p + kShards * 128);
    a.gran = reinterpret_cast<uint64_t*>(p + kWsControlBytes);
    a.rows_per_block = R;
    a.RL = (int)RL;
    a.stamps = g_stamps;
    // zero status and every granule tag (a stale tag from a previous run must never match)
    hipError_t e = hipMemsetAsync(p, 0, (size_t)persistent_ws_bytes(d, G), s);
    if (e != hipSuccess) return e;
    if (d == 2) e = gf ? launch_p_rt<2, true>(a, rt, nt, G, lds, s) : launch_p_rt<2, false>(a, rt, nt, G, lds, s);
    else e = gf ? launch_p_rt<4, true>(a, rt, nt, G, lds, s) : launch_p_rt<4, false>(a, rt, nt, G, lds, s);
    if (e == hipSuccess) *used = 1;
    return e;
}


}  // namespace st
