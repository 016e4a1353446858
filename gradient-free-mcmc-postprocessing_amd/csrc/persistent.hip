// Persistent, on-chip-resident greedy kernel (K4) for gfx950.
//
// One cooperative launch runs the whole greedy loop of the reference's _greedy_search
// (JAX_Stein_Thinning.ipynb cell 22, json ~281-295; report.tex:413-426) for one device:
//   * G <= #CU blocks of 256 threads, one per CU.  Block b owns rows [b*R, (b+1)*R).
//   * Its rows live on chip for the whole run: RT rows per thread in VGPRs/AGPRs (x, g, A[, w]),
//     RL rows in LDS (SoA), the remainder streamed from HBM each step (coalesced, like K2).
//   * Per step: every block evaluates k(x_i, x_j) for its rows, A_i += 2k, block MINLOC, and
//     publishes ONE record {A_min, index} into a two-bank SoA record array; it then signals an
//     arrival counter sharded by blockIdx % 8 (8 counters on separate 128-B lines).  Every block
//     waits until all arrivals of the step are visible (8 lanes poll the 8 shards together), reads
//     the G records (coalesced), picks the same winner (np.argmin order) and reads the winner's
//     row from the read-only x / g / w arrays -> next step.  Block 0 writes idx.
//   * Hand-off form = MI355X_MICROARCH.md "Valid forms", table row 1: payload written by ONE wave
//     with 8-B agent-scope (sc1) stores, that wave drains vmcnt(0), then ONE lane's agent-scope
//     atomic add; the consumer polls with sc1 loads, joins a workgroup barrier, reads with sc1 loads.
//   * Every spin is bounded by a wall-clock timeout (s_memrealtime); a timeout sets status[0] and
//     every block leaves the step loop, so the grid always drains.
// Arithmetic per pair: identical to K2 (stein_math.hpp), so results are bit-identical to st_greedy's
// launch-per-step path and to the C bit model.
#include "stein_math.hpp"
#include "stein_internal.hpp"

namespace st {

namespace {

constexpr int kPBlock = 256;
constexpr int kPWaves = kPBlock / 64;
constexpr int kShards = 8;
constexpr int kShardStride = 32;            // u32 words between counters (128 B)
constexpr uint64_t kTimeoutTicks = 200000000ull;   // s_memrealtime runs at 100 MHz: 2 s

__device__ __forceinline__ void st_f64(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<uint64_t*>(p), (uint64_t)__double_as_longlong(v),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_f64(const double* p) {
    return __longlong_as_double((long long)__hip_atomic_load(reinterpret_cast<const uint64_t*>(p),
                                                             __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT));
}

__device__ __forceinline__ void p_wave_minloc(double& v, int64_t& i) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double ov = __shfl_xor(v, off, 64);
        const int64_t oi = __shfl_xor(i, off, 64);
        if (better(ov, oi, v, i)) { v = ov; i = oi; }
    }
}

__device__ __forceinline__ void p_block_minloc(double& v, int64_t& i, double* s_v, int64_t* s_i) {
    p_wave_minloc(v, i);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) { s_v[wave] = v; s_i[wave] = i; }
    __syncthreads();
    v = s_v[0]; i = s_i[0];
#pragma unroll
    for (int w = 1; w < kPWaves; ++w)
        if (better(s_v[w], s_i[w], v, i)) { v = s_v[w]; i = s_i[w]; }
    __syncthreads();
}

struct Scratch {          // small per-block scratch at the start of the dynamic LDS region
    double row[2 * kMaxCtDim + 2];
    double v[kPWaves];
    int64_t i[kPWaves];
    int abort;
    int pad[3];
};

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
    double* rec_val;      // 2 banks x G: block minima
    int64_t* rec_idx;     // 2 banks x G: their row indices
    unsigned* counters;   // kShards counters, kShardStride words apart
    unsigned* status;     // [0]: 0 ok, 1 timeout
    int64_t rows_per_block;
    int RL;               // LDS-resident rows per block
};

// publish this block's {A_min, index} for step t (bank t & 1) and signal its arrival
__device__ __forceinline__ void publish(const PersistArgs& a, Scratch* sc, double v, int64_t li,
                                        int64_t t) {
    p_block_minloc(v, li, sc->v, sc->i);
    if (threadIdx.x == 0) {   // ONE lane stores the record, drains, signals
        const int64_t slot = (t & 1) * (int64_t)gridDim.x + blockIdx.x;
        st_f64(a.rec_val + slot, v);
        __hip_atomic_store(reinterpret_cast<uint64_t*>(a.rec_idx + slot), (uint64_t)li,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_fetch_add(a.counters + (blockIdx.x % kShards) * kShardStride, 1u,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

// wait until every block has published step t, reduce the G records (np.argmin order) and stage
// the winner's row (read-only x, g, w) in sc->row.  Returns the winner's index, -1 on timeout.
template <int D, bool GF>
__device__ __forceinline__ int64_t wait_and_pick(const PersistArgs& a, Scratch* sc, int64_t t) {
    const int G = gridDim.x;
    if (threadIdx.x < 64) {   // wave 0: lane s polls shard s; all shards in flight together
        const int lane = threadIdx.x;
        const unsigned ns = lane < kShards ? (unsigned)((G - lane + kShards - 1) / kShards) : 0u;
        const unsigned want = ns * (unsigned)(t + 1);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        int ok = 1;
        for (unsigned it = 0;; ++it) {
            const unsigned c = lane < kShards
                                   ? __hip_atomic_load(a.counters + lane * kShardStride, __ATOMIC_RELAXED,
                                                       __HIP_MEMORY_SCOPE_AGENT)
                                   : 0u;
            if (__all(c >= want)) break;
            __builtin_amdgcn_s_sleep(1);
            if ((it & 31) == 31) {
                const bool late = __builtin_amdgcn_s_memrealtime() - t0 > kTimeoutTicks;
                const bool other = __hip_atomic_load(a.status, __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT) != 0;
                if (late || other) { ok = 0; break; }
            }
        }
        if (lane == 0) {
            if (!ok) __hip_atomic_store(a.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            sc->abort = !ok;
        }
    }
    __syncthreads();
    if (sc->abort) return -1;
    const int64_t base = (t & 1) * (int64_t)G;
    double v = INFINITY;
    int64_t gi = INT64_MAX;
    for (int r = threadIdx.x; r < G; r += kPBlock) {
        const double rv = ld_f64(a.rec_val + base + r);
        const int64_t ri = (int64_t)__hip_atomic_load(reinterpret_cast<const uint64_t*>(a.rec_idx + base + r),
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (better(rv, ri, v, gi)) { v = rv; gi = ri; }
    }
    p_block_minloc(v, gi, sc->v, sc->i);
    const int k = threadIdx.x;
    if (k < 2 * D + (GF ? 1 : 0)) {
        double val;
        if (k < D) val = a.x[(int64_t)k * a.ld + gi];
        else if (k < 2 * D) val = a.g[(int64_t)(k - D) * a.ld + gi];
        else val = a.w[gi];
        sc->row[k] = val;
    }
    __syncthreads();
    return gi;
}

template <int D, bool GF, int RT>
__global__ __launch_bounds__(kPBlock, 1) void greedy_persistent(PersistArgs a) {
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
    double bv = INFINITY;
    int64_t bi = INT64_MAX;
#pragma unroll
    for (int q = 0; q < RT; ++q) {
        const int64_t row = r0 + (int64_t)q * kPBlock + tid;
        double kv = diag_value_ct<D>(gr[q], tr);
        if constexpr (GF) kv = (kv * wr[q]) * wr[q];
        ar[q] = kv;
        if (row < r1 && better(kv, row, bv, bi)) { bv = kv; bi = row; }
    }
    for (int e = tid; e < RL; e += kPBlock) {
        const int64_t row = lds_base + e;
        double gi[D];
#pragma unroll
        for (int k = 0; k < D; ++k) gi[k] = sg[k * RL + e];
        double kv = diag_value_ct<D>(gi, tr);
        if constexpr (GF) kv = (kv * sw[e]) * sw[e];
        sa[e] = kv;
        if (row < r1 && better(kv, row, bv, bi)) { bv = kv; bi = row; }
    }
    for (int64_t row = str_base + tid; row < r1; row += kPBlock) {
        double gi[D];
#pragma unroll
        for (int k = 0; k < D; ++k) gi[k] = a.g[k * ld + row];
        double kv = diag_value_ct<D>(gi, tr);
        if constexpr (GF) kv = (kv * a.w[row]) * a.w[row];
        a.A[row] = kv;
        if (better(kv, row, bv, bi)) { bv = kv; bi = row; }
    }
    publish(a, sc, bv, bi, 0);

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
        bv = INFINITY;
        bi = INT64_MAX;
#pragma unroll
        for (int q = 0; q < RT; ++q) {
            const int64_t row = r0 + (int64_t)q * kPBlock + tid;
            double kv = pair_value_ct<D>(xr[q], gr[q], xj, gj, l, l2, tr);
            if constexpr (GF) kv = (kv * wr[q]) * wj;
            ar[q] = ar[q] + 2.0 * kv;
            if (row < r1 && better(ar[q], row, bv, bi)) { bv = ar[q]; bi = row; }
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
            if (row < r1 && better(av, row, bv, bi)) { bv = av; bi = row; }
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
            if (better(av, row, bv, bi)) { bv = av; bi = row; }
        }
        publish(a, sc, bv, bi, t);
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
    // [control: counters 8 x 128 B + status 128 B][2 x G values][2 x G indices]
    (void)d;
    return kWsControlBytes + 4 * (int64_t)G * 8;
}

static int g_persist_rt = -1;   // st_tune key 3: -1 auto, 0 = off
int persistent_tune(int value) {
    if (value < -1 || value > 64) return -1;
    g_persist_rt = value;
    return 0;
}

template <int D, bool GF, int RT>
static hipError_t launch_p(const PersistArgs& a, int G, size_t lds, hipStream_t s) {
    auto fn = greedy_persistent<D, GF, RT>;
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    PersistArgs args = a;
    void* kargs[] = {&args};
    return hipLaunchCooperativeKernel(reinterpret_cast<const void*>(fn), dim3(G), dim3(kPBlock),
                                      kargs, lds, s);
}

template <int D, bool GF>
static hipError_t launch_p_rt(const PersistArgs& a, int rt, int G, size_t lds, hipStream_t s) {
    switch (rt) {
        case 4: return launch_p<D, GF, 4>(a, G, lds, s);
        case 8: return launch_p<D, GF, 8>(a, G, lds, s);
        default: return launch_p<D, GF, 16>(a, G, lds, s);
    }
}

// Returns hipErrorNotSupported when the persistent path does not apply (caller falls back).
hipError_t launch_greedy_persistent(const double* x, const double* g, const double* w, double* A,
                                    int64_t n, int d, int64_t ld, double l, double tr, int64_t m,
                                    uint32_t* idx_out, void* ws, int64_t ws_bytes, hipStream_t s,
                                    int* used) {
    *used = 0;
    if (g_persist_rt == 0 || (d != 2 && d != 4) || m < 1) return hipErrorNotSupported;
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
    int G = cus > kMaxBlocks ? kMaxBlocks : cus;
    const int64_t min_rows = 256;   // fewer blocks for small n: exchange cost grows with G
    if (n < (int64_t)G * min_rows) G = (int)((n + min_rows - 1) / min_rows);
    if (G < 1) G = 1;
    if (persistent_ws_bytes(d, G) > ws_bytes) return hipErrorNotSupported;
    const int64_t R = (n + G - 1) / G;
    int rt = g_persist_rt > 0 ? g_persist_rt : 16;
    if (rt != 4 && rt != 8 && rt != 16) rt = 16;
    while (rt > 4 && (int64_t)rt * kPBlock > R) rt /= 2;   // do not hold empty register rows
    const bool gf = w != nullptr;
    const size_t row_bytes = (size_t)(2 * d + 1 + (gf ? 1 : 0)) * sizeof(double);
    const size_t head = (sizeof(Scratch) + 15) / 16 * 16;
    const size_t budget = (size_t)(lds_max > 0 ? lds_max : 65536) - 1024;   // static + slack
    int64_t RL = (int64_t)((budget - head) / row_bytes);
    const int64_t need = R - (int64_t)rt * kPBlock;
    if (RL > need) RL = need > 0 ? need : 0;
    RL = RL / 64 * 64;
    if (RL < 0) RL = 0;
    const size_t lds = head + (size_t)RL * row_bytes;

    char* p = static_cast<char*>(ws);
    PersistArgs a{};
    a.x = x; a.g = g; a.w = w; a.A = A;
    a.n = n; a.ld = ld; a.l = l; a.tr = tr; a.m = m;
    a.idx_out = idx_out;
    a.counters = reinterpret_cast<unsigned*>(p);
    a.status = reinterpret_cast<unsigned*>(p + kShards * 128);
    a.rec_val = reinterpret_cast<double*>(p + kWsControlBytes);
    a.rec_idx = reinterpret_cast<int64_t*>(p + kWsControlBytes + 2 * (int64_t)G * 8);
    a.rows_per_block = R;
    a.RL = (int)RL;
    hipError_t e = hipMemsetAsync(p, 0, kWsControlBytes, s);
    if (e != hipSuccess) return e;
    if (d == 2) e = gf ? launch_p_rt<2, true>(a, rt, G, lds, s) : launch_p_rt<2, false>(a, rt, G, lds, s);
    else e = gf ? launch_p_rt<4, true>(a, rt, G, lds, s) : launch_p_rt<4, false>(a, rt, G, lds, s);
    if (e == hipSuccess) *used = 1;
    return e;
}


}  // namespace st
