// Greedy Stein-thinning step kernels for gfx950 (K1 diag, K2 fused step, K3 argmin finalize).
//
// Replaces the reference's hot loop (stein_thinning.thinning._greedy_search, restated at
// JAX_Stein_Thinning.ipynb cell 22, json ~281-295; Algorithm 3, report.tex:413-426):
//     A = integrand(:, :); idx[0] = argmin(A)
//     for t in 1..m-1:  A += 2 * integrand(:, [idx[t-1]]);  idx[t] = argmin(A)
//
// One launch per greedy step.  Every launch:
//   1. picks the previous step's winner from R rank candidates (lowest value, then lowest global
//      index; NaN counts as minimum -- np.argmin semantics) and stages its row (x_j, g_j, w_j) in LDS;
//   2. streams the candidate columns of this rank's shard (SoA, coalesced 16-B loads, two candidates
//      per lane), evaluates k(x_i, x_j), updates the running sum A_i in place;
//   3. reduces (A_i, i) to one per-block MINLOC; the last block to arrive (agent-scope ticket)
//      reduces the block partials and publishes this rank's candidate {val, gidx, x, g, w} for the
//      next launch (and, for R > 1 ranks, for the RCCL all-gather between launches).
// Inter-workgroup hand-off follows the measured valid form of MI355X_MICROARCH.md (table row 1):
// 8-B agent-scope (sc1) stores, every storing wave drained (s_waitcnt vmcnt(0)) before ONE lane's
// agent-scope atomic add; the last arriver reads with agent-scope (sc1) loads.
#include "stein_math.hpp"
#include "stein_internal.hpp"

namespace st {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

__device__ __forceinline__ void wave_minloc(double& v, int64_t& i) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const double ov = __shfl_xor(v, off, 64);
        const int64_t oi = __shfl_xor(i, off, 64);
        if (better(ov, oi, v, i)) { v = ov; i = oi; }
    }
}

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

__device__ __forceinline__ void store_agent_f64(double* p, double v) {
    __hip_atomic_store(reinterpret_cast<uint64_t*>(p), __double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_agent_f64(const double* p) {
    return __longlong_as_double(__hip_atomic_load(reinterpret_cast<const uint64_t*>(p),
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void store_agent_i64(int64_t* p, int64_t v) {
    __hip_atomic_store(reinterpret_cast<uint64_t*>(p), (uint64_t)v, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int64_t load_agent_i64(const int64_t* p) {
    return (int64_t)__hip_atomic_load(reinterpret_cast<const uint64_t*>(p), __ATOMIC_RELAXED,
                                      __HIP_MEMORY_SCOPE_AGENT);
}

// Select the winner among R candidates (deterministic, identical in every block and rank).
// Stages the winner row {x[d], g[d], w} in s_row; returns the winner's global index.
__device__ __forceinline__ int64_t select_winner(const double* __restrict__ cands, int nranks,
                                                 int d, int64_t stride, double* s_row,
                                                 int64_t* s_gidx) {
    if (threadIdx.x < 64) {
        double v = INFINITY;
        int64_t gi = INT64_MAX;
        if ((int)threadIdx.x < nranks) {
            const double* c = cands + threadIdx.x * stride;
            v = c[0];
            gi = (int64_t)__double_as_longlong(c[1]);
        }
        wave_minloc(v, gi);
        if (threadIdx.x == 0) *s_gidx = gi;
    }
    __syncthreads();
    const int64_t gidx = *s_gidx;
    // which rank slot holds it: the first slot whose gidx matches (gidx unique across ranks)
    int win = 0;
    for (int r = 0; r < nranks; ++r)
        if ((int64_t)__double_as_longlong(cands[r * stride + 1]) == gidx) { win = r; break; }
    const double* row = cands + win * stride + kCandHeader;
    for (int k = threadIdx.x; k < 2 * d + 1; k += kBlock) s_row[k] = row[k];
    __syncthreads();
    return gidx;
}

// Last-arriver epilogue: reduce block partials, publish {val, gidx, x_row, g_row, w} of the
// local best.  Called by every thread of the block that drew the last ticket.
__device__ void publish_rank_candidate(const GreedyArgs& a, double* s_v, int64_t* s_i) {
    double v = INFINITY;
    int64_t li = INT64_MAX;
    for (int b = threadIdx.x; b < (int)gridDim.x; b += kBlock) {
        const double pv = load_agent_f64(a.part_val + b);
        const int64_t pi = load_agent_i64(a.part_idx + b);
        if (better(pv, pi, v, li)) { v = pv; li = pi; }
    }
    block_minloc(v, li, s_v, s_i);
    double* out = a.cand_out;
    if (threadIdx.x == 0) {
        out[0] = v;
        out[1] = __longlong_as_double((long long)(a.row_offset + li));
    }
    const int d = a.d;
    for (int k = threadIdx.x; k < 2 * d + 1; k += kBlock) {
        double val;
        if (k < d) val = a.x[(int64_t)k * a.ld + li];
        else if (k < 2 * d) val = a.g[(int64_t)(k - d) * a.ld + li];
        else val = a.w ? a.w[li] : 1.0;
        out[kCandHeader + k] = val;
    }
}

// Per-block partial -> ticket; returns true in every thread of the last-arriving block.
__device__ __forceinline__ bool arrive(const GreedyArgs& a, double v, int64_t i, int* s_flag) {
    if (threadIdx.x == 0) {
        store_agent_f64(a.part_val + blockIdx.x, v);
        store_agent_i64(a.part_idx + blockIdx.x, i);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned target = (unsigned)((a.t + 1) * (int64_t)gridDim.x - 1);
        const unsigned old = __hip_atomic_fetch_add(a.ticket, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
        *s_flag = (old == target);
    }
    __syncthreads();
    return *s_flag != 0;
}

// ------------------------------------------------------------------------------------------
// K1/K2: compile-time d.  DIAG: A_i = k(x_i, x_i) [w_i^2]; else A_i += 2 k(x_i, x_j) [w_i w_j].
// Two adjacent candidates per lane (16-B loads of the SoA columns), grid-stride.
// ------------------------------------------------------------------------------------------
template <int D, bool GF, bool DIAG>
__global__ __launch_bounds__(kBlock) void greedy_step_ct(GreedyArgs a) {
    __shared__ double s_row[2 * D + 1];
    __shared__ int64_t s_gidx;
    __shared__ double s_v[kWaves];
    __shared__ int64_t s_i[kWaves];
    __shared__ int s_flag;

    double xj[D], gj[D];
    double wj = 1.0;
    if constexpr (!DIAG) {
        const int64_t gw = select_winner(a.cands_in, a.nranks, D, a.cand_stride, s_row, &s_gidx);
        if (blockIdx.x == 0 && threadIdx.x == 0 && a.idx_out) a.idx_out[a.t - 1] = (uint32_t)gw;
#pragma unroll
        for (int k = 0; k < D; ++k) { xj[k] = s_row[k]; gj[k] = s_row[D + k]; }
        if constexpr (GF) wj = s_row[2 * D];
    }

    const int64_t n = a.n, ld = a.ld;
    const double l = a.l, l2 = a.l * a.l, tr = a.tr;
    double best_v = INFINITY;
    int64_t best_i = INT64_MAX;
    const int64_t npairs = (n + 1) >> 1;
    for (int64_t p = (int64_t)blockIdx.x * kBlock + threadIdx.x; p < npairs;
         p += (int64_t)gridDim.x * kBlock) {
        const int64_t i0 = p * 2;
        double x0[D], x1[D], g0[D], g1[D];
#pragma unroll
        for (int k = 0; k < D; ++k) {
            const double2 xv = *reinterpret_cast<const double2*>(a.x + k * ld + i0);
            const double2 gv = *reinterpret_cast<const double2*>(a.g + k * ld + i0);
            x0[k] = xv.x; x1[k] = xv.y; g0[k] = gv.x; g1[k] = gv.y;
        }
        double2 w2 = make_double2(1.0, 1.0);
        if constexpr (GF) w2 = *reinterpret_cast<const double2*>(a.w + i0);
        double k0v, k1v;
        if constexpr (DIAG) {
            k0v = diag_value_ct<D>(g0, tr);
            k1v = diag_value_ct<D>(g1, tr);
            if constexpr (GF) {
                k0v = (k0v * w2.x) * w2.x;
                k1v = (k1v * w2.y) * w2.y;
            }
        } else {
            k0v = pair_value_ct<D>(x0, g0, xj, gj, l, l2, tr);
            k1v = pair_value_ct<D>(x1, g1, xj, gj, l, l2, tr);
            if constexpr (GF) {
                k0v = (k0v * w2.x) * wj;
                k1v = (k1v * w2.y) * wj;
            }
        }
        double2 av;
        if constexpr (DIAG) {
            av = make_double2(k0v, k1v);
        } else {
            av = *reinterpret_cast<const double2*>(a.A + i0);
            av.x = av.x + 2.0 * k0v;
            av.y = av.y + 2.0 * k1v;
        }
        *reinterpret_cast<double2*>(a.A + i0) = av;
        if (better(av.x, i0, best_v, best_i)) { best_v = av.x; best_i = i0; }
        if (i0 + 1 < n && better(av.y, i0 + 1, best_v, best_i)) { best_v = av.y; best_i = i0 + 1; }
    }
    block_minloc(best_v, best_i, s_v, s_i);
    if (arrive(a, best_v, best_i, &s_flag)) publish_rank_candidate(a, s_v, s_i);
}

// ------------------------------------------------------------------------------------------
// Runtime-d variant (any 1 <= d <= 128): one candidate per lane per iteration, selected row in LDS.
// ------------------------------------------------------------------------------------------
template <bool GF, bool DIAG>
__global__ __launch_bounds__(kBlock) void greedy_step_rt(GreedyArgs a) {
    __shared__ double s_row[2 * kMaxDim + 1];
    __shared__ int64_t s_gidx;
    __shared__ double s_v[kWaves];
    __shared__ int64_t s_i[kWaves];
    __shared__ int s_flag;
    const int d = a.d;
    double wj = 1.0;
    if constexpr (!DIAG) {
        const int64_t gw = select_winner(a.cands_in, a.nranks, d, a.cand_stride, s_row, &s_gidx);
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
            kv = pair_value_rt(a.x + i, a.g + i, ld, s_row, s_row + d, 1, d, l, l2, tr);
            if constexpr (GF) kv = (kv * a.w[i]) * wj;
            kv = a.A[i] + 2.0 * kv;
            a.A[i] = kv;
        }
        if (better(kv, i, best_v, best_i)) { best_v = kv; best_i = i; }
    }
    block_minloc(best_v, best_i, s_v, s_i);
    if (arrive(a, best_v, best_i, &s_flag)) publish_rank_candidate(a, s_v, s_i);
}

// K3: after the last step's exchange, write idx[m-1].
__global__ void greedy_finalize(const double* cands, int nranks, int64_t stride, uint32_t* idx_out,
                                int64_t t) {
    double v = INFINITY;
    int64_t gi = INT64_MAX;
    if ((int)threadIdx.x < nranks) {
        v = cands[threadIdx.x * stride];
        gi = (int64_t)__double_as_longlong(cands[threadIdx.x * stride + 1]);
    }
    wave_minloc(v, gi);
    if (threadIdx.x == 0) idx_out[t] = (uint32_t)gi;
}

// ------------------------------------------------------------------------------------------
// host-side launchers
// ------------------------------------------------------------------------------------------
int greedy_blocks(int64_t n, int d) {
    const int64_t per_block = (d <= kMaxCtDim ? 2 : 1) * (int64_t)kBlock;
    int64_t b = (n + per_block - 1) / per_block;
    if (b > kMaxBlocks) b = kMaxBlocks;
    if (b < 1) b = 1;
    return (int)b;
}

template <int D>
static hipError_t launch_ct(const GreedyArgs& a, bool diag, int blocks, hipStream_t s) {
    const bool gf = a.w != nullptr;
    if (diag) {
        if (gf) greedy_step_ct<D, true, true><<<blocks, kBlock, 0, s>>>(a);
        else greedy_step_ct<D, false, true><<<blocks, kBlock, 0, s>>>(a);
    } else {
        if (gf) greedy_step_ct<D, true, false><<<blocks, kBlock, 0, s>>>(a);
        else greedy_step_ct<D, false, false><<<blocks, kBlock, 0, s>>>(a);
    }
    return hipGetLastError();
}

hipError_t launch_greedy_step(const GreedyArgs& a, bool diag, hipStream_t s) {
    const int blocks = greedy_blocks(a.n, a.d);
    switch (a.d) {
        case 1: return launch_ct<1>(a, diag, blocks, s);
        case 2: return launch_ct<2>(a, diag, blocks, s);
        case 3: return launch_ct<3>(a, diag, blocks, s);
        case 4: return launch_ct<4>(a, diag, blocks, s);
        case 5: return launch_ct<5>(a, diag, blocks, s);
        case 6: return launch_ct<6>(a, diag, blocks, s);
        case 7: return launch_ct<7>(a, diag, blocks, s);
        case 8: return launch_ct<8>(a, diag, blocks, s);
        default: break;
    }
    const bool gf = a.w != nullptr;
    if (diag) {
        if (gf) greedy_step_rt<true, true><<<blocks, kBlock, 0, s>>>(a);
        else greedy_step_rt<false, true><<<blocks, kBlock, 0, s>>>(a);
    } else {
        if (gf) greedy_step_rt<true, false><<<blocks, kBlock, 0, s>>>(a);
        else greedy_step_rt<false, false><<<blocks, kBlock, 0, s>>>(a);
    }
    return hipGetLastError();
}

hipError_t launch_greedy_finalize(const double* cands, int nranks, int64_t stride,
                                  uint32_t* idx_out, int64_t t, hipStream_t s) {
    greedy_finalize<<<1, 64, 0, s>>>(cands, nranks, stride, idx_out, t);
    return hipGetLastError();
}

}  // namespace st
