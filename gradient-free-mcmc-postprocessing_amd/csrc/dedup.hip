// Repeated-row compaction for the greedy selection (stein_thinning.device.DeviceProblem.dedup_view).
//
// A row of an MCMC sample that repeats the row before it bit for bit (a rejected proposal) has the
// same pair values, hence the same running sum, as the first row of its run at every step, and loses
// every tie to that row's lower index (np.argmin order in the reference's _greedy_search, restated at
// JAX_Stein_Thinning.ipynb:281-295, lines 291-292 the running sum and the argmin): it is never
// selected.  Thinning only
// the run starts and mapping the winners back selects the same rows with a fraction of the pair work
// (about a quarter of the rows of a random-walk chain at acceptance ~0.23).
//
// Three launches, HBM-bound (each reads the SoA arrays once; d = 4: 72 B per row):
//   run_flags_kernel  -- starts[i] = (i == 0 or row i != row i-1 in some bit of x, g, w), and the
//                        number of starts per 1024-row tile;
//   tile_scan_kernel  -- one block: exclusive scan of the tile counts -> tile offsets, total count;
//   run_compact_kernel -- every run start scattered to its compact position (row order kept), its
//                        source row index beside it, and the padding rows [count, ld_out) zeroed.
// The host reads the count between the second and the third launch (it sizes the compact arrays).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "stein_internal.hpp"

namespace st {

namespace {

constexpr int kRunBlock = 256;
constexpr int kRunRowsPerThread = 4;
constexpr int kRunTile = kRunBlock * kRunRowsPerThread;   // rows per block
constexpr int kScanBlock = 1024;

__device__ inline bool rows_differ(const double* __restrict__ x, const double* __restrict__ g,
                                   const double* __restrict__ w, int64_t ld, int d, int64_t i) {
    const uint64_t* xu = reinterpret_cast<const uint64_t*>(x);
    const uint64_t* gu = reinterpret_cast<const uint64_t*>(g);
    bool diff = false;
    for (int k = 0; k < d; ++k) {
        const int64_t o = (int64_t)k * ld + i;
        diff |= (xu[o] != xu[o - 1]) | (gu[o] != gu[o - 1]);
    }
    if (w) {
        const uint64_t* wu = reinterpret_cast<const uint64_t*>(w);
        diff |= wu[i] != wu[i - 1];
    }
    return diff;
}

// block-wide sum of one int per thread (kRunBlock threads, 4 waves)
__device__ inline int block_sum(int v, int* sh) {
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    const int wave = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) sh[wave] = v;
    __syncthreads();
    int s = 0;
    for (int q = 0; q < kRunBlock / 64; ++q) s += sh[q];
    return s;
}

__global__ __launch_bounds__(kRunBlock) void run_flags_kernel(const double* __restrict__ x,
                                                              const double* __restrict__ g,
                                                              const double* __restrict__ w, int64_t n,
                                                              int64_t ld, int d, uint8_t* __restrict__ starts,
                                                              int32_t* __restrict__ tile_count) {
    __shared__ int sh[kRunBlock / 64];
    const int64_t base = (int64_t)blockIdx.x * kRunTile;
    int c = 0;
#pragma unroll
    for (int j = 0; j < kRunRowsPerThread; ++j) {
        const int64_t i = base + j * kRunBlock + threadIdx.x;
        if (i < n) {
            const bool s = i == 0 || rows_differ(x, g, w, ld, d, i);
            starts[i] = s ? 1 : 0;
            c += s ? 1 : 0;
        }
    }
    const int total = block_sum(c, sh);
    if (threadIdx.x == 0) tile_count[blockIdx.x] = total;
}

// exclusive scan of ntiles counts in one block; total -> *count
__global__ __launch_bounds__(kScanBlock) void tile_scan_kernel(const int32_t* __restrict__ tile_count,
                                                               int64_t ntiles, int32_t* __restrict__ tile_off,
                                                               int64_t* __restrict__ count) {
    __shared__ int64_t wsum[kScanBlock / 64];
    __shared__ int64_t carry_sh;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t carry = 0;
    for (int64_t b0 = 0; b0 < ntiles; b0 += kScanBlock) {
        const int64_t b = b0 + threadIdx.x;
        const int64_t v = b < ntiles ? tile_count[b] : 0;
        int64_t incl = v;   // inclusive wave scan
        for (int off = 1; off < 64; off <<= 1) {
            const int64_t o = __shfl_up(incl, off);
            if (lane >= off) incl += o;
        }
        if (lane == 63) wsum[wave] = incl;
        __syncthreads();
        int64_t before = carry;
        for (int q = 0; q < wave; ++q) before += wsum[q];
        if (b < ntiles) tile_off[b] = (int32_t)(before + incl - v);
        if (threadIdx.x == kScanBlock - 1) carry_sh = before + incl;
        __syncthreads();
        carry = carry_sh;
        __syncthreads();
    }
    if (threadIdx.x == 0) count[0] = carry;
}

__global__ __launch_bounds__(kRunBlock) void run_compact_kernel(
    const double* __restrict__ x, const double* __restrict__ g, const double* __restrict__ w, int64_t n,
    int64_t ld, int d, const uint8_t* __restrict__ starts, const int32_t* __restrict__ tile_off,
    int64_t count, int64_t ld_out, double* __restrict__ xo, double* __restrict__ go, double* __restrict__ wo,
    int32_t* __restrict__ rows_out) {
    __shared__ int wcnt[kRunBlock / 64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t base = (int64_t)blockIdx.x * kRunTile;
    int64_t pos0 = tile_off[blockIdx.x];
    for (int j = 0; j < kRunRowsPerThread; ++j) {   // rows in order: j-major, then thread
        const int64_t i = base + j * kRunBlock + threadIdx.x;
        const bool s = i < n && starts[i] != 0;
        const uint64_t bal = __ballot(s);
        const int before_lane = __popcll(bal & ((1ull << lane) - 1ull));
        if (lane == 0) wcnt[wave] = __popcll(bal);
        __syncthreads();
        int before_wave = 0, all = 0;
        for (int q = 0; q < kRunBlock / 64; ++q) {
            before_wave += q < wave ? wcnt[q] : 0;
            all += wcnt[q];
        }
        if (s) {
            const int64_t p = pos0 + before_wave + before_lane;
            for (int k = 0; k < d; ++k) {
                xo[(int64_t)k * ld_out + p] = x[(int64_t)k * ld + i];
                go[(int64_t)k * ld_out + p] = g[(int64_t)k * ld + i];
            }
            if (w) wo[p] = w[i];
            rows_out[p] = (int32_t)i;
        }
        pos0 += all;
        __syncthreads();
    }
    // padding rows of the compact arrays (the kernels' lane-pair loads read up to ld_out): zeros
    if (blockIdx.x == 0) {
        for (int64_t p = count + threadIdx.x; p < ld_out; p += kRunBlock) {
            for (int k = 0; k < d; ++k) {
                xo[(int64_t)k * ld_out + p] = 0.0;
                go[(int64_t)k * ld_out + p] = 0.0;
            }
            if (w) wo[p] = 0.0;
        }
    }
}

}  // namespace

int64_t run_tiles(int64_t n) { return (n + kRunTile - 1) / kRunTile; }

hipError_t launch_run_starts(const double* x, const double* g, const double* w, int64_t n, int d, int64_t ld,
                             uint8_t* starts, int32_t* tile_count, int32_t* tile_off, int64_t* count,
                             hipStream_t s) {
    const int64_t tiles = run_tiles(n);
    run_flags_kernel<<<(unsigned)tiles, kRunBlock, 0, s>>>(x, g, w, n, ld, d, starts, tile_count);
    tile_scan_kernel<<<1, kScanBlock, 0, s>>>(tile_count, tiles, tile_off, count);
    return hipGetLastError();
}

hipError_t launch_run_compact(const double* x, const double* g, const double* w, int64_t n, int d, int64_t ld,
                              const uint8_t* starts, const int32_t* tile_off, int64_t count, int64_t ld_out,
                              double* xo, double* go, double* wo, int32_t* rows_out, hipStream_t s) {
    run_compact_kernel<<<(unsigned)run_tiles(n), kRunBlock, 0, s>>>(x, g, w, n, ld, d, starts, tile_off, count,
                                                                    ld_out, xo, go, wo, rows_out);
    return hipGetLastError();
}

}  // namespace st
