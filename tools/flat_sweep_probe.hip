// Measurement probe (not product code): the exchange floor of a FLAT multi-rank winner sweep on one
// GPU.  In a flat R-rank design every block of every rank stores its per-step
// record into every rank's record array and each block sweeps all R x 256 records once, instead of
// the two levels the product uses (the 256-record sweep on the device, then one rank record per
// peer through the mailboxes, csrc/persistent.hip).  Here 256 blocks (one per CU) play rank 0: each
// stores R records per step (its own and R - 1 stand-ins for the peers' blocks, same tag), as 16-B
// sc1 stores into `nrep` replicas of an R x 256-record array (the product's record format and
// replica scheme), then one wave sweeps its replica with the product's polling rules (one 16-B sc1
// load per record, records already seen re-read out of range, polls on the 450-ns s_memrealtime
// grid), takes the minimum (key, index), broadcasts it through LDS and starts the next step.  No
// pair arithmetic: the time per step is the publish + sweep + broadcast floor for R x 256 records.
// Bounded: a sweep that has not completed within 2 s sets the abort word and every block leaves.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/flat_sweep_probe tools/flat_sweep_probe.hip
//   ./tools/flat_sweep_probe [steps]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                               \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kSync = 45;                      // poll grid, s_memrealtime ticks (the product's)
constexpr uint64_t kTimeout = 200000000ull;    // 2 s

struct Args {
    uint64_t* gran;     // 2 banks x nrep replicas x (R * 256) records x 2 granules
    int R, nrep, steps;
    int64_t rep_stride; // granules between replicas
    unsigned* abort;
    uint64_t* ticks;    // [0] start, [1] end (block 0)
    uint32_t* winners;  // per step (block 0)
};

template <int RPL>   // records per lane = R * 256 / 64
__global__ __launch_bounds__(256) void flat_sweep(Args a) {
    __shared__ uint64_t win_sh;
    const int lane = threadIdx.x & 63;
    const int nrec = a.R * 256;
    if (blockIdx.x == 0 && threadIdx.x == 0) a.ticks[0] = __builtin_amdgcn_s_memrealtime();
    uint32_t prev = 0;
    for (int t = 0; t < a.steps; ++t) {
        const uint64_t tag = (uint64_t)((t + 1) & 0xFF) << 56;
        const uint32_t want8 = (uint32_t)((t + 1) & 0xFF);
        if (threadIdx.x < 64) {
            // publish: R records (this block's and R - 1 stand-ins) into every replica, 16-B sc1 stores
            for (int q = lane; q < a.R * a.nrep; q += 64) {
                const int r = q % a.R, rep = q / a.R;
                const uint32_t idx = (uint32_t)(r * 256 + blockIdx.x);
                // a key that moves every step (depends on the previous winner: a real data dependence)
                const uint64_t key = ((uint64_t)((idx * 2654435761u) ^ (prev * 40503u) ^ (uint32_t)t) << 8) & 0x00FFFFFFFFFFFF00ull;
                const uint64_t g0 = tag | (key >> 8), g1 = tag | idx;
                const int64_t off = (((t & 1) * a.nrep + rep) * a.rep_stride + (int64_t)idx * 2) * 8;
                const auto rs = __builtin_amdgcn_make_buffer_rsrc(a.gran, 0, 0x7FFFFFFF, 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b128(u32x4{(unsigned)g0, (unsigned)(g0 >> 32), (unsigned)g1,
                                                             (unsigned)(g1 >> 32)}, rs, (int)off, 0, 16 /* sc1 */);
            }
            // sweep replica blockIdx % nrep
            const uint64_t* bank = a.gran + ((t & 1) * a.nrep + (int)blockIdx.x % a.nrep) * a.rep_stride;
            const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t*>(bank), 0, nrec * 16, 0x00020000);
            const uint32_t oob = (uint32_t)nrec * 16;
            uint32_t need = 0, seen = 0;
            for (int c = 0; c < RPL; ++c) need |= (lane + 64 * c < nrec) ? (1u << c) : 0u;
            uint64_t bk = ~0ull;
            uint32_t bi = 0xFFFFFFFFu;
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            bool ok = true;
            for (unsigned it = 0;; ++it) {
                const uint64_t now = __builtin_amdgcn_s_memrealtime();
                const uint64_t slot = (now + kSync - 1) / kSync * kSync;
                while (__builtin_amdgcn_s_memrealtime() < slot) __builtin_amdgcn_s_sleep(1);
                u32x4 qs[RPL];
#pragma unroll
                for (int c = 0; c < RPL; ++c) {
                    const uint32_t off = (uint32_t)(lane + 64 * c) * 16;
                    qs[c] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, ((need & ~seen) >> c) & 1u ? off : oob, 0, 16);
                }
                const uint32_t open = need & ~seen;
#pragma unroll
                for (int c = 0; c < RPL; ++c) {
                    const u32x4 q = qs[c];
                    const bool hit = ((open >> c) & 1u) && (q.y >> 24) == want8 && (q.w >> 24) == want8;
                    const uint64_t k = ((uint64_t)(q.y & 0x00FFFFFFu) << 32) | q.x;
                    const uint32_t ib = q.z;
                    const bool tk = hit && (k < bk || (k == bk && ib < bi));
                    bk = tk ? k : bk;
                    bi = tk ? ib : bi;
                    seen |= hit ? (1u << c) : 0u;
                }
                if (__all(seen == need)) break;
                if ((it & 15) == 15 && __any(__builtin_amdgcn_s_memrealtime() - t0 > kTimeout ||
                                             __hip_atomic_load(a.abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0)) {
                    ok = false;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            // wave minimum of (key, index)
            for (int off = 32; off >= 1; off >>= 1) {
                const uint64_t ok2 = (uint64_t)__shfl_xor((unsigned long long)bk, off);
                const uint32_t oi = __shfl_xor(bi, off);
                const bool tk = ok2 < bk || (ok2 == bk && oi < bi);
                bk = tk ? ok2 : bk;
                bi = tk ? oi : bi;
            }
            if (!ok && lane == 0) __hip_atomic_store(a.abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (lane == 0) win_sh = ok ? bi : 0xFFFFFFFFull;
        }
        __syncthreads();
        prev = (uint32_t)win_sh;
        if (blockIdx.x == 0 && threadIdx.x == 0) a.winners[t] = prev;
        if (prev == 0xFFFFFFFFu) break;
        __syncthreads();
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) a.ticks[1] = __builtin_amdgcn_s_memrealtime();
}

template <int RPL>
static double run(int R, int nrep, int steps, int G) {
    Args a{};
    a.R = R;
    a.nrep = nrep;
    a.steps = steps;
    const int64_t one = (int64_t)R * 256 * 2;
    a.rep_stride = nrep == 1 ? one : (one + 63) / 64 * 64 + 32;
    const size_t bytes = (size_t)2 * nrep * a.rep_stride * 8;
    CK(hipMalloc(&a.gran, bytes));
    CK(hipMalloc(&a.abort, 4));
    CK(hipMalloc(&a.ticks, 16));
    CK(hipMalloc(&a.winners, 4 * steps));
    double best = 1e30;
    for (int rep = 0; rep < 3; ++rep) {
        CK(hipMemset(a.gran, 0, bytes));
        CK(hipMemset(a.abort, 0, 4));
        hipLaunchKernelGGL(flat_sweep<RPL>, dim3(G), dim3(256), 0, 0, a);
        CK(hipDeviceSynchronize());
        uint64_t tk[2];
        unsigned ab;
        CK(hipMemcpy(tk, a.ticks, 16, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&ab, a.abort, 4, hipMemcpyDeviceToHost));
        if (ab) { printf("R=%d: bounded wait expired\n", R); break; }
        const double us = (double)(tk[1] - tk[0]) * 0.01 / steps;
        if (us < best) best = us;
    }
    CK(hipFree(a.gran)); CK(hipFree(a.abort)); CK(hipFree(a.ticks)); CK(hipFree(a.winners));
    return best;
}

int main(int argc, char** argv) {
    const int steps = argc > 1 ? atoi(argv[1]) : 2000;
    int dev = 0, cus = 0;
    CK(hipGetDevice(&dev));
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    if (cus != 256) { printf("expects 256 CUs (MI355X), found %d\n", cus); return 1; }
    printf("# flat winner sweep, 256 blocks (one per CU), no pair arithmetic, %d steps, best of 3\n", steps);
    for (int nrep : {16, 8}) {
        printf("R=1 (256 records)   nrep=%2d: %6.2f us per step\n", nrep, run<4>(1, nrep, steps, 256));
        printf("R=2 (512 records)   nrep=%2d: %6.2f us per step\n", nrep, run<8>(2, nrep, steps, 256));
        printf("R=4 (1024 records)  nrep=%2d: %6.2f us per step\n", nrep, run<16>(4, nrep, steps, 256));
        printf("R=8 (2048 records)  nrep=%2d: %6.2f us per step\n", nrep, run<32>(8, nrep, steps, 256));
    }
    return 0;
}
