// Pair-list, cumulative-KSD and Gram-matrix kernels (K5) for gfx950.
//
// * pairs:     out[p] = k(i1[p], i2[p]) -- the integrand protocol integrand(ind1, ind2) of the
//              reference (stein_thinning.thinning._make_stein_integrand / _make_stein_gf_integrand;
//              used at code/src/utils/ksd.py:9-16, JAX_Stein_Thinning.ipynb cells 17, 30).
// * ksd rows:  LDS-tiled lower triangle of the selected set's Gram matrix: per (row tile, column
//              tile) partial row sums r_i = 2 sum_{j<i} k_ij + k_ii (stein_thinning.stein.ksd,
//              called at code/src/utils/ksd.py:27; report.tex:311-313).
// * ksd scan:  ps_i = sum_{a<=i} r_a, ks_i = sqrt(ps_i) / (i+1).
// * kmat:      K[r, c] = integrand(min(r,c), max(r,c)) (stein_thinning.stein.kmat,
//              code/tests/test_ksd.py:20, Gaussian_mixture.ipynb cell 94).
// All operate on a compact SoA problem (leading dimension ld); fp64 VALU bound, no MFMA.
#include "stein_math.hpp"
#include "stein_internal.hpp"

namespace st {

constexpr int kTile = 64;      // rows per tile (one row per lane)
constexpr int kChunk = 16;     // columns staged in LDS per pass

__global__ __launch_bounds__(256) void pairs_kernel(PairArgs p, const int64_t* __restrict__ i1,
                                                    const int64_t* __restrict__ i2, int64_t L,
                                                    double* __restrict__ out) {
    const double l2 = p.l * p.l;
    for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < L;
         q += (int64_t)gridDim.x * blockDim.x) {
        const int64_t a = i1[q], b = i2[q];
        double kv = pair_value_rt(p.x + a, p.g + a, p.ld, p.x + b, p.g + b, p.ld, p.d, p.l, l2, p.tr);
        if (p.w) kv = (kv * p.w[a]) * p.w[b];
        out[q] = kv;
    }
}

// Stage columns [c0, c0+kChunk) of the compact problem into LDS: s[k][c], k < 2d+1.
__device__ __forceinline__ void stage_chunk(const PairArgs& p, int64_t m, int64_t c0,
                                            double (*s)[kChunk]) {
    const int d = p.d;
    const int total = (2 * d + 1) * kChunk;
    for (int e = threadIdx.x; e < total; e += blockDim.x) {
        const int k = e / kChunk, c = e % kChunk;
        const int64_t j = c0 + c;
        double v = 0.0;
        if (j < m) {
            if (k < d) v = p.x[(int64_t)k * p.ld + j];
            else if (k < 2 * d) v = p.g[(int64_t)(k - d) * p.ld + j];
            else v = p.w ? p.w[j] : 1.0;
        }
        s[k][c] = v;
    }
}

// KSD: grid (ntiles_j, ntiles_i); block 256 = 4 waves; lane <-> row i; wave w takes columns
// w, w+4, ... of each staged chunk.  part[bj * ld + i] = this tile's share of r_i.
__global__ __launch_bounds__(256) void ksd_rows_kernel(PairArgs p, int64_t m,
                                                       double* __restrict__ part) {
    const int64_t bi = blockIdx.y, bj = blockIdx.x;
    if (bj > bi) return;
    __shared__ double s[2 * kMaxDim + 1][kChunk];
    __shared__ double s_red[4][kTile];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t i = bi * kTile + lane;
    const double l2 = p.l * p.l;
    const int d = p.d;
    const double wi = (p.w && i < m) ? p.w[i] : 1.0;
    double acc = 0.0;
    const int64_t cend = (bj * kTile + kTile < m) ? bj * kTile + kTile : m;
    for (int64_t c0 = bj * kTile; c0 < cend; c0 += kChunk) {
        __syncthreads();
        stage_chunk(p, m, c0, s);
        __syncthreads();
        if (i < m) {
            for (int c = wave; c < kChunk; c += 4) {
                const int64_t j = c0 + c;
                if (j > i || j >= m) continue;
                double kv = pair_value_rt(p.x + i, p.g + i, p.ld, &s[0][c], &s[d][c], kChunk, d,
                                          p.l, l2, p.tr);
                if (p.w) kv = (kv * wi) * s[2 * d][c];
                acc += (j < i) ? 2.0 * kv : kv;
            }
        }
    }
    s_red[wave][lane] = acc;
    __syncthreads();
    if (wave == 0 && i < m)
        part[bj * p.ld + i] = ((s_red[0][lane] + s_red[1][lane]) + s_red[2][lane]) + s_red[3][lane];
}

// r_i = sum over column tiles bj <= bi of part; then a single-block prefix sum -> ks.
__global__ __launch_bounds__(1024) void ksd_scan_kernel(const double* __restrict__ part,
                                                        int64_t ld, int64_t m,
                                                        double* __restrict__ ks) {
    __shared__ double s_tot[1024];
    const int tid = threadIdx.x;
    const int64_t per = (m + blockDim.x - 1) / blockDim.x;
    const int64_t b = tid * per, e = (b + per < m) ? b + per : m;
    double run = 0.0;
    for (int64_t i = b; i < e; ++i) {
        const int64_t bi = i / kTile;
        double r = 0.0;
        for (int64_t bj = 0; bj <= bi; ++bj) r += part[bj * ld + i];
        run += r;
        ks[i] = r;  // temporarily hold r_i
    }
    s_tot[tid] = run;
    __syncthreads();
    if (tid == 0) {
        double acc = 0.0;
        for (int t = 0; t < (int)blockDim.x; ++t) {
            const double v = s_tot[t];
            s_tot[t] = acc;
            acc += v;
        }
    }
    __syncthreads();
    double ps = s_tot[tid];
    for (int64_t i = b; i < e; ++i) {
        ps += ks[i];
        ks[i] = __builtin_sqrt(ps) / (double)(i + 1);
    }
}

// kmat: grid (ntiles, ntiles); lane <-> row r of the tile, columns staged; out is (k, k) row-major
// and symmetric by construction (weights applied in (min, max) order), so the lane-contiguous
// store out[c * k + r] is coalesced.
__global__ __launch_bounds__(256) void kmat_kernel(PairArgs p, int64_t k, double* __restrict__ out) {
    const int64_t bi = blockIdx.y, bj = blockIdx.x;
    __shared__ double s[2 * kMaxDim + 1][kChunk];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t r = bi * kTile + lane;
    const double l2 = p.l * p.l;
    const int d = p.d;
    const double wr = (p.w && r < k) ? p.w[r] : 1.0;
    const int64_t cend = (bj * kTile + kTile < k) ? bj * kTile + kTile : k;
    for (int64_t c0 = bj * kTile; c0 < cend; c0 += kChunk) {
        __syncthreads();
        stage_chunk(p, k, c0, s);
        __syncthreads();
        if (r < k) {
            for (int c = wave; c < kChunk; c += 4) {
                const int64_t cc = c0 + c;
                if (cc >= k) continue;
                double kv = pair_value_rt(p.x + r, p.g + r, p.ld, &s[0][c], &s[d][c], kChunk, d,
                                          p.l, l2, p.tr);
                if (p.w) {
                    const double wc = s[2 * d][c];
                    kv = (r <= cc) ? (kv * wr) * wc : (kv * wc) * wr;
                }
                out[cc * k + r] = kv;
            }
        }
    }
}

__global__ void layout_soa_kernel(const double* __restrict__ rowmajor, int64_t n, int d, int64_t ld,
                                  double* __restrict__ soa) {
    const int64_t total = n * d;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t i = e / d;
        const int k = (int)(e - i * d);
        soa[(int64_t)k * ld + i] = rowmajor[e];
    }
}

static int grid_for(int64_t work, int block) {
    int64_t b = (work + block - 1) / block;
    if (b > 2048) b = 2048;
    if (b < 1) b = 1;
    return (int)b;
}

hipError_t launch_pairs(const PairArgs& p, const int64_t* i1, const int64_t* i2, int64_t L,
                        double* out, hipStream_t s) {
    pairs_kernel<<<grid_for(L, 256), 256, 0, s>>>(p, i1, i2, L, out);
    return hipGetLastError();
}

hipError_t launch_ksd_rows(const PairArgs& p, const int64_t* idx, int64_t m, double* part,
                           int64_t ntiles, hipStream_t s) {
    (void)idx;
    dim3 grid((unsigned)ntiles, (unsigned)ntiles);
    ksd_rows_kernel<<<grid, 256, 0, s>>>(p, m, part);
    return hipGetLastError();
}

hipError_t launch_ksd_scan(const double* part, int64_t m, int64_t ld, double* ks, hipStream_t s) {
    ksd_scan_kernel<<<1, 1024, 0, s>>>(part, ld, m, ks);
    return hipGetLastError();
}

hipError_t launch_kmat(const PairArgs& p, const int64_t* idx, int64_t k, double* out,
                       hipStream_t s) {
    (void)idx;
    const int64_t nt = (k + kTile - 1) / kTile;
    dim3 grid((unsigned)nt, (unsigned)nt);
    kmat_kernel<<<grid, 256, 0, s>>>(p, k, out);
    return hipGetLastError();
}

hipError_t launch_layout_soa(const double* rowmajor, int64_t n, int d, int64_t ld, double* soa,
                             hipStream_t s) {
    layout_soa_kernel<<<grid_for(n * d, 256), 256, 0, s>>>(rowmajor, n, d, ld, soa);
    return hipGetLastError();
}

}  // namespace st
