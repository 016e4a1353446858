// Measurement probe (not product code): achievable bandwidth for the greedy step's exact access
// pattern on this MI355X, and a sweep of the step-kernel variants exposed by st_tune().
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -o tools/probe tools/probe.hip \
//        -Lgradient-free-mcmc-postprocessing_amd/stein_thinning/_lib -lstein_hip -Wl,-rpath,<that dir>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

#include "../include/stein_thinning_hip.h"

#ifdef ST_PERSIST_STAMPS
extern "C" int st_debug_set_stamps(uint64_t* buf);
#endif

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                            \
        }                                                                       \
    } while (0)

__global__ void fill(double* p, int64_t n, uint64_t seed, double scale) {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        p[i] = ((double)(z >> 11) * 0x1.0p-53 - 0.5) * scale;
    }
}

// pure streaming of the step's traffic: 2*D column reads (+A read, +A write), double2 per lane
template <int D, bool WRITE_A, int CPT>
__global__ __launch_bounds__(256) void stream_kernel(const double* x, const double* g, double* A,
                                                     int64_t n, int64_t ld, double* out) {
    double acc = 0.0;
    const int64_t nunits = n / CPT;
    for (int64_t u = blockIdx.x * 256ll + threadIdx.x; u < nunits; u += (int64_t)gridDim.x * 256) {
        const int64_t i0 = u * CPT;
        double s[CPT];
#pragma unroll
        for (int c = 0; c < CPT; ++c) s[c] = 0.0;
#pragma unroll
        for (int k = 0; k < D; ++k)
#pragma unroll
            for (int c = 0; c < CPT; c += 2) {
                const double2 xv = *reinterpret_cast<const double2*>(x + k * ld + i0 + c);
                const double2 gv = *reinterpret_cast<const double2*>(g + k * ld + i0 + c);
                s[c] += xv.x * gv.x;
                s[c + 1] += xv.y * gv.y;
            }
#pragma unroll
        for (int c = 0; c < CPT; c += 2) {
            double2 av = *reinterpret_cast<const double2*>(A + i0 + c);
            if (WRITE_A) {
                av.x += s[c];
                av.y += s[c + 1];
                *reinterpret_cast<double2*>(A + i0 + c) = av;
            } else {
                acc += av.x + av.y + s[c] + s[c + 1];
            }
        }
    }
    if (!WRITE_A && acc == 12345.678) out[0] = acc;
}

struct Timer {
    hipEvent_t a, b;
    Timer() { CK(hipEventCreate(&a)); CK(hipEventCreate(&b)); }
    void start(hipStream_t s) { CK(hipEventRecord(a, s)); }
    float stop(hipStream_t s) {
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        return ms;
    }
};

int main(int argc, char** argv) {
    const int64_t n = argc > 1 ? atoll(argv[1]) : 2000000;
    const int d = 4;
    const int64_t ld = (n + 63) / 64 * 64;
    hipStream_t s;
    CK(hipStreamCreate(&s));
    // near-tie guard (st_tune key 20; on by default in the library): PROBE_GUARD=0 times the plain kernels
    if (getenv("PROBE_GUARD")) st_tune(20, atoi(getenv("PROBE_GUARD")));
    double *x, *g, *A, *out;
    CK(hipMalloc(&x, sizeof(double) * d * ld));
    CK(hipMalloc(&g, sizeof(double) * d * ld));
    CK(hipMalloc(&A, sizeof(double) * ld));
    CK(hipMalloc(&out, 64));
    fill<<<1024, 256, 0, s>>>(x, d * ld, 1, 4.0);
    fill<<<1024, 256, 0, s>>>(g, d * ld, 2, 6.0);
    fill<<<1024, 256, 0, s>>>(A, ld, 3, 1.0);
    CK(hipStreamSynchronize(s));
    Timer T;
    const double bytes_rw = (double)n * (16 * d + 16), bytes_r = (double)n * (16 * d + 8);
    printf("# n=%lld d=%d  step traffic %.1f MB (read %.1f MB)\n", (long long)n, d, bytes_rw / 1e6, bytes_r / 1e6);
    const int reps = 200;
    const bool persist_only = argc > 2 && (argv[2][0] == 'p' || argv[2][0] == 'r' || argv[2][0] == 'q');
    for (int blocks : {256, 512, 1024, 2048, 4096}) {
        if (persist_only) break;
        for (int wr = 0; wr < 2; ++wr) {
            for (int cpt : {2, 4}) {
                auto launch = [&]() {
                    if (wr) {
                        if (cpt == 2) stream_kernel<4, true, 2><<<blocks, 256, 0, s>>>(x, g, A, n, ld, out);
                        else stream_kernel<4, true, 4><<<blocks, 256, 0, s>>>(x, g, A, n, ld, out);
                    } else {
                        if (cpt == 2) stream_kernel<4, false, 2><<<blocks, 256, 0, s>>>(x, g, A, n, ld, out);
                        else stream_kernel<4, false, 4><<<blocks, 256, 0, s>>>(x, g, A, n, ld, out);
                    }
                };
                for (int i = 0; i < 20; ++i) launch();
                T.start(s);
                for (int i = 0; i < reps; ++i) launch();
                const float ms = T.stop(s);
                const double us = ms * 1e3 / reps;
                printf("stream blocks=%5d write_A=%d cpt=%d  %8.2f us/launch  %7.1f GB/s\n", blocks, wr, cpt, us,
                       (wr ? bytes_rw : bytes_r) / (us * 1e-6) / 1e9);
            }
        }
    }
    // greedy step variants through the C ABI (single-device run of `reps` steps)
    const int64_t ws_bytes = st_greedy_workspace_bytes(n, d, 1);
    void* ws;
    uint32_t* idx;
    CK(hipMalloc(&ws, ws_bytes));
    CK(hipMalloc(&idx, 4 * 4096));
    const double l = 0.37, tr = 4 * 0.37;
    const int M = reps + 1;
    for (int blocks : {128, 256, 512, 1024}) {
        if (persist_only) break;
        for (int cpt : {1, 2, 4}) {
            for (int pf = 0; pf < 2; ++pf) {
                st_tune(0, blocks);
                st_tune(1, cpt);
                st_tune(2, pf);
                auto run = [&](int64_t t0, int64_t t1) {
                    int rc = st_greedy_steps(x, g, nullptr, n, d, ld, l, tr, t0, t1, M, idx, A, ws, ws_bytes, s);
                    if (rc) { fprintf(stderr, "rc=%d %s\n", rc, st_last_error()); exit(1); }
                };
                run(0, 1);
                for (int t = 1; t < 11; ++t) run(t, t + 1);
                T.start(s);
                run(11, 11 + 150);
                const double us = T.stop(s) * 1e3 / 150;
                std::vector<float> v;
                for (int t = 161; t < 191; ++t) {
                    T.start(s);
                    run(t, t + 1);
                    v.push_back(T.stop(s) * 1e3f);
                }
                std::sort(v.begin(), v.end());
                printf("greedy blocks=%4d cpt=%d pf=%d  %8.2f us/step back-to-back (%7.1f GB/s)  isolated median %8.2f us\n",
                       blocks, cpt, pf, us, bytes_rw / (us * 1e-6) / 1e9, v[v.size() / 2]);
            }
        }
    }
    st_tune(0, 256); st_tune(1, -1); st_tune(2, -1);
    if (argc > 2 && argv[2][0] == 'q') {   // quick: the default persistent configuration, m = 1000
        const int Mq = 1000;
        // optional st_tune overrides: PROBE_NT (key 4), PROBE_RT (key 3), PROBE_GRID (key 5), PROBE_NREP (key 10),
        // PROBE_CMP (key 12)
        if (getenv("PROBE_NT")) st_tune(4, atoi(getenv("PROBE_NT")));
        if (getenv("PROBE_RT")) st_tune(3, atoi(getenv("PROBE_RT")));
        if (getenv("PROBE_GRID")) st_tune(5, atoi(getenv("PROBE_GRID")));
        if (getenv("PROBE_NREP")) st_tune(10, atoi(getenv("PROBE_NREP")));
        if (getenv("PROBE_CMP")) st_tune(12, atoi(getenv("PROBE_CMP")));
        std::vector<float> v;
        std::vector<uint32_t> h(Mq);
        for (int rep = 0; rep < 5; ++rep) {
            T.start(s);
            int rc = st_greedy(x, g, nullptr, n, d, ld, l, tr, Mq, idx, A, ws, ws_bytes, s);
            if (rc) { fprintf(stderr, "rc=%d %s\n", rc, st_last_error()); exit(1); }
            v.push_back(T.stop(s));
        }
        CK(hipMemcpy(h.data(), idx, 4 * Mq, hipMemcpyDeviceToHost));
        std::sort(v.begin(), v.end());
        uint64_t hs = 1469598103934665603ull;
        for (uint32_t e : h) hs = (hs ^ e) * 1099511628211ull;
        printf("quick n=%lld m=%d  best %8.3f ms  median %8.3f ms  (%6.2f us/step)  idx hash %016llx\n",
               (long long)n, Mq, v[0], v[2], v[0] * 1e3 / Mq, (unsigned long long)hs);
        return 0;
    }
    if (argc > 2 && argv[2][0] == 'r') {   // record replicas (st_tune key 10) x pitch (key 9), m = 1000
        const int Mr = 1000;
        std::vector<uint32_t> ref;
        struct RV { int nrep, pitch; };
        for (int pass = 0; pass < 2; ++pass)
        for (RV cfg : {RV{1, -1}, RV{2, 16}, RV{4, 16}, RV{8, 16}, RV{8, 64}, RV{16, 16},
                       RV{32, 16}, RV{8, 256}}) {
            if (st_tune(10, cfg.nrep) || st_tune(9, cfg.pitch)) { fprintf(stderr, "tune\n"); exit(1); }
            std::vector<float> v;
            std::vector<uint32_t> h(Mr);
            for (int rep = 0; rep < 4; ++rep) {
                T.start(s);
                int rc = st_greedy(x, g, nullptr, n, d, ld, l, tr, Mr, idx, A, ws, ws_bytes, s);
                if (rc) { fprintf(stderr, "rc=%d %s\n", rc, st_last_error()); exit(1); }
                v.push_back(T.stop(s));
            }
            CK(hipMemcpy(h.data(), idx, 4 * Mr, hipMemcpyDeviceToHost));
            if (ref.empty()) ref = h;
            std::sort(v.begin(), v.end());
            printf("replicas=%2d pitch=%4d  m=%d  best %8.3f ms  median %8.3f ms  (%6.2f us/step)  same_idx=%d\n",
                   cfg.nrep, cfg.pitch, Mr, v[0], v[2], v[0] * 1e3 / Mr, (int)(h == ref));
            fflush(stdout);
        }
        st_tune(10, -1); st_tune(9, -1);
        return 0;
    }
    // whole-run st_greedy: persistent kernel (register rows per thread rt; 0 = launch per step)
    struct V { int rt, nt; };
    for (V cfg : {V{8, 512}, V{4, 512}, V{4, 256}, V{0, 256}}) {
        const int rt = cfg.rt;
        st_tune(3, rt);
        st_tune(4, cfg.nt);
        for (int rep = 0; rep < 3; ++rep) {
            T.start(s);
            int rc = st_greedy(x, g, nullptr, n, d, ld, l, tr, M, idx, A, ws, ws_bytes, s);
            if (rc) { fprintf(stderr, "rc=%d %s\n", rc, st_last_error()); exit(1); }
            const float ms = T.stop(s);
            std::vector<uint32_t> h(M);
            CK(hipMemcpy(h.data(), idx, 4 * M, hipMemcpyDeviceToHost));
            const uint32_t mx = *std::max_element(h.begin(), h.end());
            printf("st_greedy nt=%d rt=%2d m=%d  %8.3f ms  %8.2f us/step  idx[0..2]=%u %u %u  max=%u%s\n", cfg.nt, rt, M, ms,
                   ms * 1e3 / M, h[0], h[1], h[2], mx, mx >= n ? "  POISONED" : "");
            (void)0;
        }
    }
    st_tune(3, -1);
    st_tune(4, -1);
#ifdef ST_PERSIST_STAMPS
    {   // phase breakdown of persistent steps 20..51 (s_memrealtime, 10 ns ticks)
        const int SP = 32, PH = 32, GMAX = 512;
        if (getenv("PROBE_BPC")) st_tune(8, atoi(getenv("PROBE_BPC")));
        if (getenv("PROBE_NT")) st_tune(4, atoi(getenv("PROBE_NT")));
        if (getenv("PROBE_RT")) st_tune(3, atoi(getenv("PROBE_RT")));
        if (getenv("PROBE_NREP")) st_tune(10, atoi(getenv("PROBE_NREP")));
        if (getenv("PROBE_CMP")) st_tune(12, atoi(getenv("PROBE_CMP")));
        uint64_t* dst;
        CK(hipMalloc(&dst, sizeof(uint64_t) * GMAX * SP * PH));
        CK(hipMemset(dst, 0, sizeof(uint64_t) * GMAX * SP * PH));
        st_debug_set_stamps(dst);
        st_greedy(x, g, nullptr, n, d, ld, l, tr, M, idx, A, ws, ws_bytes, s);
        CK(hipStreamSynchronize(s));
        st_debug_set_stamps(nullptr);
        std::vector<uint64_t> h(GMAX * SP * PH);
        CK(hipMemcpy(h.data(), dst, h.size() * 8, hipMemcpyDeviceToHost));
        int G = 0;
        while (G < GMAX && h[(size_t)G * SP * PH + 0] != 0) ++G;
        double acc[8] = {0}, ph_lds = 0;
        int cnt = 0;
        for (int st = 1; st + 1 < SP; ++st) {   // step st: compute (2->3), publish (3->4), exchange
            uint64_t last_pub = 0, first_start = ~(uint64_t)0, last_start = 0;
            double c_avg = 0, wait_avg = 0, row_avg = 0, pub_avg = 0, creg = 0, clds = 0;
            for (int b = 0; b < G; ++b) {
                const uint64_t* q = &h[((size_t)b * SP + st) * PH];
                last_pub = std::max<uint64_t>(last_pub, q[4]);
                c_avg += (double)(q[3] - q[2]);
                creg += (double)(q[5] - q[2]);
                clds += (double)(q[6] - q[5]);
                pub_avg += (double)(q[4] - q[3]);
                const uint64_t* nx = &h[((size_t)b * SP + st + 1) * PH];
                wait_avg += (double)(nx[1] - nx[0]);
                row_avg += (double)(nx[2] - nx[1]);
                first_start = std::min<uint64_t>(first_start, nx[2]);
                last_start = std::max<uint64_t>(last_start, nx[2]);
            }
            acc[0] += c_avg / G; acc[1] += pub_avg / G; acc[2] += wait_avg / G; acc[3] += row_avg / G;
            acc[4] += (double)(first_start - last_pub); acc[5] += (double)(last_start - first_start);
            uint64_t s0 = ~(uint64_t)0, s1 = ~(uint64_t)0;
            for (int b = 0; b < G; ++b) {
                s0 = std::min<uint64_t>(s0, h[((size_t)b * SP + st) * PH + 2]);
                s1 = std::min<uint64_t>(s1, h[((size_t)b * SP + st + 1) * PH + 2]);
            }
            acc[6] += (double)(s1 - s0);
            acc[7] += creg / G;
            ph_lds += clds / G;
            ++cnt;
        }
        printf("stamps G=%d (us): compute %.2f  publish %.2f  sweep-wait %.2f  winner-row %.2f  "
               "last-publish->first-next-start %.2f  start-skew %.2f  step period %.2f\n", G,
               acc[0] / cnt / 100, acc[1] / cnt / 100, acc[2] / cnt / 100, acc[3] / cnt / 100,
               acc[4] / cnt / 100, acc[5] / cnt / 100, acc[6] / cnt / 100);
        {
            double mloc = 0, late = 0, tot = 0;
            for (int st = 1; st < SP; ++st)
                for (int b = 0; b < G; ++b) {
                    const uint64_t* q = &h[((size_t)b * SP + st) * PH];
                    mloc += (double)(q[7] - q[1]);
                    if (q[8]) { tot += 1; late += q[8] == 2; }
                }
            double its = 0, swt = 0;
            for (int st = 1; st < SP; ++st)
                for (int b = 0; b < G; ++b) {
                    const uint64_t* q = &h[((size_t)b * SP + st) * PH];
                    its += (double)q[9];
                    swt += (double)(q[1] - q[0]);
                }
            printf("sweep: %.2f polls per step on average, %.3f us per poll\n", its / ((SP - 1) * G),
                   swt / its / 100);
            printf("sweep-done -> minloc-done %.2f us; winner row loaded after the sweep in %.0f%% of steps\n",
                   mloc / ((SP - 1) * G) / 100, tot > 0 ? 100.0 * late / tot : -1.0);
        }
        {   // publish breakdown: wave 0's compute end (3) -> its minloc (10); waves' compute ends
            // (12 + w) -> spread; barrier passed (11); record stored (4)
            double ml = 0, spread = 0, w0_to_last = 0, bar = 0, st = 0;
            int cntp = 0;
            const int NW = getenv("PROBE_NT") && atoi(getenv("PROBE_NT")) == 256 ? 4 : 8;
            for (int stp = 1; stp < SP; ++stp)
                for (int b = 0; b < G; ++b) {
                    const uint64_t* q = &h[((size_t)b * SP + stp) * PH];
                    uint64_t lo = ~(uint64_t)0, hi = 0;
                    for (int w = 0; w < NW; ++w) { lo = std::min<uint64_t>(lo, q[12 + w]); hi = std::max<uint64_t>(hi, q[12 + w]); }
                    ml += (double)(q[10] - q[12]);
                    spread += (double)(hi - lo);
                    w0_to_last += (double)(hi - q[12]);
                    bar += (double)(q[11] - hi);
                    st += (double)(q[4] - q[11]);
                    ++cntp;
                }
            printf("publish split (us): wave0 minloc %.2f  waves' compute-end spread %.2f (wave0 -> last %.2f)  "
                   "last wave end -> barrier passed %.2f  barrier -> record stored %.2f\n",
                   ml / cntp / 100, spread / cntp / 100, w0_to_last / cntp / 100, bar / cntp / 100, st / cntp / 100);
        }
        {   // near-tie guard (diagnostic): the latest wave's rescan of step st (phase 24 + w) against the block's
            // sweep of that step done (phase 1 of row st + 1): > 0 = the rescan holds the next step's barrier
            double late = 0, lat_max = 0;
            int cntr = 0;
            const int NW = getenv("PROBE_NT") && atoi(getenv("PROBE_NT")) == 256 ? 4 : 8;
            for (int stp = 1; stp + 1 < SP; ++stp)
                for (int b = 0; b < G; ++b) {
                    const uint64_t* q = &h[((size_t)b * SP + stp) * PH];
                    const uint64_t* nx = &h[((size_t)b * SP + stp + 1) * PH];
                    uint64_t hi = 0;
                    for (int w = 1; w < NW; ++w) hi = std::max<uint64_t>(hi, q[24 + w]);
                    if (hi == 0) continue;
                    const double d = ((double)hi - (double)nx[1]) / 100;
                    late += d;
                    lat_max = std::max(lat_max, d);
                    ++cntr;
                }
            if (cntr) printf("guard rescan end - sweep done: %.2f us on average, %.2f max\n", late / cntr, lat_max);
        }
        printf("compute split (us): register rows %.2f  LDS rows %.2f  streamed rows %.2f\n",
               acc[7] / cnt / 100, ph_lds / cnt / 100, (acc[0] - acc[7] - ph_lds) / cnt / 100);
        {   // speculation study: is the best record after a block's FIRST poll the step's winner?
            std::vector<uint32_t> hidx(M);
            CK(hipMemcpy(hidx.data(), idx, 4 * M, hipMemcpyDeviceToHost));
            double seen0 = 0, hits = 0, tot = 0, settle_before_last = 0, polls = 0, proc = 0;
            double hist[6] = {0};
            for (int st = 1; st < SP; ++st) {
                const int64_t t = st + 20 - 1;   // stamps row st holds the sweep that picked idx[t]
                if (t >= M) break;
                for (int b = 0; b < G; ++b) {
                    const uint64_t* q = &h[((size_t)b * SP + st) * PH];
                    seen0 += (double)q[20];
                    proc += (double)q[23];
                    hits += (int64_t)q[22] == (int64_t)hidx[t];
                    const double np = (double)q[9];
                    polls += np;
                    settle_before_last += (double)q[21] < np;
                    hist[std::min<int>(5, (int)q[21])] += 1;
                    tot += 1;
                }
            }
            printf("sweep processing: %.3f us per poll from data landed to records taken (polls %.2f)\n",
                   proc / polls / 100, polls / tot);
            printf("speculation: first poll sees %.1f of %d records; its best is the winner in %.1f%% of "
                   "block-steps; polls %.2f; best settled before the last poll in %.1f%%; settle poll histogram "
                   "1:%.1f%% 2:%.1f%% 3:%.1f%% 4:%.1f%% 5+:%.1f%%\n",
                   seen0 / tot, G, 100 * hits / tot, polls / tot, 100 * settle_before_last / tot, 100 * hist[1] / tot,
                   100 * hist[2] / tot, 100 * hist[3] / tot, 100 * hist[4] / tot, 100 * hist[5] / tot);
        }
    }
#endif
    T.start(s);
    for (int r = 0; r < 50; ++r) st_greedy_steps(x, g, nullptr, n, d, ld, l, tr, 0, 1, M, idx, A, ws, ws_bytes, s);
    printf("diag  %8.2f us/launch\n", T.stop(s) * 1e3 / 50);
    return 0;
}
