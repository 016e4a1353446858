// Test helper (not product code): holds `blocks` CUs for `ticks` of s_memrealtime (100 MHz) with
// one 64-thread block each and `lds_bytes` of LDS, so a persistent kernel launched next to it on
// another stream cannot make its grid co-resident (tests/test_gpu_fallback.py).  Every wave exits
// once its own bounded wait ends.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void occupy_kernel(uint64_t ticks, int* sink) {
    extern __shared__ int lds[];
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    lds[threadIdx.x] = (int)threadIdx.x;
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
    __syncthreads();
    if (blockIdx.x == 0 && threadIdx.x == 0) sink[0] = lds[63];
}

extern "C" int st_test_occupy(int blocks, int lds_bytes, uint64_t ticks, int* sink, void* stream) {
    if (blocks < 1 || blocks > 1024 || lds_bytes < 256 || lds_bytes > 163840 || !sink ||
        ticks > 300000000ull)
        return -1;
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(occupy_kernel),
                            hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes) != hipSuccess)
        return -2;
    hipLaunchKernelGGL(occupy_kernel, dim3(blocks), dim3(64), lds_bytes, static_cast<hipStream_t>(stream),
                       ticks, sink);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}
