#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__device__ __forceinline__ float rcp_fast(float x) {
    const float r = __builtin_amdgcn_rcpf(x);
    const float e = __builtin_fmaf(-x, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
__global__ __launch_bounds__(256) void check(unsigned long long* bad, uint32_t* first, unsigned long long* hist) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < (1ull << 32); i += stride) {
        const float x = __builtin_bit_cast(float, (uint32_t)i);
        const uint32_t a = __builtin_bit_cast(uint32_t, rcp_fast(x));
        const uint32_t b = __builtin_bit_cast(uint32_t, 1.0f / x);
        if (a != b) {
            const uint32_t ex = ((uint32_t)i >> 23) & 0xff;
            atomicAdd(&hist[ex], 1ull);
            if (ex > 2 && ex < 252) {
                const unsigned long long n = atomicAdd(bad, 1ull);
                if (n < 16) first[n] = (uint32_t)i;
            }
        }
    }
}
int main() {
    unsigned long long *bad, *hist; uint32_t* first;
    hipMalloc(&bad, 8); hipMalloc(&first, 64); hipMalloc(&hist, 256 * 8);
    hipMemset(bad, 0, 8); hipMemset(hist, 0, 256 * 8);
    hipLaunchKernelGGL(check, dim3(256 * 64), dim3(256), 0, 0, bad, first, hist);
    unsigned long long n = 0, h[256]; uint32_t f[16] = {0};
    hipMemcpy(&n, bad, 8, hipMemcpyDeviceToHost); hipMemcpy(f, first, 64, hipMemcpyDeviceToHost);
    hipMemcpy(h, hist, 256 * 8, hipMemcpyDeviceToHost);
    printf("mismatches in exponents 3..251: %llu\n", n);
    for (unsigned long long i = 0; i < n && i < 16; ++i) printf("  x = 0x%08x\n", f[i]);
    for (int e = 0; e < 256; ++e) if (h[e]) printf("  exp %3d: %llu\n", e, h[e]);
    return 0;
}
