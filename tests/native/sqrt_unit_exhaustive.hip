// geo::sqrt_unit_ (the branch-free correctly rounded sqrt of acos_pi_: rsq,
// one residual correction, the 2^-96 floor by a max) == the specification
// sqrtf(fmaxf(x, 2^-96)) (hipcc's correctly rounded builtin) for every f32 x
// in [0, 1], the domain acos_pi_ feeds it (1 - |x| for |x| <= 1).
// Prints "mismatches N"; exit status 0 iff N == 0.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../schwarzschild_raytracer_wgpu_amd/csrc/geo_math.h"

__global__ __launch_bounds__(256) void check(unsigned long long* bad, uint32_t* first) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i <= 0x3F800000ull; i += stride) {  // [0, 1]
        float x = __builtin_bit_cast(float, (uint32_t)i);
        GEO_OPAQUE(x);
        const float a = geo::sqrt_unit_(x);
        const float b = __builtin_sqrtf(__builtin_fmaxf(x, 0x1p-96f));
        if (__builtin_bit_cast(uint32_t, a) != __builtin_bit_cast(uint32_t, b)) {
            const unsigned long long n = atomicAdd(bad, 1ull);
            if (n < 8) first[n] = (uint32_t)i;
        }
    }
}

int main() {
    unsigned long long* bad;
    uint32_t* first;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&first, 32) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, 8);
    hipLaunchKernelGGL(check, dim3(256 * 64), dim3(256), 0, 0, bad, first);
    unsigned long long n = 0;
    uint32_t f[8] = {0};
    if (hipMemcpy(&n, bad, 8, hipMemcpyDeviceToHost) != hipSuccess) return 2;
    (void)hipMemcpy(f, first, 32, hipMemcpyDeviceToHost);
    printf("mismatches %llu\n", n);
    for (unsigned long long i = 0; i < n && i < 8; ++i) printf("  x = 0x%08x\n", f[i]);
    return n == 0 ? 0 : 1;
}
