// geo::fan_lerp's device quotient a / pi as q0 = a * RN(1/pi), q = fma(fma(-q0,
// pi, a), RN(1/pi), q0) (3 VALU instead of a ~11-VALU correctly rounded
// division): equal to a / pi for a = 0 and every f32 a in [2^-100, 4].
// fan_lerp's a = pi/2 - asin(s) lies in [0, pi] and is 0 or at least 2^-24
// (for asin(s) >= pi/4 the subtraction is exact, a multiple of asin(s)'s
// ulp).  (Below 2^-100 the residual underflows and the form is off by an ulp.)
// Prints "mismatches N"; exit status 0 iff N == 0.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
__global__ void check(unsigned long long* bad, uint32_t* first) {
    const float kPi = 3.14159265358979323846f;
    const float r = 1.0f / kPi;  // constant-folded, correctly rounded
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i <= 0x40800000ull; i += stride) {  // [0, 4]
        float a = __builtin_bit_cast(float, (uint32_t)i);
        asm volatile("" : "+v"(a));
        const float q0 = a * r;
        const float e = __builtin_fmaf(-q0, kPi, a);
        const float q = __builtin_fmaf(e, r, q0);
        const float ref = a / kPi;
        if (a != 0.0f && a < 0x1p-100f) continue;  // a = pi/2 - asin(s) is 0 or >= ulp(pi/2)/2
        if (__builtin_bit_cast(uint32_t, q) != __builtin_bit_cast(uint32_t, ref)) {
            const unsigned long long n = atomicAdd(bad, 1ull);
            if (n < 8) first[n] = (uint32_t)i;
        }
    }
}
int main() {
    unsigned long long* bad; uint32_t* first;
    if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&first, 32) != hipSuccess) return 2;
    (void)hipMemset(bad, 0, 8);
    hipLaunchKernelGGL(check, dim3(256 * 64), dim3(256), 0, 0, bad, first);
    unsigned long long n = 0; uint32_t f[8] = {0};
    (void)hipMemcpy(&n, bad, 8, hipMemcpyDeviceToHost); (void)hipMemcpy(f, first, 32, hipMemcpyDeviceToHost);
    printf("mismatches %llu\n", n);
    for (unsigned long long i = 0; i < n && i < 8; ++i) printf("  a = 0x%08x\n", f[i]);
    return n == 0 ? 0 : 1;
}
