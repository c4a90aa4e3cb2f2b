// Two device rewrites of the specification, checked over every f32 input of
// their domain on the GPU:
//  * geo::floor_i32_ (one v_cvt_flr_i32_f32) == (int32_t)floorf(x) for every
//    finite |x| < 2^30 (the sampler's texel coordinates lie in [-128, 2^28]);
//  * geo::sincosf_ (quadrant and rint by the 1.5 * 2^23 shifter) == the same
//    polynomial evaluation with rintf and the int cast, for every x with
//    |x| < 6.5e6 (|x * 2/pi| < 2^22).
// Prints "mismatches N"; exit status 0 iff N == 0.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../schwarzschild_raytracer_wgpu_amd/csrc/geo_pixel.h"

__device__ void sincos_rint(float x, float* s, float* c) {
    using geo::fmaf_;
    const float j = __builtin_rintf(x * geo::kTwoOverPi);
    float r = fmaf_(-j, 1.5703125f, x);
    r = fmaf_(-j, 4.837512969970703125e-4f, r);
    r = fmaf_(-j, 7.54978995489188216e-8f, r);
    const float z = r * r;
    const float ps = fmaf_(fmaf_(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
    const float sn = fmaf_(ps * z, r, r);
    const float pc = fmaf_(fmaf_(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
    const float cs = fmaf_(pc * z, z, fmaf_(-0.5f, z, 1.0f));
    const int q = ((int)j) & 3;
    const float sa = (q & 1) ? cs : sn;
    const float ca = (q & 1) ? sn : cs;
    *s = (q & 2) ? -sa : sa;
    *c = ((q + 1) & 2) ? -ca : ca;
}

__global__ __launch_bounds__(256) void check(unsigned long long* bad, uint32_t* first) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < (1ull << 32); i += stride) {
        float x = __builtin_bit_cast(float, (uint32_t)i);
        GEO_OPAQUE(x);
        const float ax = __builtin_fabsf(x);
        bool ok = true;
        if (ax < 0x1p30f) ok = geo::floor_i32_(x) == (int32_t)__builtin_floorf(x);
        if (ax < 6.5e6f) {
            float s0, c0, s1, c1;
            geo::sincosf_(x, &s0, &c0);
            sincos_rint(x, &s1, &c1);
            ok = ok && __builtin_bit_cast(uint32_t, s0) == __builtin_bit_cast(uint32_t, s1) &&
                 __builtin_bit_cast(uint32_t, c0) == __builtin_bit_cast(uint32_t, c1);
        }
        if (!ok) {
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
