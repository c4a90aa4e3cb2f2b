// The sky UV clamp of the specification (geo_pixel.h sky_uv): y = x + 0, then
// NaN -> 0 and [0, 1] clamping, as ONE v_med3_f32(y, 0, 1) on the device
// (geo::med3_); and sin theta's clamp (geo::central_sin: NaN -> -1, [-1, 1]).  Checked for all 2^32 f32 bit patterns against the same rule
// evaluated on the IEEE bit pattern (no float compares the compiler could
// fold back into a med3).  Prints "mismatches N"; exit status 0 iff N == 0.
#include <hip/hip_runtime.h>

#include <cstdio>

#include "../../schwarzschild_raytracer_wgpu_amd/csrc/geo_pixel.h"

__device__ __forceinline__ uint32_t rule(uint32_t yb) {
    if ((yb & 0x7fffffffu) > 0x7f800000u) return 0u;          // NaN -> +0
    if (yb & 0x80000000u) return (yb == 0x80000000u) ? yb : 0u;  // negative -> +0 (-0 cannot occur: y = x + 0)
    if (yb > 0x3f800000u) return 0x3f800000u;                 // > 1 (incl. +inf) -> 1
    return yb;
}

// geo::central_sin: med3(x, -1, 1); NaN -> -1, else clamped (-0 stays -0)
__device__ __forceinline__ uint32_t rule_sin(uint32_t xb) {
    if ((xb & 0x7fffffffu) > 0x7f800000u) return 0xbf800000u;                    // NaN -> -1
    if ((xb & 0x7fffffffu) > 0x3f800000u) return (xb & 0x80000000u) | 0x3f800000u;  // |x| > 1 -> +-1
    return xb;
}

__global__ __launch_bounds__(256) void check(unsigned long long* bad, uint32_t* first) {
    const uint64_t stride = (uint64_t)gridDim.x * 256u;
    for (uint64_t i = (uint64_t)blockIdx.x * 256u + threadIdx.x; i < (1ull << 32); i += stride) {
        float x = __builtin_bit_cast(float, (uint32_t)i);
        GEO_OPAQUE(x);
        const float y = x + 0.0f;
        const uint32_t a = __builtin_bit_cast(uint32_t, geo::med3_(y, 0.0f, 1.0f));
        const uint32_t b = rule(__builtin_bit_cast(uint32_t, y));
        // c2z is always an arithmetic result: a signaling NaN cannot reach the
        // clamp (and v_med3_f32 would quiet one instead of returning -1), so
        // the input passes a multiply first (x * 1 keeps -0; `one` is opaque)
        float one = 1.0f;
        GEO_OPAQUE(one);
        const float z = x * one;
        const uint32_t c = __builtin_bit_cast(uint32_t, geo::central_sin(z));
        const uint32_t d = rule_sin(__builtin_bit_cast(uint32_t, z));
        if (a != b || c != d) {
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
