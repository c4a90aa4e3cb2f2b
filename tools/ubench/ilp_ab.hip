// Is the RK4 loop issue-bound or latency-bound?  The render loop's step is a
// dependent chain (depth ~9 of its 14 ops), one ray per lane.  Variants of
// the same 14-op scaled RK4 step (geo_pixel.h rk4_step) with no exit test,
// fixed step count, 32 waves/CU:
//   1x        one ray per lane (the product's loop body)
//   2x        two independent rays per lane, scalar ops interleaved
//   2x-pk     two rays per lane as float2: v_pk_fma_f32 / v_pk_add_f32
// Reported as RK4 steps per second (rays x steps / time).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f2 __attribute__((ext_vector_type(2)));

struct H {
    float h, hh, hh2, hhh, h6, h2_6;
};

__device__ __forceinline__ float F(float u) { return __builtin_fmaf(u, u, -u); }
__device__ __forceinline__ void step1(float& U, float& B, const H& c) {
    const float fu = F(U);
    const float au = __builtin_fmaf(c.hh, B, U);
    const float uh = __builtin_fmaf(c.h, B, U);
    const float fa = F(au);
    const float bu = __builtin_fmaf(c.hh2, fu, au);
    const float fb = F(bu);
    const float cu = __builtin_fmaf(c.hhh, fa, uh);
    const float fc = F(cu);
    const float fab = fa + fb;
    U = __builtin_fmaf(c.h2_6, fu + fab, uh);
    B = __builtin_fmaf(c.h6, __builtin_fmaf(2.0f, fab, fu) + fc, B);
}

__device__ __forceinline__ f2 F2(f2 u) { return __builtin_elementwise_fma(u, u, -u); }
__device__ __forceinline__ f2 fma2(float a, f2 b, f2 c) { return __builtin_elementwise_fma(f2{a, a}, b, c); }
__device__ __forceinline__ void step2(f2& U, f2& B, const H& c) {
    const f2 fu = F2(U);
    const f2 au = fma2(c.hh, B, U);
    const f2 uh = fma2(c.h, B, U);
    const f2 fa = F2(au);
    const f2 bu = fma2(c.hh2, fu, au);
    const f2 fb = F2(bu);
    const f2 cu = fma2(c.hhh, fa, uh);
    const f2 fc = F2(cu);
    const f2 fab = fa + fb;
    U = fma2(c.h2_6, fu + fab, uh);
    B = fma2(c.h6, __builtin_elementwise_fma(f2{2.0f, 2.0f}, fab, fu) + fc, B);
}

__global__ __launch_bounds__(256) void k1(float* out, int steps, H c) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    float U = 0.03f + 1e-9f * i, B = 0.01f;
    for (int s = 0; s < steps; s += 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) step1(U, B, c);
    }
    out[i] = U + B;
}

__global__ __launch_bounds__(256) void k2(float* out, int steps, H c) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    float U0 = 0.03f + 1e-9f * i, B0 = 0.01f, U1 = 0.031f + 1e-9f * i, B1 = 0.011f;
    for (int s = 0; s < steps; s += 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            step1(U0, B0, c);
            step1(U1, B1, c);
        }
    }
    out[i] = U0 + B0 + U1 + B1;
}

__global__ __launch_bounds__(256) void k2p(float* out, int steps, H c) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    f2 U = {0.03f + 1e-9f * i, 0.031f + 1e-9f * i}, B = {0.01f, 0.011f};
    for (int s = 0; s < steps; s += 4) {
#pragma unroll
        for (int j = 0; j < 4; ++j) step2(U, B, c);
    }
    out[i] = U.x + B.x + U.y + B.y;
}

int main() {
    const float h = 3.14159265f / 100.0f;
    H c{h, h * 0.5f, h * h * 0.25f, h * h * 0.5f, h / 6.0f, h * h / 6.0f};
    const int blocks = 256 * 8 * 8;  // 8 resident blocks/CU, 8 rounds
    float* out;
    hipMalloc(&out, (size_t)blocks * 256 * 4);
    const int steps = 512;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    struct V { const char* name; void (*fn)(float*, int, H); int rays; };
    V vs[] = {{"1x", k1, 1}, {"2x", k2, 2}, {"2x-pk", k2p, 2}};
    std::vector<std::vector<float>> t(3);
    for (int r = 0; r < 25; ++r)
        for (int v = 0; v < 3; ++v) {
            // equal ray counts: the 2-ray kernels run half the blocks
            const int nb = blocks / vs[v].rays;
            hipEventRecord(e0);
            hipLaunchKernelGGL(vs[v].fn, dim3(nb), dim3(256), 0, 0, out, steps, c);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (r >= 5) t[v].push_back(ms);
        }
    const double rays = (double)blocks * 256;
    for (int v = 0; v < 3; ++v) {
        std::sort(t[v].begin(), t[v].end());
        const double ms = t[v][t[v].size() / 2];
        printf("%-6s median %.4f ms  %.3e RK4 steps/s  (%.1f TF at 40 flop/step)\n", vs[v].name, ms,
               rays * steps / (ms * 1e-3), rays * steps * 40 / (ms * 1e-3) / 1e12);
    }
    return 0;
}
