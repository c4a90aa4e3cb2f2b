// Microbenchmark: sustained FP32 VALU throughput on gfx950 for
//   v_fma_f32 (scalar), v_pk_fma_f32 (2 x f32 per lane), and the
// dependent-chain latency, to calibrate the roofline of geo_render_kernel.
// CAUTION: built without -fno-slp-vectorize, hipcc packs fma_scalar's
// independent chains into v_pk_fma_f32 too, so both kernels measure packed
// code; tools/ubench/op_rates.hip pins the opcodes with inline asm.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int CHAINS>
__global__ __launch_bounds__(256) void fma_scalar(float* out, int iters, float a, float b) {
    float x[CHAINS];
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = threadIdx.x * 1e-3f + c;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_fmaf(x[c], a, b);
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <int CHAINS>
__global__ __launch_bounds__(256) void fma_packed(float* out, int iters, float a, float b) {
    f2 x[CHAINS];
    const f2 av = {a, a}, bv = {b, b};
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) x[c] = f2{threadIdx.x * 1e-3f + c, c * 0.5f};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int c = 0; c < CHAINS; ++c) x[c] = __builtin_elementwise_fma(x[c], av, bv);
    }
    float s = 0;
#pragma unroll
    for (int c = 0; c < CHAINS; ++c) s += x[c].x + x[c].y;
    if (s == 12345.f) out[threadIdx.x] = s;
}

template <typename K>
double run(K k, int blocks, int iters, double flops_per_thread_iter) {
    float* out;
    hipMalloc(&out, 1024 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f, 1e-4f);
    hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        hipEventRecord(e0);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f, 1e-4f);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    hipFree(out);
    return flops_per_thread_iter * iters * 256.0 * blocks / (best * 1e-3) / 1e12;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    printf("device %s, %d CUs, clock %d kHz\n", p.name, cus, p.clockRate);
    const int iters = 20000;
    for (int wpc : {4, 8, 16, 32}) {
        const int blocks = cus * wpc / 4;  // 4 waves per block
        printf("waves/CU %2d: scalar fma x8 %.1f TF | x4 %.1f TF | packed x4 %.1f TF | packed x8 %.1f TF\n", wpc,
               run(fma_scalar<8>, blocks, iters, 16), run(fma_scalar<4>, blocks, iters, 8),
               run(fma_packed<4>, blocks, iters, 16), run(fma_packed<8>, blocks, iters, 32));
    }
    return 0;
}
