// Microbenchmark: issue cost of single VALU opcodes on gfx950 relative to
// v_fma_f32.  Each kernel runs 16 independent chains per lane in ONE inline-asm
// block per iteration (separate asm statements get an s_nop each from the
// hazard recognizer, which halves the issue rate), second operand an SGPR as
// the kernel's frame constants are, 32 waves per CU.  Prices the per-pixel
// preamble: correctly rounded division (v_div_scale/v_rcp/v_div_fmas/
// v_div_fixup), v_sqrt_f32, transcendentals, integer multiplies.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/op_rates.hip -o tools/ubench/op_rates
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_fma(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_fma_f32 %0, %0, %16, %0\nv_fma_f32 %1, %1, %16, %1\nv_fma_f32 %2, %2, %16, %2\nv_fma_f32 %3, %3, %16, %3\nv_fma_f32 %4, %4, %16, %4\nv_fma_f32 %5, %5, %16, %5\nv_fma_f32 %6, %6, %16, %6\nv_fma_f32 %7, %7, %16, %7\nv_fma_f32 %8, %8, %16, %8\nv_fma_f32 %9, %9, %16, %9\nv_fma_f32 %10, %10, %16, %10\nv_fma_f32 %11, %11, %16, %11\nv_fma_f32 %12, %12, %16, %12\nv_fma_f32 %13, %13, %16, %13\nv_fma_f32 %14, %14, %16, %14\nv_fma_f32 %15, %15, %16, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_fmac(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_fmac_f32 %0, %16, %0\nv_fmac_f32 %1, %16, %1\nv_fmac_f32 %2, %16, %2\nv_fmac_f32 %3, %16, %3\nv_fmac_f32 %4, %16, %4\nv_fmac_f32 %5, %16, %5\nv_fmac_f32 %6, %16, %6\nv_fmac_f32 %7, %16, %7\nv_fmac_f32 %8, %16, %8\nv_fmac_f32 %9, %16, %9\nv_fmac_f32 %10, %16, %10\nv_fmac_f32 %11, %16, %11\nv_fmac_f32 %12, %16, %12\nv_fmac_f32 %13, %16, %13\nv_fmac_f32 %14, %16, %14\nv_fmac_f32 %15, %16, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_add(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_add_f32 %0, %16, %0\nv_add_f32 %1, %16, %1\nv_add_f32 %2, %16, %2\nv_add_f32 %3, %16, %3\nv_add_f32 %4, %16, %4\nv_add_f32 %5, %16, %5\nv_add_f32 %6, %16, %6\nv_add_f32 %7, %16, %7\nv_add_f32 %8, %16, %8\nv_add_f32 %9, %16, %9\nv_add_f32 %10, %16, %10\nv_add_f32 %11, %16, %11\nv_add_f32 %12, %16, %12\nv_add_f32 %13, %16, %13\nv_add_f32 %14, %16, %14\nv_add_f32 %15, %16, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_mul(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_mul_f32 %0, %16, %0\nv_mul_f32 %1, %16, %1\nv_mul_f32 %2, %16, %2\nv_mul_f32 %3, %16, %3\nv_mul_f32 %4, %16, %4\nv_mul_f32 %5, %16, %5\nv_mul_f32 %6, %16, %6\nv_mul_f32 %7, %16, %7\nv_mul_f32 %8, %16, %8\nv_mul_f32 %9, %16, %9\nv_mul_f32 %10, %16, %10\nv_mul_f32 %11, %16, %11\nv_mul_f32 %12, %16, %12\nv_mul_f32 %13, %16, %13\nv_mul_f32 %14, %16, %14\nv_mul_f32 %15, %16, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_pkfma(float* out, int iters, float a) {
    f2 x[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) x[c] = f2{threadIdx.x * 1e-3f + c + 1.0f, a};
    for (int i = 0; i < iters; ++i)
        asm volatile("v_pk_fma_f32 %0, %0, %0, %0\nv_pk_fma_f32 %1, %1, %1, %1\nv_pk_fma_f32 %2, %2, %2, %2\nv_pk_fma_f32 %3, %3, %3, %3\nv_pk_fma_f32 %4, %4, %4, %4\nv_pk_fma_f32 %5, %5, %5, %5\nv_pk_fma_f32 %6, %6, %6, %6\nv_pk_fma_f32 %7, %7, %7, %7" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
    float s = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) s += x[c].x + x[c].y;
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_rcp(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_rcp_f32 %0, %0\nv_rcp_f32 %1, %1\nv_rcp_f32 %2, %2\nv_rcp_f32 %3, %3\nv_rcp_f32 %4, %4\nv_rcp_f32 %5, %5\nv_rcp_f32 %6, %6\nv_rcp_f32 %7, %7\nv_rcp_f32 %8, %8\nv_rcp_f32 %9, %9\nv_rcp_f32 %10, %10\nv_rcp_f32 %11, %11\nv_rcp_f32 %12, %12\nv_rcp_f32 %13, %13\nv_rcp_f32 %14, %14\nv_rcp_f32 %15, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_sqrt(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_sqrt_f32 %0, %0\nv_sqrt_f32 %1, %1\nv_sqrt_f32 %2, %2\nv_sqrt_f32 %3, %3\nv_sqrt_f32 %4, %4\nv_sqrt_f32 %5, %5\nv_sqrt_f32 %6, %6\nv_sqrt_f32 %7, %7\nv_sqrt_f32 %8, %8\nv_sqrt_f32 %9, %9\nv_sqrt_f32 %10, %10\nv_sqrt_f32 %11, %11\nv_sqrt_f32 %12, %12\nv_sqrt_f32 %13, %13\nv_sqrt_f32 %14, %14\nv_sqrt_f32 %15, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_rsq(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_rsq_f32 %0, %0\nv_rsq_f32 %1, %1\nv_rsq_f32 %2, %2\nv_rsq_f32 %3, %3\nv_rsq_f32 %4, %4\nv_rsq_f32 %5, %5\nv_rsq_f32 %6, %6\nv_rsq_f32 %7, %7\nv_rsq_f32 %8, %8\nv_rsq_f32 %9, %9\nv_rsq_f32 %10, %10\nv_rsq_f32 %11, %11\nv_rsq_f32 %12, %12\nv_rsq_f32 %13, %13\nv_rsq_f32 %14, %14\nv_rsq_f32 %15, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_divscale(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_div_scale_f32 %0, vcc, %0, %16, %0\nv_div_scale_f32 %1, vcc, %1, %16, %1\nv_div_scale_f32 %2, vcc, %2, %16, %2\nv_div_scale_f32 %3, vcc, %3, %16, %3\nv_div_scale_f32 %4, vcc, %4, %16, %4\nv_div_scale_f32 %5, vcc, %5, %16, %5\nv_div_scale_f32 %6, vcc, %6, %16, %6\nv_div_scale_f32 %7, vcc, %7, %16, %7\nv_div_scale_f32 %8, vcc, %8, %16, %8\nv_div_scale_f32 %9, vcc, %9, %16, %9\nv_div_scale_f32 %10, vcc, %10, %16, %10\nv_div_scale_f32 %11, vcc, %11, %16, %11\nv_div_scale_f32 %12, vcc, %12, %16, %12\nv_div_scale_f32 %13, vcc, %13, %16, %13\nv_div_scale_f32 %14, vcc, %14, %16, %14\nv_div_scale_f32 %15, vcc, %15, %16, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_divfmas(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_div_fmas_f32 %0, %0, %0, %0\nv_div_fmas_f32 %1, %1, %1, %1\nv_div_fmas_f32 %2, %2, %2, %2\nv_div_fmas_f32 %3, %3, %3, %3\nv_div_fmas_f32 %4, %4, %4, %4\nv_div_fmas_f32 %5, %5, %5, %5\nv_div_fmas_f32 %6, %6, %6, %6\nv_div_fmas_f32 %7, %7, %7, %7\nv_div_fmas_f32 %8, %8, %8, %8\nv_div_fmas_f32 %9, %9, %9, %9\nv_div_fmas_f32 %10, %10, %10, %10\nv_div_fmas_f32 %11, %11, %11, %11\nv_div_fmas_f32 %12, %12, %12, %12\nv_div_fmas_f32 %13, %13, %13, %13\nv_div_fmas_f32 %14, %14, %14, %14\nv_div_fmas_f32 %15, %15, %15, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_divfixup(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_div_fixup_f32 %0, %0, %16, %0\nv_div_fixup_f32 %1, %1, %16, %1\nv_div_fixup_f32 %2, %2, %16, %2\nv_div_fixup_f32 %3, %3, %16, %3\nv_div_fixup_f32 %4, %4, %16, %4\nv_div_fixup_f32 %5, %5, %16, %5\nv_div_fixup_f32 %6, %6, %16, %6\nv_div_fixup_f32 %7, %7, %16, %7\nv_div_fixup_f32 %8, %8, %16, %8\nv_div_fixup_f32 %9, %9, %16, %9\nv_div_fixup_f32 %10, %10, %16, %10\nv_div_fixup_f32 %11, %11, %16, %11\nv_div_fixup_f32 %12, %12, %16, %12\nv_div_fixup_f32 %13, %13, %16, %13\nv_div_fixup_f32 %14, %14, %16, %14\nv_div_fixup_f32 %15, %15, %16, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_med3(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_med3_f32 %0, %0, %16, %0\nv_med3_f32 %1, %1, %16, %1\nv_med3_f32 %2, %2, %16, %2\nv_med3_f32 %3, %3, %16, %3\nv_med3_f32 %4, %4, %16, %4\nv_med3_f32 %5, %5, %16, %5\nv_med3_f32 %6, %6, %16, %6\nv_med3_f32 %7, %7, %16, %7\nv_med3_f32 %8, %8, %16, %8\nv_med3_f32 %9, %9, %16, %9\nv_med3_f32 %10, %10, %16, %10\nv_med3_f32 %11, %11, %16, %11\nv_med3_f32 %12, %12, %16, %12\nv_med3_f32 %13, %13, %16, %13\nv_med3_f32 %14, %14, %16, %14\nv_med3_f32 %15, %15, %16, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_floor(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_floor_f32 %0, %0\nv_floor_f32 %1, %1\nv_floor_f32 %2, %2\nv_floor_f32 %3, %3\nv_floor_f32 %4, %4\nv_floor_f32 %5, %5\nv_floor_f32 %6, %6\nv_floor_f32 %7, %7\nv_floor_f32 %8, %8\nv_floor_f32 %9, %9\nv_floor_f32 %10, %10\nv_floor_f32 %11, %11\nv_floor_f32 %12, %12\nv_floor_f32 %13, %13\nv_floor_f32 %14, %14\nv_floor_f32 %15, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_cvt(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_cvt_f32_u32 %0, %0\nv_cvt_f32_u32 %1, %1\nv_cvt_f32_u32 %2, %2\nv_cvt_f32_u32 %3, %3\nv_cvt_f32_u32 %4, %4\nv_cvt_f32_u32 %5, %5\nv_cvt_f32_u32 %6, %6\nv_cvt_f32_u32 %7, %7\nv_cvt_f32_u32 %8, %8\nv_cvt_f32_u32 %9, %9\nv_cvt_f32_u32 %10, %10\nv_cvt_f32_u32 %11, %11\nv_cvt_f32_u32 %12, %12\nv_cvt_f32_u32 %13, %13\nv_cvt_f32_u32 %14, %14\nv_cvt_f32_u32 %15, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_mul24(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_mul_u32_u24 %0, %16, %0\nv_mul_u32_u24 %1, %16, %1\nv_mul_u32_u24 %2, %16, %2\nv_mul_u32_u24 %3, %16, %3\nv_mul_u32_u24 %4, %16, %4\nv_mul_u32_u24 %5, %16, %5\nv_mul_u32_u24 %6, %16, %6\nv_mul_u32_u24 %7, %16, %7\nv_mul_u32_u24 %8, %16, %8\nv_mul_u32_u24 %9, %16, %9\nv_mul_u32_u24 %10, %16, %10\nv_mul_u32_u24 %11, %16, %11\nv_mul_u32_u24 %12, %16, %12\nv_mul_u32_u24 %13, %16, %13\nv_mul_u32_u24 %14, %16, %14\nv_mul_u32_u24 %15, %16, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_mullo(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_mul_lo_u32 %0, %16, %0\nv_mul_lo_u32 %1, %16, %1\nv_mul_lo_u32 %2, %16, %2\nv_mul_lo_u32 %3, %16, %3\nv_mul_lo_u32 %4, %16, %4\nv_mul_lo_u32 %5, %16, %5\nv_mul_lo_u32 %6, %16, %6\nv_mul_lo_u32 %7, %16, %7\nv_mul_lo_u32 %8, %16, %8\nv_mul_lo_u32 %9, %16, %9\nv_mul_lo_u32 %10, %16, %10\nv_mul_lo_u32 %11, %16, %11\nv_mul_lo_u32 %12, %16, %12\nv_mul_lo_u32 %13, %16, %13\nv_mul_lo_u32 %14, %16, %14\nv_mul_lo_u32 %15, %16, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_cndmask(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_cndmask_b32 %0, %0, %0, vcc\nv_cndmask_b32 %1, %1, %1, vcc\nv_cndmask_b32 %2, %2, %2, vcc\nv_cndmask_b32 %3, %3, %3, vcc\nv_cndmask_b32 %4, %4, %4, vcc\nv_cndmask_b32 %5, %5, %5, vcc\nv_cndmask_b32 %6, %6, %6, vcc\nv_cndmask_b32 %7, %7, %7, vcc\nv_cndmask_b32 %8, %8, %8, vcc\nv_cndmask_b32 %9, %9, %9, vcc\nv_cndmask_b32 %10, %10, %10, vcc\nv_cndmask_b32 %11, %11, %11, vcc\nv_cndmask_b32 %12, %12, %12, vcc\nv_cndmask_b32 %13, %13, %13, vcc\nv_cndmask_b32 %14, %14, %14, vcc\nv_cndmask_b32 %15, %15, %15, vcc" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_sin(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_sin_f32 %0, %0\nv_sin_f32 %1, %1\nv_sin_f32 %2, %2\nv_sin_f32 %3, %3\nv_sin_f32 %4, %4\nv_sin_f32 %5, %5\nv_sin_f32 %6, %6\nv_sin_f32 %7, %7\nv_sin_f32 %8, %8\nv_sin_f32 %9, %9\nv_sin_f32 %10, %10\nv_sin_f32 %11, %11\nv_sin_f32 %12, %12\nv_sin_f32 %13, %13\nv_sin_f32 %14, %14\nv_sin_f32 %15, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_exp(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_exp_f32 %0, %0\nv_exp_f32 %1, %1\nv_exp_f32 %2, %2\nv_exp_f32 %3, %3\nv_exp_f32 %4, %4\nv_exp_f32 %5, %5\nv_exp_f32 %6, %6\nv_exp_f32 %7, %7\nv_exp_f32 %8, %8\nv_exp_f32 %9, %9\nv_exp_f32 %10, %10\nv_exp_f32 %11, %11\nv_exp_f32 %12, %12\nv_exp_f32 %13, %13\nv_exp_f32 %14, %14\nv_exp_f32 %15, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_fma2(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_fma_f32 %0, %16, %1, %0\nv_fma_f32 %1, %16, %2, %1\nv_fma_f32 %2, %16, %3, %2\nv_fma_f32 %3, %16, %4, %3\nv_fma_f32 %4, %16, %5, %4\nv_fma_f32 %5, %16, %6, %5\nv_fma_f32 %6, %16, %7, %6\nv_fma_f32 %7, %16, %8, %7\nv_fma_f32 %8, %16, %9, %8\nv_fma_f32 %9, %16, %10, %9\nv_fma_f32 %10, %16, %11, %10\nv_fma_f32 %11, %16, %12, %11\nv_fma_f32 %12, %16, %13, %12\nv_fma_f32 %13, %16, %14, %13\nv_fma_f32 %14, %16, %15, %14\nv_fma_f32 %15, %16, %0, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_fma3(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_fma_f32 %0, %1, %1, %0\nv_fma_f32 %1, %2, %2, %1\nv_fma_f32 %2, %3, %3, %2\nv_fma_f32 %3, %4, %4, %3\nv_fma_f32 %4, %5, %5, %4\nv_fma_f32 %5, %6, %6, %5\nv_fma_f32 %6, %7, %7, %6\nv_fma_f32 %7, %8, %8, %7\nv_fma_f32 %8, %9, %9, %8\nv_fma_f32 %9, %10, %10, %9\nv_fma_f32 %10, %11, %11, %10\nv_fma_f32 %11, %12, %12, %11\nv_fma_f32 %12, %13, %13, %12\nv_fma_f32 %13, %14, %14, %13\nv_fma_f32 %14, %15, %15, %14\nv_fma_f32 %15, %0, %0, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_pkfma2(float* out, int iters, float a) {
    f2 x[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) x[c] = f2{threadIdx.x * 1e-3f + c + 1.0f, a};
    for (int i = 0; i < iters; ++i)
        asm volatile("v_pk_fma_f32 %0, %1, %1, %0\nv_pk_fma_f32 %1, %2, %2, %1\nv_pk_fma_f32 %2, %3, %3, %2\nv_pk_fma_f32 %3, %4, %4, %3\nv_pk_fma_f32 %4, %5, %5, %4\nv_pk_fma_f32 %5, %6, %6, %5\nv_pk_fma_f32 %6, %7, %7, %6\nv_pk_fma_f32 %7, %0, %0, %7" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]));
    float s = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) s += x[c].x + x[c].y;
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_fma_alt(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_fma_f32 %0, %0, %16, %0\nv_fma_f32 %1, %2, %2, %1\nv_fma_f32 %2, %2, %16, %2\nv_fma_f32 %3, %4, %4, %3\nv_fma_f32 %4, %4, %16, %4\nv_fma_f32 %5, %6, %6, %5\nv_fma_f32 %6, %6, %16, %6\nv_fma_f32 %7, %8, %8, %7\nv_fma_f32 %8, %8, %16, %8\nv_fma_f32 %9, %10, %10, %9\nv_fma_f32 %10, %10, %16, %10\nv_fma_f32 %11, %12, %12, %11\nv_fma_f32 %12, %12, %16, %12\nv_fma_f32 %13, %14, %14, %13\nv_fma_f32 %14, %14, %16, %14\nv_fma_f32 %15, %0, %0, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_lit(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_fmac_f32 %0, 0x3e99999a, %1\nv_fmac_f32 %1, 0x3f4ccccd, %2\nv_fmac_f32 %2, 0x3e99999a, %3\nv_fmac_f32 %3, 0x3f4ccccd, %4\nv_fmac_f32 %4, 0x3e99999a, %5\nv_fmac_f32 %5, 0x3f4ccccd, %6\nv_fmac_f32 %6, 0x3e99999a, %7\nv_fmac_f32 %7, 0x3f4ccccd, %8\nv_fmac_f32 %8, 0x3e99999a, %9\nv_fmac_f32 %9, 0x3f4ccccd, %10\nv_fmac_f32 %10, 0x3e99999a, %11\nv_fmac_f32 %11, 0x3f4ccccd, %12\nv_fmac_f32 %12, 0x3e99999a, %13\nv_fmac_f32 %13, 0x3f4ccccd, %14\nv_fmac_f32 %14, 0x3e99999a, %15\nv_fmac_f32 %15, 0x3f4ccccd, %0" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_lit_alt(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_fmac_f32 %0, 0x3e99999a, %1\nv_fma_f32 %1, %2, %2, %1\nv_fmac_f32 %2, 0x3e99999a, %3\nv_fma_f32 %3, %4, %4, %3\nv_fmac_f32 %4, 0x3e99999a, %5\nv_fma_f32 %5, %6, %6, %5\nv_fmac_f32 %6, 0x3e99999a, %7\nv_fma_f32 %7, %8, %8, %7\nv_fmac_f32 %8, 0x3e99999a, %9\nv_fma_f32 %9, %10, %10, %9\nv_fmac_f32 %10, 0x3e99999a, %11\nv_fma_f32 %11, %12, %12, %11\nv_fmac_f32 %12, 0x3e99999a, %13\nv_fma_f32 %13, %14, %14, %13\nv_fmac_f32 %14, 0x3e99999a, %15\nv_fma_f32 %15, %0, %0, %15" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void k_inl(float* out, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    for (int i = 0; i < iters; ++i)
        asm volatile("v_fmac_f32 %0, 0.5, %1\nv_fmac_f32 %1, 2.0, %2\nv_fmac_f32 %2, 0.5, %3\nv_fmac_f32 %3, 2.0, %4\nv_fmac_f32 %4, 0.5, %5\nv_fmac_f32 %5, 2.0, %6\nv_fmac_f32 %6, 0.5, %7\nv_fmac_f32 %7, 2.0, %8\nv_fmac_f32 %8, 0.5, %9\nv_fmac_f32 %9, 2.0, %10\nv_fmac_f32 %10, 0.5, %11\nv_fmac_f32 %11, 2.0, %12\nv_fmac_f32 %12, 0.5, %13\nv_fmac_f32 %13, 2.0, %14\nv_fmac_f32 %14, 0.5, %15\nv_fmac_f32 %15, 2.0, %0" : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]), "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]), "+v"(x[14]), "+v"(x[15]) : "s"(a) : "vcc");
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    if (s == 12345.f) out[threadIdx.x] = s;
}
template <typename K>
float run(K k, int blocks, int iters) {
    float* out;
    (void)hipMalloc(&out, 1024 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
    (void)hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; ++r) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, out, iters, 0.999f);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (ms < best) best = ms;
    }
    (void)hipFree(out);
    return best;
}

int main() {
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 8;  // 32 waves per CU
    const int iters = 2048;
    // clock spin-up: ~0.5 s of FMA work before anything is timed (a cold
    // GPU runs its first milliseconds at a fraction of the boost clock)
    for (int w = 0; w < 200; ++w) hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, nullptr, iters, 0.999f);
    (void)hipDeviceSynchronize();
    const float base = run(k_fma, blocks, iters);
    const double winstr = (double)blocks * 4 * iters * 16;  // wave-instructions
    printf("v_fma_f32: %.3f ms = %.3f wave-instr per SIMD per ns (%.1f TFLOP/s)\n", base,
           winstr / (cus * 4.0) / (base * 1e6), winstr * 64 * 2 / (base * 1e-3) / 1e12);
    struct { const char* n; void (*k)(float*, int, float); int per; } ks[] = {
        {"v_fma_f32 d, s, v_other, d", k_fma2, 16},
        {"v_fma_f32 d, v_o, v_o, d", k_fma3, 16},
        {"v_pk_fma_f32 d, v_o, v_o, d", k_pkfma2, 8},
        {"alternating SGPR / all-VGPR fma", k_fma_alt, 16},
        {"v_fmac_f32 d, literal, v", k_lit, 16},
        {"alternating literal / all-VGPR", k_lit_alt, 16},
        {"v_fmac_f32 d, inline const, v", k_inl, 16},
        {"v_fmac_f32", k_fmac, 16},
        {"v_add_f32", k_add, 16},
        {"v_mul_f32", k_mul, 16},
        {"v_pk_fma_f32 (2 lanes' worth)", k_pkfma, 8},
        {"v_rcp_f32", k_rcp, 16},
        {"v_sqrt_f32", k_sqrt, 16},
        {"v_rsq_f32", k_rsq, 16},
        {"v_div_scale_f32", k_divscale, 16},
        {"v_div_fmas_f32", k_divfmas, 16},
        {"v_div_fixup_f32", k_divfixup, 16},
        {"v_med3_f32", k_med3, 16},
        {"v_floor_f32", k_floor, 16},
        {"v_cvt_f32_u32", k_cvt, 16},
        {"v_mul_u32_u24", k_mul24, 16},
        {"v_mul_lo_u32", k_mullo, 16},
        {"v_cndmask_b32", k_cndmask, 16},
        {"v_sin_f32", k_sin, 16},
        {"v_exp_f32", k_exp, 16},
    };
    for (auto& e : ks) {
        const float t = run(e.k, blocks, iters);
        printf("%-30s %.3f ms  cost %.2f x v_fma_f32 per instruction\n", e.n, t, t / base * 16.0 / e.per);
    }
    const float again = run(k_fma, blocks, iters);
    printf("v_fma_f32 again: %.3f ms (clock drift check)\n", again);
    return 0;
}
