// Microbenchmark: the VALU issue rate of gfx950 per SIMD-cycle of the clock
// the chip actually holds.  Each wave runs N iterations
// of one inline-asm block of 16 VALU instructions over CH independent chains
// (16 / CH dependent instructions per chain per block), and stamps
// s_memtime (the shader clock) and s_memrealtime (100 MHz) at its start and
// end.  Per configuration:
//   clock  = median over waves of d(memtime) / d(memrealtime) x 100 MHz
//   issue  = waves per SIMD x 16 N / median d(memtime) of the waves
//            (VALU wave-instructions per SIMD-cycle, all waves running
//            together: the grid is one wave-slot generation)
//   event  = the same instructions / (event-timed kernel x 2.4 GHz)
// Swept: waves per SIMD (1, 2, 4, 8), chains (1, 2, 4, 8, 16), and the
// instruction form: v_fma_f32 all-VGPR (VOP3, 8 bytes), v_fmac_f32 all-VGPR
// (VOP2, 4 bytes), v_fma_f32 with an SGPR operand, v_add_f32 (VOP2),
// v_fma_f64 (the band's f64 path).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/issue_sweep.hip -o tools/ubench/issue_sweep
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define R16(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)

// register of chain c for instruction i of the block: 16 / CH instructions per chain
template <int CH>
struct Blk;

// %0..%15 are 16 VGPRs; instruction i writes register (i % CH) so CH chains interleave
#define FMA_I(i) "v_fma_f32 %" #i ", %" #i ", %16, %" #i "\n"
#define FMAC_I(i) "v_fmac_f32 %" #i ", %16, %17\n"
#define ADD_I(i) "v_add_f32 %" #i ", %16, %" #i "\n"

enum Form { kFma = 0, kFmac, kFmaSgpr, kAdd, kFma64, kForms };
static const char* kFormName[kForms] = {"v_fma_f32 v,v,v (VOP3)", "v_fmac_f32 v,v (VOP2)", "v_fma_f32 v,s,v (SGPR)",
                                         "v_add_f32 v,v (VOP2)", "v_fma_f64 v,v,v"};

struct Stamp {
    unsigned long long t0, t1, r0, r1;
};

// CH chains: the 16 instructions of a block cycle through registers x[0..CH-1]
template <int FORM, int CH>
__global__ __launch_bounds__(256) void k_issue(Stamp* st, int iters, float a) {
    float x[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) x[c] = threadIdx.x * 1e-3f + c + 1.0f;
    float b = a + threadIdx.x * 1e-7f;
    double y[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) y[c] = threadIdx.x * 1e-3 + c + 1.0;
    const double da = (double)b;
    __builtin_amdgcn_s_barrier();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < iters; ++i) {
        if constexpr (FORM == kFma) {
            if constexpr (CH == 16)
                asm volatile(R16(FMA_I)
                             : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                               "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]),
                               "+v"(x[13]), "+v"(x[14]), "+v"(x[15])
                             : "v"(b));
            else if constexpr (CH == 8)
                asm volatile(FMA_I(0) FMA_I(1) FMA_I(2) FMA_I(3) FMA_I(4) FMA_I(5) FMA_I(6) FMA_I(7) FMA_I(0) FMA_I(1)
                                 FMA_I(2) FMA_I(3) FMA_I(4) FMA_I(5) FMA_I(6) FMA_I(7)
                             : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                               "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]),
                               "+v"(x[13]), "+v"(x[14]), "+v"(x[15])
                             : "v"(b));
            else if constexpr (CH == 4)
                asm volatile(FMA_I(0) FMA_I(1) FMA_I(2) FMA_I(3) FMA_I(0) FMA_I(1) FMA_I(2) FMA_I(3) FMA_I(0) FMA_I(1)
                                 FMA_I(2) FMA_I(3) FMA_I(0) FMA_I(1) FMA_I(2) FMA_I(3)
                             : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                               "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]),
                               "+v"(x[13]), "+v"(x[14]), "+v"(x[15])
                             : "v"(b));
            else if constexpr (CH == 2)
                asm volatile(FMA_I(0) FMA_I(1) FMA_I(0) FMA_I(1) FMA_I(0) FMA_I(1) FMA_I(0) FMA_I(1) FMA_I(0) FMA_I(1)
                                 FMA_I(0) FMA_I(1) FMA_I(0) FMA_I(1) FMA_I(0) FMA_I(1)
                             : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                               "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]),
                               "+v"(x[13]), "+v"(x[14]), "+v"(x[15])
                             : "v"(b));
            else
                asm volatile(FMA_I(0) FMA_I(0) FMA_I(0) FMA_I(0) FMA_I(0) FMA_I(0) FMA_I(0) FMA_I(0) FMA_I(0) FMA_I(0)
                                 FMA_I(0) FMA_I(0) FMA_I(0) FMA_I(0) FMA_I(0) FMA_I(0)
                             : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                               "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]),
                               "+v"(x[13]), "+v"(x[14]), "+v"(x[15])
                             : "v"(b));
        } else if constexpr (FORM == kFmac) {
            asm volatile(R16(FMAC_I)
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                           "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]),
                           "+v"(x[14]), "+v"(x[15])
                         : "v"(b), "v"(a));
        } else if constexpr (FORM == kFmaSgpr) {
            asm volatile(R16(FMA_I)
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                           "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]),
                           "+v"(x[14]), "+v"(x[15])
                         : "s"(a));
        } else if constexpr (FORM == kAdd) {
            asm volatile(R16(ADD_I)
                         : "+v"(x[0]), "+v"(x[1]), "+v"(x[2]), "+v"(x[3]), "+v"(x[4]), "+v"(x[5]), "+v"(x[6]),
                           "+v"(x[7]), "+v"(x[8]), "+v"(x[9]), "+v"(x[10]), "+v"(x[11]), "+v"(x[12]), "+v"(x[13]),
                           "+v"(x[14]), "+v"(x[15])
                         : "v"(b));
        } else {  // v_fma_f64 over 8 register pairs, twice
            asm volatile(
                "v_fma_f64 %0, %0, %8, %0\nv_fma_f64 %1, %1, %8, %1\nv_fma_f64 %2, %2, %8, %2\nv_fma_f64 %3, %3, %8, %3\n"
                "v_fma_f64 %4, %4, %8, %4\nv_fma_f64 %5, %5, %8, %5\nv_fma_f64 %6, %6, %8, %6\nv_fma_f64 %7, %7, %8, %7\n"
                "v_fma_f64 %0, %0, %8, %0\nv_fma_f64 %1, %1, %8, %1\nv_fma_f64 %2, %2, %8, %2\nv_fma_f64 %3, %3, %8, %3\n"
                "v_fma_f64 %4, %4, %8, %4\nv_fma_f64 %5, %5, %8, %5\nv_fma_f64 %6, %6, %8, %6\nv_fma_f64 %7, %7, %8, %7\n"
                : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7])
                : "v"(da));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0;
#pragma unroll
    for (int c = 0; c < 16; ++c) s += x[c];
    double sd = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) sd += y[c];
    if ((threadIdx.x & 63) == 0) {
        const size_t w = (size_t)blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64;
        st[w] = Stamp{t0, t1, r0, r1 + (s == 12345.f || sd == 12345.0 ? 1ull : 0ull)};
    }
}

template <int FORM, int CH>
static void run(int cus, int wps, int iters, Stamp* d_st, std::vector<Stamp>& h) {
    const int blocks = cus * wps;  // 256-thread blocks: one wave per SIMD each
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((k_issue<FORM, CH>), dim3(blocks), dim3(256), 0, 0, d_st, iters, 0.999f);
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL((k_issue<FORM, CH>), dim3(blocks), dim3(256), 0, 0, d_st, iters, 0.999f);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const size_t nw = (size_t)blocks * 4;
    h.resize(nw);
    (void)hipMemcpy(h.data(), d_st, nw * sizeof(Stamp), hipMemcpyDeviceToHost);
    std::vector<double> dt(nw), clk(nw);
    for (size_t i = 0; i < nw; ++i) {
        const double t = (double)(h[i].t1 - h[i].t0), r = (double)(h[i].r1 - h[i].r0);
        dt[i] = t;
        clk[i] = r > 0 ? t / r * 100.0 : 0.0;  // MHz
    }
    std::sort(dt.begin(), dt.end());
    std::sort(clk.begin(), clk.end());
    const double med_dt = dt[nw / 2], med_clk = clk[nw / 2];
    const double per_wave = 16.0 * iters * (FORM == kFma64 ? 1.0 : 1.0);
    const double issue = wps * per_wave / med_dt;                        // per SIMD-cycle of the held clock
    const double issue_ev = wps * per_wave / (ms * 1e-3 * 2.4e9);        // per 2.4-GHz cycle, event time
    printf("%-24s chains %2d  waves/SIMD %d  clock %6.0f MHz  issue %.3f /SIMD-cycle (held clock)  %.3f /2.4GHz-cycle (events, %.3f ms)\n",
           kFormName[FORM], CH, wps, med_clk, issue, issue_ev, ms);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
}

int main() {
    int cus = 256;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    Stamp* d_st;
    (void)hipMalloc(&d_st, sizeof(Stamp) * (size_t)cus * 8 * 4);
    std::vector<Stamp> h;
    const int iters = 4096;
    // clock spin-up: ~1 s of FMA work
    for (int w = 0; w < 150; ++w)
        hipLaunchKernelGGL((k_issue<kFma, 16>), dim3(cus * 8), dim3(256), 0, 0, d_st, iters, 0.999f);
    (void)hipDeviceSynchronize();
    for (int wps : {1, 2, 4, 8}) {
        run<kFma, 16>(cus, wps, iters, d_st, h);
        run<kFma, 8>(cus, wps, iters, d_st, h);
        run<kFma, 4>(cus, wps, iters, d_st, h);
        run<kFma, 2>(cus, wps, iters, d_st, h);
        run<kFma, 1>(cus, wps, iters, d_st, h);
        run<kFmac, 16>(cus, wps, iters, d_st, h);
        run<kFmaSgpr, 16>(cus, wps, iters, d_st, h);
        run<kAdd, 16>(cus, wps, iters, d_st, h);
        run<kFma64, 8>(cus, wps, iters, d_st, h);
    }
    run<kFma, 16>(cus, 8, iters, d_st, h);  // clock drift check
    (void)hipFree(d_st);
    return 0;
}
