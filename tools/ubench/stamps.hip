// Diagnostic build (never the product): per-stage wave-cycle shares of the
// render pipeline via s_memtime stamps (cdna_hip_programming.md §7 "In-kernel
// stamps").  Read the SHARES, not the absolute time (stamps add waits).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "../../include/geo/geo.h"
#include "../../schwarzschild_raytracer_wgpu_amd/csrc/geo_pixel.h"

struct Args {
    geo_frame f;
    geo::PixelConsts k;
    uint32_t w, h, tiles_x;
    float inv_w, inv_h, kt;
    const uint32_t* sky;
    uint32_t sw, sh;
    uint32_t* out;
    unsigned long long* acc;  // [6] cycle sums + [1] waves
};

__device__ __forceinline__ unsigned long long stamp() {
    unsigned long long t;
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
    __builtin_amdgcn_sched_barrier(0);
    return t;
}

__global__ __launch_bounds__(256) void kern(const Args a) {
    const unsigned long long t0 = stamp();
    const uint32_t tx = blockIdx.x % a.tiles_x, ty = blockIdx.x / a.tiles_x;
    const uint32_t px = tx * 8 + threadIdx.x % 8, py = ty * 32 + threadIdx.x / 8;
    const bool in = px < a.w && py < a.h;
    float c2x = 0, c2y = 0, c2z = 1;
    if (in)
        geo::pixel_central_dir(a.f.display_to_movement, a.f.movement_to_central, a.f.psi_factor_and_position[0],
                               a.kt, a.w, a.h, a.inv_w, a.inv_h, px, py, &c2x, &c2y, &c2z);
    const float st = geo::clampf_(c2z, -1.0f, 1.0f);
    const float ct = geo::central_rho(c2x, c2y);
    const unsigned long long t1 = stamp();
    uint32_t steps = 0;
    float lam = 0;
    if (in) lam = geo::kPi2 - geo::geodesic_angle_v<4, geo::kCurvedOut>(a.k, st, ct, &steps);
    const unsigned long long t2 = stamp();
    float U = 0, V = 0;
    const bool bh = lam < geo::kBlackHoleLambda;
    if (in) geo::sky_uv(a.f.central_to_uv, c2x, c2y, ct, lam, &U, &V);
    const unsigned long long t3 = stamp();
    if (in) {
        const uint32_t* sky = a.sky;
        a.out[(size_t)py * a.w + px] =
            bh ? geo::kBlackRGBA : geo::sample_sky([sky](uint32_t i) { return sky[i]; }, a.sw, a.sh, true, U, V);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t4 = stamp();
    if ((threadIdx.x & 63) == 0) {
        unsigned long long* r = a.acc + ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * 5;
        r[0] = t1 - t0;
        r[1] = t2 - t1;
        r[2] = t3 - t2;
        r[3] = t4 - t3;
        r[4] = t4 - t0;
    }
}

int main() {
    const uint32_t W = 3840, H = 2160;
    geo_observer* o;
    geo_observer_create(1.0, M_PI / 2, W, H, &o);
    geo_observer_set_position(o, 2.5, 0.0, 0.1);
    Args a;
    geo_observer_calc_transformation_pipeline(o, &a.f);
    a.k = geo::make_consts(1.0f, 50.0f, (float)geo_observer_radial_position(o), (float)(M_PI / 100.0), 2048);
    a.w = W; a.h = H; a.inv_w = 1.0f / W; a.inv_h = 1.0f / H;
    a.kt = geo::aberration_kt(a.f.psi_factor_and_position[0]);
    a.sw = 4096; a.sh = 2048;
    std::vector<uint32_t> sky(a.sw * a.sh);
    for (size_t i = 0; i < sky.size(); ++i) sky[i] = 0xFF000000u | (uint32_t)(i * 2654435761u >> 8);
    uint32_t* dsky;
    hipMalloc(&dsky, sky.size() * 4);
    hipMemcpy(dsky, sky.data(), sky.size() * 4, hipMemcpyHostToDevice);
    a.sky = dsky;
    hipMalloc(&a.out, (size_t)W * H * 4);
    a.tiles_x = W / 8;
    const uint32_t grid = a.tiles_x * ((H + 31) / 32);
    const size_t nw = (size_t)grid * 4;
    hipMalloc(&a.acc, nw * 5 * 8);
    for (int r = 0; r < 20; ++r) {
        hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a);
        hipDeviceSynchronize();
    }
    std::vector<unsigned long long> rec(nw * 5);
    hipMemcpy(rec.data(), a.acc, rec.size() * 8, hipMemcpyDeviceToHost);
    unsigned long long acc[8] = {0};
    for (size_t i = 0; i < nw; ++i)
        for (int j = 0; j < 5; ++j) acc[j] += rec[i * 5 + j];
    acc[5] = nw;
    const char* names[] = {"central dir", "geodesic (init+loop+newton)", "sky uv", "sample+store", "total"};
    for (int i = 0; i < 5; ++i)
        printf("%-30s %6.1f%%  %8.0f cycles/wave\n", names[i], 100.0 * acc[i] / acc[4], (double)acc[i] / acc[5]);
    return 0;
}
