// Does the workgroup dispatch ORDER matter for the config-3 frame?  The
// per-tile cost varies ~30x (78 RK4 steps/pixel on average, up to 512 near
// the photon ring), so a long tile dispatched late can stretch the kernel's
// tail.  Variants (timing only; the product-like pixel of parts_ab.hip):
//   natural   row-major tiles (the product's 2-D grid order)
//   lpt       tiles sorted by measured cost, most expensive first
//   reverse   cheapest first (the worst case)
// plus a wave-occupancy profile of the natural order from s_memrealtime
// stamps (active waves per 5 % of the kernel span).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <numeric>
#include <vector>

#include "../../include/geo/geo.h"
#include "../../schwarzschild_raytracer_wgpu_amd/csrc/geo_pixel.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Args {
    geo_frame f;
    geo::PixelConsts k;
    uint32_t w, h, tiles_x;
    float inv_w, inv_h, kt;
    const uint32_t* sky;
    uint32_t sw, sh;
    uint32_t* out;
    const uint32_t* order;      // tile permutation (nullptr = natural)
    uint32_t* steps;            // per-pixel steps (cost probe) or nullptr
    unsigned long long* stamps;  // per-wave (start, end) or nullptr
};

__global__ __launch_bounds__(256) void kern(const Args a) {
    unsigned long long t0 = 0;
    if (a.stamps) t0 = __builtin_amdgcn_s_memrealtime();
    const uint32_t lin = blockIdx.x;
    const uint32_t tile = a.order ? a.order[lin] : lin;
    const uint32_t px = (tile % a.tiles_x) * 8 + (threadIdx.x % 8);
    const uint32_t py = (tile / a.tiles_x) * 32 + (threadIdx.x / 8);
    if (px < a.w && py < a.h) {
        float c2x, c2y, c2z;
        geo::pixel_central_dir(a.f.display_to_movement, a.f.movement_to_central, a.f.psi_factor_and_position[0],
                               a.kt, a.w, a.h, a.inv_w, a.inv_h, px, py, &c2x, &c2y, &c2z);
        const float st = geo::clampf_(c2z, -1.0f, 1.0f);
        const float ct = geo::central_rho(c2x, c2y);
        uint32_t steps = 0;
        const float lam = geo::kPi2 - geo::geodesic_angle_v<4, geo::kCurvedOut>(a.k, st, ct, &steps);
        float U, V;
        geo::sky_uv(a.f.central_to_uv, c2x, c2y, ct, lam, &U, &V);
        const uint32_t* sky = a.sky;
        a.out[(size_t)py * a.w + px] = lam < geo::kBlackHoleLambda
                                           ? geo::kBlackRGBA
                                           : geo::sample_sky([sky](uint32_t i) { return sky[i]; }, a.sw, a.sh,
                                                             true, U, V);
        if (a.steps) a.steps[(size_t)py * a.w + px] = steps;
    }
    if (a.stamps) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        if ((threadIdx.x & 63) == 0) {
            unsigned long long* r = a.stamps + ((size_t)lin * 4 + (threadIdx.x >> 6)) * 2;
            r[0] = t0;
            r[1] = t1;
        }
    }
}

// Persistent variant: 8 blocks of 256 per CU; each WAVE pulls 8x8-pixel tiles
// from its XCD's queue head (one returning atomicAdd per tile, the next ticket
// fetched before the current tile is shaded).  XCD x owns tiles x, x+8, ...
__device__ __forceinline__ uint32_t xcc_id() {
    uint32_t v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 7u;
}

__device__ __forceinline__ void shade(const Args& a, uint32_t px, uint32_t py) {
    float c2x, c2y, c2z;
    geo::pixel_central_dir(a.f.display_to_movement, a.f.movement_to_central, a.f.psi_factor_and_position[0], a.kt,
                           a.w, a.h, a.inv_w, a.inv_h, px, py, &c2x, &c2y, &c2z);
    const float st = geo::clampf_(c2z, -1.0f, 1.0f);
    const float ct = geo::central_rho(c2x, c2y);
    uint32_t steps = 0;
    const float lam = geo::kPi2 - geo::geodesic_angle_v<4, geo::kCurvedOut>(a.k, st, ct, &steps);
    float U, V;
    geo::sky_uv(a.f.central_to_uv, c2x, c2y, ct, lam, &U, &V);
    const uint32_t* sky = a.sky;
    a.out[(size_t)py * a.w + px] =
        lam < geo::kBlackHoleLambda
            ? geo::kBlackRGBA
            : geo::sample_sky([sky](uint32_t i) { return sky[i]; }, a.sw, a.sh, true, U, V);
}

template <int PER>
__global__ __launch_bounds__(256) void kern_persist(const Args a, uint32_t* heads, uint32_t ntiles) {
    const uint32_t x = xcc_id();
    const uint32_t tx = a.w / 8;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t tk = 0;
    if (lane == 0) tk = atomicAdd(&heads[x * 32], 1u);
    tk = __builtin_amdgcn_readfirstlane(tk);
    while (true) {
        const uint32_t t0 = (tk * PER) * 8 + x;
        if (t0 >= ntiles) break;
        uint32_t nx = 0;
        if (lane == 0) nx = atomicAdd(&heads[x * 32], 1u);
#pragma unroll
        for (int j = 0; j < PER; ++j) {
            const uint32_t t = t0 + 8u * j;
            if (t < ntiles) {
                const uint32_t px = (t % tx) * 8 + lane % 8, py = (t / tx) * 8 + lane / 8;
                if (py < a.h) shade(a, px, py);
            }
        }
        tk = __builtin_amdgcn_readfirstlane(nx);
    }
}

int main() {
    const uint32_t W = 3840, H = 2160;
    geo_observer* o;
    geo_observer_create(1.0, M_PI / 2, W, H, &o);
    geo_observer_set_position(o, 2.5, 0.0, 0.1);
    Args a{};
    geo_observer_calc_transformation_pipeline(o, &a.f);
    a.k = geo::make_consts(1.0f, 50.0f, (float)geo_observer_radial_position(o), (float)(M_PI / 100.0), 2048);
    a.w = W; a.h = H; a.inv_w = 1.0f / W; a.inv_h = 1.0f / H;
    a.kt = geo::aberration_kt(a.f.psi_factor_and_position[0]);
    a.sw = 4096; a.sh = 2048;
    std::vector<uint32_t> sky(a.sw * a.sh);
    for (size_t i = 0; i < sky.size(); ++i) sky[i] = 0xFF000000u | (uint32_t)(i * 2654435761u >> 8);
    uint32_t* dsky;
    CK(hipMalloc(&dsky, sky.size() * 4));
    CK(hipMemcpy(dsky, sky.data(), sky.size() * 4, hipMemcpyHostToDevice));
    a.sky = dsky;
    CK(hipMalloc(&a.out, (size_t)W * H * 4));
    a.tiles_x = W / 8;
    const uint32_t tiles_y = (H + 31) / 32, ntiles = a.tiles_x * tiles_y;

    // cost probe: per-tile sum of per-wave max steps
    uint32_t* dsteps;
    CK(hipMalloc(&dsteps, (size_t)W * H * 4));
    a.steps = dsteps;
    hipLaunchKernelGGL(kern, dim3(ntiles), dim3(256), 0, 0, a);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> st((size_t)W * H);
    CK(hipMemcpy(st.data(), dsteps, st.size() * 4, hipMemcpyDeviceToHost));
    a.steps = nullptr;
    std::vector<double> cost(ntiles, 0.0);
    for (uint32_t t = 0; t < ntiles; ++t)
        for (int wv = 0; wv < 4; ++wv) {
            uint32_t m = 0;
            for (int l = 0; l < 64; ++l) {
                const uint32_t px = (t % a.tiles_x) * 8 + l % 8, py = (t / a.tiles_x) * 32 + wv * 8 + l / 8;
                if (py < H) m = std::max(m, st[(size_t)py * W + px]);
            }
            cost[t] += m + 40.0;  // + the per-pixel preamble/epilogue in step units (~0.5 of the frame's 78)
        }
    std::vector<uint32_t> lpt(ntiles), rev(ntiles);
    std::iota(lpt.begin(), lpt.end(), 0u);
    std::stable_sort(lpt.begin(), lpt.end(), [&](uint32_t x, uint32_t y) { return cost[x] > cost[y]; });
    rev.assign(lpt.rbegin(), lpt.rend());
    uint32_t *dlpt, *drev;
    CK(hipMalloc(&dlpt, ntiles * 4));
    CK(hipMalloc(&drev, ntiles * 4));
    CK(hipMemcpy(dlpt, lpt.data(), ntiles * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(drev, rev.data(), ntiles * 4, hipMemcpyHostToDevice));
    const double cmax = *std::max_element(cost.begin(), cost.end());
    const double csum = std::accumulate(cost.begin(), cost.end(), 0.0);
    printf("tiles %u  cost max/mean %.1f\n", ntiles, cmax / (csum / ntiles));

    struct Var { const char* name; const uint32_t* order; };
    Var vars[] = {{"natural", nullptr}, {"lpt", dlpt}, {"reverse", drev}};
    const int NV = 3;
    std::vector<std::vector<float>> tm(NV);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int round = 0; round < 60; ++round)
        for (int v = 0; v < NV; ++v) {
            a.order = vars[v].order;
            hipEventRecord(e0);
            hipLaunchKernelGGL(kern, dim3(ntiles), dim3(256), 0, 0, a);
            hipEventRecord(e1);
            CK(hipEventSynchronize(e1));
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (round >= 10) tm[v].push_back(ms);
        }
    uint32_t* dheads;
    CK(hipMalloc(&dheads, 8 * 32 * 4));
    const uint32_t wtiles = (W / 8) * ((H + 7) / 8);
    int nblk_list[] = {2048, 1024, 4096};
    std::vector<std::vector<float>> tp(6);
    for (int round = 0; round < 60; ++round)
        for (int v = 0; v < 6; ++v) {
            CK(hipMemsetAsync(dheads, 0, 8 * 32 * 4));
            hipEventRecord(e0);
            if (v < 3) hipLaunchKernelGGL(kern_persist<1>, dim3(nblk_list[v]), dim3(256), 0, 0, a, dheads, wtiles);
            else hipLaunchKernelGGL(kern_persist<2>, dim3(nblk_list[v - 3]), dim3(256), 0, 0, a, dheads, wtiles);
            hipEventRecord(e1);
            CK(hipEventSynchronize(e1));
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (round >= 10) tp[v].push_back(ms);
        }
    {  // persistent output == natural output
        std::vector<uint32_t> o1((size_t)W * H), o2((size_t)W * H);
        CK(hipMemcpy(o1.data(), a.out, o1.size() * 4, hipMemcpyDeviceToHost));
        a.order = nullptr;
        hipLaunchKernelGGL(kern, dim3(ntiles), dim3(256), 0, 0, a);
        CK(hipMemcpy(o2.data(), a.out, o2.size() * 4, hipMemcpyDeviceToHost));
        printf("persistent output %s natural\n", o1 == o2 ? "==" : "!=");
    }
    for (int v = 0; v < 6; ++v) {
        std::sort(tp[v].begin(), tp[v].end());
        printf("persist PER=%d blocks=%d  median %.4f ms  min %.4f ms\n", v < 3 ? 1 : 2, nblk_list[v % 3],
               tp[v][tp[v].size() / 2], tp[v][0]);
    }
    for (int v = 0; v < NV; ++v) {
        std::sort(tm[v].begin(), tm[v].end());
        printf("%-10s median %.4f ms  min %.4f ms\n", vars[v].name, tm[v][tm[v].size() / 2], tm[v][0]);
    }

    // occupancy profile (natural and lpt orders)
    unsigned long long* dst;
    const size_t nw = (size_t)ntiles * 4;
    CK(hipMalloc(&dst, nw * 16));
    for (int v = 0; v < 2; ++v) {
        a.order = vars[v].order;
        a.stamps = dst;
        for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(kern, dim3(ntiles), dim3(256), 0, 0, a);
        CK(hipDeviceSynchronize());
        std::vector<unsigned long long> s(nw * 2);
        CK(hipMemcpy(s.data(), dst, s.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull, t1 = 0;
        for (size_t i = 0; i < nw; ++i) {
            t0 = std::min(t0, s[2 * i]);
            t1 = std::max(t1, s[2 * i + 1]);
        }
        const double span = (double)(t1 - t0);
        const int NB = 20;
        std::vector<double> busy(NB, 0.0);  // wave-ticks per bin
        for (size_t i = 0; i < nw; ++i) {
            const double b = s[2 * i] - t0, e = s[2 * i + 1] - t0;
            for (int k = 0; k < NB; ++k) {
                const double lo = span * k / NB, hi = span * (k + 1) / NB;
                const double ov = std::min(e, hi) - std::max(b, lo);
                if (ov > 0) busy[k] += ov;
            }
        }
        printf("%s: span %.1f us (100 MHz clock); mean active waves per 5%% bin:\n  ", vars[v].name, span / 100.0);
        for (int k = 0; k < NB; ++k) printf("%.0f ", busy[k] / (span / NB));
        printf("\n");
    }
    a.stamps = nullptr;
    return 0;
}
