// Cost breakdown of the per-pixel pipeline OUTSIDE the RK4 loop on the
// config-3 frame (3840x2160): variants drop one part each (outputs differ;
// timing only), interleaved rounds in one process.  Product-like launch:
// 2-D grid of 8x32-pixel tiles, one pixel per lane.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

#include "../../include/geo/geo.h"
#include "../../schwarzschild_raytracer_wgpu_amd/csrc/geo_pixel.h"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

struct Args {
    geo_frame f;
    geo::PixelConsts k;
    uint32_t w, h;
    float inv_w, inv_h, kt;
    const uint32_t* sky;
    uint32_t sw, sh;
    uint32_t* out;
};

enum { kInit = 1, kNewton = 2, kUV = 4, kSample = 8, kLoop = 16 };

template <int P>
__global__ __launch_bounds__(256) void kern(const Args a) {
    const uint32_t px = blockIdx.x * 8 + (threadIdx.x % 8);
    const uint32_t py = blockIdx.y * 32 + (threadIdx.x / 8);
    if (px >= a.w || py >= a.h) return;
    float c2x, c2y, c2z;
    geo::pixel_central_dir(a.f.display_to_movement, a.f.movement_to_central, a.f.psi_factor_and_position[0], a.kt,
                           a.w, a.h, a.inv_w, a.inv_h, px, py, &c2x, &c2y, &c2z);
    const float st = geo::clampf_(c2z, -1.0f, 1.0f);
    const float ct = geo::central_rho(c2x, c2y);
    float ang = 0.3f * st;
    uint32_t steps = 0;
    if constexpr ((P & kLoop) != 0) {
        ang = geo::geodesic_angle_v<4, geo::kCurvedOut>(a.k, st, ct, &steps);
    } else if constexpr ((P & kInit) != 0) {
        float U, UB, early;
        if (!geo::geodesic_init(a.k, st, ct, &early, &U, &UB)) {
            ang = early;
        } else if constexpr ((P & kNewton) != 0) {
            float NU, NUB;
            geo::rk4_step<geo::kCurvedOut>(U, UB, a.k.step, a.k.hh, a.k.hh2, a.k.hhh, a.k.h6, a.k.h2_6, &NU, &NUB);
            ang = geo::newton_angle<geo::kCurvedOut>(a.k, U, UB, NU, NUB, 1);
        } else {
            ang = U + UB;
        }
    }
    const float lam = geo::kPi2 - ang;
    float U = 0.5f + 0.5f * c2x, V = 0.5f + 0.5f * c2y;
    if constexpr ((P & kUV) != 0) geo::sky_uv(a.f.central_to_uv, c2x, c2y, ct, lam, &U, &V);
    uint32_t rgba;
    if constexpr ((P & kSample) != 0) {
        const uint32_t* sky = a.sky;
        rgba = lam < geo::kBlackHoleLambda ? geo::kBlackRGBA
                                           : geo::sample_sky([sky](uint32_t i) { return sky[i]; }, a.sw, a.sh, true, U, V);
    } else {
        rgba = __float_as_uint(U) ^ __float_as_uint(V) ^ __float_as_uint(lam) ^ steps;
    }
    a.out[(size_t)py * a.w + px] = rgba;
}

typedef void (*KFn)(Args);

int main() {
    const uint32_t W = 3840, H = 2160;
    geo_observer* o;
    geo_observer_create(1.0, M_PI / 2, W, H, &o);
    geo_observer_set_position(o, 2.5, 0.0, 0.1);
    Args a;
    geo_observer_calc_transformation_pipeline(o, &a.f);
    a.k = geo::make_consts(1.0f, 50.0f, (float)geo_observer_radial_position(o), (float)(M_PI / 100.0), 2048);
    a.w = W; a.h = H;
    a.inv_w = 1.0f / W; a.inv_h = 1.0f / H;
    a.kt = geo::aberration_kt(a.f.psi_factor_and_position[0]);
    a.sw = 4096; a.sh = 2048;
    std::vector<uint32_t> sky(a.sw * a.sh);
    for (size_t i = 0; i < sky.size(); ++i) sky[i] = 0xFF000000u | (uint32_t)(i * 2654435761u >> 8);
    uint32_t* dsky;
    CK(hipMalloc(&dsky, sky.size() * 4));
    CK(hipMemcpy(dsky, sky.data(), sky.size() * 4, hipMemcpyHostToDevice));
    a.sky = dsky;
    CK(hipMalloc(&a.out, (size_t)W * H * 4));
    struct Var { const char* name; KFn fn; };
    Var vars[] = {
        {"camera + store", kern<0>},
        {"+ init", kern<kInit>},
        {"+ init + 1 step + Newton", kern<kInit | kNewton>},
        {"+ init + Newton + UV", kern<kInit | kNewton | kUV>},
        {"no-loop pipeline (all parts)", kern<kInit | kNewton | kUV | kSample>},
        {"all but UV (sample at c2)", kern<kInit | kNewton | kSample>},
        {"all but Newton", kern<kInit | kUV | kSample>},
        {"full product pixel (loop)", kern<kLoop | kUV | kSample>},
        {"loop, no UV/sample", kern<kLoop>},
    };
    const int NV = sizeof(vars) / sizeof(vars[0]);
    std::vector<std::vector<float>> t(NV);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const dim3 grid((W + 7) / 8, (H + 31) / 32);
    for (int round = 0; round < 40; ++round) {
        for (int v = 0; v < NV; ++v) {
            hipEventRecord(e0);
            hipLaunchKernelGGL(vars[v].fn, grid, dim3(256), 0, 0, a);
            hipEventRecord(e1);
            CK(hipEventSynchronize(e1));
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (round >= 10) t[v].push_back(ms);
        }
    }
    for (int v = 0; v < NV; ++v) {
        std::sort(t[v].begin(), t[v].end());
        printf("%-34s median %.4f ms  min %.4f ms\n", vars[v].name, t[v][t[v].size() / 2], t[v][0]);
    }
    return 0;
}
