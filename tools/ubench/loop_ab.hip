// A/B harness: times the RK4 loop variants of geo_pixel.h (geodesic_angle_v<V>)
// inside the full per-pixel pipeline on the config-3 frame (3840x2160, 2048
// budget), interleaved rounds in ONE process (cdna_hip_programming.md §5.4
// rule 24), and checks every variant's output equals variant 0's bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
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
    unsigned long long* slots;
};

// Everything but the RK4 loop: ray set-up, ONE step, Newton, UV, sample.
template <int KIND>
__device__ float noloop_angle(const geo::PixelConsts& k, float st, float ct, uint32_t* steps) {
    *steps = 1;
    float U, UB, early;
    if (!geo::geodesic_init(k, st, ct, &early, &U, &UB)) return early;
    float NU, NUB;
    geo::rk4_step<KIND>(U, UB, k.step, k.hh, k.hh2, k.hhh, k.h6, k.h2_6, &NU, &NUB);
    return geo::newton_angle<KIND>(k, U, UB, NU, NUB, 1);
}

template <int V, int TW, int T = 1>
__global__ __launch_bounds__(256) void kern(const Args a) {
    constexpr int TH = 256 / TW;
    __shared__ unsigned long long red[4];
    const uint32_t ntiles = a.tiles_x * ((a.h + TH - 1) / TH);
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    __syncthreads();
    const uint32_t tx = tile % a.tiles_x, ty = tile / a.tiles_x;
    const uint32_t px = tx * TW + threadIdx.x % TW, py = ty * TH + threadIdx.x / TW;
    uint32_t steps = 0;
    if (px < a.w && py < a.h) {
        float c2x, c2y, c2z;
        geo::pixel_central_dir(a.f.display_to_movement, a.f.movement_to_central, a.f.psi_factor_and_position[0],
                               a.kt, a.w, a.h, a.inv_w, a.inv_h, px, py, &c2x, &c2y, &c2z);
        const float st = geo::clampf_(c2z, -1.0f, 1.0f);
        const float ct = geo::central_rho(c2x, c2y);
        const float lam = geo::kPi2 - (V == 0 ? noloop_angle<geo::kCurvedOut>(a.k, st, ct, &steps)
                                              : geo::geodesic_angle_v<(V > 0 ? V : 1), geo::kCurvedOut>(a.k, st, ct, &steps));
        const bool bh = lam < geo::kBlackHoleLambda;
        float U, V2;
        geo::sky_uv(a.f.central_to_uv, c2x, c2y, ct, lam, &U, &V2);
        const uint32_t* sky = a.sky;
        a.out[(size_t)py * a.w + px] =
            bh ? geo::kBlackRGBA : geo::sample_sky([sky](uint32_t i) { return sky[i]; }, a.sw, a.sh, true, U, V2);
    }
    unsigned long long s = steps;
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(&a.slots[(blockIdx.x % 64) * 16], red[0] + red[1] + red[2] + red[3]);
  }
}

// Loop-only ceiling: every lane runs exactly max_steps RK4 steps (the stop
// flags can never fire: su < 0, bound = -inf, hu = +inf), bounded orbit.
template <int V>
__global__ __launch_bounds__(256) void loop_only(geo::PixelConsts k, float* out) {
    // never stops: inside-sphere interval [SU+, HU] = (-inf, inf)
    k.U0 = 0.1f;  // bounded orbit (U = 1 is the unstable photon-sphere equilibrium)
    k.SU = -__builtin_inff();
    k.SUp = -__builtin_inff();
    k.BD = -__builtin_inff();
    k.HU = __builtin_inff();
    k.pf_always = k.pf_eneg = k.pf_barrier = k.pf_falling = k.pf_outgoing = false;
    uint32_t steps;
    // st, ct chosen so rotation > 1e-10 and the ray is slightly off radial
    const float st = 0.3f + 1e-6f * (threadIdx.x & 63), ct = 0.9f;
    const float a = geo::geodesic_angle_v<V, geo::kCurvedOut>(k, st, ct, &steps);
    if (a == 12345.0f) out[blockIdx.x] = (float)steps;
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
    CK(hipMalloc(&a.slots, 64 * 16 * 8));
    struct Var { const char* name; KFn fn; int tw; int flat_sky; int tpb; };
    Var vars[] = {
        {"NO-LOOP 8x32", kern<0, 8>, 8}, {"NO-LOOP 8x32 T=2", kern<0, 8, 2>, 8, 0, 2},
        {"NO-LOOP 8x32 T=4", kern<0, 8, 4>, 8, 0, 4}, {"G=4 8x32 T=2", kern<4, 8, 2>, 8, 0, 2},
        {"G=4 8x32 T=4", kern<4, 8, 4>, 8, 0, 4}, {"G=1 8x32", kern<1, 8>, 8}, {"G=2 8x32", kern<2, 8>, 8}, {"G=3 8x32", kern<3, 8>, 8},
        {"G=4 8x32", kern<4, 8>, 8}, {"G=2 16x16", kern<2, 16>, 16}, {"G=4 16x16", kern<4, 16>, 16},
        {"G=4 32x8", kern<4, 32>, 32},
    };
    const int NV = sizeof(vars) / sizeof(vars[0]);
    std::vector<uint32_t*> outs(NV);
    for (int v = 0; v < NV; ++v) CK(hipMalloc(&outs[v], (size_t)W * H * 4));
    std::vector<std::vector<float>> t(NV);
    std::vector<unsigned long long> steps(NV);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int round = 0; round < 12; ++round) {
        for (int v = 0; v < NV; ++v) {
            a.out = outs[v];
            a.sw = vars[v].flat_sky ? 1 : 4096;
            a.sh = vars[v].flat_sky ? 1 : 2048;
            a.tiles_x = (W + vars[v].tw - 1) / vars[v].tw;
            const uint32_t th = 256 / vars[v].tw;
            const uint32_t tpb = vars[v].tpb ? vars[v].tpb : 1;
            const uint32_t grid = (a.tiles_x * ((H + th - 1) / th) + tpb - 1) / tpb;
            CK(hipMemset(a.slots, 0, 64 * 16 * 8));
            hipEventRecord(e0);
            hipLaunchKernelGGL(vars[v].fn, dim3(grid), dim3(256), 0, 0, a);
            hipEventRecord(e1);
            CK(hipEventSynchronize(e1));
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            if (round >= 2) t[v].push_back(ms);
            std::vector<unsigned long long> sl(64 * 16);
            CK(hipMemcpy(sl.data(), a.slots, sl.size() * 8, hipMemcpyDeviceToHost));
            unsigned long long sum = 0;
            for (int i = 0; i < 64; ++i) sum += sl[i * 16];
            steps[v] = sum;
        }
    }
    {
        // loop-only ceiling: 2048 x 256 blocks x 4 waves per CU-generation
        geo::PixelConsts kk = a.k;
        kk.max_steps = 2000;
        float* dummy;
        CK(hipMalloc(&dummy, 1 << 20));
        const int blocks = 256 * 8 * 4;
        void (*lk[4])(geo::PixelConsts, float*) = {loop_only<1>, loop_only<2>, loop_only<3>, loop_only<4>};
        for (int v = 0; v < 4; ++v) {
            std::vector<float> tt;
            for (int r = 0; r < 7; ++r) {
                hipEventRecord(e0);
                hipLaunchKernelGGL(lk[v], dim3(blocks), dim3(256), 0, 0, kk, dummy);
                hipEventRecord(e1);
                CK(hipEventSynchronize(e1));
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (r) tt.push_back(ms);
            }
            std::sort(tt.begin(), tt.end());
            const double st = 2000.0 * blocks * 256;
            printf("loop-only G=%d: %.3f ms, %.3e steps/s = %.1f TF(alg 40 flop/step)\n", v + 1, tt[tt.size() / 2],
                   st / (tt[tt.size() / 2] * 1e-3), 40.0 * st / (tt[tt.size() / 2] * 1e-3) / 1e12);
        }
    }
    std::vector<uint32_t> ref((size_t)W * H), got((size_t)W * H);
    CK(hipMemcpy(ref.data(), outs[6], ref.size() * 4, hipMemcpyDeviceToHost));
    for (int v = 0; v < NV; ++v) {
        CK(hipMemcpy(got.data(), outs[v], got.size() * 4, hipMemcpyDeviceToHost));
        const bool same = vars[v].flat_sky || memcmp(ref.data(), got.data(), ref.size() * 4) == 0;
        std::sort(t[v].begin(), t[v].end());
        const double med = t[v][t[v].size() / 2];
        const double tf = 40.0 * steps[v] / (med * 1e-3) / 1e12;
        printf("%-28s median %.4f ms min %.4f ms  steps %llu  ~%.1f TF(alg, w/o newton)  %s\n", vars[v].name, med,
               t[v][0], steps[v], tf, same ? "bit-identical" : "MISMATCH");
    }
    return 0;
}
