// VALU per pixel of each block of the fan-mode draw (the reference's display
// path, shader.wgsl:58-105) and of the direct mode's out-of-loop work, from
// the device code itself: every block is compiled alone between per-lane
// loads and stores, and its VALU count is that kernel's minus the count of
// the same kernel with the block replaced by a pass-through (the loads,
// stores and addressing).  Never run: compiled to gfx950 assembly only.
//
//   python tools/fan_blocks.py          (compiles this file, prints the table)
#include <hip/hip_runtime.h>

#include "../../schwarzschild_raytracer_wgpu_amd/csrc/geo_pixel.h"

namespace {

struct Args {
    geo::CameraConsts cam;
    float m1[16], m2[16];
    float psi_k, kt;
    const float* fan;
    uint32_t n_fan;
    __amdgpu_buffer_rsrc_t sky;
    uint32_t pitch_b;
    float tw256, th256;
};

struct Quad {  // the padded sky's 2 x 2 block (geo_render.hip PaddedSkyQuad)
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t pitch_b;
    __device__ __forceinline__ void operator()(int ix0, int iy0, uint32_t (&t)[4]) const {
        const uint32_t off = __umul24((uint32_t)(iy0 + 1), pitch_b) + ((uint32_t)(ix0 + 1) << 2);
        t[0] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, 0, 0);
        t[1] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 4u, 0, 0);
        t[2] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, (int)pitch_b, 0);
        t[3] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off + 4u, (int)pitch_b, 0);
    }
};

enum Block { kPass, kRay, kCentral, kFanIndex, kFanLerp, kSkyUV, kSincos, kAtan2, kAsin, kSample, kBlend };

template <int B>
__global__ __launch_bounds__(256) void blk(const float4* __restrict__ in, float4* __restrict__ out, const Args a) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    const float4 x = in[i];
    float4 y = x;
    if constexpr (B == kRay) {
        const uint32_t px = blockIdx.x * 32u + (threadIdx.x & 31u), py = threadIdx.x >> 5;
        geo::pixel_central_dir(a.cam, a.m1, a.psi_k, a.kt, px, py, &y.x, &y.y, &y.z);
    } else if constexpr (B == kCentral) {
        y.x = geo::central_sin(x.z);
        y.y = geo::central_rho(x.x, x.y);
        y.z = geo::rcpf_(y.y);
    } else if constexpr (B == kFanIndex) {
        const geo::FanPos p = geo::fan_pos(a.n_fan, x.x);
        y.x = __uint_as_float(p.i);
        y.y = __uint_as_float(p.i1);
        y.z = p.w;
    } else if constexpr (B == kFanLerp) {
        const geo::FanPos p{__float_as_uint(x.x), __float_as_uint(x.y), x.z};
        y.x = geo::fan_at(a.fan, p);
    } else if constexpr (B == kSkyUV) {
        geo::sky_uv(a.m2, x.x, x.y, x.z, x.w, y.w, &y.x, &y.y);
    } else if constexpr (B == kSincos) {
        geo::sincos_sky_(x.x, &y.x, &y.y);
    } else if constexpr (B == kAtan2) {
        y.x = geo::med3_(geo::atan2_turns_(x.x, x.y), 0.0f, 1.0f);
    } else if constexpr (B == kAsin) {
        y.x = geo::acos_pi_(x.x);
    } else if constexpr (B == kSample) {
        const Quad q{a.sky, a.pitch_b};
        y.x = __uint_as_float(geo::sample_sky_quad_f(q, a.tw256, a.th256, x.x, x.y));
    } else if constexpr (B == kBlend) {
        y.x = __uint_as_float(geo::over_clear(__float_as_uint(x.x), x.y > 0.0f));
    }
    out[i] = y;
}

template __global__ void blk<kPass>(const float4*, float4*, const Args);
template __global__ void blk<kRay>(const float4*, float4*, const Args);
template __global__ void blk<kCentral>(const float4*, float4*, const Args);
template __global__ void blk<kFanIndex>(const float4*, float4*, const Args);
template __global__ void blk<kFanLerp>(const float4*, float4*, const Args);
template __global__ void blk<kSkyUV>(const float4*, float4*, const Args);
template __global__ void blk<kSincos>(const float4*, float4*, const Args);
template __global__ void blk<kAtan2>(const float4*, float4*, const Args);
template __global__ void blk<kAsin>(const float4*, float4*, const Args);
template __global__ void blk<kSample>(const float4*, float4*, const Args);
template __global__ void blk<kBlend>(const float4*, float4*, const Args);

}  // namespace
