// geo_pixel.h — the per-pixel f32 path: camera ray, relativistic aberration,
// null-geodesic RK4 + Newton sphere crossing, sky-sphere UV, bilinear sample.
//
// Restates, per pixel and in f32:
//   fs_main                SR/schwarzschild_sphere_shader/shader.wgsl:57-106
//   solve_ray_fan (1 node) SR/simulation/sphere_ray_tracer.rs:35-56
//   solve_geodesic         SR/simulation/sphere_ray_tracer.rs:60-193
// with the node angle theta replaced by the pixel's own angle to the black
// hole.
//
// Evaluation order is fixed (explicit fmaf, no contraction); the CPU oracle
// (oracle/geo_oracle.c, geo_oracle_pixel_f32) restates the same sequence
// independently and tests/ require bit-identical mask, UV, steps and RGBA.
// Any change here must be mirrored there.
#pragma once

#include <stdint.h>

#include "geo_math.h"

namespace geo {

constexpr float kNoValue = 15.0f;          // SphereRayTracer::NO_VALUE, sphere_ray_tracer.rs:22
constexpr float kBlackHoleLambda = -7.0f;  // hit_black_hole threshold, shader.wgsl:88
constexpr int kNewtonIters = 3;            // final_newton_refinements, sphere_ray_tracer.rs:129

// Frame-constant scalars derived from the scene, evaluated identically on
// every lane (and by the oracle).  Names follow sphere_ray_tracer.rs:60-132.
struct PixelConsts {
    float rs, sphere_r, r, step;
    uint32_t max_steps;
    float hh, h6;          // step/2 (step_half :130), step/6
    float r3_2;            // 3*rs/2 (:109)
    float sphere_u;        // 1/sphere_r (:131)
    float schwarz_u;       // 1/rs (:132)
    float u0;              // 1/r (:122)
    float h_over_r2;       // (1 - rs/r)/(r*r) (:123)
    float bound;           // 0.9*min(u0, 1/max(sphere_r, r3_2)) (:127)
    float e_out;           // sqrt(1 - rs/r) (solve_ray_fan :48)
    float e_in;            // sqrt(-1 + rs/r) (:44)
    float barrier_thresh;  // 4/(27 rs^2) (:107)
    bool r_inside_h;       // r < rs (:42)
    bool outside;          // r > rs (:62)
    bool sphere_outside;   // sphere_r > rs (:63)
    bool inside_sphere;    // r < sphere_r (:64)
    bool diff_sides;       // different_sides_3r_2 (:110)
    bool rs_nonzero;
};

GEO_HD PixelConsts make_consts(float rs, float sphere_r, float r, float step, uint32_t max_steps) {
    PixelConsts k;
    k.rs = rs;
    k.sphere_r = sphere_r;
    k.r = r;
    k.step = step;
    k.max_steps = max_steps;
    k.hh = step * 0.5f;
    k.h6 = step / 6.0f;
    k.r3_2 = 1.5f * rs;
    k.sphere_u = 1.0f / sphere_r;
    k.schwarz_u = 1.0f / rs;
    k.u0 = 1.0f / r;
    k.h_over_r2 = (1.0f - rs / r) / (r * r);
    const float um = 1.0f / (sphere_r > k.r3_2 ? sphere_r : k.r3_2);
    k.bound = 0.9f * (k.u0 < um ? k.u0 : um);
    k.e_out = __builtin_sqrtf(1.0f - rs / r);
    k.e_in = __builtin_sqrtf(-1.0f + rs / r);
    k.barrier_thresh = 4.0f / (27.0f * rs * rs);
    k.r_inside_h = r < rs;
    k.outside = r > rs;
    k.sphere_outside = sphere_r > rs;
    k.inside_sphere = r < sphere_r;
    const float dr = r - k.r3_2;
    k.diff_sides = ((r < k.r3_2) != (sphere_r < k.r3_2)) && (__builtin_fabsf(dr) > 1e-10f);
    k.rs_nonzero = rs != 0.0f;
    return k;
}

// One classic RK4 step of u'' = -u + c u^2 (sphere_ray_tracer.rs:137-146),
// f(x) = x (c x - 1).
GEO_HD void rk4_step(float u, float ub, float h, float hh, float h6, float c, float* nu,
                     float* nub) {
    const float fu = fmaf_(c, u, -1.0f) * u;
    const float au = fmaf_(hh, ub, u);
    const float aub = fmaf_(hh, fu, ub);
    const float fa = fmaf_(c, au, -1.0f) * au;
    const float bu = fmaf_(hh, aub, u);
    const float bub = fmaf_(hh, fa, ub);
    const float fb = fmaf_(c, bu, -1.0f) * bu;
    const float cu = fmaf_(h, bub, u);
    const float cub = fmaf_(h, fb, ub);
    const float fc = fmaf_(c, cu, -1.0f) * cu;
    const float s1 = fmaf_(2.0f, aub + bub, ub) + cub;
    const float s2 = fmaf_(2.0f, fa + fb, fu) + fc;
    *nu = fmaf_(h6, s1, u);
    *nub = fmaf_(h6, s2, ub);
}

// Traveled angle of the ray seen at angle theta from the black hole
// (st = sin theta), or kNoValue.  *steps = executed main-loop RK4 steps.
GEO_HD float geodesic_angle(const PixelConsts& k, float st, uint32_t* steps) {
    *steps = 0;
    // solve_ray_fan per node (sphere_ray_tracer.rs:38-49), theta = asin(st)
    const float ct = __builtin_sqrtf(fmaxf_(0.0f, (1.0f - st) * (1.0f + st)));
    const float rotation = k.r * ct;
    bool falling;
    float energy;
    if (k.r_inside_h) {
        falling = false;
        energy = (-st) * k.e_in;
    } else {
        falling = st > 0.0f;
        energy = k.e_out;
    }
    // radial rays (:67-104)
    if (rotation < 1e-10f) {
        if (k.inside_sphere) {
            if (k.outside) {
                if (falling) return k.rs_nonzero ? kNoValue : kPi;
                return 0.0f;
            }
            if (k.sphere_outside) return energy > 0.0f ? 0.0f : kNoValue;
            return 0.0f;
        }
        return (k.sphere_outside && falling) ? 0.0f : kNoValue;
    }
    const float b = rotation / energy;
    const float inv_b2 = 1.0f / (b * b);
    // pre-filters (:106-119)
    const bool barrier = k.rs > 0.0f && inv_b2 < k.barrier_thresh;
    if ((k.inside_sphere && !k.sphere_outside) || (!k.outside && k.sphere_outside && energy < 0.0f) ||
        (barrier && k.diff_sides) || (k.r < k.r3_2 && k.inside_sphere && falling) ||
        (k.r > k.r3_2 && !k.inside_sphere && !falling)) {
        return kNoValue;
    }
    // RK4 init (:122-132); the radicand is clamped at 0 (the reference yields
    // NaN there only for |theta| < ~1e-8, never at a fan node).
    float u = k.u0;
    float ub = __builtin_sqrtf(fmaxf_(0.0f, inv_b2 - k.h_over_r2));
    if (!falling) ub = -ub;
    const float su = k.sphere_u;
    const float c = k.r3_2;
    uint32_t it = 0;
    // main loop (:134-191)
    while (!(k.rs_nonzero && u > k.schwarz_u && ub > 0.0f) && it < k.max_steps && u > 0.0f) {
        float nu, nub;
        rk4_step(u, ub, k.step, k.hh, k.h6, c, &nu, &nub);
        ++it;
        if ((nu > su) != (u > su)) {
            // Newton on the step length from the steeper end (:150-182)
            float ns, wu, wub;
            if (__builtin_fabsf(ub) > __builtin_fabsf(nub)) {
                ns = 0.0f;
                wu = u;
                wub = ub;
            } else {
                ns = k.step;
                wu = nu;
                wub = nub;
            }
            for (int n = 0; n < kNewtonIters; ++n) {
                ns = ns - (wu - su) / wub;
                rk4_step(u, ub, ns, ns * 0.5f, ns / 6.0f, c, &wu, &wub);
            }
            *steps = it;
            return (float)(it - 1u) * k.step + ns;
        }
        if (nu < k.bound) {
            *steps = it;
            return kNoValue;
        }
        u = nu;
        ub = nub;
    }
    *steps = it;
    return kNoValue;
}

// 3x3 part of a column-major mat4 times v (w = 0).
GEO_HD void mat3_mul(const float* m, float x, float y, float z, float* ox, float* oy, float* oz) {
    *ox = fmaf_(m[8], z, fmaf_(m[4], y, m[0] * x));
    *oy = fmaf_(m[9], z, fmaf_(m[5], y, m[1] * x));
    *oz = fmaf_(m[10], z, fmaf_(m[6], y, m[2] * x));
}

// shader.wgsl:60-75 — pixel (px, py) of a width x height frame to the unit
// direction in the black-hole-central frame.  The aberration is applied to
// sin(lambda) directly; cos/sin of phi come from the direction itself, so
// steps 3-5 need no transcendental (the f64 oracle keeps the literal form).
GEO_HD void pixel_central_dir(const float* m0, const float* m1, float psi_k, uint32_t width,
                              uint32_t height, uint32_t px, uint32_t py, float* c2x, float* c2y,
                              float* c2z) {
    const float nx = ((float)(2u * px + 1u) - (float)width) / (float)width;
    const float ny = ((float)height - (float)(2u * py + 1u)) / (float)height;
    // carthesic = (-pos.y, -pos.x, 1, 0) * screen_to_movement.w (:60-63)
    const float cx = -ny * m0[12];
    const float cy = -nx * m0[13];
    const float cz = m0[14];
    float dx, dy, dz;
    mat3_mul(m0, cx, cy, cz, &dx, &dy, &dz);
    const float inv = 1.0f / __builtin_sqrtf(fmaf_(dz, dz, fmaf_(dy, dy, dx * dx)));
    dx *= inv;
    dy *= inv;
    dz *= inv;
    // aberration (:69-70): sin(lambda') = (s - k)/(1 - s k)
    const float s = clampf_(dz, -1.0f, 1.0f);
    const float q = clampf_((s - psi_k) / fmaf_(-s, psi_k, 1.0f), -1.0f, 1.0f);
    const float cl = __builtin_sqrtf(fmaxf_(0.0f, (1.0f - q) * (1.0f + q)));
    const float rho = __builtin_sqrtf(fmaf_(dy, dy, dx * dx));
    float cp = 1.0f, sp = 0.0f;
    if (rho > 0.0f) {
        cp = dx / rho;
        sp = dy / rho;
    }
    // to_cart, then movement_to_central (:72-74)
    mat3_mul(m1, cp * cl, sp * cl, q, c2x, c2y, c2z);
}

// Fan lookup (shader.wgsl:77-84); i+1 clamped to n-1 (weight 0 there).
GEO_HD float fan_lerp(const float* fan, uint32_t n, float st) {
    const float theta = asinf_(st);
    float t = clampf_((kPi2 - theta) / kPi, 0.0f, 1.0f);
    t = t * (float)(n - 1u);
    const float fl = __builtin_floorf(t);
    const uint32_t i = (uint32_t)fl;
    const float w = t - fl;
    const uint32_t i1 = (i + 1u < n) ? i + 1u : n - 1u;
    return fan[i] * (1.0f - w) + fan[i1] * w;
}

// shader.wgsl:90-100 — (phi of c2, lambda') to sky-sphere (U, V).
GEO_HD void sky_uv(const float* m2, float c2x, float c2y, float lam, float* U, float* V) {
    const float rho = __builtin_sqrtf(fmaf_(c2y, c2y, c2x * c2x));
    float cp = 1.0f, sp = 0.0f;
    if (rho > 0.0f) {
        cp = c2x / rho;
        sp = c2y / rho;
    }
    float sl, cl;
    sincosf_(lam, &sl, &cl);
    float x, y, z;
    mat3_mul(m2, cp * cl, sp * cl, sl, &x, &y, &z);
    float u = atan2f_(y, x) * kInvTwoPi;
    if (u < 0.0f) u += 1.0f;
    float v = 0.5f - asinf_(z) * kInvPi;
    if (!(u == u)) u = 0.0f;  // NaN guard
    if (!(v == v)) v = 0.0f;
    *U = clampf_(u, 0.0f, 1.0f);
    *V = clampf_(v, 0.0f, 1.0f);
}

GEO_HD float lerpf_(float a, float b, float t) { return fmaf_(t, b - a, a); }

GEO_HD float texel_channel(uint32_t t, int ch) { return (float)((t >> (8 * ch)) & 255u); }

GEO_HD uint32_t to_u8(float v) {
    v = clampf_(v + 0.5f, 0.0f, 255.0f);
    return (uint32_t)v;
}

// LOD-0 bilinear sample of an RGBA8 equirect (U wraps, V clamps), then the
// reference's alpha blend over the clear colour (0,0,0,1): rgb*a, alpha 1.
template <typename Fetch>
GEO_HD uint32_t sample_sky(Fetch fetch, uint32_t tw, uint32_t th, float U, float V) {
    const float x = fmaf_(U, (float)tw, -0.5f);
    const float y = fmaf_(V, (float)th, -0.5f);
    const float fx0 = __builtin_floorf(x);
    const float fy0 = __builtin_floorf(y);
    const float fx = x - fx0;
    const float fy = y - fy0;
    int ix0 = (int)fx0;
    int iy0 = (int)fy0;
    const int w = (int)tw, h = (int)th;
    if (ix0 < 0) ix0 += w;
    if (ix0 >= w) ix0 -= w;
    const int ix1 = (ix0 + 1 == w) ? 0 : ix0 + 1;
    int iy1 = iy0 + 1;
    iy0 = iy0 < 0 ? 0 : (iy0 > h - 1 ? h - 1 : iy0);
    iy1 = iy1 < 0 ? 0 : (iy1 > h - 1 ? h - 1 : iy1);
    const uint32_t t00 = fetch((uint32_t)iy0 * tw + (uint32_t)ix0);
    const uint32_t t10 = fetch((uint32_t)iy0 * tw + (uint32_t)ix1);
    const uint32_t t01 = fetch((uint32_t)iy1 * tw + (uint32_t)ix0);
    const uint32_t t11 = fetch((uint32_t)iy1 * tw + (uint32_t)ix1);
    float c[4];
    for (int ch = 0; ch < 4; ++ch) {
        const float a = lerpf_(texel_channel(t00, ch), texel_channel(t10, ch), fx);
        const float b = lerpf_(texel_channel(t01, ch), texel_channel(t11, ch), fx);
        c[ch] = lerpf_(a, b, fy);
    }
    const float alpha = c[3] * (1.0f / 255.0f);
    return to_u8(c[0] * alpha) | (to_u8(c[1] * alpha) << 8) | (to_u8(c[2] * alpha) << 16) |
           (255u << 24);
}

constexpr uint32_t kBlackRGBA = 0xFF000000u;  // clear colour (0,0,0,1), renderer.rs:233-238

}  // namespace geo
