// geo_rays.h — the accretion-disk point path in f32, shared
// by the HIP kernels (geo_points.hip) and the host-compiled tests:
//
//   RayConnector::{reset_ray, update_ray, calc_ray_angle}
//                              SR/simulation/ray_connector.rs:27-157
//   vs_main (point pipeline)   SR/schwarzschild_point_shader/shader.wgsl:36-68
//
// The RayConnector is restated in the reference's own f32 expression order
// (Rust does not contract: every product and sum rounds separately; this file
// is compiled with -ffp-contract=off), the Vec3 helpers as glam 0.25 evaluates
// them.  Transcendentals: glam's Vec3::angle_between uses its acos_approx (the
// DirectXMath XMScalarAcos 7-degree minimax, restated below — the glam source
// is not in this image, so this is restated from its published form); f32::acos,
// f32::atan come from geo_math.h (<= 4 ulp from libm).  Reciprocals 1.0 / x
// go through rcpf_ (geo_math.h), equal to the IEEE quotient for every input,
// so the oracle's `1.0f / x` is unchanged.  The oracle
// (oracle/geo_oracle_points.c) restates the same sequence; tests require bit
// equality with it, and the reference's own RayConnector tests (tests.rs:15-79,
// 5e-4 rad) on both.
#pragma once

#include <stdint.h>

#include "geo_math.h"

namespace geo {

constexpr int kRayNodes = 48;                      // NR_NODES, ray_connector.rs:3
constexpr float kSmallestAngle = 0.05f;           // SMALLEST_ANGLE, :4
constexpr int kResetIterations = 5;                // reset_ray's update_ray(.., 5), :43
constexpr float kTauF = 6.28318530717958647692f;   // std::f32::consts::TAU
constexpr uint32_t kPointRGBA = 0xFF0000FFu;       // fs_main colour (1,0,0,1), shader.wgsl:71-73

// glam Vec3 (f32, scalar): dot = x*x' + y*y' + z*z' left to right, length = sqrt(dot)
GEO_HD float dot3_(float ax, float ay, float az, float bx, float by, float bz) {
    return ax * bx + ay * by + az * bz;
}
GEO_HD float len3_(float x, float y, float z) { return __builtin_sqrtf(dot3_(x, y, z, x, y, z)); }

// glam acos_approx: acos of v clamped to [-1, 1], XMScalarAcos polynomial (no FMA)
GEO_HD float acos_approx_(float v) {
    const bool nonnegative = v >= 0.0f;
    const float x = __builtin_fabsf(v);
    float omx = 1.0f - x;
    if (omx < 0.0f) omx = 0.0f;
    const float root = __builtin_sqrtf(omx);
    float r = ((((((-0.0012624911f * x + 0.0066700901f) * x - 0.0170881256f) * x + 0.0308918810f) * x -
                 0.0501743046f) * x + 0.0889789874f) * x - 0.2145988016f) * x + 1.5707963050f;
    r *= root;
    return nonnegative ? r : kPi - r;
}

// glam Vec3::angle_between: acos_approx(dot / sqrt(|a|^2 |b|^2))
GEO_HD float angle_between_(float ax, float ay, float az, float bx, float by, float bz) {
    return acos_approx_(dot3_(ax, ay, az, bx, by, bz) /
                        __builtin_sqrtf(dot3_(ax, ay, az, ax, ay, az) * dot3_(bx, by, bz, bx, by, bz)));
}

GEO_HD float signum_(float x) { return x != x ? x : __builtin_copysignf(1.0f, x); }  // Rust f32::signum

// calc_ray_angle (:141-157)
GEO_HD float calc_ray_angle(float rs, bool lt180, float u_bar, float r) {
    float theta;
    if (r > rs) {
        theta = signum_(u_bar) * acosf_(__builtin_sqrtf(rcpf_(1.0f + (r * r * u_bar * u_bar) / (1.0f - rs / r))));
    } else {
        const float inter = -(r * r * u_bar * u_bar) / (1.0f - rs / r) - 1.0f;
        theta = inter > 0.0f ? -kPi2 + atanf_(__builtin_sqrtf(rcpf_(inter))) : 0.0f;
    }
    return (kPi2 - theta) * (lt180 ? 1.0f : -1.0f);
}

// One RayConnector call for a connector at (px,py,pz) and the other end
// (ox,oy,oz): reset_ray(other) when `reset`, else update_ray(other, iterations)
// (which resets by itself when needs_reset is set or the other end jumped by
// more than 0.5).  load(i): the connector's stored node value i, read only
// when no reset replaces it (so the stored and the reset values are never
// live together); u: the 48 node values after the call.  Returns the
// incoming angle (vertex w).
template <typename Load>
GEO_HD float ray_connect(float rs, bool lt180, float px, float py, float pz, float ox, float oy, float oz,
                         bool reset, uint32_t iterations, bool* needs_reset, Load load, float* u) {
    float phi = angle_between_(px, py, pz, ox, oy, oz);  // last_phi (:31-34, :53-56)
    if (!lt180) phi = kTauF - phi;
    bool do_reset = reset || *needs_reset;
    if (!do_reset && !(phi < kSmallestAngle)) {
        // the jump test of update_ray (:82-84)
        const float u0 = rcpf_(len3_(ox, oy, oz));
        if (__builtin_fabsf(rcpf_(u0) - rcpf_(load(0))) > 0.5f) do_reset = true;
    }
    if (do_reset) {
        // reset_ray (:28-40): linear initial guess between the two ends
        *needs_reset = false;
        const float u0 = rcpf_(len3_(ox, oy, oz));
        const float u1 = rcpf_(len3_(px, py, pz));
#pragma unroll
        for (int i = 0; i < kRayNodes; ++i) {
            const float w = (float)i / (float)(kRayNodes - 1);
            u[i] = u0 * (1.0f - w) + u1 * w;
        }
    } else {
#pragma unroll
        for (int i = 0; i < kRayNodes; ++i) u[i] = load(i);
    }
    if (phi < kSmallestAngle) {
        // nearly straight ray (:61-76): no solve; reset on the next call
        *needs_reset = true;
        if (phi == 0.0f) return len3_(ox, oy, oz) > len3_(px, py, pz) ? 0.0f : kPi;
        const float u0 = rcpf_(len3_(ox, oy, oz));
        const float u_bar =
            (rcpf_(len3_(px, py, pz)) - u0) / phi - phi / 2.0f * (-u0 + 1.5f * rs * u0 * u0);
        return calc_ray_angle(rs, lt180, u_bar, rcpf_(u0));
    }
    // update_ray (:78-131); after a reset the end deltas are exactly 0
    const float u0 = rcpf_(len3_(ox, oy, oz));
    const float u1 = rcpf_(len3_(px, py, pz));
    const float u0_delta = u0 - u[0];
    const float u1_delta = u1 - u[kRayNodes - 1];
#pragma unroll
    for (int i = 0; i < kRayNodes; ++i) {
        const float w = (float)i / (float)(kRayNodes - 1);
        u[i] += u0_delta * (1.0f - w) + u1_delta * w;
    }
    // Newton on the 46 interior nodes of u'' + u = 3rs/2 u^2 (finite
    // differences, fixed ends), each step one tridiagonal solve (Thomas;
    // off-diagonals all -scale) (:94-126)
    const float h = phi / (float)(kRayNodes - 1);
    const float scale = rcpf_(h * h);
    const uint32_t iters = do_reset ? (uint32_t)kResetIterations : iterations;
    float res[kRayNodes - 2], tc[kRayNodes - 2];
    for (uint32_t k = 0; k < iters; ++k) {
#pragma unroll
        for (int i = 1; i < kRayNodes - 1; ++i)
            res[i - 1] = scale * (-u[i - 1] + 2.0f * u[i] - u[i + 1]) - u[i] + 3.0f * rs / 2.0f * u[i] * u[i];
        float mdi = rcpf_(2.0f * scale - 1.0f + 3.0f * rs * u[1]);
        tc[0] = (-scale) * mdi;
        res[0] = res[0] * mdi;
#pragma unroll
        for (int i = 1; i < kRayNodes - 2; ++i) {
            mdi = rcpf_(2.0f * scale - 1.0f + 3.0f * rs * u[i + 1] + scale * tc[i - 1]);
            tc[i] = (-scale) * mdi;
            res[i] = (res[i] + scale * res[i - 1]) * mdi;
        }
        u[kRayNodes - 2] -= res[kRayNodes - 3];
#pragma unroll
        for (int i = kRayNodes - 4; i >= 0; --i) {
            res[i] = res[i] - tc[i] * res[i + 1];
            u[i + 1] -= res[i];
        }
    }
    // incoming angle from the second-order one-sided derivative at node 0 (:129-130)
    const float u_bar = (u[1] - u[0]) / h - h / 2.0f * (-u[0] + 1.5f * rs * u[0] * u[0]);
    return calc_ray_angle(rs, lt180, u_bar, rcpf_(u0));
}

// vs_main (shader.wgsl:36-68) for the vertex (x, y, z, incoming angle):
// WGSL `v * M` is the transposed product, c_j = dot(v, column j) (evaluated
// here as an fma chain in component order).  Returns false when the point is
// clipped (behind the camera or outside the frame); else its pixel.
GEO_HD void vmul4_t_(const float* m, float x, float y, float z, float w, float* o) {
#pragma unroll
    for (int j = 0; j < 4; ++j) o[j] = fmaf_(m[4 * j + 3], w, fmaf_(m[4 * j + 2], z, fmaf_(m[4 * j + 1], y, m[4 * j] * x)));
}

GEO_HD bool project_point(const float* m0, const float* m1, const float* m2, float psi_k, float x, float y, float z,
                          float w, uint32_t width, uint32_t height, uint32_t* ix, uint32_t* iy) {
    float c[4];
    vmul4_t_(m2, x, y, z, w, c);  // onto the observer's normal plane
    float pphi = atan2f_(c[1], c[0]);
    float plam = c[3];
    if (plam < 0.0f) pphi += 2.0f * kPi2;  // far-side ray
    plam = kPi2 - __builtin_fabsf(plam);
    float sp, cp, sl, cl;
    sincosf_(pphi, &sp, &cp);
    sincosf_(plam, &sl, &cl);
    vmul4_t_(m1, cp * cl, sp * cl, sl, 0.0f, c);
    pphi = atan2f_(c[1], c[0]);
    plam = asinf_(c[2]);
    // aberration, inverted (:61-64)
    float sr, cr;
    sincosf_(-plam, &sr, &cr);
    plam = -asinf_((sr - psi_k) / (1.0f - sr * psi_k));
    sincosf_(pphi, &sp, &cp);
    sincosf_(plam, &sl, &cl);
    vmul4_t_(m0, cp * cl, sp * cl, sl, 0.0f, c);
    // screen scaling by the FOV column (:66)
    const float sx = c[0] / m0[12];
    const float sy = c[1] / m0[13];
    const float sz = c[2] / m0[14];
    // clip position (-sy, -sx, sz, |sz|): inside iff 0 <= z <= w, |x|,|y| <= w, w > 0
    const float cw = __builtin_fabsf(sz);
    if (!(sz > 0.0f) || !(__builtin_fabsf(sy) <= cw) || !(__builtin_fabsf(sx) <= cw)) return false;
    const float nx = -sy / cw, ny = -sx / cw;
    const float fx = (nx + 1.0f) * 0.5f * (float)width;
    const float fy = (1.0f - ny) * 0.5f * (float)height;
    const float flx = __builtin_floorf(fx), fly = __builtin_floorf(fy);
    if (!(flx >= 0.0f && flx < (float)width && fly >= 0.0f && fly < (float)height)) return false;
    *ix = (uint32_t)flx;
    *iy = (uint32_t)fly;
    return true;
}

}  // namespace geo
