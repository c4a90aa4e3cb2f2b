// geo_band.h — GEO_FLAG_RING_F64: the capture-orbit band in f64 (geo.h,
// DESIGN.md §2 "The capture band in f64").
//
// Next to the capture orbit (impact parameter b near b_c = 3 sqrt(3) rs / 2)
// the orbit's instability amplifies an f32 evaluation's roundings past the
// 1e-4 UV bar.  The pixels of the band |b/b_c - 1| < GEO_RING_X, decided on
// the f32 ray exactly as the f32 draw computes it, take their traveled angle
// from this f64 path instead of the f32 integrator, inside the same kernel
// (geo_render_kernel<..., RING>): the lane skips the f32 loop and runs
//   * the camera ray and the aberration in f64 (the f32 path's algebra,
//     pixel_central_dir, on the unrounded f64 frame constants);
//   * solve_ray_fan's node set-up and solve_geodesic's radial cases,
//     pre-filters and initial slope as the reference writes them
//     (sphere_ray_tracer.rs:38-49, 60-132), in f64;
//   * the RK4 main loop with its exits and step count as the reference's
//     (:134-191), on the scaled state U = (3 rs/2) u (F(U) = U(U - 1), one
//     FMA; geo_pixel.h rk4_step in f64), four steps per exit branch with a
//     conservative test and the stopping group replayed step by step;
//   * Newton's three refinements (:150-182);
// and returns lambda' = pi/2 - angle in f64.  The mask is decided in f64
// (lambda' < -7); the sky direction and the sample are the f32 draw's own
// (sky_uv on the pixel's f32 ray and lambda' rounded to f32).  Every
// operation is IEEE f64 + - * / sqrt fma (no contraction, correctly rounded
// divide and sqrt), so the host build of this header and the gfx950 kernel
// agree bit for bit, and the oracle restates it (geo_oracle.c band_lambda).
#pragma once

#include <stdint.h>

#include "../../include/geo/geo.h"
#include "geo_pixel.h"

namespace geo {

// Frame + scene constants of the band (host, f64; a kernel argument).
struct BandConsts {
    double a[3], b[3], c[3];  // the camera ray d = py a + px b + c (camera_consts, not rounded to f32)
    double m1[9];             // movement_to_central's 3 x 3 part (column-major), unless m1_identity
    double k, kt;             // psi_k and sqrt(1 - k^2) (shader.wgsl:69-70 as a z-boost)
    double r;                 // r_obs
    double energy;            // sqrt(1 - rs/r)            (solve_ray_fan :48, r > rs)
    double hor;               // (1 - rs/r)/(r r)          (:123)
    double barrier_lim;       // 4/(27 rs^2) if r, sphere_r lie on different sides of 3rs/2 (:106-110), else -inf
    double radial_falling, radial_outgoing;  // the radial case's result (:67-104; r > rs)
    double scale;             // 3 rs/2: U = scale u
    double U0, SU, BD, HU;    // scale x: 1/r, 1/sphere_r, bound (:127), 1/rs
    double lo, hi;            // the group exit: a state outside [lo, hi] (or NaN) may stop the loop
    double h, hh, hh2, hhh, h6, h2_6;  // step, step/2, step^2/4, step^2/2, step/6, step^2/6
    float kx;                 // r / (energy b_c) rounded once: the band test |kx cos(theta) - 1| (f32)
    uint32_t max_steps;
    uint32_t above0;          // U0 > SU: the observer inside the sphere (the group exit's short form)
    uint32_t pf_always, pf_falling, pf_outgoing;  // the pre-filters' frame-uniform terms (:113-117)
    uint32_t m1_identity;
};

// The band test on the f32 draw's cos(theta) (central_rho).
#if !defined(GEO_BAND_X)  // (A/B variants only; the specification is GEO_RING_X)
#define GEO_BAND_X GEO_RING_X
#endif
GEO_HD bool in_band(float kx, float ct) { return __builtin_fabsf(kx * ct - 1.0f) < GEO_BAND_X; }

// kx = r / (E b_c) rounded once: the band test's factor (rs > 0, r_obs > rs).
GEO_HD float band_kx(float rs, float r_obs) {
    const double r = (double)r_obs, rsd = (double)rs;
    return (float)(r / (__builtin_sqrt(1.0 - rsd / r) * (1.5 * __builtin_sqrt(3.0) * rsd)));
}

// The next double above a positive finite x (nextafter(x, +inf)).
GEO_HD double next_up_pos_(double x) {
    uint64_t b;
    __builtin_memcpy(&b, &x, 8);
    ++b;
    __builtin_memcpy(&x, &b, 8);
    return x;
}

// The constants for a frame and scene with rs > 0 and r_obs > rs, written
// field by field into k (on the device: a wave's LDS slot, so that a batched
// launch derives each frame's constants where it needs them; the same IEEE
// f64 operations on the host and the device).
GEO_HD void band_consts_into(BandConsts& k, const geo_frame& f, float rs_f, float sphere_r_f, float r_obs_f,
                             float step_f, uint32_t max_steps, uint32_t width, uint32_t height) {
    const float* m0 = f.display_to_movement;
    const double w = (double)width, hgt = (double)height;
    const double sx = 2.0 / w, ox = (1.0 - w) / w, sy = -2.0 / hgt, oy = (hgt - 1.0) / hgt;
    for (int i = 0; i < 3; ++i) {
        const double p = -(double)m0[12] * (double)m0[i];
        const double q = -(double)m0[13] * (double)m0[4 + i];
        const double rr = (double)m0[14] * (double)m0[8 + i];
        k.a[i] = sy * p;
        k.b[i] = sx * q;
        k.c[i] = (oy * p + ox * q) + rr;
    }
    const float* m1 = f.movement_to_central;
    for (int j = 0; j < 3; ++j)
        for (int i = 0; i < 3; ++i) k.m1[3 * j + i] = (double)m1[4 * j + i];
    k.m1_identity = (m1[0] == 1.0f && m1[1] == 0.0f && m1[2] == 0.0f && m1[4] == 0.0f && m1[5] == 1.0f &&
                     m1[6] == 0.0f && m1[8] == 0.0f && m1[9] == 0.0f && m1[10] == 1.0f)
                        ? 1u
                        : 0u;
    const double psi = (double)f.psi_factor_and_position[0];
    k.k = psi;
    k.kt = __builtin_sqrt(1.0 - psi * psi);
    const double rs = (double)rs_f, sr = (double)sphere_r_f, r = (double)r_obs_f, step = (double)step_f;
    k.r = r;
    k.energy = __builtin_sqrt(1.0 - rs / r);
    k.hor = (1.0 - rs / r) / (r * r);
    const double r3_2 = 3.0 * rs / 2.0;
    const bool diff_sides = ((r < r3_2) != (sr < r3_2)) && __builtin_fabs(r - r3_2) > 1e-10;
    k.barrier_lim = diff_sides ? 4.0 / (27.0 * rs * rs) : -__builtin_inf();
    const bool inside_sphere = r < sr, sphere_outside = sr > rs;
    k.radial_falling = inside_sphere ? GEO_NO_VALUE : (sphere_outside ? 0.0 : GEO_NO_VALUE);
    k.radial_outgoing = inside_sphere ? 0.0 : GEO_NO_VALUE;
    k.pf_always = (inside_sphere && !sphere_outside) ? 1u : 0u;
    k.pf_falling = (r < r3_2 && inside_sphere) ? 1u : 0u;
    k.pf_outgoing = (r > r3_2 && !inside_sphere) ? 1u : 0u;
    const double c = r3_2;
    k.scale = c;
    const double u0 = 1.0 / r;
    const double U0 = c * u0, SU = c / sr, HU = c / rs;
    k.U0 = U0;
    k.SU = SU;
    k.BD = c * (0.9 * __builtin_fmin(u0, 1.0 / __builtin_fmax(sr, r3_2)));
    k.HU = HU;
    k.above0 = U0 > SU ? 1u : 0u;
    if (U0 > SU) {  // inside the sphere: stops below SU (crossing, escape) or above HU (horizon)
        k.lo = next_up_pos_(SU);
        k.hi = HU;
    } else {  // outside it: stops above SU (crossing, horizon) or below BD (escape)
        k.lo = k.BD;
        k.hi = __builtin_fmin(SU, HU);
    }
    k.h = step;
    k.hh = step / 2.0;
    k.hh2 = step * step / 4.0;
    k.hhh = step * step / 2.0;
    k.h6 = step / 6.0;
    k.h2_6 = step * step / 6.0;
    k.kx = band_kx(rs_f, r_obs_f);
    k.max_steps = max_steps;
}

// Host: the constants for a frame and scene with rs > 0 and r_obs > rs.
inline BandConsts band_consts(const geo_frame& f, const geo_scene& s, uint32_t width, uint32_t height) {
    BandConsts k;
    band_consts_into(k, f, s.rs, s.sphere_r, s.r_obs, s.step, s.max_steps, width, height);
    return k;
}

GEO_HD double fma64_(double a, double b, double c) { return __builtin_fma(a, b, c); }

// One RK4 step of U'' = U(U - 1) in f64 (rk4_step's 14 operations).
GEO_HD void band_rk4(double U, double V, double h, double hh, double hh2, double hhh, double h6, double h2_6,
                     double* NU, double* NV) {
    const double fu = fma64_(U, U, -U);
    const double au = fma64_(hh, V, U);
    const double uh = fma64_(h, V, U);
    const double fa = fma64_(au, au, -au);
    const double bu = fma64_(hh2, fu, au);
    const double fb = fma64_(bu, bu, -bu);
    const double cu = fma64_(hhh, fa, uh);
    const double fc = fma64_(cu, cu, -cu);
    const double fab = fa + fb;
    *NU = fma64_(h2_6, fu + fab, uh);
    *NV = fma64_(h6, fma64_(2.0, fab, fu) + fc, V);
}

// A state the group exit must look at: outside [lo, hi] or NaN.  Every stop
// of the reference's loop is at such a state: a crossing from inside the
// sphere (U <= SU < lo), an escape (U < BD <= lo), the horizon test on the
// state after a step (U > HU >= hi), a crossing from outside (U > SU >= hi).
GEO_HD bool band_out(const BandConsts& k, double x) { return !(x >= k.lo) | (x > k.hi); }

// IEEE minNum of two doubles (a NaN operand yields the other) as one
// v_min_f64 (hipcc would canonicalise both operands first; the states are
// arithmetic results, never signaling NaNs).
GEO_HD double min64_(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
#else
    return __builtin_fmin(a, b);
#endif
}

// The group exit for the four states u1..u4 of a group: true if any of them
// is one band_out must look at.  Inside the sphere (above0) in five
// operations: a state above hi = HU with U' > 0 keeps every later state
// above it (U > 1 makes every RK4 stage slope U(U - 1) positive, so the map
// raises U and U'), so only u4 needs the upper test; a state above hi with
// U' <= 0 is no stop; below lo, the minimum of u1..u3 (a NaN state makes
// every later one NaN, which u4's tests see: minNum skips NaN operands).
GEO_HD bool band_group_out(const BandConsts& k, double u1, double u2, double u3, double u4) {
    if (k.above0)
        return (int)(min64_(min64_(u1, u2), u3) < k.lo) | (int)!(u4 >= k.lo) | (int)(u4 > k.hi);
    return (int)band_out(k, u1) | (int)band_out(k, u2) | (int)band_out(k, u3) | (int)band_out(k, u4);
}

// The reference's main loop (sphere_ray_tracer.rs:134-191) from the scaled
// state (U, V) at step `it`: its exits, its step count (*steps = the RK4
// steps taken) and Newton's refinement.  The traveled angle before step it,
// the reference's `angle += step` summed it times, is it x step exactly:
// step is an f32 value (24 significant bits), so every partial sum k step
// (k < 2^24, at most 48 significant bits) is a double and no addition rounds.
GEO_HD double band_steps(const BandConsts& k, double U, double V, uint32_t it, uint32_t* steps) {
    for (; it < k.max_steps; ++it) {
        if ((U > k.HU && V > 0.0) || !(U > 0.0)) {  // the loop test (:134-135)
            *steps = it;
            return GEO_NO_VALUE;
        }
        double NU, NV;
        band_rk4(U, V, k.h, k.hh, k.hh2, k.hhh, k.h6, k.h2_6, &NU, &NV);
        if ((NU > k.SU) != (U > k.SU)) {
            // Newton on the step length from the steeper end (:150-182)
            double ns, wu, wv;
            if (__builtin_fabs(V) > __builtin_fabs(NV)) {
                ns = 0.0;
                wu = U;
                wv = V;
            } else {
                ns = k.h;
                wu = NU;
                wv = NV;
            }
            for (int n = 0; n < kNewtonIters; ++n) {
                ns -= (wu - k.SU) / wv;
                const double n2 = ns * ns;
                band_rk4(U, V, ns, ns / 2.0, n2 / 4.0, n2 / 2.0, ns / 6.0, n2 / 6.0, &wu, &wv);
            }
            *steps = it + 1u;
            return (double)it * k.h + ns;
        }
        if (NU < k.BD) {
            *steps = it + 1u;
            return GEO_NO_VALUE;
        }
        U = NU;
        V = NV;
    }
    *steps = k.max_steps;
    return GEO_NO_VALUE;
}

// lambda' = pi/2 - (the traveled angle) of pixel (px, py) in f64; *steps the
// RK4 steps taken.
GEO_HD double band_lambda(const BandConsts& k, uint32_t px, uint32_t py, uint32_t* steps) {
    constexpr double kHalfPi = 1.57079632679489661923;
    // the camera ray and the aberration (pixel_central_dir in f64)
    const double fx = (double)px, fy = (double)py;
    const double dx = fma64_(fy, k.a[0], fma64_(fx, k.b[0], k.c[0]));
    const double dy = fma64_(fy, k.a[1], fma64_(fx, k.b[1], k.c[1]));
    const double dz = fma64_(fy, k.a[2], fma64_(fx, k.b[2], k.c[2]));
    const double len = __builtin_sqrt(fma64_(dz, dz, fma64_(dy, dy, dx * dx)));
    const double id = 1.0 / fma64_(-k.k, dz, len);
    const double g = k.kt * id;
    double ex = dx * g, ey = dy * g, ez = fma64_(-k.k, len, dz) * id;
    if (!k.m1_identity) {
        const double x = fma64_(k.m1[6], ez, fma64_(k.m1[3], ey, k.m1[0] * ex));
        const double y = fma64_(k.m1[7], ez, fma64_(k.m1[4], ey, k.m1[1] * ex));
        const double z = fma64_(k.m1[8], ez, fma64_(k.m1[5], ey, k.m1[2] * ex));
        ex = x;
        ey = y;
        ez = z;
    }
    // sin and cos of theta (to_polar, shader.wgsl:75): sin clamped to [-1, 1]
    const double st = ez > -1.0 ? (ez < 1.0 ? ez : 1.0) : -1.0;
    const double ct = __builtin_sqrt(fma64_(ey, ey, ex * ex));
    // solve_ray_fan's node (:38-49, r > rs) and solve_geodesic's set-up (:60-132)
    *steps = 0;
    const bool falling = st > 0.0;
    const double rotation = k.r * ct;
    if (rotation < 1e-10) return kHalfPi - (falling ? k.radial_falling : k.radial_outgoing);
    const double b = rotation / k.energy;
    const double ib2 = 1.0 / (b * b);
    if (k.pf_always || ib2 < k.barrier_lim || (falling ? k.pf_falling : k.pf_outgoing))
        return kHalfPi - GEO_NO_VALUE;
    const double ub = __builtin_sqrt(ib2 - k.hor);
    double U = k.U0;
    double V = k.scale * (falling ? ub : -ub);
    // four RK4 steps per exit branch; a group with a state the exit must
    // look at is replayed step by step from its start (band_steps)
    uint32_t it = 0;
    while (it + 4u <= k.max_steps) {
        double u1, v1, u2, v2, u3, v3, u4, v4;
        band_rk4(U, V, k.h, k.hh, k.hh2, k.hhh, k.h6, k.h2_6, &u1, &v1);
        band_rk4(u1, v1, k.h, k.hh, k.hh2, k.hhh, k.h6, k.h2_6, &u2, &v2);
        band_rk4(u2, v2, k.h, k.hh, k.hh2, k.hhh, k.h6, k.h2_6, &u3, &v3);
        band_rk4(u3, v3, k.h, k.hh, k.hh2, k.hhh, k.h6, k.h2_6, &u4, &v4);
        if (band_group_out(k, u1, u2, u3, u4)) break;  // one exit branch per group
        U = u4;
        V = v4;
        it += 4u;
    }
    return kHalfPi - band_steps(k, U, V, it, steps);
}

}  // namespace geo
