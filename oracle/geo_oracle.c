/*
 * geo_oracle.c — ORACLE (test infrastructure only).  See geo_oracle.h for the
 * contract and the "parity unpinned" statement.
 *
 * Two independent restatements of the reference hot path:
 *   (1) f64, literal: every arithmetic expression of
 *       SR/simulation/sphere_ray_tracer.rs:35-193 and
 *       SR/schwarzschild_sphere_shader/shader.wgsl:57-106 in its source order,
 *       with libm transcendentals;
 *   (2) f32, the kernel's documented evaluation order (geo_pixel.h), written
 *       here from the specification in DESIGN.md §3, not shared with the
 *       product sources: tests require the HIP output to equal it bit for bit.
 *
 * Build: make -C oracle   (gcc, -ffp-contract=off so no implicit FMA).
 */
#include "geo_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define O_PI 3.14159265358979323846
#define O_FRAC_PI_2 1.57079632679489661923
#define O_NO_VALUE 15.0

/* ------------------------------------------------------------------ */
/* (1) f64 literal restatement                                          */
/* ------------------------------------------------------------------ */

/* sphere_ray_tracer.rs:60-193 */
double geo_oracle_solve_geodesic_f64(double sphere_r, double schwarz_r, uint32_t max_iter,
                                     double default_step, double r, double energy,
                                     double rotation, int r_falling, uint32_t* steps) {
    uint32_t dummy;
    if (!steps) steps = &dummy;
    *steps = 0;
    double b = rotation / energy;
    int outside = r > schwarz_r;
    int sphere_outside = sphere_r > schwarz_r;
    int inside_sphere = r < sphere_r;

    if (rotation < 1e-10) { /* :67-104 */
        if (inside_sphere) {
            if (outside) {
                if (r_falling) {
                    if (schwarz_r == 0.) return O_PI;
                    return O_NO_VALUE;
                }
                return 0.;
            } else {
                if (sphere_outside) {
                    if (energy > 0.) return 0.;
                    return O_NO_VALUE;
                }
                return 0.;
            }
        } else {
            if (sphere_outside && r_falling) return 0.;
            return O_NO_VALUE;
        }
    }
    /* :107-119 */
    int barrier_3r_2 = (schwarz_r > 0.) && 1. / (b * b) < 4. / (27. * schwarz_r * schwarz_r);
    double r3_2 = 3. * schwarz_r / 2.;
    int different_sides_3r_2 = ((r < r3_2) ^ (sphere_r < r3_2)) && fabs(r - r3_2) > 1e-10;
    if ((inside_sphere && !sphere_outside) || (!outside && sphere_outside && energy < 0.) ||
        (barrier_3r_2 && different_sides_3r_2) || (r < r3_2 && inside_sphere && r_falling) ||
        (r > r3_2 && !inside_sphere && !r_falling)) {
        return O_NO_VALUE;
    }
    /* :122-132 */
    double u_k = 1. / r;
    double u_bar_k = (r_falling ? 1. : -1.) * sqrt(1. / (b * b) - (1. - schwarz_r / r) / (r * r));
    double angle = 0.;
    uint32_t iteration = 0;
    double bound = 0.9 * fmin(u_k, 1. / fmax(sphere_r, r3_2));
    double step = default_step;
    double step_half = step / 2.;
    double sphere_u = 1. / sphere_r;
    double schwarz_u = 1. / schwarz_r;
    /* :134-191 */
    while (!(schwarz_r != 0. && u_k > schwarz_u && u_bar_k > 0.) && iteration < max_iter && u_k > 0.) {
        double a_u = u_k + step_half * u_bar_k;
        double a_u_bar = u_bar_k + step_half * (-u_k + r3_2 * u_k * u_k);
        double b_u = u_k + step_half * a_u_bar;
        double b_u_bar = u_bar_k + step_half * (-a_u + r3_2 * a_u * a_u);
        double c_u = u_k + step * b_u_bar;
        double c_u_bar = u_bar_k + step * (-b_u + r3_2 * b_u * b_u);
        double next_u = u_k + step * (u_bar_k + 2. * a_u_bar + 2. * b_u_bar + c_u_bar) / 6.;
        double next_u_bar = u_bar_k + step * ((-u_k + r3_2 * u_k * u_k) + 2. * (-a_u + r3_2 * a_u * a_u) +
                                              2. * (-b_u + r3_2 * b_u * b_u) + (-c_u + r3_2 * c_u * c_u)) / 6.;
        *steps = iteration + 1;
        if ((next_u > sphere_u) ^ (u_k > sphere_u)) {
            double newton_u, newton_u_bar, newton_step;
            if (fabs(u_bar_k) > fabs(next_u_bar)) {
                newton_step = 0.;
                newton_u = u_k;
                newton_u_bar = u_bar_k;
            } else {
                newton_step = step;
                newton_u = next_u;
                newton_u_bar = next_u_bar;
            }
            for (int n = 0; n < 3; ++n) {
                newton_step -= (newton_u - sphere_u) / newton_u_bar;
                double newton_step_half = newton_step / 2.;
                a_u = u_k + newton_step_half * u_bar_k;
                a_u_bar = u_bar_k + newton_step_half * (-u_k + r3_2 * u_k * u_k);
                b_u = u_k + newton_step_half * a_u_bar;
                b_u_bar = u_bar_k + newton_step_half * (-a_u + r3_2 * a_u * a_u);
                c_u = u_k + newton_step * b_u_bar;
                c_u_bar = u_bar_k + newton_step * (-b_u + r3_2 * b_u * b_u);
                newton_u = u_k + newton_step * (u_bar_k + 2. * a_u_bar + 2. * b_u_bar + c_u_bar) / 6.;
                newton_u_bar = u_bar_k + newton_step * ((-u_k + r3_2 * u_k * u_k) + 2. * (-a_u + r3_2 * a_u * a_u) +
                                                        2. * (-b_u + r3_2 * b_u * b_u) + (-c_u + r3_2 * c_u * c_u)) / 6.;
            }
            return angle + newton_step;
        }
        if (next_u < bound) return O_NO_VALUE;
        u_k = next_u;
        u_bar_k = next_u_bar;
        iteration += 1;
        angle += step;
    }
    return O_NO_VALUE;
}

/* sphere_ray_tracer.rs:38-52 for one theta */
double geo_oracle_geodesic_at_theta_f64(double sphere_r, double schwarz_r, uint32_t max_iter,
                                        double step, double r, double theta, uint32_t* steps) {
    double rotation = r * cos(theta);
    int r_falling;
    double energy;
    if (r < schwarz_r) {
        r_falling = 0;
        energy = sin(-theta) * sqrt(-1. + schwarz_r / r);
    } else {
        r_falling = theta > 0.;
        energy = sqrt(1. - schwarz_r / r);
    }
    return geo_oracle_solve_geodesic_f64(sphere_r, schwarz_r, max_iter, step, r, energy, rotation,
                                         r_falling, steps);
}

/* sphere_ray_tracer.rs:35-56 */
void geo_oracle_solve_ray_fan_f64(double sphere_r, double schwarz_r, uint32_t max_iter,
                                  double step, uint32_t nr_nodes, double r, float* fan_out) {
    for (uint32_t i = 0; i < nr_nodes; ++i) {
        double theta = O_FRAC_PI_2 - O_PI * (double)i / ((double)nr_nodes - 1.);
        fan_out[i] = (float)(O_FRAC_PI_2 -
                             geo_oracle_geodesic_at_theta_f64(sphere_r, schwarz_r, max_iter, step, r, theta, NULL));
    }
}

/* mat4x4<f32> * vec4 (w = 0), column-major, evaluated in f64 */
static void m3v_d(const float* m, const double* v, double* o) {
    for (int i = 0; i < 3; ++i) o[i] = (double)m[i] * v[0] + (double)m[4 + i] * v[1] + (double)m[8 + i] * v[2];
}

/* shader.wgsl:47-55 */
static void to_cart_d(double phi, double lam, double* c) {
    c[0] = cos(phi) * cos(lam);
    c[1] = sin(phi) * cos(lam);
    c[2] = sin(lam);
}

/* shader.wgsl:57-106 in f64; the fan lookup (:77-84) in fan mode, else the
 * per-pixel geodesic at theta = lambda. */
void geo_oracle_pixel_f64(const geo_frame* f, const geo_scene* s, const float* fan, uint32_t n_fan,
                          uint32_t width, uint32_t height, uint32_t px, uint32_t py,
                          geo_oracle_px* out) {
    /* full-screen quad position at the pixel centre (basic_sphere_buffer.rs:63-83) */
    double ndc_x = ((double)px + 0.5) / (double)width * 2. - 1.;
    double ndc_y = 1. - ((double)py + 0.5) / (double)height * 2.;
    const float* m0 = f->display_to_movement;
    double c[3] = {-ndc_y * (double)m0[12], -ndc_x * (double)m0[13], 1. * (double)m0[14]};
    double d[3];
    m3v_d(m0, c, d);
    double len = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
    d[0] /= len;
    d[1] /= len;
    d[2] /= len;
    double phi = atan2(d[1], d[0]);
    double lam = asin(d[2]);
    double k = (double)f->psi_factor_and_position[0];
    double sin_result = sin(lam);
    lam = asin((sin_result - k) / (1. - sin_result * k));
    to_cart_d(phi, lam, c);
    m3v_d(f->movement_to_central, c, d);
    phi = atan2(d[1], d[0]);
    lam = asin(d[2]);
    out->theta = lam;
    out->steps = 0;
    double lam2;
    if (s->mode == GEO_MODE_FAN) {
        double t = (O_FRAC_PI_2 - lam) / (O_FRAC_PI_2 * 2.);
        t = t < 0. ? 0. : (t > 1. ? 1. : t);
        t = t * (double)(n_fan - 1u);
        double fl = floor(t);
        uint32_t i = (uint32_t)fl;
        double w = t - fl;
        uint32_t i1 = i + 1u < n_fan ? i + 1u : n_fan - 1u;
        lam2 = (double)fan[i] * (1. - w) + (double)fan[i1] * w;
    } else if (s->mode == GEO_MODE_ADAPTIVE) {
        /* the adaptive mode has no reference counterpart: its f64 check is the
         * fixed-step integration at step/32 */
        lam2 = O_FRAC_PI_2 - geo_oracle_geodesic_at_theta_f64((double)s->sphere_r, (double)s->rs,
                                                              GEO_ORACLE_FINE_BUDGET, (double)s->step / 32.,
                                                              (double)s->r_obs, lam, &out->steps);
    } else {
        lam2 = O_FRAC_PI_2 - geo_oracle_geodesic_at_theta_f64((double)s->sphere_r, (double)s->rs, s->max_steps,
                                                              (double)s->step, (double)s->r_obs, lam, &out->steps);
    }
    out->lam = lam2;
    out->bh = lam2 < -7.;
    to_cart_d(phi, lam2, c);
    m3v_d(f->central_to_uv, c, d);
    phi = atan2(d[1], d[0]);
    lam = asin(d[2]);
    double u = phi / (O_FRAC_PI_2 * 4.);
    if (u < 0.) u += 1.;
    out->u = u;
    out->v = 0.5 - lam / (O_FRAC_PI_2 * 2.);
}

/* ------------------------------------------------------------------ */
/* (2) f32 restatement of the kernel's evaluation order                 */
/* ------------------------------------------------------------------ */

#define F_PI 3.14159265358979323846f
#define F_PI2 1.57079632679489661923f
#define F_PI4 0.785398163397448309616f

static inline float clampf(float x, float lo, float hi) { return x < lo ? lo : (x > hi ? hi : x); }
static inline float maxz(float a, float b) { return a > b ? a : b; }

void geo_oracle_sincosf(float x, float* so, float* co) {
    float j = rintf(x * 0.636619772367581343076f);
    float r = fmaf(-j, 1.5703125f, x);
    r = fmaf(-j, 4.837512969970703125e-4f, r);
    r = fmaf(-j, 7.54978995489188216e-8f, r);
    float z = r * r;
    float ps = fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f);
    float sn = fmaf(ps * z, r, r);
    float pc = fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f);
    float cs = fmaf(pc * z, z, fmaf(-0.5f, z, 1.0f));
    int q = ((int)j) & 3;
    float sv, cv;
    switch (q) {
        case 0: sv = sn; cv = cs; break;
        case 1: sv = cs; cv = -sn; break;
        case 2: sv = -sn; cv = -cs; break;
        default: sv = -cs; cv = sn; break;
    }
    *so = sv;
    *co = cv;
}

float geo_oracle_asinf(float x) {
    float a = fminf(fabsf(x), 1.0f); /* NaN -> 1 (geo_math.h asinf_) */
    int big = a > 0.5f;
    float z, sq;
    if (big) {
        z = 0.5f * (1.0f - a);
        sq = sqrtf(z);
    } else {
        z = a * a;
        sq = a;
    }
    float p = fmaf(fmaf(fmaf(fmaf(4.2163199048e-2f, z, 2.4181311049e-2f), z, 4.5470025998e-2f), z,
                        7.4953002686e-2f), z, 1.6666752422e-1f);
    float r = fmaf(p * z, sq, sq);
    if (big) r = fmaf(-2.0f, r, F_PI2);
    return copysignf(r, x);
}

float geo_oracle_atan2f(float y, float x) {
    float ay = fabsf(y), ax = fabsf(x);
    float num, den, y0;
    if (ay > 2.414213562373095f * ax) {
        num = -ax; den = ay; y0 = F_PI2;
    } else if (ay > 0.4142135623730950f * ax) {
        num = ay - ax; den = ay + ax; y0 = F_PI4;
    } else {
        num = ay; den = ax; y0 = 0.0f;
    }
    float t = den > 0.0f ? num * (1.0f / den) : 0.0f; /* divf_ */
    float z = t * t;
    float p = fmaf(fmaf(fmaf(8.05374449538e-2f, z, -1.38776856032e-1f), z, 1.99777106478e-1f), z,
                   -3.33329491539e-1f);
    float r = y0 + fmaf(p * z, t, t);
    if (x < 0.0f) r = F_PI - r;
    return copysignf(r, y);
}

/* The per-pixel sky-direction transcendentals (round 6; geo_math.h
 * sincos_sky_, acos_pi_, atan2_turns_): restated with C's fmaf / sqrtf /
 * fmaxf, the same coefficients and order. */
static float o_sqrt_unit(float x) { return sqrtf(fmaxf(x, 0x1p-96f)); }

void geo_oracle_sincos_sky(float x, float* so, float* co) {
    float tj = fmaf(x, 0.318309886183790671538f, 12582912.0f);
    float j = tj - 12582912.0f;
    uint32_t tb;
    memcpy(&tb, &tj, 4);
    float r = fmaf(-j, 3.140625f, x);
    r = fmaf(-j, 9.67653584666550159e-4f, r);
    float z = r * r;
    float ps = fmaf(fmaf(fmaf(2.600061634e-06f, z, -1.980661764e-04f), z, 8.333017118e-03f), z, -1.666665673e-01f);
    float sn = fmaf(r * z, ps, r);
    float pc = fmaf(fmaf(fmaf(2.319447049e-05f, z, -1.385593088e-03f), z, 4.166398942e-02f), z, -4.999993145e-01f);
    float cs = fmaf(z, pc, 1.0f);
    if (tb & 1u) { /* odd j: both signs flip */
        sn = -sn;
        cs = -cs;
    }
    *so = sn;
    *co = cs;
}

float geo_oracle_acos_pi(float x) {
    float a = fminf(fabsf(x), 1.0f); /* NaN -> 1 */
    float s = o_sqrt_unit(1.0f - a);
    float p = fmaf(8.312922437e-04f, a, -3.820668207e-03f);
    p = fmaf(p, a, 8.837061934e-03f);
    p = fmaf(p, a, -1.565995067e-02f);
    p = fmaf(p, a, 2.827732079e-02f);
    p = fmaf(p, a, -6.830646098e-02f);
    p = fmaf(p, a, 4.999999702e-01f);
    float h = s * p;
    return x < 0.0f ? 1.0f - h : h;
}

float geo_oracle_atan2_turns(float y, float x) {
    float ay = fabsf(y), ax = fabsf(x);
    float num, den, y0;
    if (ay > 2.414213562373095f * ax) {
        num = -ax; den = ay; y0 = 0.25f;
    } else if (ay > 0.4142135623730950f * ax) {
        num = ay - ax; den = ay + ax; y0 = 0.125f;
    } else {
        num = ay; den = ax; y0 = 0.0f;
    }
    float t = den > 0.0f ? num * (1.0f / den) : 0.0f; /* divf_ */
    float z = t * t;
    float p = fmaf(fmaf(fmaf(-1.715674624e-02f, z, 3.116416559e-02f), z, -5.302115157e-02f), z, 1.591545641e-01f);
    float r = fmaf(t, p, y0);
    float h = x < 0.0f ? 0.5f - r : r;
    return y < 0.0f ? 1.0f - h : h;
}

typedef struct {
    float rs, sphere_r, r, step;
    uint32_t max_steps;
    float hh, h6, hh2, hhh, h2_6, r3_2, sphere_u, schwarz_u, u0, h_over_r2, inv_r2, bound, e_out, e_in, barrier;
    int r_inside_h, outside, sphere_outside, inside_sphere, diff_sides, rs_nonzero;
    float scale, U0, SU, BD, HU; /* scaled state U = scale*u */
    float ubk;                   /* scale * (E/r) outside the horizon: UB0 = ubk |st|/ct */
    float tolU, tolG, hmax;      /* GEO_MODE_ADAPTIVE step control */
} fconsts;

static fconsts make_fconsts(const geo_scene* s) {
    fconsts k;
    k.rs = s->rs;
    k.sphere_r = s->sphere_r;
    k.r = s->r_obs;
    k.step = s->step;
    k.max_steps = s->max_steps;
    k.hh = k.step * 0.5f;
    k.h6 = k.step / 6.0f;
    k.hh2 = (k.step * k.step) * 0.25f;
    k.hhh = (k.step * k.step) * 0.5f;
    k.h2_6 = (k.step * k.step) / 6.0f;
    k.r3_2 = 1.5f * k.rs;
    k.sphere_u = 1.0f / k.sphere_r;
    k.schwarz_u = 1.0f / k.rs;
    k.u0 = 1.0f / k.r;
    k.h_over_r2 = (1.0f - k.rs / k.r) / (k.r * k.r);
    k.inv_r2 = 1.0f / (k.r * k.r);
    float mx = k.sphere_r > k.r3_2 ? k.sphere_r : k.r3_2;
    float um = 1.0f / mx;
    k.bound = 0.9f * (k.u0 < um ? k.u0 : um);
    k.e_out = sqrtf(1.0f - k.rs / k.r);
    k.e_in = sqrtf(-1.0f + k.rs / k.r);
        k.barrier = 4.0f / (27.0f * k.rs * k.rs);
    k.r_inside_h = k.r < k.rs;
    k.outside = k.r > k.rs;
    k.sphere_outside = k.sphere_r > k.rs;
    k.inside_sphere = k.r < k.sphere_r;
    k.diff_sides = ((k.r < k.r3_2) != (k.sphere_r < k.r3_2)) && (fabsf(k.r - k.r3_2) > 1e-10f);
    k.rs_nonzero = k.rs != 0.0f;
    k.scale = k.rs_nonzero ? k.r3_2 : 1.0f;
    k.U0 = k.scale * k.u0;
    k.SU = k.scale * k.sphere_u;
    k.BD = k.scale * k.bound;
    k.HU = k.scale * k.schwarz_u;
    k.ubk = k.scale * (k.e_out * k.u0);
    k.tolU = k.scale * (s->tol > 0.0f ? s->tol : GEO_ADAPTIVE_DEFAULT_TOL);
    k.tolG = k.tolU * (1.0f / 64.0f);
    k.hmax = k.step * (float)GEO_ADAPTIVE_MAX_GROWTH;
    return k;
}

/* the RK4 step of sphere_ray_tracer.rs:137-146 on the scaled state U = c*u
 * (c = 3rs/2; c*f(u) = F(U) = U*(U - 1), or F(U) = -U for rs = 0), stage
 * values in the algebraically identical forms of DESIGN.md §3:
 *   a = U + h/2 UB, b = a + h^2/4 F(U), U_h = U + h UB, c = U_h + h^2/2 F(a),
 *   next_U = U_h + h^2/6 (F(U)+F(a)+F(b)), next_UB = UB + h/6 (F(U)+2F(a)+2F(b)+F(c)). */
static inline float Ff(float U, int flat) { return flat ? -U : fmaf(U, U, -U); }

static inline void rk4f(float U, float UB, float h, float hh, float hh2, float hhh, float h6, float h2_6,
                        int flat, float* NU, float* NUB) {
    float fu = Ff(U, flat);
    float au = fmaf(hh, UB, U);
    float uh = fmaf(h, UB, U);
    float fa = Ff(au, flat);
    float bu = fmaf(hh2, fu, au);
    float fb = Ff(bu, flat);
    float cu = fmaf(hhh, fa, uh);
    float fc = Ff(cu, flat);
    float fab = fa + fb;
    *NU = fmaf(h2_6, fu + fab, uh);
    *NUB = fmaf(h6, fmaf(2.0f, fab, fu) + fc, UB);
}

/* GEO_MODE_ADAPTIVE (config 5, a build extension): Dormand-Prince RK5(4)
 * (J. Comput. Appl. Math. 6 (1980) 19-26) on the scaled state in Nystrom form,
 *   U_i = U + c_i h V + h^2 sum_j (A^2)_ij G_j,  G_j = F(U_j),
 *   NU = U + h V + h^2 sum_j (bA)_j G_j,  NV = V + h sum_j b_j G_j,
 *   error estimate |sum_j ((b - b*)A)_j G_j| h^2  (in U),
 * coefficients = the exact rationals rounded once to f32 (tools/dp5_coeffs.py
 * prints this table).  Evaluation order: DESIGN.md §3a. */
static const float DP_C2 = 0x1.99999ap-3f, DP_C3 = 0x1.333334p-2f, DP_C4 = 0x1.99999ap-1f,
                   DP_C5 = 0x1.c71c72p-1f;
static const float DP_A31 = 0x1.70a3d8p-5f, DP_A41 = -0x1.eb851ep-2f, DP_A42 = 0x1.99999ap-1f,
                   DP_A51 = -0x1.dde5dcp+0f, DP_A52 = 0x1.a5de0ep+1f, DP_A53 = -0x1.08b37cp+0f,
                   DP_A61 = -0x1.026c9cp+1f, DP_A62 = 0x1.08ba2ep+2f, DP_A63 = -0x1.b26c9cp+0f,
                   DP_A64 = 0x1.45d174p-4f;
static const float DP_Q[6] = {0x1.755556p-4f, 0.0f, 0x1.420338p-2f, 0x1.0aaaaap-3f, -0x1.256f18p-5f, 0.0f};
static const float DP_B[6] = {0x1.755556p-4f, 0.0f, 0x1.cc049ap-2f, 0x1.4d5556p-1f, -0x1.4a1cfcp-2f,
                              0x1.0c30c4p-3f};
static const float DP_E[6] = {0x1.5b9754p-9f, 0.0f, -0x1.938a4p-8f, 0x1.4da74p-7f, -0x1.be0506p-9f,
                              -0x1.ad1ad2p-9f};

/* sum_j w_j G_j over the nonzero w_j, first term a product, then FMAs in j order */
static float wsum(const float* w, const float* G, int n) {
    float acc = 0.0f;
    int first = 1;
    for (int j = 0; j < n; ++j) {
        if (w[j] == 0.0f) continue;
        acc = first ? w[j] * G[j] : fmaf(w[j], G[j], acc);
        first = 0;
    }
    return acc;
}

static void dp5f(float U, float V, float h, int flat, float* NU, float* NV, float* SE) {
    float G[6], Ui;
    const float A2[6][4] = {{0}, {0}, {DP_A31}, {DP_A41, DP_A42}, {DP_A51, DP_A52, DP_A53},
                            {DP_A61, DP_A62, DP_A63, DP_A64}};
    const float C[6] = {0.0f, DP_C2, DP_C3, DP_C4, DP_C5, 1.0f};
    /* U_i = (U + c_i hV) + h^2 S_i, S_i over j < i-1 ((A^2)_{i,i-1} = 0);
     * c6 = 1: U + hV itself, shared with NU */
    const float hv = h * V, hh = h * h, w = U + hv;
    G[0] = Ff(U, flat);
    for (int i = 1; i < 6; ++i) {
        if (i == 1)
            Ui = fmaf(C[i], hv, U);
        else if (i == 5)
            Ui = fmaf(hh, wsum(A2[i], G, i - 1), w);
        else
            Ui = fmaf(hh, wsum(A2[i], G, i - 1), fmaf(C[i], hv, U));
        G[i] = Ff(Ui, flat);
    }
    *NU = fmaf(hh, wsum(DP_Q, G, 6), w);
    *NV = fmaf(h, wsum(DP_B, G, 6), V);
    *SE = wsum(DP_E, G, 6);
}

/* the literal adaptive loop: stop checks in the reference's order
 * (crossing :150, escape :184, loop test :134-135) on accepted steps only */
static float adaptive_f32(const fconsts* k, float U, float V, int flat, uint32_t* steps) {
    float h = k->step, ang = 0.0f;
    uint32_t it = 0;
    while (it < k->max_steps) {
        float NU, NV, SE;
        ++it;
        dp5f(U, V, h, flat, &NU, &NV, &SE);
        float err = fabsf(SE) * (h * h);
        if (err > k->tolU) {
            h = h * 0.5f;
            continue;
        }
        if ((NU > k->SU) != (U > k->SU)) {
            float ns, wu, wv, se;
            if (fabsf(V) > fabsf(NV)) {
                ns = 0.0f; wu = U; wv = V;
            } else {
                ns = h; wu = NU; wv = NV;
            }
            for (int n = 0; n < 3; ++n) {
                ns = ns - (wu - k->SU) * (1.0f / wv); /* divf_ */
                dp5f(U, V, ns, flat, &wu, &wv, &se);
            }
            *steps = it;
            return ang + ns;
        }
        if (NU < k->BD) break;
        U = NU;
        V = NV;
        ang = ang + h;
        if (err < k->tolG) h = fminf(h + h, k->hmax);
        if ((k->rs_nonzero && U > k->HU && V > 0.0f) || !(U > 0.0f)) break;
    }
    *steps = it;
    return 15.0f;
}

static float geodesic_f32(const fconsts* k, float st, float ct, float rct, int adaptive, uint32_t* steps) {
    *steps = 0;
    float rotation = k->r * ct;
    int falling;
    float energy;
    if (k->r_inside_h) {
        falling = 0;
        energy = (-st) * k->e_in;
    } else {
        falling = st > 0.0f;
        energy = k->e_out;
    }
    if (rotation < 1e-10f) {
        if (k->inside_sphere) {
            if (k->outside) {
                if (falling) return k->rs_nonzero ? 15.0f : F_PI;
                return 0.0f;
            }
            if (k->sphere_outside) return energy > 0.0f ? 0.0f : 15.0f;
            return 0.0f;
        }
        return (k->sphere_outside && falling) ? 0.0f : 15.0f;
    }
    /* 1/b^2, b = L/E = r ct/E, from the pixel's rct = 1/ct (shared with its sky direction) */
    float inv_b2 = (energy * energy) * ((rct * rct) * k->inv_r2);
    int barrier = k->rs > 0.0f && inv_b2 < k->barrier;
    if ((k->inside_sphere && !k->sphere_outside) || (!k->outside && k->sphere_outside && energy < 0.0f) ||
        (barrier && k->diff_sides) || (k->r < k->r3_2 && k->inside_sphere && falling) ||
        (k->r > k->r3_2 && !k->inside_sphere && !falling))
        return 15.0f;
    /* u'0 = sqrt(1/b^2 - (1 - rs/r)/r^2) (:123), scaled: UB = c u'0.  Outside
     * the horizon E^2 = 1 - rs/r, so the radicand is (E/r)^2 (1/ct^2 - 1) =
     * (E/r)^2 tan^2 theta and UB = (c E/r) |st|/ct: well conditioned where the
     * literal difference cancels (|theta| << 1, a tangential ray: up to 4e-4
     * rad of traveled angle in f32).  Inside the horizon both terms of the
     * radicand are positive and the literal form is kept. */
    float UB;
    if (k->r_inside_h) {
        float ub = sqrtf(maxz(0.0f, inv_b2 - k->h_over_r2));
        if (!falling) ub = -ub;
        UB = k->scale * ub;
    } else {
        UB = (k->ubk * fabsf(st)) * rct;
        if (!falling) UB = -UB;
    }
    /* loop test (:134-135) for the initial state (u' > 0 <=> UB > 0) */
    if ((k->rs_nonzero && k->u0 > k->schwarz_u && UB > 0.0f) || k->max_steps == 0u || !(k->u0 > 0.0f)) return 15.0f;
    int flat = !k->rs_nonzero;
    float U = k->U0;
    if (adaptive) return adaptive_f32(k, U, UB, flat, steps);
    uint32_t it = 0;
    for (;;) { /* :134-191, one step per iteration */
        float NU, NUB;
        rk4f(U, UB, k->step, k->hh, k->hh2, k->hhh, k->h6, k->h2_6, flat, &NU, &NUB);
        ++it;
        if ((NU > k->SU) != (U > k->SU)) {
            float ns, wu, wub;
            if (fabsf(UB) > fabsf(NUB)) {
                ns = 0.0f; wu = U; wub = UB;
            } else {
                ns = k->step; wu = NU; wub = NUB;
            }
            for (int n = 0; n < 3; ++n) {
                ns = ns - (wu - k->SU) * (1.0f / wub); /* divf_ */
                float n2 = ns * ns;
                float n6 = ns * (1.0f / 6.0f);
                rk4f(U, UB, ns, ns * 0.5f, n2 * 0.25f, n2 * 0.5f, n6, ns * n6, flat, &wu, &wub);
            }
            *steps = it;
            return (float)(it - 1u) * k->step + ns;
        }
        if (NU < k->BD) {
            *steps = it;
            return 15.0f;
        }
        U = NU;
        UB = NUB;
        /* loop test: not inside the horizon and falling, budget, u > 0 */
        if ((k->rs_nonzero && U > k->HU && UB > 0.0f) || !(it < k->max_steps) || !(U > 0.0f)) break;
    }
    *steps = it;
    return 15.0f;
}

float geo_oracle_geodesic_f32(const geo_scene* s, float st, float ct, uint32_t* steps) {
    fconsts k = make_fconsts(s);
    uint32_t n = 0;
    float a = geodesic_f32(&k, st, ct, 1.0f / ct, s->mode == GEO_MODE_ADAPTIVE, &n);
    if (steps) *steps = n;
    return a;
}

static inline void m3vf(const float* m, float x, float y, float z, float* o) {
    o[0] = fmaf(m[8], z, fmaf(m[4], y, m[0] * x));
    o[1] = fmaf(m[9], z, fmaf(m[5], y, m[1] * x));
    o[2] = fmaf(m[10], z, fmaf(m[6], y, m[2] * x));
}


typedef struct {
    float a[3], b[3], c[3]; /* d = py a + px b + c */
    int m1_identity;
} cam_f32;

static cam_f32 camera_f32(const geo_frame* f, uint32_t width, uint32_t height) {
    const float* m0 = f->display_to_movement;
    const float* m1 = f->movement_to_central;
    cam_f32 cc;
    double w = (double)width, h = (double)height;
    double sx = 2.0 / w, ox = (1.0 - w) / w, sy = -2.0 / h, oy = (h - 1.0) / h;
    for (int i = 0; i < 3; ++i) {
        double p = -(double)m0[12] * (double)m0[i];
        double q = -(double)m0[13] * (double)m0[4 + i];
        double r = (double)m0[14] * (double)m0[8 + i];
        cc.a[i] = (float)(sy * p);
        cc.b[i] = (float)(sx * q);
        cc.c[i] = (float)((oy * p + ox * q) + r);
    }
    cc.m1_identity = m1[0] == 1.0f && m1[1] == 0.0f && m1[2] == 0.0f && m1[4] == 0.0f && m1[5] == 1.0f &&
                     m1[6] == 0.0f && m1[8] == 0.0f && m1[9] == 0.0f && m1[10] == 1.0f;
    return cc;
}

/* bilinear sample of one sw x sh level, U wraps, V clamps, 8-bit sub-texel
 * weights; per channel: horizontal lerp truncated to 8 bits, vertical lerp
 * rounded.  Texel coordinates in 1/256 texel units: n = floor(256 (U sw -
 * 1/2)); texel floor(n / 256), 8-bit weight n mod 256. */
static uint32_t bilinear_level(const uint32_t* sky, uint32_t sw, uint32_t sh, float U, float V) {
    int nx = (int)floorf(fmaf(U, (float)sw * 256.0f, -128.0f));
    int ny = (int)floorf(fmaf(V, (float)sh * 256.0f, -128.0f));
    uint32_t wx = (uint32_t)nx & 255u;
    uint32_t wy = (uint32_t)ny & 255u;
    int ix0 = nx >> 8, iy0 = ny >> 8;
    int w = (int)sw, h = (int)sh;
    if (ix0 < 0) ix0 += w;
    if (ix0 >= w) ix0 -= w;
    int ix1 = (ix0 + 1 == w) ? 0 : ix0 + 1;
    int iy1 = iy0 + 1;
    iy0 = iy0 < 0 ? 0 : (iy0 > h - 1 ? h - 1 : iy0);
    iy1 = iy1 < 0 ? 0 : (iy1 > h - 1 ? h - 1 : iy1);
    uint32_t t[4] = {sky[(uint32_t)iy0 * sw + (uint32_t)ix0], sky[(uint32_t)iy0 * sw + (uint32_t)ix1],
                     sky[(uint32_t)iy1 * sw + (uint32_t)ix0], sky[(uint32_t)iy1 * sw + (uint32_t)ix1]};
    uint32_t c = 0;
    for (int ch = 0; ch < 4; ++ch) {
        uint32_t v00 = (t[0] >> (8 * ch)) & 255u, v10 = (t[1] >> (8 * ch)) & 255u;
        uint32_t v01 = (t[2] >> (8 * ch)) & 255u, v11 = (t[3] >> (8 * ch)) & 255u;
        uint32_t top = (v00 * (256u - wx) + v10 * wx) >> 8;
        uint32_t bot = (v01 * (256u - wx) + v11 * wx) >> 8;
        c |= ((top * (256u - wy) + bot * wy + 128u) >> 8) << (8 * ch);
    }
    return c;
}

/* BlendState::ALPHA_BLENDING (pipeline.rs:49) of the sample s over the target
 * d, 8-bit fixed point: rgb = round((s a + d (255 - a))/255), alpha =
 * round((255 a + d_a (255 - a))/255); without GEO_FLAG_COMPOSITE d = the
 * clear colour (0,0,0,255). */
static uint32_t blend_over(uint32_t s, uint32_t dst) {
    uint32_t a = s >> 24, out = 0;
    for (int ch = 0; ch < 4; ++ch) {
        uint32_t sv = ch < 3 ? (s >> (8 * ch)) & 255u : 255u;
        uint32_t p = sv * a + ((dst >> (8 * ch)) & 255u) * (255u - a) + 128u;
        out |= ((p + (p >> 8)) >> 8) << (8 * ch);
    }
    return out;
}

/* The pixel's unit ray in the central frame, c2 (shader.wgsl:58-75). */
static void camera_c2(const geo_frame* f, const cam_f32* cam, uint32_t px, uint32_t py, float* c2) {
    /* camera ray (shader.wgsl:60-64): d = M0 (-ny M0[12], -nx M0[13], M0[14]) with the pixel-centre NDC
     * nx = (2 px + 1 - W)/W, ny = (H - 2 py - 1)/H, affine in (px, py): d = py A + px B + C, the frame
     * constants in f64 rounded once to f32 (cam_f32) */
    const cam_f32* cc = cam;
    float d[3];
    for (int i = 0; i < 3; ++i) d[i] = fmaf((float)py, cc->a[i], fmaf((float)px, cc->b[i], cc->c[i]));
    /* aberration (shader.wgsl:69-70) as a boost along z on the unnormalised ray */
    float kk = f->psi_factor_and_position[0];
    float kt = sqrtf(fmaf(-kk, kk, 1.0f));
    float len = sqrtf(fmaf(d[2], d[2], fmaf(d[1], d[1], d[0] * d[0])));
    float id = 1.0f / fmaf(-kk, d[2], len);
    float g = kt * id;
    float e[3] = {d[0] * g, d[1] * g, fmaf(-kk, len, d[2]) * id};
    if (cc->m1_identity) { /* movement_to_central = I (observer.rs:243-246): skipped, -0 stays -0 */
        c2[0] = e[0]; c2[1] = e[1]; c2[2] = e[2];
    } else {
        m3vf(f->movement_to_central, e[0], e[1], e[2], c2);
    }
}

/* GEO_FLAG_RING_F64 (geo.h; DESIGN.md §2 "The capture band in f64"): the
 * traveled angle of a band pixel in f64, restated from the specification
 * (the product's geo_band.h is not shared):
 *   - the camera ray d = py a + px b + c with the frame constants of
 *     camera_f32 in f64, not rounded, and the aberration as the f32 path's
 *     z-boost (shader.wgsl:60-75), in f64;
 *   - solve_ray_fan's node (sphere_ray_tracer.rs:38-49, r > rs) and
 *     solve_geodesic's radial cases, pre-filters and initial slope
 *     (:60-132) as written;
 *   - the main loop (:134-191) one step at a time, on the scaled state
 *     U = (3 rs/2) u with the 14-operation RK4 form,
 *     the loop test, the crossing, the escape, Newton's three refinements;
 * returns lambda' = pi/2 - angle; *steps = the RK4 steps taken. */
static void band_rk4(double U, double V, double h, double hh, double hh2, double hhh, double h6, double h2_6,
                     double* NU, double* NV) {
    double fu = fma(U, U, -U);
    double au = fma(hh, V, U);
    double uh = fma(h, V, U);
    double fa = fma(au, au, -au);
    double bu = fma(hh2, fu, au);
    double fb = fma(bu, bu, -bu);
    double cu = fma(hhh, fa, uh);
    double fc = fma(cu, cu, -cu);
    double fab = fa + fb;
    *NU = fma(h2_6, fu + fab, uh);
    *NV = fma(h6, fma(2.0, fab, fu) + fc, V);
}

static double band_lambda(const geo_frame* f, const geo_scene* s, uint32_t width, uint32_t height, uint32_t px,
                          uint32_t py, uint32_t* steps) {
    const float* m0 = f->display_to_movement;
    const float* m1 = f->movement_to_central;
    double w = (double)width, hgt = (double)height;
    double sx = 2.0 / w, ox = (1.0 - w) / w, sy = -2.0 / hgt, oy = (hgt - 1.0) / hgt;
    double d[3];
    for (int i = 0; i < 3; ++i) {
        double p = -(double)m0[12] * (double)m0[i];
        double q = -(double)m0[13] * (double)m0[4 + i];
        double r_ = (double)m0[14] * (double)m0[8 + i];
        double a = sy * p, b = sx * q, c = (oy * p + ox * q) + r_;
        d[i] = fma((double)py, a, fma((double)px, b, c));
    }
    double k = (double)f->psi_factor_and_position[0];
    double kt = sqrt(1.0 - k * k);
    double len = sqrt(fma(d[2], d[2], fma(d[1], d[1], d[0] * d[0])));
    double id = 1.0 / fma(-k, d[2], len);
    double g = kt * id;
    double e[3] = {d[0] * g, d[1] * g, fma(-k, len, d[2]) * id};
    int ident = m1[0] == 1.0f && m1[1] == 0.0f && m1[2] == 0.0f && m1[4] == 0.0f && m1[5] == 1.0f &&
                m1[6] == 0.0f && m1[8] == 0.0f && m1[9] == 0.0f && m1[10] == 1.0f;
    double c2[3];
    if (ident) {
        c2[0] = e[0]; c2[1] = e[1]; c2[2] = e[2];
    } else {
        for (int i = 0; i < 3; ++i)
            c2[i] = fma((double)m1[8 + i], e[2], fma((double)m1[4 + i], e[1], (double)m1[i] * e[0]));
    }
    double st = c2[2] > -1.0 ? (c2[2] < 1.0 ? c2[2] : 1.0) : -1.0;
    double ct = sqrt(fma(c2[1], c2[1], c2[0] * c2[0]));
    /* solve_ray_fan (:38-49), r > rs */
    double schwarz_r = (double)s->rs, sphere_r = (double)s->sphere_r, r = (double)s->r_obs;
    double rotation = r * ct;
    int r_falling = st > 0.0;
    double energy = sqrt(1. - schwarz_r / r);
    /* solve_geodesic (:60-132) */
    *steps = 0;
    int sphere_outside = sphere_r > schwarz_r;
    int inside_sphere = r < sphere_r;
    double lam0 = O_FRAC_PI_2;
    if (rotation < 1e-10) {
        if (inside_sphere) return lam0 - (r_falling ? O_NO_VALUE : 0.);
        return lam0 - ((sphere_outside && r_falling) ? 0. : O_NO_VALUE);
    }
    double b = rotation / energy;
    int barrier_3r_2 = 1. / (b * b) < 4. / (27. * schwarz_r * schwarz_r);
    double r3_2 = 3. * schwarz_r / 2.;
    int different_sides_3r_2 = ((r < r3_2) ^ (sphere_r < r3_2)) && fabs(r - r3_2) > 1e-10;
    if ((inside_sphere && !sphere_outside) || (barrier_3r_2 && different_sides_3r_2) ||
        (r < r3_2 && inside_sphere && r_falling) || (r > r3_2 && !inside_sphere && !r_falling))
        return lam0 - O_NO_VALUE;
    double u_bar0 = (r_falling ? 1. : -1.) * sqrt(1. / (b * b) - (1. - schwarz_r / r) / (r * r));
    /* the scaled state and thresholds (U = c u, c = 3 rs/2) */
    double c = r3_2;
    double u0 = 1. / r;
    double U = c * u0, V = c * u_bar0;
    double SU = c / sphere_r;
    double BD = c * (0.9 * fmin(u0, 1. / fmax(sphere_r, r3_2)));
    double HU = c / schwarz_r;
    double h = (double)s->step;
    double hh = h / 2., hh2 = h * h / 4., hhh = h * h / 2., h6 = h / 6., h2_6 = h * h / 6.;
    double angle = 0.;
    uint32_t it = 0;
    for (;;) {
        if ((U > HU && V > 0.) || it >= s->max_steps || !(U > 0.)) { /* :134-135 */
            *steps = it;
            return lam0 - O_NO_VALUE;
        }
        double NU, NV;
        band_rk4(U, V, h, hh, hh2, hhh, h6, h2_6, &NU, &NV);
        *steps = it + 1;
        if ((NU > SU) != (U > SU)) { /* :150-182 */
            double ns, wu, wv;
            if (fabs(V) > fabs(NV)) {
                ns = 0.; wu = U; wv = V;
            } else {
                ns = h; wu = NU; wv = NV;
            }
            for (int n = 0; n < 3; ++n) {
                ns -= (wu - SU) / wv;
                double n2 = ns * ns;
                band_rk4(U, V, ns, ns / 2., n2 / 4., n2 / 2., ns / 6., n2 / 6., &wu, &wv);
            }
            return lam0 - (angle + ns);
        }
        if (NU < BD) return lam0 - O_NO_VALUE; /* :184 */
        U = NU;
        V = NV;
        it += 1;
        angle += h;
    }
}

/* ring_kx > 0: GEO_FLAG_RING_F64 applies (the band test |kx ct - 1| < GEO_RING_X on the f32 ray) */
static void pixel_f32(const geo_frame* f, const cam_f32* cam, const fconsts* k, int mode, const float* fan, uint32_t n_fan,
                      const uint32_t* sky, uint32_t sw, uint32_t sh, int opaque, int composite, uint32_t width,
                      uint32_t height, uint32_t px, uint32_t py, uint32_t* rgba, uint8_t* bh_out, float* uv,
                      uint32_t* steps, float ring_kx, const geo_scene* s) {
    float c2[3];
    camera_c2(f, cam, px, py, c2);
    float st = c2[2] > -1.0f ? c2[2] : -1.0f; /* med3(c2z, -1, 1): NaN -> -1 */
    st = st < 1.0f ? st : 1.0f;
    float rho2 = sqrtf(fmaf(c2[1], c2[1], c2[0] * c2[0])); /* cos theta */
    float rrho = 1.0f / rho2;
    float lam;
    int bh;
    *steps = 0;
    if (ring_kx > 0.0f && fabsf(ring_kx * rho2 - 1.0f) < GEO_RING_X) {
        /* the capture-orbit band: lambda' and the mask in f64, the sky from the f32 ray */
        double l = band_lambda(f, s, width, height, px, py, steps);
        lam = (float)l;
        bh = l < -7.0;
    } else if (mode == (int)GEO_MODE_FAN) {
        float t = geo_oracle_acos_pi(st) * (float)(n_fan - 1u); /* (pi/2 - asin st) / pi, in [0, 1] */
        float fl = floorf(t);
        uint32_t i = (uint32_t)fl;
        float w = t - fl;
        uint32_t i1 = (i + 1u < n_fan) ? i + 1u : n_fan - 1u;
        lam = fan[i] * (1.0f - w) + fan[i1] * w;
        bh = lam < -7.0f;
    } else {
        lam = F_PI2 - geodesic_f32(k, st, rho2, rrho, mode == (int)GEO_MODE_ADAPTIVE, steps);
        bh = lam < -7.0f;
    }
    /* sky_uv */
    float sl, cll;
    geo_oracle_sincos_sky(lam, &sl, &cll);
    float ex = cll, ey = 0.0f;
    if (rho2 > 0.0f) {
        float w = cll * rrho;
        ex = c2[0] * w;
        ey = c2[1] * w;
    }
    float c3[3];
    m3vf(f->central_to_uv, ex, ey, sl, c3);
    float U = geo_oracle_atan2_turns(c3[1], c3[0]); /* atan2 / 2pi taken into [0, 1] */
    if (!(U == U)) U = 0.0f;
    U = clampf(U, 0.0f, 1.0f);
    float V = geo_oracle_acos_pi(c3[2]); /* 1/2 - asin(z) / pi */
    uv[0] = U;
    uv[1] = V;
    *bh_out = (uint8_t)bh;
    if (bh) {
        if (!composite) *rgba = 0xFF000000u; /* composite: a discarded fragment keeps the target */
        return;
    }
    *rgba = blend_over(bilinear_level(sky, sw, sh, U, V), composite ? *rgba : 0xFF000000u);
    (void)opaque; /* all-opaque skies take the same formula (a = 255: out = s) */
}

typedef struct {
    const geo_frame* f;
    const geo_scene* s;
    fconsts k;
    cam_f32 cam;
    const float* fan;
    uint32_t n_fan;
    const uint32_t* sky;
    uint32_t sw, sh, width, height, row0, nrows, row_step;
    int opaque;
    int threads, tid;
    uint8_t* rgba;
    uint8_t* mask;
    float* uv;
    uint32_t* steps;
    double* lam;
    double* theta;
    uint64_t total;
    int ring;      /* GEO_FLAG_RING_F64 applies (ring_kx) */
    float ring_kx; /* r_obs / (sqrt(1 - rs/r_obs) 3 sqrt(3)/2 rs), rounded once to f32 */
} job_t;

/* GEO_FLAG_RING_F64 (geo.h): the f32 ray's |b/b_c - 1| = |kx cos(theta) - 1|,
 * kx from the scene in f64 rounded once (the library computes the same
 * expression on its host). */
float geo_oracle_ring_kx(const geo_scene* s) {
    double rs = (double)s->rs, r = (double)s->r_obs;
    double e = sqrt(1.0 - rs / r);
    return (float)(r / (e * (1.5 * sqrt(3.0) * rs)));
}

static int ring_applies(const geo_scene* s) {
    return (s->flags & GEO_FLAG_RING_F64) != 0 && s->rs > 0.0f && s->r_obs > s->rs;
}

/* the band test on the f32 ray's cos(theta) */
static int in_ring(float kx, float ct) { return fabsf(kx * ct - 1.0f) < GEO_RING_X; }

/* |kx cos(theta) - 1| of every pixel's f32 ray on rows row0 + i row_step
 * (the band test's quantity; the scene's kx whatever its flags). */
int geo_oracle_ring_x(const geo_frame* f, const geo_scene* s, uint32_t width, uint32_t height, uint32_t row0,
                      uint32_t nrows, uint32_t row_step, float* x) {
    if (!f || !s || !x || width == 0 || height == 0 || row_step == 0) return -1;
    if ((uint64_t)row0 + (uint64_t)(nrows ? nrows - 1 : 0) * row_step >= height) return -1;
    float kx = geo_oracle_ring_kx(s);
    cam_f32 cam = camera_f32(f, width, height);
    for (uint32_t r = 0; r < nrows; ++r)
        for (uint32_t px = 0; px < width; ++px) {
            float c2[3];
            camera_c2(f, &cam, px, row0 + r * row_step, c2);
            x[(size_t)r * width + px] = fabsf(kx * sqrtf(fmaf(c2[1], c2[1], c2[0] * c2[0])) - 1.0f);
        }
    return 0;
}

int geo_oracle_ring_band(const geo_frame* f, const geo_scene* s, uint32_t width, uint32_t height, uint32_t row0,
                         uint32_t nrows, uint32_t row_step, uint8_t* band) {
    if (!f || !s || !band || width == 0 || height == 0 || row_step == 0) return -1;
    if ((uint64_t)row0 + (uint64_t)(nrows ? nrows - 1 : 0) * row_step >= height) return -1;
    int ring = ring_applies(s) && s->mode != GEO_MODE_FAN;
    float kx = ring ? geo_oracle_ring_kx(s) : 0.0f;
    cam_f32 cam = camera_f32(f, width, height);
    for (uint32_t r = 0; r < nrows; ++r)
        for (uint32_t px = 0; px < width; ++px) {
            uint8_t b = 0;
            if (ring) {
                float c2[3];
                camera_c2(f, &cam, px, row0 + r * row_step, c2);
                b = (uint8_t)in_ring(kx, sqrtf(fmaf(c2[1], c2[1], c2[0] * c2[0])));
            }
            band[(size_t)r * width + px] = b;
        }
    return 0;
}

static void* job_f32(void* arg) {
    job_t* j = (job_t*)arg;
    uint64_t total = 0;
    for (uint32_t r = (uint32_t)j->tid; r < j->nrows; r += (uint32_t)j->threads) {
        uint32_t py = j->row0 + r * j->row_step;
        for (uint32_t px = 0; px < j->width; ++px) {
            size_t o = (size_t)r * j->width + px;
            uint32_t rgba, st;
            uint8_t bh;
            float uv[2];
            memcpy(&rgba, j->rgba + 4 * o, 4); /* the target, for GEO_FLAG_COMPOSITE */
            pixel_f32(j->f, &j->cam, &j->k, (int)j->s->mode, j->fan, j->n_fan, j->sky, j->sw, j->sh, j->opaque,
                      (j->s->flags & GEO_FLAG_COMPOSITE) != 0, j->width, j->height, px, py, &rgba, &bh, uv, &st,
                      j->ring ? j->ring_kx : 0.0f, j->s);
            total += st; /* the steps each pixel reports (the band's: its f64 steps) */
            memcpy(j->rgba + 4 * o, &rgba, 4);
            if (j->mask) j->mask[o] = bh;
            if (j->uv) {
                j->uv[2 * o] = uv[0];
                j->uv[2 * o + 1] = uv[1];
            }
            if (j->steps) j->steps[o] = st;
        }
    }
    j->total = total;
    return NULL;
}

static void* job_f64(void* arg) {
    job_t* j = (job_t*)arg;
    for (uint32_t r = (uint32_t)j->tid; r < j->nrows; r += (uint32_t)j->threads) {
        uint32_t py = j->row0 + r * j->row_step;
        for (uint32_t px = 0; px < j->width; ++px) {
            size_t o = (size_t)r * j->width + px;
            geo_oracle_px p;
            geo_oracle_pixel_f64(j->f, j->s, j->fan, j->n_fan, j->width, j->height, px, py, &p);
            if (j->mask) j->mask[o] = (uint8_t)p.bh;
            if (j->uv) {
                j->uv[2 * o] = (float)p.u;
                j->uv[2 * o + 1] = (float)p.v;
            }
            if (j->steps) j->steps[o] = p.steps;
            if (j->lam) j->lam[o] = p.lam;
            if (j->theta) j->theta[o] = p.theta;
        }
    }
    return NULL;
}

static int run_jobs(job_t* base, int threads, void* (*fn)(void*), uint64_t* total) {
    if (threads < 1) threads = 1;
    if (threads > 256) threads = 256;
    job_t* jobs = (job_t*)calloc((size_t)threads, sizeof(job_t));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    if (!jobs || !th) {
        free(jobs);
        free(th);
        return -3;
    }
    for (int t = 0; t < threads; ++t) {
        jobs[t] = *base;
        jobs[t].threads = threads;
        jobs[t].tid = t;
        if (t > 0 && pthread_create(&th[t], NULL, fn, &jobs[t]) != 0) {
            jobs[t].tid = -1; /* run inline below */
        }
    }
    fn(&jobs[0]);
    for (int t = 1; t < threads; ++t) {
        if (jobs[t].tid < 0) {
            jobs[t].tid = t;
            fn(&jobs[t]);
        } else {
            pthread_join(th[t], NULL);
        }
    }
    uint64_t sum = 0;
    for (int t = 0; t < threads; ++t) sum += jobs[t].total;
    if (total) *total = sum;
    free(jobs);
    free(th);
    return 0;
}

int geo_oracle_render_f32(const geo_frame* f, const geo_scene* s, const float* fan, uint32_t n_fan,
                          const uint8_t* sky, uint32_t sky_w, uint32_t sky_h, uint32_t width,
                          uint32_t height, uint32_t row0, uint32_t nrows, uint32_t row_step,
                          int threads, uint8_t* rgba, uint8_t* mask, float* uv, uint32_t* steps,
                          uint64_t* steps_total) {
    if (!f || !s || !sky || !rgba || width == 0 || height == 0 || row_step == 0) return -1;
    if ((uint64_t)row0 + (uint64_t)(nrows ? nrows - 1 : 0) * row_step >= height) return -1;
    if (s->mode == GEO_MODE_FAN && (!fan || n_fan < 2)) return -1;
    if ((s->flags & GEO_FLAG_RING_F64) &&
        (s->mode == GEO_MODE_FAN || (s->flags & (GEO_FLAG_COMPOSITE | GEO_FLAG_MIPS))))
        return -1; /* the library's GEO_EINVAL */
    job_t j;
    memset(&j, 0, sizeof(j));
    j.f = f;
    j.s = s;
    j.ring = ring_applies(s);
    j.ring_kx = j.ring ? geo_oracle_ring_kx(s) : 0.0f;
    j.k = make_fconsts(s);
    j.cam = camera_f32(f, width, height);
    j.fan = fan;
    j.n_fan = n_fan;
    j.sky = (const uint32_t*)sky;
    j.sw = sky_w;
    j.sh = sky_h;
    j.opaque = 1;
    for (size_t i = 0; i < (size_t)sky_w * sky_h; ++i)
        if (sky[4 * i + 3] != 255u) {
            j.opaque = 0;
            break;
        }
    j.width = width;
    j.height = height;
    j.row0 = row0;
    j.nrows = nrows;
    j.row_step = row_step;
    j.rgba = rgba;
    j.mask = mask;
    j.uv = uv;
    j.steps = steps;
    return run_jobs(&j, threads, job_f32, steps_total);
}

/* ---- GEO_FLAG_MIPS: the specification of geo_pixel.h restated ---------
 * (DESIGN.md §3): a 4-level box-filtered mip chain (basic_sphere_buffer.rs:
 * 31-36), the level of detail from the UV differences across each frame-
 * aligned 2 x 2 pixel quad, trilinear between two bilinear level samples
 * (textureSample, shader.wgsl:101). */
#define O_MIP_LEVELS 4

static uint32_t mipdim(uint32_t d, int l) {
    uint32_t r = d >> l;
    return r ? r : 1u;
}

uint64_t geo_oracle_mip_chain_texels(uint32_t w, uint32_t h) {
    uint64_t n = 0;
    for (int l = 0; l < O_MIP_LEVELS; ++l) n += (uint64_t)mipdim(w, l) * mipdim(h, l);
    return n;
}

/* out: the levels one after another, level 0 = the texture; texel (x, y) of
 * level l+1 = (a + b + c + d + 2) >> 2 per channel over (2x..2x+1, 2y..2y+1)
 * of level l, indices clamped to level l */
void geo_oracle_mip_chain(const uint8_t* rgba8, uint32_t w, uint32_t h, uint32_t* out) {
    memcpy(out, rgba8, (size_t)w * h * 4);
    const uint32_t* src = out;
    uint32_t sw = w, sh = h;
    uint32_t* dst = out + (size_t)w * h;
    for (int l = 1; l < O_MIP_LEVELS; ++l) {
        uint32_t dw = mipdim(w, l), dh = mipdim(h, l);
        for (uint32_t y = 0; y < dh; ++y)
            for (uint32_t x = 0; x < dw; ++x) {
                uint32_t xs[2] = {2 * x < sw ? 2 * x : sw - 1, 2 * x + 1 < sw ? 2 * x + 1 : sw - 1};
                uint32_t ys[2] = {2 * y < sh ? 2 * y : sh - 1, 2 * y + 1 < sh ? 2 * y + 1 : sh - 1};
                uint32_t o = 0;
                for (int ch = 0; ch < 4; ++ch) {
                    uint32_t sum = 2;
                    for (int j = 0; j < 2; ++j)
                        for (int i = 0; i < 2; ++i) sum += (src[(size_t)ys[j] * sw + xs[i]] >> (8 * ch)) & 255u;
                    o |= (sum >> 2) << (8 * ch);
                }
                dst[(size_t)y * dw + x] = o;
            }
        src = dst;
        dst += (size_t)dw * dh;
        sw = dw;
        sh = dh;
    }
}

/* 256 lambda, lambda = log2(rho2)/2 clamped to [0, 3]; log2(1 + t) by the
 * fixed polynomial t (c1 + t (c2 + t (c3 + t c4))) */
static uint32_t lod_q8(float rho2) {
    if (!(rho2 > 1.0f)) return 0u;
    if (!(rho2 < 64.0f)) return 768u;
    uint32_t b;
    memcpy(&b, &rho2, 4);
    float e = (float)((int32_t)(b >> 23) - 127);
    uint32_t mb = (b & 0x007FFFFFu) | 0x3F800000u;
    float m;
    memcpy(&m, &mb, 4);
    float t = m - 1.0f;
    float p = t * fmaf(t, fmaf(t, fmaf(t, -0x1.59455ap-4f, 0x1.4b69f0p-2f), -0x1.5b2e8ap-1f), 0x1.7044aep+0f);
    float l2 = e + p;
    int32_t q = (int32_t)floorf(l2 * 128.0f);
    return q < 0 ? 0u : ((uint32_t)q < 768u ? (uint32_t)q : 768u);
}

void geo_oracle_lod_q8_n(const float* rho2, uint32_t n, uint32_t* out) {
    for (uint32_t i = 0; i < n; ++i) out[i] = lod_q8(rho2[i]);
}

/* the quad footprint in level-0 texels^2: max over the x and y differences */
static float mip_rho2(float dux, float dvx, float duy, float dvy, float w, float h) {
    float ax = dux * w, bx = dvx * h, ay = duy * w, by = dvy * h;
    float rx = fmaf(bx, bx, ax * ax), ry = fmaf(by, by, ay * ay);
    return rx > ry ? rx : ry;
}

typedef struct {
    const geo_frame* f;
    const cam_f32* cam;
    const fconsts* k;
    int mode;
    const float* fan;
    uint32_t n_fan;
    const uint32_t* sky;
    uint32_t sw, sh, width, height, r_lo, gw, gh;
    int threads, tid;
    float* uv;
    uint8_t* bh;
    uint32_t* steps;
} grid_job;

/* UV, black-hole flag and steps of every pixel of the quad-aligned grid
 * (columns 0..gw-1, rows r_lo..r_lo+gh-1), the quads' helpers outside the
 * frame included (the camera of the width x height frame, extrapolated) */
static void* job_grid(void* arg) {
    grid_job* g = (grid_job*)arg;
    for (uint32_t r = (uint32_t)g->tid; r < g->gh; r += (uint32_t)g->threads)
        for (uint32_t x = 0; x < g->gw; ++x) {
            size_t o = (size_t)r * g->gw + x;
            uint32_t rgba = 0;
            pixel_f32(g->f, g->cam, g->k, g->mode, g->fan, g->n_fan, g->sky, g->sw, g->sh, 1, 0, g->width, g->height,
                      x, g->r_lo + r, &rgba, &g->bh[o], &g->uv[2 * o], &g->steps[o], 0.0f, NULL);
        }
    return NULL;
}

int geo_oracle_render_mips_f32(const geo_frame* f, const geo_scene* s, const float* fan, uint32_t n_fan,
                               const uint8_t* sky, uint32_t sky_w, uint32_t sky_h, uint32_t width, uint32_t height,
                               uint32_t row0, uint32_t nrows, int threads, uint8_t* rgba, uint8_t* mask, float* uv,
                               uint32_t* steps, uint64_t* steps_total) {
    if (!f || !s || !sky || !rgba || width == 0 || height == 0 || nrows == 0 || (row0 & 1u)) return -1;
    if ((uint64_t)row0 + nrows > height) return -1;
    if (s->mode == GEO_MODE_FAN && (!fan || n_fan < 2)) return -1;
    if (s->flags & GEO_FLAG_RING_F64) return -1; /* not with GEO_FLAG_MIPS (geo.h) */
    if (threads < 1) threads = 1;
    if (threads > 64) threads = 64;
    uint32_t* chain = (uint32_t*)malloc(geo_oracle_mip_chain_texels(sky_w, sky_h) * 4);
    uint32_t gw = width + (width & 1u), gh = nrows + (nrows & 1u);
    float* guv = (float*)malloc((size_t)gw * gh * 2 * sizeof(float));
    uint8_t* gbh = (uint8_t*)malloc((size_t)gw * gh);
    uint32_t* gst = (uint32_t*)malloc((size_t)gw * gh * 4);
    grid_job* jobs = (grid_job*)calloc((size_t)threads, sizeof(grid_job));
    pthread_t* th = (pthread_t*)calloc((size_t)threads, sizeof(pthread_t));
    if (!chain || !guv || !gbh || !gst || !jobs || !th) {
        free(chain); free(guv); free(gbh); free(gst); free(jobs); free(th);
        return -3;
    }
    geo_oracle_mip_chain(sky, sky_w, sky_h, chain);
    int opaque = 1;
    for (size_t i = 0; i < (size_t)sky_w * sky_h; ++i)
        if (sky[4 * i + 3] != 255u) {
            opaque = 0;
            break;
        }
    fconsts k = make_fconsts(s);
    cam_f32 cam = camera_f32(f, width, height);
    for (int t = 0; t < threads; ++t) {
        grid_job g = {f, &cam, &k, (int)s->mode, fan, n_fan, chain, sky_w, sky_h, width, height, row0, gw, gh,
                      threads, t, guv, gbh, gst};
        jobs[t] = g;
        if (t > 0 && pthread_create(&th[t], NULL, job_grid, &jobs[t]) != 0) jobs[t].tid = -1;
    }
    job_grid(&jobs[0]);
    for (int t = 1; t < threads; ++t) {
        if (jobs[t].tid < 0) {
            jobs[t].tid = t;
            job_grid(&jobs[t]);
        } else {
            pthread_join(th[t], NULL);
        }
    }
    const uint32_t* lvl[O_MIP_LEVELS];
    uint32_t lw[O_MIP_LEVELS], lh[O_MIP_LEVELS];
    const uint32_t* p = chain;
    for (int l = 0; l < O_MIP_LEVELS; ++l) {
        lvl[l] = p;
        lw[l] = mipdim(sky_w, l);
        lh[l] = mipdim(sky_h, l);
        p += (size_t)lw[l] * lh[l];
    }
    int composite = (s->flags & GEO_FLAG_COMPOSITE) != 0;
    uint64_t total = 0;
    for (uint32_t r = 0; r < nrows; ++r)
        for (uint32_t x = 0; x < width; ++x) {
            size_t o = (size_t)r * gw + x, oo = (size_t)r * width + x;
            size_t ox = (size_t)r * gw + (x ^ 1u), oy = (size_t)(r ^ 1u) * gw + x;
            float U = guv[2 * o], V = guv[2 * o + 1];
            /* each row's and each column's own difference, the higher-index pixel minus the lower */
            float dux = (x & 1u) ? U - guv[2 * ox] : guv[2 * ox] - U;
            float dvx = (x & 1u) ? V - guv[2 * ox + 1] : guv[2 * ox + 1] - V;
            float duy = (r & 1u) ? U - guv[2 * oy] : guv[2 * oy] - U;
            float dvy = (r & 1u) ? V - guv[2 * oy + 1] : guv[2 * oy + 1] - V;
            uint32_t q = lod_q8(mip_rho2(dux, dvx, duy, dvy, (float)sky_w, (float)sky_h));
            uint32_t l0 = q >> 8, wf = q & 255u, l1 = l0 + 1 < O_MIP_LEVELS ? l0 + 1 : l0;
            uint32_t s0 = bilinear_level(lvl[l0], lw[l0], lh[l0], U, V);
            uint32_t s1 = bilinear_level(lvl[l1], lw[l1], lh[l1], U, V);
            uint32_t sm = 0;
            for (int ch = 0; ch < 4; ++ch) {
                uint32_t a0 = (s0 >> (8 * ch)) & 255u, a1 = (s1 >> (8 * ch)) & 255u;
                sm |= ((a0 * (256u - wf) + a1 * wf + 128u) >> 8) << (8 * ch);
            }
            uint32_t dst;
            memcpy(&dst, rgba + 4 * oo, 4);
            uint32_t out;
            if (gbh[o])
                out = composite ? dst : 0xFF000000u;
            else
                out = blend_over(sm, composite ? dst : 0xFF000000u);
            (void)opaque;
            memcpy(rgba + 4 * oo, &out, 4);
            if (mask) mask[oo] = gbh[o];
            if (uv) {
                uv[2 * oo] = U;
                uv[2 * oo + 1] = V;
            }
            if (steps) steps[oo] = gst[o];
            total += gst[o];
        }
    if (steps_total) *steps_total = total;
    free(chain); free(guv); free(gbh); free(gst); free(jobs); free(th);
    return 0;
}

int geo_oracle_render_f64(const geo_frame* f, const geo_scene* s, const float* fan, uint32_t n_fan,
                          uint32_t width, uint32_t height, uint32_t row0, uint32_t nrows, uint32_t row_step,
                          int threads, uint8_t* mask, float* uv, uint32_t* steps, double* lam, double* theta) {
    if (!f || !s || width == 0 || height == 0 || row_step == 0) return -1;
    if ((uint64_t)row0 + (uint64_t)(nrows ? nrows - 1 : 0) * row_step >= height) return -1;
    if (s->mode == GEO_MODE_FAN && (!fan || n_fan < 2)) return -1;
    job_t j;
    memset(&j, 0, sizeof(j));
    j.f = f;
    j.s = s;
    j.fan = fan;
    j.n_fan = n_fan;
    j.width = width;
    j.height = height;
    j.row0 = row0;
    j.nrows = nrows;
    j.row_step = row_step;
    j.mask = mask;
    j.uv = uv;
    j.steps = steps;
    j.lam = lam;
    j.theta = theta;
    return run_jobs(&j, threads, job_f64, NULL);
}

/* ------------------------------------------------------------------ */
/* Observer (observer.rs:68-87, 141-160, 197-262; glam 0.25 semantics)  */
/* ------------------------------------------------------------------ */

typedef struct { double x, y, z; } ov3;
typedef struct { ov3 c[3]; } om3; /* column-major */

static double olen(ov3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }
static ov3 ocross(ov3 a, ov3 b) {
    ov3 r = {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
    return r;
}
static ov3 omv(const om3* m, ov3 v) {
    ov3 r;
    r.x = m->c[0].x * v.x + m->c[1].x * v.y + m->c[2].x * v.z;
    r.y = m->c[0].y * v.x + m->c[1].y * v.y + m->c[2].y * v.z;
    r.z = m->c[0].z * v.x + m->c[1].z * v.y + m->c[2].z * v.z;
    return r;
}
static om3 omm(const om3* a, const om3* b) {
    om3 r;
    for (int i = 0; i < 3; ++i) r.c[i] = omv(a, b->c[i]);
    return r;
}
static om3 otr(const om3* m) {
    om3 r;
    r.c[0].x = m->c[0].x; r.c[0].y = m->c[1].x; r.c[0].z = m->c[2].x;
    r.c[1].x = m->c[0].y; r.c[1].y = m->c[1].y; r.c[1].z = m->c[2].y;
    r.c[2].x = m->c[0].z; r.c[2].y = m->c[1].z; r.c[2].z = m->c[2].z;
    return r;
}
/* polar_transformations.rs:43-51 */
static om3 olook(ov3 t) {
    double inv = 1.0 / olen(t);
    ov3 z = {t.x * inv, t.y * inv, t.z * inv};
    double pr = olen(z), pphi = 0., plam = 0.;
    if (pr != 0.) {
        pphi = atan2(z.y, z.x);
        plam = asin(z.z / pr);
    }
    plam -= O_FRAC_PI_2;
    ov3 x = {pr * cos(pphi) * cos(plam), pr * sin(pphi) * cos(plam), pr * sin(plam)};
    ov3 y = ocross(z, x);
    om3 m = {{x, y, z}};
    return m;
}

void geo_oracle_observer_frame(double rs, double fov, double width, double height, const double pos[3],
                               double cam_phi, double cam_theta, int state, double energy, geo_frame* out) {
    ov3 p = {pos[0], pos[1], pos[2]};
    double r = olen(p);
    double hr = 1. - rs / r;
    double vx, vy;
    /* unmoving_velocity / frozen_fall_velocity (observer.rs:141-160) */
    int unmoving = (state == GEO_OBSERVER_UNMOVING) || (energy * energy < hr);
    if (unmoving) {
        if (r > rs) {
            vx = 1. / sqrt(hr);
            vy = 0.;
        } else {
            vx = 0.;
            vy = -sqrt(-hr);
        }
    } else {
        vx = energy / hr;
        vy = sqrt(energy * energy - hr);
    }
    double psi = r > rs ? vx * vx * hr : -vy * vy / hr;
    if (psi - 1. < 1e-10) psi = 1.;
    ov3 np = {-p.x, -p.y, -p.z};
    om3 l = olook(np);
    om3 std_to_central = otr(&l);
    om3 cu = olook(p);
    om3 flip = {{{1, 0, 0}, {0, -1, 0}, {0, 0, 1}}};
    om3 central_to_uv = omm(&cu, &flip);
    ov3 camv = {cos(cam_phi) * cos(cam_theta), sin(cam_phi) * cos(cam_theta), sin(cam_theta)};
    om3 cam_to_std = olook(camv);
    om3 cam = omm(&std_to_central, &cam_to_std);
    double t = tan(fov / 2.);
    double fov_scaling[4] = {t, t * (width / height), 1., 1.};
    memset(out, 0, sizeof(*out));
    for (int c = 0; c < 3; ++c) {
        out->display_to_movement[c * 4 + 0] = (float)cam.c[c].x;
        out->display_to_movement[c * 4 + 1] = (float)cam.c[c].y;
        out->display_to_movement[c * 4 + 2] = (float)cam.c[c].z;
        out->central_to_uv[c * 4 + 0] = (float)central_to_uv.c[c].x;
        out->central_to_uv[c * 4 + 1] = (float)central_to_uv.c[c].y;
        out->central_to_uv[c * 4 + 2] = (float)central_to_uv.c[c].z;
        out->movement_to_central[c * 4 + c] = 1.f;
    }
    for (int i = 0; i < 4; ++i) out->display_to_movement[12 + i] = (float)fov_scaling[i];
    out->movement_to_central[15] = 1.f;
    out->central_to_uv[15] = 1.f;
    out->psi_factor_and_position[0] = (float)sqrt((psi - 1.) / psi);
    out->psi_factor_and_position[1] = (float)p.x;
    out->psi_factor_and_position[2] = (float)p.y;
    out->psi_factor_and_position[3] = (float)p.z;
}
