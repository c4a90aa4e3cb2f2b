/*
 * geo_oracle_points.c — ORACLE (test infrastructure only; never linked into,
 * called by, or shipped with libgeo.so) for the accretion-disk point path
 * (SURVEY.md §8f N3).  Independent C restatements, in the reference's own
 * structure:
 *
 *   RayConnector           SR/simulation/ray_connector.rs:6-157 (f32; reset_ray /
 *                          update_ray keep the reference's mutual recursion)
 *   Orbit                  SR/simulation/orbit.rs:28-182 (f64)
 *   PointCloud::new/update SR/schwarzschild_point_shader/point_cloud.rs:20-65, 117-148
 *   vs_main                SR/schwarzschild_point_shader/shader.wgsl:36-68 (f32)
 *
 * Transcendentals: `libm` = 1 uses the C library's acosf/atanf where the
 * reference calls f32::acos/f32::atan (the reference-faithful variant; the
 * reference's own tests, tests.rs:15-79, run on it); `libm` = 0 uses the
 * fixed polynomials of the f32 kernel (the bit-exact checker of the HIP path).
 * glam's Vec3::angle_between is its acos_approx (DirectXMath XMScalarAcos) in
 * both.  Pinned by the reference's RayConnector tests (5e-4 rad); parity of
 * the rest is unpinned (no reference run is possible here, see geo_oracle.h).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "geo_oracle.h"

#define NR_NODES 48
#define SMALLEST_ANGLE 0.05f
#define F32_PI 3.14159265358979323846f
#define F32_FRAC_PI_2 1.57079632679489661923f
#define F32_TAU 6.28318530717958647692f

/* the kernel's f32 acos (geo_math.h acosf_) from the asin kernel */
float geo_oracle_acosf(float x) {
    x = x < -1.0f ? -1.0f : (x > 1.0f ? 1.0f : x);
    float a = fabsf(x);
    if (a <= 0.5f) return F32_FRAC_PI_2 - geo_oracle_asinf(x);
    float z = 0.5f * (1.0f - a);
    float s = sqrtf(z);
    float p = fmaf(fmaf(fmaf(fmaf(4.2163199048e-2f, z, 2.4181311049e-2f), z, 4.5470025998e-2f), z,
                        7.4953002686e-2f), z, 1.6666752422e-1f);
    float r = 2.0f * fmaf(p * z, s, s);
    return x > 0.0f ? r : F32_PI - r;
}

static float o_acos(float x, int libm) { return libm ? acosf(x) : geo_oracle_acosf(x); }
static float o_atan(float x, int libm) { return libm ? atanf(x) : geo_oracle_atan2f(x, 1.0f); }

/* glam 0.25 Vec3 (scalar f32) */
typedef struct { float x, y, z; } fv3;
static float fdot(fv3 a, fv3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static float flen(fv3 a) { return sqrtf(fdot(a, a)); }
static float flen_recip(fv3 a) { return 1.0f / flen(a); }
static float acos_approx(float v) {
    int nonnegative = v >= 0.0f;
    float x = fabsf(v);
    float omx = 1.0f - x;
    if (omx < 0.0f) omx = 0.0f;
    float root = sqrtf(omx);
    float result = ((((((-0.0012624911f * x + 0.0066700901f) * x - 0.0170881256f) * x + 0.0308918810f) * x -
                      0.0501743046f) * x + 0.0889789874f) * x - 0.2145988016f) * x + 1.5707963050f;
    result *= root;
    return nonnegative ? result : F32_PI - result;
}
static float fangle_between(fv3 a, fv3 b) { return acos_approx(fdot(a, b) / sqrtf(fdot(a, a) * fdot(b, b))); }
static float fsignum(float x) { return x != x ? x : copysignf(1.0f, x); }

typedef struct {
    float schwarz_r;
    fv3 pos;
    float last_phi;
    int less_than_180;
    int needs_reset;
    float u_ray[NR_NODES];
    int libm;
} ray_connector;

/* ray_connector.rs:141-157 */
static float calc_ray_angle(const ray_connector* s, float u_bar, float r) {
    float theta;
    if (r > s->schwarz_r) {
        theta = fsignum(u_bar) *
                o_acos(sqrtf(1.f / (1.f + (r * r * u_bar * u_bar) / (1.f - s->schwarz_r / r))), s->libm);
    } else {
        float intermediate = -(r * r * u_bar * u_bar) / (1.f - s->schwarz_r / r) - 1.f;
        if (intermediate > 0.f)
            theta = -F32_FRAC_PI_2 + o_atan(sqrtf(1.f / intermediate), s->libm);
        else
            theta = 0.f;
    }
    return (F32_FRAC_PI_2 - theta) * (s->less_than_180 ? 1.f : -1.f);
}

static float update_ray(ray_connector* s, fv3 other, int iterations);

/* ray_connector.rs:27-44 */
static float reset_ray(ray_connector* s, fv3 other) {
    s->needs_reset = 0;
    float u0 = 1.f / flen(other);
    float u1 = 1.f / flen(s->pos);
    s->last_phi = fangle_between(s->pos, other);
    if (!s->less_than_180) s->last_phi = F32_TAU - s->last_phi;
    for (int i = 0; i < NR_NODES; ++i) {
        float weight = (float)i / ((float)NR_NODES - 1.f);
        s->u_ray[i] = u0 * (1.f - weight) + u1 * weight;
    }
    return update_ray(s, other, 5);
}

/* ray_connector.rs:48-132 */
static float update_ray(ray_connector* s, fv3 other, int iterations) {
    if (s->needs_reset) return reset_ray(s, other);
    s->last_phi = fangle_between(s->pos, other);
    if (!s->less_than_180) s->last_phi = F32_TAU - s->last_phi;
    if (s->last_phi < SMALLEST_ANGLE) {
        s->needs_reset = 1;
        float incoming_angle;
        if (s->last_phi == 0.f) {
            incoming_angle = flen(other) > flen(s->pos) ? 0.f : F32_PI;
        } else {
            float u0 = flen_recip(other);
            float u_bar = (flen_recip(s->pos) - u0) / s->last_phi -
                          s->last_phi / 2.f * (-u0 + 1.5f * s->schwarz_r * u0 * u0);
            incoming_angle = calc_ray_angle(s, u_bar, 1.f / u0);
        }
        return incoming_angle;
    }
    float u0 = flen_recip(other);
    float u1 = flen_recip(s->pos);
    if (fabsf(1.f / u0 - 1.f / s->u_ray[0]) > 0.5f) return reset_ray(s, other);
    float u0_delta = u0 - s->u_ray[0];
    float u1_delta = u1 - s->u_ray[NR_NODES - 1];
    for (int i = 0; i < NR_NODES; ++i) {
        float weight = (float)i / ((float)NR_NODES - 1.f);
        s->u_ray[i] += u0_delta * (1.f - weight) + u1_delta * weight;
    }
    float residual[NR_NODES - 2];
    float thomas_c[NR_NODES - 2];
    memset(residual, 0, sizeof(residual));
    memset(thomas_c, 0, sizeof(thomas_c));
    float h = s->last_phi / (float)(NR_NODES - 1);
    float scale = 1.f / (h * h);
    float* u = s->u_ray;
    float R = s->schwarz_r;
    for (int k = 0; k < iterations; ++k) {
        for (int i = 1; i < NR_NODES - 1; ++i)
            residual[i - 1] = scale * (-u[i - 1] + 2.f * u[i] - u[i + 1]) - u[i] + 3.f * R / 2.f * u[i] * u[i];
        float main_diag_inv = 1.f / (2.f * scale - 1.f + 3.f * R * u[1]);
        thomas_c[0] = (-scale) * main_diag_inv;
        residual[0] = residual[0] * main_diag_inv;
        for (int i = 1; i < NR_NODES - 2; ++i) {
            float mdi = 1.f / (2.f * scale - 1.f + 3.f * R * u[i + 1] + scale * thomas_c[i - 1]);
            thomas_c[i] = (-scale) * mdi;
            residual[i] = (residual[i] + scale * residual[i - 1]) * mdi;
        }
        u[NR_NODES - 2] -= residual[NR_NODES - 3];
        for (int i = NR_NODES - 4; i >= 0; --i) {
            residual[i] = residual[i] - thomas_c[i] * residual[i + 1];
            u[i + 1] -= residual[i];
        }
    }
    float u_bar = (u[1] - u[0]) / h - h / 2.f * (-u[0] + 1.5f * R * u[0] * u[0]);
    return calc_ray_angle(s, u_bar, 1.f / u0);
}

/* Batch form of the device API (geo_rays_update): connectors c < n near side
 * (when sides & 1), then far side; state u[c*48 + i], needs[c]. */
int geo_oracle_rays_update(float rs, uint32_t n_points, uint32_t sides, const float* pos, float* u, uint8_t* needs,
                           const float* other, int per_point, int iterations, int reset, float* out, int libm) {
    uint32_t nside = ((sides & 1u) ? 1u : 0u) + ((sides & 2u) ? 1u : 0u);
    for (uint32_t c = 0; c < n_points * nside; ++c) {
        uint32_t p = c % n_points;
        int far = (sides == 2u) ? 1 : (c >= n_points);
        ray_connector s;
        s.schwarz_r = rs;
        s.pos.x = pos[3 * p];
        s.pos.y = pos[3 * p + 1];
        s.pos.z = pos[3 * p + 2];
        s.last_phi = 1.f;
        s.less_than_180 = !far;
        s.needs_reset = needs[c];
        s.libm = libm;
        memcpy(s.u_ray, u + (size_t)c * NR_NODES, sizeof(s.u_ray));
        const float* o = per_point ? other + 3 * (size_t)p : other;
        fv3 ov = {o[0], o[1], o[2]};
        float a = reset ? reset_ray(&s, ov) : update_ray(&s, ov, iterations);
        memcpy(u + (size_t)c * NR_NODES, s.u_ray, sizeof(s.u_ray));
        needs[c] = (uint8_t)s.needs_reset;
        if (out) {
            out[4 * c] = s.pos.x;
            out[4 * c + 1] = s.pos.y;
            out[4 * c + 2] = s.pos.z;
            out[4 * c + 3] = a;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* Orbit (orbit.rs) in f64, glam DVec3/DMat3 semantics                   */
/* ------------------------------------------------------------------ */

typedef struct { double x, y, z; } dv3;
static dv3 d3(double x, double y, double z) { dv3 r = {x, y, z}; return r; }
static double ddot(dv3 a, dv3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static double dlen(dv3 a) { return sqrt(ddot(a, a)); }
static dv3 dcross(dv3 a, dv3 b) { return d3(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y); }
static double dangle_between(dv3 a, dv3 b) {
    double c = ddot(a, b) / sqrt(ddot(a, a) * ddot(b, b));
    c = c < -1. ? -1. : (c > 1. ? 1. : c);
    return acos(c);
}
static dv3 polar_to_carthesic(dv3 p) { return d3(p.x * cos(p.y) * cos(p.z), p.x * sin(p.y) * cos(p.z), p.x * sin(p.z)); }
static dv3 carthesic_to_polar(dv3 v) {
    dv3 p = d3(0, 0, 0);
    p.x = dlen(v);
    if (p.x != 0.) {
        p.y = atan2(v.y, v.x);
        p.z = asin(v.z / p.x);
    }
    return p;
}
typedef struct { dv3 c[3]; } dm3;
static dv3 dmv(const dm3* m, dv3 v) {
    dv3 r = d3(m->c[0].x * v.x, m->c[0].y * v.x, m->c[0].z * v.x);
    r = d3(r.x + m->c[1].x * v.y, r.y + m->c[1].y * v.y, r.z + m->c[1].z * v.y);
    return d3(r.x + m->c[2].x * v.z, r.y + m->c[2].y * v.z, r.z + m->c[2].z * v.z);
}

typedef struct {
    double schwarz_r, start_phi, tilt_angle, orbit_angle;
    dm3 plane_tilt_mat;
    double energy, rotation, r, u, u_bar, last_r;
    int has_hit_singularity;
} orbit;

static int orbit_new(double schwarz_r, dv3 position, dv3 desired_direction, double rotation, orbit* o) {
    double r = dlen(position);
    if (r <= schwarz_r) return 0;
    if (rotation < schwarz_r * 1e-5) rotation = 0.;
    double u = 1. / r;
    double energy = sqrt((1. - schwarz_r / r) * (1. + rotation * rotation / (r * r)));
    dv3 plane_normal = dcross(position, desired_direction);
    double tilt_angle = dangle_between(plane_normal, d3(0, 0, 1));
    double pos_phi = atan2(position.y, position.x);
    if (tilt_angle < 1e-10 || 3.14159265358979323846 - tilt_angle < 1e-10) {
        tilt_angle = 0.;
        o->start_phi = 0.;
        o->orbit_angle = pos_phi;
        o->plane_tilt_mat.c[0] = d3(1, 0, 0);
        o->plane_tilt_mat.c[1] = d3(0, 1, 0);
        o->plane_tilt_mat.c[2] = d3(0, 0, 1);
    } else {
        dv3 horizontal_cut = dcross(d3(0, 0, 1), plane_normal);
        double orbit_angle = dangle_between(horizontal_cut, position);
        if (position.z < 0.) orbit_angle = 6.28318530717958647692 - orbit_angle;
        o->orbit_angle = orbit_angle;
        o->start_phi = atan2(horizontal_cut.y, horizontal_cut.x);
        double s = sin(tilt_angle), c = cos(tilt_angle);
        o->plane_tilt_mat.c[0] = d3(1, 0, 0);
        o->plane_tilt_mat.c[1] = d3(0, c, s);
        o->plane_tilt_mat.c[2] = d3(0, -s, c);
    }
    o->schwarz_r = schwarz_r;
    o->tilt_angle = tilt_angle;
    o->energy = energy;
    o->rotation = rotation;
    o->r = r;
    o->u = u;
    o->u_bar = 0.;
    o->last_r = r;
    o->has_hit_singularity = 0;
    return 1;
}

static void orbit_do_angle_step(orbit* o, double delta_phi) {
    double l = o->rotation, u = o->u, u_bar = o->u_bar, schwarz_r = o->schwarz_r;
    double a_u = u + delta_phi / 2. * u_bar;
    double a_u_bar = u_bar + delta_phi / 2. * (schwarz_r * (1. / (2. * l * l) + 3. / 2. * u * u) - u);
    double b_u = u + delta_phi / 2. * a_u_bar;
    double b_u_bar = u_bar + delta_phi / 2. * (schwarz_r * (1. / (2. * l * l) + 3. / 2. * a_u * a_u) - a_u);
    double c_u = u + delta_phi * b_u_bar;
    double c_u_bar = u_bar + delta_phi * (schwarz_r * (1. / (2. * l * l) + 3. / 2. * b_u * b_u) - b_u);
    double next_u = u + delta_phi * (u_bar / 6. + a_u_bar / 3. + b_u_bar / 3. + c_u_bar / 6.);
    double next_u_bar = u_bar + delta_phi * (schwarz_r / (2. * l * l) +
                                             3. * schwarz_r / 2. * (u * u / 6. + a_u * a_u / 3. + b_u * b_u / 3. + c_u * c_u / 6.) -
                                             (u + 2. * a_u + 2. * b_u + c_u) / 6.);
    o->u = next_u;
    o->u_bar = next_u_bar;
    if (isinf(o->u) || o->u > 100.) {
        o->has_hit_singularity = 1;
    } else {
        o->r = 1. / o->u;
        o->orbit_angle += delta_phi;
    }
}

static void orbit_do_step(orbit* o, double time_step) {
    if (o->has_hit_singularity) return;
    if (o->rotation == 0.) {
        double next_r = 2. * o->r - o->last_r - time_step * time_step * o->schwarz_r / (2. * o->r * o->r);
        if (next_r < 0.) {
            o->has_hit_singularity = 1;
        } else {
            o->last_r = o->r;
            o->r = next_r;
        }
        return;
    }
    double l = o->rotation, u = o->u, u_bar = o->u_bar;
    double delta_phi = time_step * l * u * u / 2.;
    double next_u = u + delta_phi * u_bar;
    delta_phi = time_step * l / 4. * (u * u + next_u * next_u);
    next_u = u + delta_phi * u_bar;
    delta_phi = time_step * l / 4. * (u * u + next_u * next_u);
    next_u = u + delta_phi * u_bar;
    delta_phi = time_step * l / 4. * (u * u + next_u * next_u);
    if (next_u > 50.) {
        o->has_hit_singularity = 1;
        return;
    }
    double fr = 1. + floor(delta_phi * 100.);
    unsigned step_fragments = fr > 1000. ? 1000u : (unsigned)fr;
    for (unsigned i = 0; i < step_fragments; ++i) {
        orbit_do_angle_step(o, delta_phi / (double)step_fragments);
        if (o->has_hit_singularity) return;
    }
}

static dv3 orbit_get_position(const orbit* o) {
    dv3 p = carthesic_to_polar(dmv(&o->plane_tilt_mat, polar_to_carthesic(d3(o->r, o->orbit_angle, 0.))));
    p.y += o->start_phi;
    return polar_to_carthesic(p);
}

/* fastrand 2.0.1 wyrand + f64 mapping, one stream per point (same seeding as
 * the device path: seed ^ (golden * (i + 1))) */
static uint64_t wy_u64(uint64_t* s) {
    uint64_t x = *s + 0xA0761D6478BD642Full;
    *s = x;
    unsigned __int128 t = (unsigned __int128)x * (unsigned __int128)(x ^ 0xE7037ED1A0B428DBull);
    return (uint64_t)t ^ (uint64_t)(t >> 64);
}
static double wy_f64(uint64_t* s) {
    uint64_t bits = (1ull << 62) - (1ull << 52) + (wy_u64(s) >> 12);
    double d;
    memcpy(&d, &bits, 8);
    return d - 1.0;
}
static uint64_t stream_seed(uint64_t seed, uint32_t i) { return seed ^ (0x9E3779B97F4A7C15ull * ((uint64_t)i + 1u)); }

static void spawn(double rs, uint64_t* s, orbit* o) {
    double r = 16. + 10. * wy_f64(s);
    double phi = wy_f64(s) * 6.283185307179586;
    double theta = 0.2 * (wy_f64(s) - 0.5);
    dv3 pos = polar_to_carthesic(d3(r, phi, theta));
    (void)orbit_new(rs, pos, d3(-pos.y, pos.x, 0.), 18. + 2. * wy_f64(s), o);
}

/* PointCloud::new + `nframes` PointCloud::update calls (point_cloud.rs:20-65,
 * 117-148), sequentially.  observers: 3 floats per frame (+1 for new); dts:
 * seconds per frame.  out_near/out_far (4 floats per point; far may be NULL),
 * out_pos (3 floats per point): the state after the last frame. */
int geo_oracle_points_run(float rs, const float* model, uint32_t n, int farside, int orbits, uint64_t seed,
                          uint32_t nframes, const float* observers, const double* dts, float* out_near,
                          float* out_far, float* out_pos, int libm) {
    ray_connector* near_ = (ray_connector*)calloc(n, sizeof(ray_connector));
    ray_connector* far_ = farside ? (ray_connector*)calloc(n, sizeof(ray_connector)) : NULL;
    orbit* orb = orbits ? (orbit*)calloc(n, sizeof(orbit)) : NULL;
    uint64_t* rng = orbits ? (uint64_t*)calloc(n, sizeof(uint64_t)) : NULL;
    if (!near_ || (farside && !far_) || (orbits && (!orb || !rng))) {
        free(near_); free(far_); free(orb); free(rng);
        return -3;
    }
    fv3 obs = {observers[0], observers[1], observers[2]};
    float *vn = out_near, *vf = out_far;
    for (uint32_t i = 0; i < n; ++i) {
        fv3 p = {model[3 * i], model[3 * i + 1], model[3 * i + 2]};
        ray_connector* sides[2] = {&near_[i], farside ? &far_[i] : NULL};
        for (int k = 0; k < 2; ++k) {
            if (!sides[k]) continue;
            ray_connector* s = sides[k];
            s->schwarz_r = rs;
            s->pos = p;
            s->last_phi = 1.f;
            s->less_than_180 = k == 0;
            s->needs_reset = 1;
            s->libm = libm;
            for (int j = 0; j < NR_NODES; ++j) s->u_ray[j] = 1.f;
            float a = reset_ray(s, obs);
            float* v = k == 0 ? vn : vf;
            if (v) {
                v[4 * i] = p.x; v[4 * i + 1] = p.y; v[4 * i + 2] = p.z; v[4 * i + 3] = a;
            }
        }
        if (orbits) {
            uint64_t s = stream_seed(seed, i);
            if (!orbit_new(rs, d3(p.x, p.y, p.z), d3(-(double)p.y, p.x, 0.), 18. + 2. * wy_f64(&s), &orb[i])) {
                free(near_); free(far_); free(orb); free(rng);
                return -1;
            }
            rng[i] = s;
        }
    }
    for (uint32_t f = 0; f < nframes; ++f) {
        fv3 ob = {observers[3 * (f + 1)], observers[3 * (f + 1) + 1], observers[3 * (f + 1) + 2]};
        for (uint32_t i = 0; i < n; ++i) {
            if (orbits) {
                orbit_do_step(&orb[i], dts[f]);
                dv3 op = orbit_get_position(&orb[i]);
                fv3 orbit_pos = {(float)op.x, (float)op.y, (float)op.z};
                if (orb[i].has_hit_singularity || fdot(orbit_pos, orbit_pos) <= rs * rs) {
                    spawn(rs, &rng[i], &orb[i]);
                    dv3 np = orbit_get_position(&orb[i]);
                    fv3 npf = {(float)np.x, (float)np.y, (float)np.z};
                    near_[i].pos = npf;
                    reset_ray(&near_[i], ob);
                    if (farside) {
                        far_[i].pos = npf;
                        reset_ray(&far_[i], ob);
                    }
                }
                near_[i].pos = orbit_pos;
                if (farside) far_[i].pos = orbit_pos;
            }
            float a = update_ray(&near_[i], ob, 1);
            if (vn) {
                vn[4 * i] = near_[i].pos.x; vn[4 * i + 1] = near_[i].pos.y; vn[4 * i + 2] = near_[i].pos.z;
                vn[4 * i + 3] = a;
            }
            if (farside) {
                float b = update_ray(&far_[i], ob, 1);
                if (vf) {
                    vf[4 * i] = far_[i].pos.x; vf[4 * i + 1] = far_[i].pos.y; vf[4 * i + 2] = far_[i].pos.z;
                    vf[4 * i + 3] = b;
                }
            }
        }
    }
    if (out_pos)
        for (uint32_t i = 0; i < n; ++i) {
            out_pos[3 * i] = near_[i].pos.x;
            out_pos[3 * i + 1] = near_[i].pos.y;
            out_pos[3 * i + 2] = near_[i].pos.z;
        }
    free(near_); free(far_); free(orb); free(rng);
    return 0;
}

/* ------------------------------------------------------------------ */
/* vs_main (shader.wgsl:36-68) in the kernel's f32 order + PointList raster */
/* ------------------------------------------------------------------ */

static void vmul4_t(const float* m, float x, float y, float z, float w, float* o) {
    for (int j = 0; j < 4; ++j) o[j] = fmaf(m[4 * j + 3], w, fmaf(m[4 * j + 2], z, fmaf(m[4 * j + 1], y, m[4 * j] * x)));
}

int geo_oracle_project_point(const geo_frame* f, const float* v, uint32_t width, uint32_t height, int* ix, int* iy) {
    const float *m0 = f->display_to_movement, *m1 = f->movement_to_central, *m2 = f->central_to_uv;
    float k = f->psi_factor_and_position[0];
    float c[4];
    vmul4_t(m2, v[0], v[1], v[2], v[3], c);
    float pphi = geo_oracle_atan2f(c[1], c[0]);
    float plam = c[3];
    if (plam < 0.0f) pphi += 2.0f * F32_FRAC_PI_2;
    plam = F32_FRAC_PI_2 - fabsf(plam);
    float sp, cp, sl, cl;
    geo_oracle_sincosf(pphi, &sp, &cp);
    geo_oracle_sincosf(plam, &sl, &cl);
    vmul4_t(m1, cp * cl, sp * cl, sl, 0.0f, c);
    pphi = geo_oracle_atan2f(c[1], c[0]);
    plam = geo_oracle_asinf(c[2]);
    float sr, cr;
    geo_oracle_sincosf(-plam, &sr, &cr);
    plam = -geo_oracle_asinf((sr - k) / (1.0f - sr * k));
    geo_oracle_sincosf(pphi, &sp, &cp);
    geo_oracle_sincosf(plam, &sl, &cl);
    vmul4_t(m0, cp * cl, sp * cl, sl, 0.0f, c);
    float sx = c[0] / m0[12], sy = c[1] / m0[13], sz = c[2] / m0[14];
    float cw = fabsf(sz);
    *ix = -1;
    *iy = -1;
    if (!(sz > 0.0f) || !(fabsf(sy) <= cw) || !(fabsf(sx) <= cw)) return 0;
    float nx = -sy / cw, ny = -sx / cw;
    float fx = (nx + 1.0f) * 0.5f * (float)width;
    float fy = (1.0f - ny) * 0.5f * (float)height;
    float flx = floorf(fx), fly = floorf(fy);
    if (!(flx >= 0.0f && flx < (float)width && fly >= 0.0f && fly < (float)height)) return 0;
    *ix = (int)flx;
    *iy = (int)fly;
    return 1;
}

int geo_oracle_draw_points(const geo_frame* f, const float* verts, uint32_t n, uint32_t width, uint32_t height,
                           uint32_t row0, uint32_t nrows, uint8_t* rgba, int* out_xy) {
    for (uint32_t i = 0; i < n; ++i) {
        int x, y;
        int vis = geo_oracle_project_point(f, verts + 4 * (size_t)i, width, height, &x, &y);
        if (out_xy) {
            out_xy[2 * i] = x;
            out_xy[2 * i + 1] = y;
        }
        if (vis && (uint32_t)y >= row0 && (uint32_t)y - row0 < nrows) {
            uint8_t* px = rgba + 4 * ((size_t)((uint32_t)y - row0) * width + (uint32_t)x);
            px[0] = 255; px[1] = 0; px[2] = 0; px[3] = 255;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------ */
/* Orbiting observer (observer.rs:104-124, 162-169, 197-262): start_orbit,  */
/* then per frame update_position + calc_transformation_pipeline            */
/* ------------------------------------------------------------------ */

static dm3 dm_cols(dv3 x, dv3 y, dv3 z) { dm3 m; m.c[0] = x; m.c[1] = y; m.c[2] = z; return m; }
static dm3 dmm(const dm3* a, const dm3* b) { return dm_cols(dmv(a, b->c[0]), dmv(a, b->c[1]), dmv(a, b->c[2])); }
static dm3 dtr(const dm3* m) {
    return dm_cols(d3(m->c[0].x, m->c[1].x, m->c[2].x), d3(m->c[0].y, m->c[1].y, m->c[2].y),
                   d3(m->c[0].z, m->c[1].z, m->c[2].z));
}
static dm3 drot_x(double a) { double s = sin(a), c = cos(a); return dm_cols(d3(1, 0, 0), d3(0, c, s), d3(0, -s, c)); }
static dm3 drot_z(double a) { double s = sin(a), c = cos(a); return dm_cols(d3(c, s, 0), d3(-s, c, 0), d3(0, 0, 1)); }
static dm3 dlook(dv3 t) { /* polar_transformations.rs:43-51 */
    double inv = 1. / dlen(t);
    dv3 z = d3(t.x * inv, t.y * inv, t.z * inv);
    dv3 xp = carthesic_to_polar(z);
    xp.z -= 1.57079632679489661923;
    dv3 x = polar_to_carthesic(xp);
    return dm_cols(x, dcross(z, x), z);
}
static double dsignum(double x) { return signbit(x) ? -1. : 1.; }

/* orbit.rs:185-208 */
static dv3 orbit_get_velocity(const orbit* o) {
    double hr = 1. - o->schwarz_r / o->r;
    double falling = o->rotation == 0. ? -dsignum(o->r - o->last_r) : dsignum(o->u_bar);
    return d3(o->energy / hr,
              -falling * sqrt(o->energy * o->energy - hr * (1. + o->rotation * o->rotation / (o->r * o->r))),
              o->rotation / (o->r * o->r));
}
static double orbit_current_tilt_angle(const orbit* o) {
    dv3 p = carthesic_to_polar(dmv(&o->plane_tilt_mat, polar_to_carthesic(d3(o->r, o->orbit_angle, 0.))));
    return o->tilt_angle * cos(p.y);
}

/* Replays an orbiting observer: start_orbit(rotation) at pos, then nframes x
 * (update_position(_, dt), calc_transformation_pipeline).  Returns -1 when the
 * orbit cannot start (Orbit::new is None). */
int geo_oracle_orbit_frames(double rs, double fov, double width, double height, const double pos[3], double cam_phi,
                            double cam_theta, double rotation, uint32_t nframes, double dt, geo_frame* frames,
                            double* positions) {
    dv3 p = d3(pos[0], pos[1], pos[2]);
    orbit o;
    if (!orbit_new(rs, p, d3(-p.y, p.x, 0.), rotation, &o)) return -1;
    double psi = 1.;
    dm3 std_to_mov = dm_cols(d3(1, 0, 0), d3(0, 1, 0), d3(0, 0, 1));
    dm3 mov_to_central = std_to_mov, central_to_uv = std_to_mov;
    double t = tan(fov / 2.);
    double fov_scaling[4] = {t, t * (width / height), 1., 1.};
    for (uint32_t f = 0; f < nframes; ++f) {
        orbit_do_step(&o, 1. * dt); /* time_speedup 1 */
        p = orbit_get_position(&o);
        double r = dlen(p);
        int singular = fabs(r - rs) < 1e-10 || o.has_hit_singularity;
        if (!singular) {
            dv3 vel = orbit_get_velocity(&o);
            double hr = 1. - rs / dlen(p);
            psi = r > rs ? vel.x * vel.x * hr : -vel.y * vel.y / hr;
            if (psi - 1. < 1e-10) psi = 1.;
            dm3 l = dlook(d3(-p.x, -p.y, -p.z));
            dm3 standard_to_central = dtr(&l);
            if (o.rotation != 0.) {
                double tilt_angle = orbit_current_tilt_angle(&o);
                double plane_angle1 = acos(-vel.x * vel.y * dsignum(r - rs) /
                                           sqrt((1. + r * r * vel.z * vel.z) * psi * (psi - 1.)));
                double plane_angle2 = r > rs ? acos(-vel.y / sqrt(hr * (psi - 1.)))
                                             : acos(-vel.x * sqrt(-hr / (psi - 1.)));
                dm3 opt = drot_z(-tilt_angle), tc1 = drot_x(-plane_angle1), m2 = drot_x(plane_angle2);
                dm3 a = dmm(&tc1, &opt);
                std_to_mov = dmm(&a, &standard_to_central);
                dm3 optt = dtr(&opt);
                mov_to_central = dmm(&optt, &m2);
            } else {
                std_to_mov = standard_to_central;
                mov_to_central = dm_cols(d3(1, 0, 0), d3(0, 1, 0), d3(0, 0, 1));
            }
            dm3 lu = dlook(p), flip = dm_cols(d3(1, 0, 0), d3(0, -1, 0), d3(0, 0, 1));
            central_to_uv = dmm(&lu, &flip);
        }
        dm3 cam_to_std = dlook(d3(cos(cam_phi) * cos(cam_theta), sin(cam_phi) * cos(cam_theta), sin(cam_theta)));
        dm3 cam = dmm(&std_to_mov, &cam_to_std);
        geo_frame* out = &frames[f];
        memset(out, 0, sizeof(*out));
        const dm3* src[3] = {&cam, &mov_to_central, &central_to_uv};
        float* dst[3] = {out->display_to_movement, out->movement_to_central, out->central_to_uv};
        for (int k = 0; k < 3; ++k)
            for (int c = 0; c < 3; ++c) {
                dst[k][c * 4 + 0] = (float)src[k]->c[c].x;
                dst[k][c * 4 + 1] = (float)src[k]->c[c].y;
                dst[k][c * 4 + 2] = (float)src[k]->c[c].z;
            }
        for (int i = 0; i < 4; ++i) out->display_to_movement[12 + i] = (float)fov_scaling[i];
        out->movement_to_central[15] = 1.f;
        out->central_to_uv[15] = 1.f;
        out->psi_factor_and_position[0] = (float)sqrt((psi - 1.) / psi);
        out->psi_factor_and_position[1] = (float)p.x;
        out->psi_factor_and_position[2] = (float)p.y;
        out->psi_factor_and_position[3] = (float)p.z;
        if (positions) {
            positions[3 * f] = p.x;
            positions[3 * f + 1] = p.y;
            positions[3 * f + 2] = p.z;
        }
    }
    return 0;
}
