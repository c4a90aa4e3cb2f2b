/*
 * geo_oracle.h — ORACLE (test infrastructure only; never linked into, called
 * by, or shipped with libgeo.so).  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it, and only as the checker.
 *
 * PARITY UNPINNED against the reference's own outputs: the reference
 * (Rust + WGSL, wgpu 0.19) cannot be built here (no cargo/rustc; the
 * wgpu_renderer submodule is empty) and its only hot-path test,
 * sphere_geodesics_test (SR/simulation/tests.rs:8-13), asserts nothing.  The
 * oracle is pinned instead by analytic known-answer tests (flat space,
 * capture threshold, scale invariance, radial rays: tests/test_oracle_kat.py),
 * by an independent high-precision solution of the reference's initial value
 * problem and stop rules (scipy DOP853, tests/test_oracle_physics.py: within
 * 5.2e-8 rad, hit/capture identical) and by committed golden vectors of its
 * own output (tests/golden/).  The point-path oracle (geo_oracle_points.c) is
 * pinned by the reference's own RayConnector tests (tests.rs:15-79).
 *
 * Contents:
 *   f64 restatements, operation for operation, of the reference:
 *     geo_oracle_solve_geodesic_f64   sphere_ray_tracer.rs:60-193
 *     geo_oracle_solve_ray_fan_f64    sphere_ray_tracer.rs:35-56
 *     geo_oracle_pixel_f64            shader.wgsl:57-106 (direct or fan mode)
 *     geo_oracle_observer_frame       observer.rs:197-262 + polar_transformations.rs
 *   f32 restatement of the kernel's fixed evaluation order (bit-exact checker):
 *     geo_oracle_pixel_f32 / geo_oracle_render_f32 (all three modes; the
 *     adaptive RK5(4) mode is a build extension without a reference
 *     counterpart, checked in f64 against the fixed step/32 integration)
 */
#ifndef GEO_ORACLE_H
#define GEO_ORACLE_H

#include <stdint.h>

#include "../include/geo/geo.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct geo_oracle_px {
    double lam;     /* PI/2 - traveled angle (or fan lerp) */
    double u, v;    /* sky-sphere UV */
    double theta;   /* angle to the black hole (lambda after movement_to_central) */
    uint32_t steps; /* executed main-loop RK4 steps */
    int bh;         /* 1 = black hole / discard */
} geo_oracle_px;

double geo_oracle_solve_geodesic_f64(double sphere_r, double schwarz_r, uint32_t max_iter,
                                     double step, double r, double energy, double rotation,
                                     int r_falling, uint32_t* steps);
void geo_oracle_solve_ray_fan_f64(double sphere_r, double schwarz_r, uint32_t max_iter,
                                  double step, uint32_t nr_nodes, double r, float* fan_out);
/* One node of solve_ray_fan at an arbitrary theta (sphere_ray_tracer.rs:38-52),
 * returning the traveled angle. */
double geo_oracle_geodesic_at_theta_f64(double sphere_r, double schwarz_r, uint32_t max_iter,
                                        double step, double r, double theta, uint32_t* steps);

/* GEO_MODE_ADAPTIVE in the f64 pixel: fixed RK4 at step/32 with this budget */
#define GEO_ORACLE_FINE_BUDGET (1u << 22)

void geo_oracle_pixel_f64(const geo_frame* f, const geo_scene* s, const float* fan, uint32_t n_fan,
                          uint32_t width, uint32_t height, uint32_t px, uint32_t py,
                          geo_oracle_px* out);
/* rows row0, row0 + row_step, ... (nrows of them); any output may be NULL.
 * theta: the pixel's angle to the black hole (the solve_ray_fan node angle
 * it stands for). */
int geo_oracle_render_f64(const geo_frame* f, const geo_scene* s, const float* fan, uint32_t n_fan,
                          uint32_t width, uint32_t height, uint32_t row0, uint32_t nrows, uint32_t row_step,
                          int threads, uint8_t* mask, float* uv, uint32_t* steps, double* lam, double* theta);

/* f32 kernel mirror.  rgba/mask/uv/steps may be NULL (except rgba). */
int geo_oracle_render_f32(const geo_frame* f, const geo_scene* s, const float* fan, uint32_t n_fan,
                          const uint8_t* sky, uint32_t sky_w, uint32_t sky_h, uint32_t width,
                          uint32_t height, uint32_t row0, uint32_t nrows, uint32_t row_step,
                          int threads, uint8_t* rgba, uint8_t* mask, float* uv, uint32_t* steps,
                          uint64_t* steps_total);

/* GEO_FLAG_RING_F64 (geo.h): render_f32 draws the band's pixels with
 * geo_oracle_pixel_f64 (UV rounded to f32, the f32 sampler); the band is
 * |kx cos(theta) - 1| < GEO_RING_X on the f32 ray.  ring_band: that band
 * (1/0 per pixel) on rows row0 + i row_step. */
float geo_oracle_ring_kx(const geo_scene* s);
int geo_oracle_ring_band(const geo_frame* f, const geo_scene* s, uint32_t width, uint32_t height, uint32_t row0,
                         uint32_t nrows, uint32_t row_step, uint8_t* band);
int geo_oracle_ring_x(const geo_frame* f, const geo_scene* s, uint32_t width, uint32_t height, uint32_t row0,
                      uint32_t nrows, uint32_t row_step, float* x);

/* GEO_FLAG_MIPS mirror (geo_pixel.h): the 4-level box-filtered mip chain
 * (levels one after another, geo_oracle_mip_chain_texels(w, h) texels), and
 * rows [row0, row0 + nrows) (row0 even) sampled trilinearly with the level of
 * detail from each frame-aligned 2 x 2 quad's UV differences. */
uint64_t geo_oracle_mip_chain_texels(uint32_t w, uint32_t h);
void geo_oracle_mip_chain(const uint8_t* rgba8, uint32_t w, uint32_t h, uint32_t* out);
void geo_oracle_lod_q8_n(const float* rho2, uint32_t n, uint32_t* out); /* 256 lambda per footprint */
int geo_oracle_render_mips_f32(const geo_frame* f, const geo_scene* s, const float* fan, uint32_t n_fan,
                               const uint8_t* sky, uint32_t sky_w, uint32_t sky_h, uint32_t width, uint32_t height,
                               uint32_t row0, uint32_t nrows, int threads, uint8_t* rgba, uint8_t* mask, float* uv,
                               uint32_t* steps, uint64_t* steps_total);

/* Traveled angle of one ray in the f32 kernel order (direct or adaptive mode
 * by s->mode) for (sin theta, cos theta) of the central-frame direction. */
float geo_oracle_geodesic_f32(const geo_scene* s, float st, float ct, uint32_t* steps);

/* Observer::calc_transformation_pipeline for a fixed pose (observer.rs:68-87,
 * 141-160, 197-262); state = GEO_OBSERVER_UNMOVING or GEO_OBSERVER_FROZEN_FALL. */
void geo_oracle_observer_frame(double schwarz_r, double fov, double width, double height,
                               const double pos[3], double cam_phi, double cam_theta, int state,
                               double energy, geo_frame* out);

/* ---- accretion-disk points (geo_oracle_points.c) ----------------------
 * libm = 1: the C library's acosf/atanf where the reference calls
 * f32::acos/atan (reference-faithful); 0: the kernel's polynomials (the
 * bit-exact checker of the HIP path). */
/* RayConnector batch, as geo_rays_update: connectors near side first; state
 * u[c*48 + i] and needs[c] in/out; other: 3 floats or 3 per point. */
int geo_oracle_rays_update(float rs, uint32_t n_points, uint32_t sides, const float* pos, float* u, uint8_t* needs,
                           const float* other, int per_point, int iterations, int reset, float* out, int libm);
/* PointCloud::new, then nframes PointCloud::update calls (observers: 3 floats
 * for new + 3 per frame; dts per frame). */
int geo_oracle_points_run(float rs, const float* model, uint32_t n, int farside, int orbits, uint64_t seed,
                          uint32_t nframes, const float* observers, const double* dts, float* out_near,
                          float* out_far, float* out_pos, int libm);
/* Orbiting observer replay (observer.rs:104-124, 162-169, 197-262):
 * start_orbit(rotation) at pos, then nframes x (update_position(dt),
 * calc_transformation_pipeline).  -1 when no orbit can start. */
int geo_oracle_orbit_frames(double rs, double fov, double width, double height, const double pos[3], double cam_phi,
                            double cam_theta, double rotation, uint32_t nframes, double dt, geo_frame* frames,
                            double* positions);
/* vs_main + raster of one vertex / a vertex list (kernel f32 order) */
int geo_oracle_project_point(const geo_frame* f, const float* v, uint32_t width, uint32_t height, int* ix, int* iy);
int geo_oracle_draw_points(const geo_frame* f, const float* verts, uint32_t n, uint32_t width, uint32_t height,
                           uint32_t row0, uint32_t nrows, uint8_t* rgba, int* out_xy);

/* f32 math kernels, exported for accuracy tests */
float geo_oracle_acosf(float x);
float geo_oracle_asinf(float x);
float geo_oracle_atan2f(float y, float x);
void geo_oracle_sincosf(float x, float* s, float* c);
/* the per-pixel sky-direction forms (round 6; geo_math.h sincos_sky_, acos_pi_, atan2_turns_) */
void geo_oracle_sincos_sky(float x, float* s, float* c);
float geo_oracle_acos_pi(float x);
float geo_oracle_atan2_turns(float y, float x);

#ifdef __cplusplus
}
#endif

#endif
