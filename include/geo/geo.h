/*
 * geo.h — C-ABI of libgeo.so, the MI355X-native per-pixel Schwarzschild
 * geodesic renderer (drop-in for the sky-sphere hot path of
 * FirePrincess01/schwarzschild_raytracer_wgpu).
 *
 * Plain C, plain pointers and sizes: no HIP, no torch types.  A HIP stream is
 * passed as `void*` (a hipStream_t; NULL = the legacy default stream).
 *
 * Reference interfaces replaced (paths relative to the reference repo,
 * `SR/` = schwarzschild_raytracer/src/):
 *
 *   geo_frame                  TransformationPipeline            SR/simulation/observer.rs:21-28
 *                              (WGSL twin ObserverTransformations SR/schwarzschild_sphere_shader/shader.wgsl:26-33)
 *   geo_observer_*             Observer::{new, calc_transformation_pipeline,
 *                              update_screen_format, move_camera, start_*}
 *                                                                SR/simulation/observer.rs:68-296
 *   geo_set_sky                Texture::new_with_mipmaps (group 2, 4 levels)
 *                                                                SR/schwarzschild_sphere_shader/sphere_buffer/basic_sphere_buffer.rs:29-36
 *   geo_solve_ray_fan          SphereRayTracer::solve_ray_fan + BasicSphereBuffer::update_ray_fan
 *                                                                SR/simulation/sphere_ray_tracer.rs:35-56,
 *                                                                .../basic_sphere_buffer.rs:85-88
 *   geo_set_fan                RayFanTexture::update             SR/schwarzschild_sphere_shader/ray_fan_texture.rs:65-90
 *   geo_rays_* / geo_points_*  RayConnector / PointCloud      SR/simulation/ray_connector.rs:6-157,
 *                                                                SR/schwarzschild_point_shader/point_cloud.rs:7-156
 *   geo_draw_points            point pipeline vs_main + fs_main  SR/schwarzschild_point_shader/shader.wgsl:36-74
 *   geo_render_rows            SchwarzschildSphereShaderDraw::draw + fs_main
 *                                                                SR/schwarzschild_sphere_shader/schwarzschild_sphere_shader_draw.rs:3-6,
 *                                                                .../basic_sphere_buffer.rs:92-100,
 *                                                                SR/schwarzschild_sphere_shader/shader.wgsl:57-106
 *
 * Conventions: every int-returning entry point returns GEO_OK (0) or a
 * negative geo_status.  All output buffers are caller-owned.  A geo_ctx is
 * bound to one device and is not thread-safe; calls that take a stream are
 * asynchronous on it unless documented otherwise.
 */
#ifndef GEO_GEO_H
#define GEO_GEO_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GEO_ABI_VERSION 8  /* 4: geo_render_band_set_frames, geo_assemble_shares;
                                5: geo_render_band_set_batch, geo_dispatch_stats;
                                6: GEO_FLAG_RING_F64;
                                7: GEO_FLAG_RING_F64 inside the render kernel (any stream,
                                   no context memory), in GEO_MODE_ADAPTIVE too; steps_total
                                   counts the band's f64 steps;
                                8: GEO_RING_X 5e-3 (was 8e-3); GEO_FLAG_RING_F64 in batched
                                   launches (geo_render_band_set_frames / _batch) */

typedef enum geo_status {
    GEO_OK = 0,
    GEO_EINVAL = -1,  /* bad argument (null pointer, zero size, out-of-range rows) */
    GEO_EHIP = -2,    /* a HIP runtime call failed */
    GEO_ENOMEM = -3,  /* device or host allocation failed */
    GEO_ENODEV = -4,  /* no such HIP device */
    GEO_ESTATE = -5   /* call out of order (e.g. render before geo_set_sky) */
} geo_status;

/* Render modes (geo_scene.mode). */
#define GEO_MODE_DIRECT 0u /* per-pixel RK4 of the null geodesic at the pixel's own angle */
#define GEO_MODE_FAN 1u    /* reference-exact: lerp into the ray fan (shader.wgsl:77-84) */
#define GEO_MODE_ADAPTIVE 2u /* per-pixel, error-controlled Dormand-Prince RK5(4) steps (config 5;
                                a build extension, not in the reference): geo_scene.step is the
                                initial step, max_steps the budget of step ATTEMPTS, tol the
                                local error tolerance in u */

/* geo_scene.flags */
#define GEO_FLAG_DEFER_STEPS 1u /* executed steps accumulate in the context (no per-call
                                   fold); read them with geo_steps_flush.  steps_total
                                   must then be NULL. */
#define GEO_FLAG_COMPOSITE 2u   /* draw OVER the current contents of out_rgba8 with the
                                   reference's alpha blending (BlendState::ALPHA_BLENDING,
                                   pipeline.rs:49) and leave discarded (black-hole / no-hit)
                                   pixels untouched: the 2nd, 3rd... sphere of a frame
                                   (lib.rs:67-89).  Without it a sphere is drawn over the
                                   cleared target (0,0,0,1). */
#define GEO_FLAG_MIPS 4u        /* (parity unpinned: the reference's mip generator and sampler
                                   are in its absent wgpu_renderer submodule; this is the
                                   repo's own specification of them)
                                   sample the sky through its 4-level mip chain, trilinear,
                                   with the level of detail from the UV differences across
                                   each 2x2 pixel quad, as textureSample does
                                   (basic_sphere_buffer.rs:31-36, shader.wgsl:101; the
                                   level-0 bilinear sample otherwise).  Quads are frame-
                                   aligned, so row0 must be even (GEO_EINVAL otherwise);
                                   band layouts keep bands 8-row aligned. */
#define GEO_FLAG_RING_F64 8u    /* (off on the benchmarked path) GEO_MODE_DIRECT or
                                   GEO_MODE_ADAPTIVE: the pixels next to the capture orbit,
                                   |b/b_c - 1| < GEO_RING_X by the f32 ray (b = r_obs
                                   cos(theta) / sqrt(1 - rs/r_obs), b_c = 3 sqrt(3) rs / 2;
                                   rs > 0, r_obs > rs), take their traveled angle from an
                                   f64 path inside the render kernel: the camera ray, the
                                   reference's set-up and fixed-step RK4 loop at
                                   geo_scene.step (with its exits, step count and Newton,
                                   sphere_ray_tracer.rs:38-191) in f64; the mask is decided
                                   in f64, the sky drawn from the f32 ray with lambda'
                                   rounded to f32 (geo_band.h).  There the orbit amplifies
                                   the f32 roundings (and, in the adaptive mode, its
                                   tolerance) past the 1e-4 UV bar.  The
                                   band's out_steps and steps_total are its f64 steps.  A
                                   one-frame ring render launches one wave per workgroup; a
                                   batch (geo_render_band_set_frames / _batch) carries each
                                   frame's band factor and derives its constants on the
                                   device; no state is kept in the context.  Not with
                                   GEO_MODE_FAN, GEO_FLAG_COMPOSITE or GEO_FLAG_MIPS
                                   (GEO_EINVAL). */
#define GEO_RING_X 5e-3f  /* (8e-3 before ABI 8; tools/ring_width_margin.py) */

/* Observer motion states, ObserverState (SR/simulation/observer.rs:12-16). */
#define GEO_OBSERVER_UNMOVING 0
#define GEO_OBSERVER_FROZEN_FALL 1
#define GEO_OBSERVER_ORBITING 2

/* GEO_MODE_ADAPTIVE step control (geo_pixel.h, geodesic_angle_adaptive). */
#define GEO_ADAPTIVE_DEFAULT_TOL 1e-6f
#define GEO_ADAPTIVE_MAX_GROWTH 16u /* largest step = 16 x geo_scene.step */

/* Sentinel for a ray that never reaches the sphere, SphereRayTracer::NO_VALUE
 * (sphere_ray_tracer.rs:22).  Fan / traveled-angle space. */
#define GEO_NO_VALUE 15.0

/* Byte-for-byte TransformationPipeline (observer.rs:21-28): three column-major
 * 4x4 f32 matrices and [sqrt((psi-1)/psi), x, y, z].  208 bytes. */
typedef struct geo_frame {
    float display_to_movement[16]; /* camera rotation; column 3 = FOV scale (observer.rs:253-254) */
    float movement_to_central[16];
    float central_to_uv[16];
    float psi_factor_and_position[4];
} geo_frame;

/* Per-draw scene constants.  The reference fixes these per sphere
 * (basic_sphere_buffer.rs:42-51, lib.rs:72, renderer.rs:83). */
typedef struct geo_scene {
    float rs;           /* Schwarzschild radius */
    float sphere_r;     /* radius of the textured sky sphere */
    float r_obs;        /* observer radial position |pos| (lib.rs:292) */
    float step;         /* RK4 step in traveled angle (PI/100 in the reference);
                           GEO_MODE_ADAPTIVE: the initial step */
    uint32_t max_steps; /* RK4 budget per ray (1000 in the reference), <= 2^24;
                           GEO_MODE_ADAPTIVE: budget of step attempts */
    uint32_t mode;      /* GEO_MODE_* */
    uint32_t flags;     /* GEO_FLAG_* */
    float tol;          /* GEO_MODE_ADAPTIVE: local error tolerance in u (0 = 1e-6);
                           must be 0 in the other modes */
} geo_scene;

typedef struct geo_ctx geo_ctx;
typedef struct geo_observer geo_observer;

/* ---- library ---------------------------------------------------------- */
/* Every call that launches device work first clears the calling thread's HIP
 * last-error state (hipGetLastError), so that an earlier, unrelated failure
 * of the caller is not reported as the call's: a caller that checks its own
 * launches with hipGetLastError must do so before calling into libgeo. */
int geo_abi_version(void);
const char* geo_status_str(int status);

/* ---- device context --------------------------------------------------- */
/* Creates a context on HIP device `device`.  Fails with GEO_ENODEV when the
 * device does not exist (there is no CPU fallback). */
int geo_ctx_create(int device, geo_ctx** out);
void geo_ctx_destroy(geo_ctx* ctx);

/* Uploads an equirect RGBA8 sky (row-major, w*h*4 bytes, host memory; the
 * bytes are copied, synchronously, after this context's renders in flight on
 * any stream have finished, so no frame samples a half-written sky; other
 * contexts' work and collectives are not waited for).  On failure the
 * context has no sky (renders return GEO_ESTATE).  U wraps, V clamps,
 * bilinear with 8-bit sub-texel weights: level 0, or with GEO_FLAG_MIPS the
 * 4-level mip chain built here (box filter; Texture::new_with_mipmaps(..., 4),
 * basic_sphere_buffer.rs:31-36).  The device keeps every level padded by one
 * texel on every side, which must stay below 2^31 bytes in all:
 * sum over l < 4 of (max(1, w >> l) + 2) * (max(1, h >> l) + 2) * 4 < 2^31,
 * w, h <= 2^20 (GEO_EINVAL otherwise). */
int geo_set_sky(geo_ctx* ctx, const uint8_t* rgba8, uint32_t w, uint32_t h);

/* Uploads a ray fan of n >= 2 nodes (host memory, copied synchronously after
 * the last solve and draws of the buffer it goes to; geo_solve_ray_fan
 * replaces it stream-ordered):
 * node i is PI/2 - traveled angle of the ray at theta_i = PI/2 - PI*i/(n-1). */
int geo_set_fan(geo_ctx* ctx, const float* fan, uint32_t n);

/* Computes the ray fan on the GPU in f64 (SphereRayTracer::solve_ray_fan,
 * sphere_ray_tracer.rs:35-193) for nr_nodes nodes at observer radius r and
 * makes it the context's fan: fan-mode renders issued after this call read
 * it.  Asynchronous on `stream`; the context keeps two fan buffers and
 * orders them itself, so the stream need not be the renders' stream: the
 * solve waits for the renders that read the buffer it overwrites (issued
 * before the previous solve), and a render waits for the solve of the fan it
 * reads.  A fan solved on a side stream thus overlaps the previous frame's
 * draws.  When fan_out (host) is non-NULL the call synchronises `stream` and
 * copies the nr_nodes f32 values there. */
int geo_solve_ray_fan(geo_ctx* ctx, double sphere_r, double schwarz_r, uint32_t max_iter,
                      double step, uint32_t nr_nodes, double r, float* fan_out, void* stream);

/* Renders rows [row0, row0+nrows) of a width x height frame (fs_main,
 * shader.wgsl:57-106, composited onto the clear colour (0,0,0,1) with the
 * reference's alpha blend, pipeline.rs:49 / renderer.rs:233-238).
 * Outputs are DEVICE pointers laid out row-major relative to row0:
 *   out_rgba8    nrows*width*4 bytes (required)
 *   out_mask     nrows*width bytes, 1 = black hole / discard (optional)
 *   out_uv       nrows*width*2 floats, sky-sphere (U,V) (optional)
 *   out_steps    nrows*width u32, executed RK4 main-loop steps (optional)
 *   steps_total  one u64 that the executed steps of this call are ADDED to (optional;
 *                exactly this call's steps, also while other renders of the context
 *                run on other streams: the call counts into a counter set of its own,
 *                reused only after that set's previous fold)
 * Asynchronous on `stream`. */
int geo_render_rows(geo_ctx* ctx, const geo_frame* frame, const geo_scene* scene,
                    uint32_t width, uint32_t height, uint32_t row0, uint32_t nrows,
                    uint8_t* out_rgba8, uint8_t* out_mask, float* out_uv,
                    uint32_t* out_steps, unsigned long long* steps_total, void* stream);

/* Renders an interleaved set of row bands (balanced multi-GPU sharding): bands
 * band0, band0+band_step, ..., nbands of them, each band_rows tall (a
 * power of two >= 8, the pixel rows of one wave); band b
 * covers rows [b*band_rows, (b+1)*band_rows) clipped to height.  Outputs are
 * packed band after band (nbands*band_rows rows; clipped rows are not
 * written).  geo_render_rows(row0, nrows) is the single-band case. */
int geo_render_bands(geo_ctx* ctx, const geo_frame* frame, const geo_scene* scene,
                     uint32_t width, uint32_t height, uint32_t band_rows, uint32_t band0,
                     uint32_t band_step, uint32_t nbands, uint8_t* out_rgba8, uint8_t* out_mask,
                     float* out_uv, uint32_t* out_steps, unsigned long long* steps_total,
                     void* stream);

/* Rank 0's reassembly after gathering every rank's geo_render_bands output
 * (multi-GPU present): `src` (device) holds `world` rank blocks
 * of rank_stride bytes, rank r's block being its packed bands (bands r,
 * r+world, r+2*world, ... of band_rows rows) for nframes frames at
 * frame_stride bytes apart, src_bpp bytes per pixel (4: RGBA8 as rendered,
 * 3: RGB24 from geo_pack_rgb, width % 4 == 0).  Writes nframes width x height
 * RGBA8 frames back to back to `dst` (device).  Asynchronous on `stream`. */
int geo_assemble_bands(geo_ctx* ctx, const uint8_t* src, size_t rank_stride, size_t frame_stride, uint32_t world,
                       uint32_t band_rows, uint32_t width, uint32_t height, uint32_t nframes, uint32_t src_bpp,
                       uint8_t* dst, void* stream);

/* The general strided band set: bands starting at rows row0, row0+row_stride,
 * ..., nbands of them, each band_rows tall (a multiple of 8; at most 4096
 * unless a power of two) and clipped
 * to height; row_stride >= band_rows.  Outputs packed band after band as in
 * geo_render_bands (which is the case row0 = band0*band_rows,
 * row_stride = band_step*band_rows).  Used for the lead layout below, where
 * rank 0 renders taller bands than its peers. */
int geo_render_band_set(geo_ctx* ctx, const geo_frame* frame, const geo_scene* scene,
                        uint32_t width, uint32_t height, uint32_t band_rows, uint32_t row0,
                        uint32_t row_stride, uint32_t nbands, uint8_t* out_rgba8, uint8_t* out_mask,
                        float* out_uv, uint32_t* out_steps, unsigned long long* steps_total,
                        void* stream);

/* A batch of nframes (1 .. GEO_MAX_BATCH_FRAMES) frames of one scene in ONE
 * launch: frame f's uniform is frames[f], its packed bands (the layout of
 * geo_render_band_set) go to out_rgba8 + f*out_frame_stride bytes
 * (out_frame_stride a multiple of 4, at least the packed bands' bytes).  The
 * frames share the scene (observer radius, step, budget, mode): frames of an
 * observer at one radius (a camera pan, or the same pose drawn again); a
 * moving observer's frames go through geo_render_band_set_batch below.  Fan
 * mode reads the context's current fan for every frame.
 * Colour only (no mask, UV or per-pixel steps; no GEO_FLAG_MIPS); the
 * executed steps of all frames go to steps_total or, with
 * GEO_FLAG_DEFER_STEPS, to the context's accumulator.  One launch pays the
 * dispatch, ramp and drain of a render once for the whole batch: a rank's
 * share of a 4K frame at N = 8 (about two waves per slot) draws 10-12 %
 * faster per frame.  Asynchronous on `stream`. */
#define GEO_MAX_BATCH_FRAMES 8
int geo_render_band_set_frames(geo_ctx* ctx, const geo_frame* frames, uint32_t nframes, const geo_scene* scene,
                               uint32_t width, uint32_t height, uint32_t band_rows, uint32_t row0,
                               uint32_t row_stride, uint32_t nbands, uint8_t* out_rgba8, size_t out_frame_stride,
                               unsigned long long* steps_total, void* stream);

/* geo_render_band_set_frames with a scene per frame (scenes[f] for frames[f]):
 * a moving observer's frames, whose radius r_obs changes every frame, in one
 * launch.  The scenes may differ in r_obs only (every other field equal, the
 * same integration kind: all outside or all inside the horizon; a fan-mode
 * batch draws one fan, so r_obs must agree too), else GEO_EINVAL. */
int geo_render_band_set_batch(geo_ctx* ctx, const geo_frame* frames, const geo_scene* scenes, uint32_t nframes,
                              uint32_t width, uint32_t height, uint32_t band_rows, uint32_t row0,
                              uint32_t row_stride, uint32_t nbands, uint8_t* out_rgba8, size_t out_frame_stride,
                              unsigned long long* steps_total, void* stream);

/* Rank 0's reassembly for the LEAD layout (multi-GPU present with rank 0
 * taking a larger share: it renders but never sends its rows, while the peers'
 * rows cross the xGMI links).  The frame is cut into cycles of
 * (lead + world - 1) * band_rows rows: the first lead*band_rows rows of each
 * cycle are rank 0's (one band of that height), then one band_rows band per
 * peer r = 1..world-1 in order.  lead = 1 is geo_assemble_bands' layout.
 *   lead_src  rank 0's packed RGBA8 bands (geo_render_band_set output), nframes
 *             frames lead_frame_stride bytes apart
 *   src       the gathered peer blocks: rank r's packed bands at
 *             src + r*rank_stride + f*frame_stride, src_bpp bytes per pixel
 *             (4 or 3 = RGB24 from geo_pack_rgb); block 0 is not read
 * Writes nframes RGBA8 frames back to back to dst.  width % 4 == 0 and
 * 16-byte aligned device buffers (4-byte for src with src_bpp 3).
 * Asynchronous on `stream`. */
int geo_assemble_lead(geo_ctx* ctx, const uint8_t* lead_src, size_t lead_frame_stride, uint32_t lead,
                      const uint8_t* src, size_t rank_stride, size_t frame_stride, uint32_t world,
                      uint32_t band_rows, uint32_t width, uint32_t height, uint32_t nframes, uint32_t src_bpp,
                      uint8_t* dst, void* stream);

/* geo_assemble_lead with rank 0's rows per cycle given directly: cycles of
 * lead_rows + (world - 1) * band_rows rows, rank 0's first (one lead_rows
 * band), then one band_rows band per peer.  Any lead_rows, so rank 0's share
 * need not be a whole number of peer bands (e.g. 24 rows against peers' 16:
 * bench.py --rank0-lead 3:2).  geo_assemble_lead(lead) is
 * geo_assemble_shares(lead * band_rows).  Same buffers and alignment rules. */
int geo_assemble_shares(geo_ctx* ctx, const uint8_t* lead_src, size_t lead_frame_stride, uint32_t lead_rows,
                        const uint8_t* src, size_t rank_stride, size_t frame_stride, uint32_t world,
                        uint32_t band_rows, uint32_t width, uint32_t height, uint32_t nframes, uint32_t src_bpp,
                        uint8_t* dst, void* stream);

/* RGBA8 -> RGB24 (the alpha byte dropped: frames are opaque after the clear,
 * renderer.rs:233-238) of npixels (a multiple of 4) device pixels: 25 % fewer
 * bytes on the links for the multi-GPU present.  Asynchronous on `stream`. */
int geo_pack_rgb(geo_ctx* ctx, const uint8_t* rgba, uint64_t npixels, uint8_t* rgb, void* stream);

/* The workgroup dispatch order of this context's renders.
 * A frame's tiles differ ~30x in cost (steps per pixel peak at the photon
 * ring), and the hardware dispatches workgroups in launch order, so a long
 * tile dispatched late stretches the kernel's tail.
 *   GEO_DISPATCH_LONGEST_FIRST (the default): every period-th render of a grid
 *     (period 1: every render; 16: renders 1, 17, 33, ...)
 *     (same width, height, rows, bands, mode and sampler) records each 32 x 8
 *     tile's cost on the device, and two small kernels after it build the
 *     order, most expensive tile first, for the renders that follow; the
 *     first render of a new grid records and uses row-major order.  Nothing
 *     is read back to the host.
 *   GEO_DISPATCH_ROW_MAJOR: the launch order.
 * Fan-mode renders (uniform cost) and frames of more than 65 535 tile rows
 * always use row-major order.  The output is the same in any order.
 * period: 1 .. 2^20 (default 16). */
#define GEO_DISPATCH_ROW_MAJOR 0
#define GEO_DISPATCH_LONGEST_FIRST 1
#define GEO_DISPATCH_EXPLICIT 2 /* set by geo_set_tile_order */
int geo_set_dispatch(geo_ctx* ctx, int mode, uint32_t period);

/* GEO_DISPATCH_LONGEST_FIRST's counters since the context was created: the
 * renders that recorded tile costs, and the rebuilt orders renders have
 * adopted.  A rebuild runs on the context's own stream after every render
 * issued before it; renders adopt its order once the host sees it complete
 * (an event query, never a wait), so a recording render due while the last
 * rebuild is still running is deferred to the next render.  Either pointer
 * may be NULL. */
int geo_dispatch_stats(geo_ctx* ctx, unsigned long long* costs_recorded, unsigned long long* orders_adopted);

/* Times the next render of this context (geo_render_rows/bands/band_set, on
 * any stream): its kernel dispatch carries start_event and stop_event
 * (hipEvent_t created with timing), so hipEventElapsedTime gives the
 * kernel's own execution time, as a profiler's dispatch timestamps do, with
 * no marker packets around it.  (A frame of more than 65 535 tile rows: from
 * the first launch's start to the last one's end.)  Consumed by the next
 * render call whether it succeeds or not: a refused call (GEO_EINVAL,
 * GEO_ESTATE, ...) records neither event and drops the pair. */
int geo_time_next_render(geo_ctx* ctx, void* start_event, void* stop_event);

/* An explicit dispatch order (GEO_DISPATCH_EXPLICIT): workgroup i draws tile
 * (order[i] & 0xFFFF, order[i] >> 16) of a tiles_x x tiles_y grid of
 * 32 x 8-pixel tiles over the rendered rows; order (host) must be a
 * permutation of the grid's tiles.  Renders whose grid is exactly
 * tiles_x x tiles_y use it, others row-major order.  order = NULL selects
 * GEO_DISPATCH_ROW_MAJOR.  Waits for the context's renders in flight. */
int geo_set_tile_order(geo_ctx* ctx, uint32_t tiles_x, uint32_t tiles_y, const uint32_t* order);

/* Adds the steps accumulated under GEO_FLAG_DEFER_STEPS to *steps_total
 * (device u64) and clears the context's counter.  Asynchronous on `stream`. */
int geo_steps_flush(geo_ctx* ctx, unsigned long long* steps_total, void* stream);

/* ---- accretion-disk points ------------------------- */
/* A batch of RayConnectors (SR/simulation/ray_connector.rs:6-25) on n points:
 * per point a near-side connector (less_than_180 = true) and/or a far-side one
 * (false).  Connector order: the n near-side ones, then the n far-side ones.
 * State (48 node values per connector, needs_reset) stays on the device. */
#define GEO_RAYS_NEAR 1u
#define GEO_RAYS_FAR 2u
typedef struct geo_rays geo_rays;
typedef struct geo_points geo_points;

/* RayConnector::new for every (point, side); pos_xyz: host, 3 floats per point. */
int geo_rays_create(geo_ctx* ctx, float schwarz_r, uint32_t n_points, uint32_t sides, const float* pos_xyz,
                    geo_rays** out);
void geo_rays_destroy(geo_rays* rays);
/* number of connectors */
int geo_rays_count(const geo_rays* rays);
/* RayConnector::set_position (:134-136) for every point (host, 3 floats per
 * point).  Synchronous: waits for the batch's last update first. */
int geo_rays_set_positions(geo_rays* rays, const float* pos_xyz);
/* update_ray(other, iterations) (ray_connector.rs:48-132) for every connector,
 * or reset_ray(other) (:27-44) when reset != 0.  other_xyz (host): 3 floats
 * (one other end for all) or 3 per point when per_point != 0 (then the call
 * synchronises `stream` after uploading them).  out_vertices: device, 4 floats
 * per connector [x, y, z, incoming angle], or NULL for the batch's own buffer
 * (geo_rays_vertices).  Asynchronous on `stream`; it waits for the batch's
 * previous update, whichever stream that ran on.  Readers of the vertices
 * (geo_draw_points) are the caller's to order: an update overwrites them. */
int geo_rays_update(geo_rays* rays, const float* other_xyz, int per_point, uint32_t iterations, int reset,
                    float* out_vertices, void* stream);
const float* geo_rays_vertices(const geo_rays* rays);

/* PointCloud::new (SR/schwarzschild_point_shader/point_cloud.rs:20-65): one
 * near-side RayConnector per model vertex (host, 3 floats each), plus a
 * far-side one when farside != 0, all reset against observer_xyz; with
 * orbits != 0 every vertex also becomes a particle on an Orbit (f64,
 * orbit.rs) with direction (-y, x, 0) and rotation 18 + 2 rand.  seed: the
 * per-point random streams (wyrand) for those rotations and for respawns.
 * Synchronous. */
int geo_points_create(geo_ctx* ctx, float schwarz_r, const float* model_xyz, uint32_t n,
                      const float* observer_xyz, int farside, int orbits, unsigned long long seed,
                      geo_points** out);
void geo_points_destroy(geo_points* pts);
int geo_points_count(const geo_points* pts);
/* PointCloud::update (point_cloud.rs:117-148): orbit step by dt seconds and
 * respawn (orbits), then update_ray(observer, 1) for every connector, in
 * one kernel launch (two, orbit step then rays, from 131072 connectors on).
 * Asynchronous on `stream`; it waits for the cloud's
 * previous update and for every geo_points_draw before it, whichever streams
 * they ran on. */
int geo_points_update(geo_points* pts, const float* observer_xyz, double dt, void* stream);
/* get_vertices / get_vertices_farside: device pointer, 4 floats per point
 * (NULL for the far side of a cloud without one). */
const float* geo_points_vertices(const geo_points* pts, int farside);
/* current point positions (host, 3 floats per point); `stream` waits for the
 * last update, then the call synchronises it. */
int geo_points_positions(const geo_points* pts, float* out_xyz, void* stream);

/* The point pipeline (SR/schwarzschild_point_shader/shader.wgsl:36-74,
 * pipeline.rs:55-74: PointList, colour (1,0,0,1), REPLACE) drawn over rows
 * [row0, row0+nrows) of an RGBA8 frame (device, laid out as geo_render_rows'
 * out_rgba8).  vertices: device, 4 floats each.  out_xy (device, optional):
 * the pixel (x, y) of every vertex, (-1, -1) when clipped.  Async on `stream`. */
int geo_draw_points(geo_ctx* ctx, const geo_frame* frame, const float* vertices, uint32_t n, uint32_t width,
                    uint32_t height, uint32_t row0, uint32_t nrows, uint8_t* out_rgba8, int* out_xy,
                    void* stream);

/* The point meshes of a PointCloud (the near-side vertices, then the
 * far-side ones; lib.rs:415-418, renderer.rs:256-264) drawn as by
 * geo_draw_points, both in one launch (every point writes the same colour,
 * so their order cannot show).  out_xy (device, optional): 2 ints per
 * connector, near side first.  Stream order: the draw waits for the cloud's last
 * geo_points_update and the next update waits for this draw and every draw
 * before it (events owned by the cloud), whichever streams they run on, so a caller may put the update
 * on a side stream where it overlaps the sphere draws.  Async on `stream`. */
int geo_points_draw(geo_points* pts, const geo_frame* frame, uint32_t width, uint32_t height, uint32_t row0,
                    uint32_t nrows, uint8_t* out_rgba8, int* out_xy, void* stream);

/* ---- observer (host, f64; SR/simulation/observer.rs) ----------------- */
/* Observer::new (observer.rs:68-87): pos (25,0,1), camera (PI,0), FrozenFall,
 * energy 1, fov scale (tan(fov/2), tan(fov/2)*w/h, 1, 1). */
int geo_observer_create(double schwarz_r, double fov, double width, double height,
                        geo_observer** out);
void geo_observer_destroy(geo_observer* obs);
int geo_observer_set_position(geo_observer* obs, double x, double y, double z);
int geo_observer_get_position(const geo_observer* obs, double* xyz3);
int geo_observer_set_camera(geo_observer* obs, double phi, double theta);
int geo_observer_set_energy(geo_observer* obs, double energy);
/* GEO_OBSERVER_UNMOVING / GEO_OBSERVER_FROZEN_FALL (start_unmoving / start_frozen_fall,
 * observer.rs:173-181). */
int geo_observer_set_state(geo_observer* obs, int state);
/* Observer::start_orbit (observer.rs:162-169); returns GEO_ESTATE when no orbit
 * can start there (inside the horizon, orbit.rs:33-35). */
int geo_observer_start_orbit(geo_observer* obs, double rotation);
int geo_observer_get_state(const geo_observer* obs);
double geo_observer_radial_position(const geo_observer* obs);
/* Observer::update_position (observer.rs:105-125); dir = (forward, left, up). */
int geo_observer_update_position(geo_observer* obs, double fwd, double left, double up, double dt);
int geo_observer_move_camera(geo_observer* obs, double dx_pixels, double dy_pixels);
int geo_observer_update_screen_format(geo_observer* obs, double width, double height);
int geo_observer_is_singular(const geo_observer* obs);
/* Observer::calc_transformation_pipeline (observer.rs:197-262). */
int geo_observer_calc_transformation_pipeline(geo_observer* obs, geo_frame* out);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* GEO_GEO_H */
