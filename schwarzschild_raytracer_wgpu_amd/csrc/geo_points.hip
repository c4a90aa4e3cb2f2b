// geo_points.hip — the accretion-disk point path on gfx950.
//
//   geo_rays_kernel     RayConnector::{reset_ray, update_ray} for a batch of
//                       connectors, one lane each (SR/simulation/ray_connector.rs:27-132);
//                       <kOrbitsFused>: the whole PointCloud::update with orbits in
//                       one launch: each connector's lane steps its point's f64
//                       orbit (Orbit::do_step + the respawn of fallen particles),
//                       then its respawn reset and its update_ray (small clouds);
//                       <kOrbitsStepped>: the same after geo_orbits_kernel (large ones)
//                       (SR/schwarzschild_point_shader/point_cloud.rs:117-148, orbit.rs:84-167)
//   geo_orbits_kernel   the orbit half alone, one lane per point
//   geo_draw_kernel     the point pipeline: vs_main + PointList raster of the
//                       red fs_main colour, REPLACE blend (shader.wgsl:36-74, pipeline.rs:55-74)
//
// Layout (HBM): node values in 64-connector tiles of node quads,
// u[(c/64)*48*64 + (node/4)*256 + (c%64)*4 + node%4] (48 x 4 B per connector;
// a lane moves them with 12 16-B loads, a wave's 12 loads one contiguous 12-KB
// block), point positions x[n] y[n] z[n], one needs_reset byte per connector,
// vertices float4 per connector (near-side connectors first, then far-side:
// get_vertices / get_vertices_farside), orbit states and generators twice
// (read one copy, write the other).  The 48-node state, the Thomas factors
// and residuals live in VGPRs for the whole call (no LDS, no scratch).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/geo/geo.h"
#include "geo_ctx.h"
#include "geo_orbit.h"
#include "geo_rays.h"

namespace {

// one wave per block: +2 % over 256 (tools/gpu_ab.sh).  Node values in
// 64-connector tiles of node quads (16-B loads and stores): +4.5 % over
// single-node tiles, which were +4.5 % over node-major SoA.
constexpr int kRaysBlock = 64;
// geo_rays_kernel's modes: plain RayConnector calls, or PointCloud::update
// with orbits stepped in the ray lanes (fused) or by geo_orbits_kernel first
enum RaysMode { kPlain = 0, kOrbitsFused = 1, kOrbitsStepped = 2 };
// From this many connectors on (two waves per SIMD of the chip), the fused
// update's doubled orbit work (a point's near and far lanes both step it)
// costs more than the launch it saves: 2 M points with orbits 0.49 -> 0.54 ms
// fused (profiles/r04u_disk_fused/points_bench_ab.txt), 5000 points 3 -> 1
// launches and the reference's frame -12 to -16 %.
constexpr uint32_t kFusedMaxConnectors = 1024u * 64u * 2u;

// fastrand 2.0.1's generator (wyrand) and its f64 mapping, restated: one
// independent stream per point (the reference draws from one OS-seeded stream
// in point order, which no parallel or repeated run can reproduce).
__host__ __device__ inline uint64_t mulhi64_(uint64_t a, uint64_t b) {
    const uint64_t a0 = a & 0xffffffffu, a1 = a >> 32, b0 = b & 0xffffffffu, b1 = b >> 32;
    const uint64_t p00 = a0 * b0, p01 = a0 * b1, p10 = a1 * b0, p11 = a1 * b1;
    const uint64_t mid = (p00 >> 32) + (p01 & 0xffffffffu) + (p10 & 0xffffffffu);
    return p11 + (p01 >> 32) + (p10 >> 32) + (mid >> 32);
}
__host__ __device__ inline uint64_t wyrand_u64(uint64_t* s) {
    const uint64_t x = *s + 0xA0761D6478BD642Full;
    *s = x;
    const uint64_t y = x ^ 0xE7037ED1A0B428DBull;
    return (x * y) ^ mulhi64_(x, y);
}
__host__ __device__ inline double wyrand_f64(uint64_t* s) {
    const uint64_t bits = (1ull << 62) - (1ull << 52) + (wyrand_u64(s) >> 12);  // [1, 2)
    double d;
    std::memcpy(&d, &bits, 8);
    return d - 1.0;
}
__host__ __device__ inline uint64_t point_stream_seed(uint64_t seed, uint32_t i) {
    return seed ^ (0x9E3779B97F4A7C15ull * ((uint64_t)i + 1u));
}

// A new particle of new_accretion_disk / the respawn (point_cloud.rs:90-96, 124-128):
// r in [16, 26), phi in [0, 2pi), theta in [-0.1, 0.1); rotation 18 + 2 rand.
__host__ __device__ inline bool spawn_orbit(double rs, uint64_t* s, geo64::Orbit* o) {
    const double r = 16. + 10. * wyrand_f64(s);
    const double phi = wyrand_f64(s) * 6.283185307179586;
    const double theta = 0.2 * (wyrand_f64(s) - 0.5);
    const geo64::V3 pos = geo64::polar_to_carthesic(geo64::v3(r, phi, theta));
    return geo64::Orbit::make(rs, pos, geo64::v3(-pos.y, pos.x, 0.), 18. + 2. * wyrand_f64(s), o);
}

struct RaysArgs {
    uint32_t n_points, n_conn, sides, iterations, reset;
    float rs;
    float ox, oy, oz;            // the other end, when `other` is null
    const float* other;          // per-point other ends (x,y,z interleaved) or null
    float* pos;                  // SoA x[n] y[n] z[n] (ORBITS: written, the stepped positions)
    float* u;                    // [48][n_conn]
    uint8_t* needs_reset;        // [n_conn]
    float4* out;                 // [n_conn]
    // kOrbitsFused: the orbit state in and out (two buffers, swapped per
    // update: both connectors of a point step it from the same input)
    double dt;
    const geo64::Orbit* orb_in;
    geo64::Orbit* orb_out;
    const uint64_t* rng_in;
    uint64_t* rng_out;
    // kOrbitsStepped: geo_orbits_kernel's output (the stepped positions in
    // pos, per point whether it respawned and where)
    const uint8_t* step_respawn;
    const float* step_respawn_pos;
};

// Node-value stream: read once and written once per call, with non-temporal
// hints (+5.5 %, tools/gpu_ab.sh, bench_points).
typedef float f4_ __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4_ ld4_(const float* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const f4_*>(p));
}
__device__ __forceinline__ void st4_(float* p, f4_ v) {
    __builtin_nontemporal_store(v, reinterpret_cast<f4_*>(p));
}

// One RayConnector call per connector (update_ray / reset_ray).
// ORBITS: PointCloud::update with orbits (point_cloud.rs:117-148) in one
// launch.  The lane first steps its point's orbit (f64, Orbit::do_step) and
// respawns a particle that hit the singularity or fell inside rs; the near
// side's lane stores the orbit, its generator and the position.  A respawned
// point's connector then runs reset_ray at the NEW position (:129-134), whose
// nodes feed this frame's update_ray at the PRE-respawn position: the
// reference sets the new position, resets the rays, then sets orbit_pos --
// computed before the respawn -- again (:129-140).  Both calls run in the
// lane's VGPRs (the first writes the nodes the second loads); before round 4
// they were three launches (orbits, respawn resets, updates) whose boundaries
// were most of a 5000-point update's latency.
template <int MODE>
__global__ __launch_bounds__(kRaysBlock) void geo_rays_kernel(const RaysArgs a) {
    const uint32_t c = blockIdx.x * kRaysBlock + threadIdx.x;
    if (c >= a.n_conn) return;
    // connector c: point c mod n, near side (less_than_180) first
    const bool far = a.sides == GEO_RAYS_FAR ? true : c >= a.n_points;
    const uint32_t p = c >= a.n_points ? c - a.n_points : c;
    const uint32_t n = a.n_points;
    bool needs = a.needs_reset[c] != 0;
    float ox = a.ox, oy = a.oy, oz = a.oz;
    if (a.other) {
        ox = a.other[3 * (size_t)p];
        oy = a.other[3 * (size_t)p + 1];
        oz = a.other[3 * (size_t)p + 2];
    }
    float px, py, pz;
    bool respawned = false;
    float qx = 0.f, qy = 0.f, qz = 0.f;  // the respawn position
    if (MODE == kOrbitsFused) {
        geo64::Orbit o = a.orb_in[p];
        o.do_step(a.dt);
        const geo64::V3 op = o.get_position();
        px = (float)op.x;
        py = (float)op.y;
        pz = (float)op.z;
        uint64_t rng = a.rng_in[p];
        if (o.is_singular() || geo::dot3_(px, py, pz, px, py, pz) <= a.rs * a.rs) {
            (void)spawn_orbit((double)a.rs, &rng, &o);  // r >= 16 > rs (checked at create): never None
            const geo64::V3 np = o.get_position();
            qx = (float)np.x;
            qy = (float)np.y;
            qz = (float)np.z;
            respawned = true;
        }
        if (c < n) {  // the point's first connector stores its state
            a.orb_out[p] = o;
            a.rng_out[p] = rng;
            a.pos[p] = px;
            a.pos[n + p] = py;
            a.pos[2 * n + p] = pz;
        }
    } else {
        px = a.pos[p];
        py = a.pos[n + p];
        pz = a.pos[2 * n + p];
        if (MODE == kOrbitsStepped && a.step_respawn[p]) {
            qx = a.step_respawn_pos[p];
            qy = a.step_respawn_pos[n + p];
            qz = a.step_respawn_pos[2 * n + p];
            respawned = true;
        }
    }
    const bool reset = a.reset != 0;
    // node quads in 64-connector tiles, u[(c/64)*48*64 + (i/4)*256 + (c%64)*4 + i%4]: a lane moves
    // its 48 nodes with 12 16-B loads and stores, a wave's quad q is one contiguous 1-KB block.
    // Without a reset pending, ray_connect reads every node (the jump test reads node 0 first),
    // so they are loaded up front; with one, none is read.
    float* const ug = a.u + (size_t)(c / 64u) * (geo::kRayNodes * 64u) + (c % 64u) * 4u;
    float u[geo::kRayNodes], v[geo::kRayNodes];
    if (MODE != kPlain && respawned) {
        // reset_ray at the new position (reads no node): its nodes are v
        (void)geo::ray_connect(a.rs, !far, qx, qy, qz, ox, oy, oz, true, a.iterations, &needs,
                               [&](int i) { return v[i]; }, v);
    } else if (!reset && !needs) {
#pragma unroll
        for (int q = 0; q < geo::kRayNodes / 4; ++q) {
            const f4_ t = ld4_(ug + q * 256);
            v[4 * q] = t.x;
            v[4 * q + 1] = t.y;
            v[4 * q + 2] = t.z;
            v[4 * q + 3] = t.w;
        }
    }
    const float angle = geo::ray_connect(a.rs, !far, px, py, pz, ox, oy, oz, reset, a.iterations, &needs,
                                         [&](int i) { return v[i]; }, u);
#pragma unroll
    for (int q = 0; q < geo::kRayNodes / 4; ++q)
        st4_(ug + q * 256, f4_{u[4 * q], u[4 * q + 1], u[4 * q + 2], u[4 * q + 3]});
    a.needs_reset[c] = needs ? 1 : 0;
    if (a.out) a.out[c] = make_float4(px, py, pz, angle);
}

// PointCloud::update, orbit half (point_cloud.rs:119-141), for large clouds
// (kOrbitsStepped): step, then respawn a particle that hit the singularity or
// fell inside rs.  pos gets the PRE-respawn position (this frame's
// update_ray), respawn_pos the new one (the respawn's reset_ray).
__global__ __launch_bounds__(kRaysBlock) void geo_orbits_kernel(uint32_t n, double dt, float rs,
                                                                const geo64::Orbit* orb_in, geo64::Orbit* orb_out,
                                                                const uint64_t* rng_in, uint64_t* rng_out, float* pos,
                                                                uint8_t* respawn, float* respawn_pos) {
    const uint32_t i = blockIdx.x * kRaysBlock + threadIdx.x;
    if (i >= n) return;
    geo64::Orbit o = orb_in[i];
    o.do_step(dt);
    const geo64::V3 op = o.get_position();
    const float x = (float)op.x, y = (float)op.y, z = (float)op.z;
    uint64_t s = rng_in[i];
    uint8_t rsp = 0;
    if (o.is_singular() || geo::dot3_(x, y, z, x, y, z) <= rs * rs) {
        (void)spawn_orbit((double)rs, &s, &o);  // r >= 16 > rs (checked at create): never None
        const geo64::V3 np = o.get_position();
        respawn_pos[i] = (float)np.x;
        respawn_pos[n + i] = (float)np.y;
        respawn_pos[2 * n + i] = (float)np.z;
        rsp = 1;
    }
    orb_out[i] = o;
    rng_out[i] = s;
    respawn[i] = rsp;
    pos[i] = x;
    pos[n + i] = y;
    pos[2 * n + i] = z;
}

struct DrawArgs {
    geo_frame frame;
    const float4* verts;
    uint32_t n, width, height, row0, nrows;
    uint32_t* out_rgba;
    int2* out_xy;
};

__global__ __launch_bounds__(kRaysBlock) void geo_draw_kernel(const DrawArgs a) {
    const uint32_t i = blockIdx.x * kRaysBlock + threadIdx.x;
    if (i >= a.n) return;
    const float4 v = a.verts[i];
    uint32_t ix = 0, iy = 0;
    const bool vis = geo::project_point(a.frame.display_to_movement, a.frame.movement_to_central,
                                        a.frame.central_to_uv, a.frame.psi_factor_and_position[0], v.x, v.y, v.z,
                                        v.w, a.width, a.height, &ix, &iy);
    if (a.out_xy) a.out_xy[i] = vis ? make_int2((int)ix, (int)iy) : make_int2(-1, -1);
    if (vis && iy >= a.row0 && iy - a.row0 < a.nrows) a.out_rgba[(size_t)(iy - a.row0) * a.width + ix] = geo::kPointRGBA;
}

template <typename T>
int dmalloc(T** p, size_t count) {
    return hipMalloc(reinterpret_cast<void**>(p), sizeof(T) * (count ? count : 1)) == hipSuccess ? GEO_OK
                                                                                               : GEO_ENOMEM;
}

}  // namespace

struct geo_rays {
    int device;
    float rs;
    uint32_t n_points, sides, n_conn;
    float* pos = nullptr;          // SoA [3][n_points]
    float* u = nullptr;            // [48][n_conn]
    uint8_t* needs_reset = nullptr;
    float* other = nullptr;        // per-point staging [n_points][3]
    float4* verts = nullptr;       // [n_conn]
    // orbits (geo_points only): two copies of the state, [2][n_points];
    // the update reads copy orb_cur and writes the other
    geo64::Orbit* orbits = nullptr;
    uint64_t* rng = nullptr;
    uint32_t orb_cur = 0;
    uint8_t* step_respawn = nullptr;  // kOrbitsStepped: [n_points], and positions [3][n_points]
    float* step_respawn_pos = nullptr;
    // geo_rays handles: the last geo_rays_update (whatever its stream).  The
    // next update waits for it (it reads and writes the same state), and
    // geo_rays_set_positions waits for it before overwriting the positions.
    hipEvent_t updated = nullptr;
    bool updated_rec = false;
};

struct geo_points {
    geo_rays rays;
    bool has_orbits;
    // Cross-stream order of the update and the draw (geo_points_draw): the
    // draw waits for the last update, the next update for the last update
    // and every draw before it, so a caller may run the update on a side
    // stream, overlapping the VALU-bound sphere draw with this latency-bound
    // work.  `drawn` is a chain: each draw records it only after waiting for
    // the previous draw's `drawn` (behind its own launches, so the draws
    // themselves still overlap), so it completes after every draw so far,
    // on whatever streams they ran.
    hipEvent_t updated = nullptr, drawn = nullptr;
    bool updated_rec = false, drawn_rec = false;
};

namespace {

void rays_free(geo_rays* r) {
    for (void* p : {(void*)r->pos, (void*)r->u, (void*)r->needs_reset, (void*)r->other, (void*)r->verts,
                    (void*)r->orbits, (void*)r->rng, (void*)r->step_respawn, (void*)r->step_respawn_pos})
        if (p) (void)hipFree(p);
}

int rays_init(geo_rays* r, geo_ctx* ctx, float rs, uint32_t n_points, uint32_t sides, const float* pos_xyz) {
    r->device = ctx->device;
    r->rs = rs;
    r->n_points = n_points;
    r->sides = sides;
    r->n_conn = n_points * ((sides & GEO_RAYS_NEAR ? 1u : 0u) + (sides & GEO_RAYS_FAR ? 1u : 0u));
    int st;
    if ((st = dmalloc(&r->pos, 3 * (size_t)n_points)) || (st = dmalloc(&r->u, (size_t)geo::kRayNodes * ((r->n_conn + 63u) / 64u * 64u))) ||
        (st = dmalloc(&r->needs_reset, r->n_conn)) || (st = dmalloc(&r->other, 3 * (size_t)n_points)) ||
        (st = dmalloc(&r->verts, r->n_conn)))
        return st;
    // RayConnector::new (:16-25): u_ray = 1, needs_reset
    std::vector<float> ones((size_t)geo::kRayNodes * ((r->n_conn + 63u) / 64u * 64u), 1.0f);
    if (hipMemcpy(r->u, ones.data(), ones.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemset(r->needs_reset, 1, r->n_conn) != hipSuccess ||
        hipMemset(r->verts, 0, sizeof(float4) * r->n_conn) != hipSuccess)
        return GEO_EHIP;
    std::vector<float> soa(3 * (size_t)n_points);
    for (uint32_t i = 0; i < n_points; ++i)
        for (int k = 0; k < 3; ++k) soa[(size_t)k * n_points + i] = pos_xyz[3 * (size_t)i + k];
    if (hipMemcpy(r->pos, soa.data(), soa.size() * sizeof(float), hipMemcpyHostToDevice) != hipSuccess)
        return GEO_EHIP;
    return GEO_OK;
}

// ORBITS (dt >= 0): PointCloud::update with orbits, one launch (geo_rays_kernel<true>)
int rays_launch(geo_rays* r, float ox, float oy, float oz, const float* other_dev, uint32_t iterations, int reset,
                double dt, float* out, hipStream_t s) {
    RaysArgs a;
    a.n_points = r->n_points;
    a.n_conn = r->n_conn;
    a.sides = r->sides;
    a.iterations = iterations;
    a.reset = reset ? 1u : 0u;
    a.rs = r->rs;
    a.ox = ox;
    a.oy = oy;
    a.oz = oz;
    a.other = other_dev;
    a.pos = r->pos;
    a.u = r->u;
    a.needs_reset = r->needs_reset;
    a.out = out ? reinterpret_cast<float4*>(out) : r->verts;
    const bool orbits = dt >= 0.0;
    a.dt = orbits ? dt : 0.0;
    const size_t n = r->n_points;
    a.orb_in = orbits ? r->orbits + r->orb_cur * n : nullptr;
    a.orb_out = orbits ? r->orbits + (1u - r->orb_cur) * n : nullptr;
    a.rng_in = orbits ? r->rng + r->orb_cur * n : nullptr;
    a.rng_out = orbits ? r->rng + (1u - r->orb_cur) * n : nullptr;
    a.step_respawn = r->step_respawn;
    a.step_respawn_pos = r->step_respawn_pos;
    if (r->n_conn == 0) return GEO_OK;
    const dim3 grid((r->n_conn + kRaysBlock - 1) / kRaysBlock);
    if (!orbits) {
        hipLaunchKernelGGL(geo_rays_kernel<kPlain>, grid, dim3(kRaysBlock), 0, s, a);
    } else if (r->n_conn < kFusedMaxConnectors) {
        hipLaunchKernelGGL(geo_rays_kernel<kOrbitsFused>, grid, dim3(kRaysBlock), 0, s, a);
    } else {
        hipLaunchKernelGGL(geo_orbits_kernel, dim3((r->n_points + kRaysBlock - 1) / kRaysBlock), dim3(kRaysBlock), 0,
                           s, r->n_points, dt, r->rs, a.orb_in, a.orb_out, a.rng_in, a.rng_out, r->pos,
                           r->step_respawn, r->step_respawn_pos);
        if (hipGetLastError() != hipSuccess) return GEO_EHIP;
        hipLaunchKernelGGL(geo_rays_kernel<kOrbitsStepped>, grid, dim3(kRaysBlock), 0, s, a);
    }
    if (hipGetLastError() != hipSuccess) return GEO_EHIP;
    if (orbits) r->orb_cur ^= 1u;
    return GEO_OK;
}

bool finite3(const float* v) {
    return v && __builtin_isfinite(v[0]) && __builtin_isfinite(v[1]) && __builtin_isfinite(v[2]);
}

}  // namespace

extern "C" {

int geo_rays_create(geo_ctx* ctx, float schwarz_r, uint32_t n_points, uint32_t sides, const float* pos_xyz,
                    geo_rays** out) {
    if (!out) return GEO_EINVAL;
    *out = nullptr;
    if (!ctx || !pos_xyz || n_points == 0 || n_points > (1u << 26) || (sides & ~3u) || !sides ||
        !(schwarz_r >= 0.0f))
        return GEO_EINVAL;
    DeviceGuard g(ctx->device);
    if (!g.ok) return GEO_EHIP;
    geo_rays* r = new (std::nothrow) geo_rays();
    if (!r) return GEO_ENOMEM;
    int st = rays_init(r, ctx, schwarz_r, n_points, sides, pos_xyz);
    if (!st && hipEventCreateWithFlags(&r->updated, hipEventDisableTiming) != hipSuccess) {
        r->updated = nullptr;
        st = GEO_EHIP;
    }
    if (st) {
        rays_free(r);
        delete r;
        return st;
    }
    *out = r;
    return GEO_OK;
}

void geo_rays_destroy(geo_rays* r) {
    if (!r) return;
    DeviceGuard g(r->device);
    if (r->updated) {
        (void)hipEventSynchronize(r->updated);  // an update in flight still uses the buffers
        (void)hipEventDestroy(r->updated);
    }
    rays_free(r);
    delete r;
}

int geo_rays_count(const geo_rays* r) { return r ? (int)r->n_conn : GEO_EINVAL; }

int geo_rays_set_positions(geo_rays* r, const float* pos_xyz) {
    if (!r || !pos_xyz) return GEO_EINVAL;
    DeviceGuard g(r->device);
    if (!g.ok) return GEO_EHIP;
    // the blocking copy below is not ordered against an update still running
    // on a caller's non-blocking stream, which reads the positions
    if (r->updated_rec && hipEventSynchronize(r->updated) != hipSuccess) return GEO_EHIP;
    std::vector<float> soa(3 * (size_t)r->n_points);
    for (uint32_t i = 0; i < r->n_points; ++i)
        for (int k = 0; k < 3; ++k) soa[(size_t)k * r->n_points + i] = pos_xyz[3 * (size_t)i + k];
    return hipMemcpy(r->pos, soa.data(), soa.size() * sizeof(float), hipMemcpyHostToDevice) == hipSuccess ? GEO_OK
                                                                                                      : GEO_EHIP;
}

int geo_rays_update(geo_rays* r, const float* other_xyz, int per_point, uint32_t iterations, int reset,
                    float* out_vertices, void* stream) {
    if (!r || !other_xyz || iterations > 1024) return GEO_EINVAL;
    DeviceGuard g(r->device);
    if (!g.ok) return GEO_EHIP;
    hipStream_t s = (hipStream_t)stream;
    // after the previous update (its state, and the per-point staging buffer)
    if (r->updated_rec && hipStreamWaitEvent(s, r->updated, 0) != hipSuccess) return GEO_EHIP;
    int st;
    if (per_point) {
        if (hipMemcpyAsync(r->other, other_xyz, sizeof(float) * 3 * r->n_points, hipMemcpyHostToDevice, s) !=
                hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return GEO_EHIP;
        st = rays_launch(r, 0.f, 0.f, 0.f, r->other, iterations, reset, -1.0, out_vertices, s);
    } else {
        st = rays_launch(r, other_xyz[0], other_xyz[1], other_xyz[2], nullptr, iterations, reset, -1.0,
                         out_vertices, s);
    }
    if (st) return st;
    if (hipEventRecord(r->updated, s) != hipSuccess) return GEO_EHIP;
    r->updated_rec = true;
    return GEO_OK;
}

const float* geo_rays_vertices(const geo_rays* r) { return r ? reinterpret_cast<const float*>(r->verts) : nullptr; }

int geo_points_create(geo_ctx* ctx, float schwarz_r, const float* model_xyz, uint32_t n, const float* observer_xyz,
                      int farside, int orbits, unsigned long long seed, geo_points** out) {
    if (!out) return GEO_EINVAL;
    *out = nullptr;
    if (!ctx || !model_xyz || !finite3(observer_xyz) || n == 0 || n > (1u << 26) || !(schwarz_r >= 0.0f))
        return GEO_EINVAL;
    if (orbits && !(schwarz_r < 16.0f)) return GEO_EINVAL;  // respawns start at r >= 16 (point_cloud.rs:124)
    DeviceGuard g(ctx->device);
    if (!g.ok) return GEO_EHIP;
    geo_points* p = new (std::nothrow) geo_points();
    if (!p) return GEO_ENOMEM;
    p->has_orbits = orbits != 0;
    geo_rays* r = &p->rays;
    int st = rays_init(r, ctx, schwarz_r, n, farside ? (GEO_RAYS_NEAR | GEO_RAYS_FAR) : GEO_RAYS_NEAR, model_xyz);
    if (!st && p->has_orbits) {
        // Orbit::new per vertex, direction (-y, x, 0), rotation 18 + 2 rand (point_cloud.rs:48-51), on the host
        std::vector<geo64::Orbit> orb(n);
        std::vector<uint64_t> rng(n);
        for (uint32_t i = 0; i < n && !st; ++i) {
            uint64_t s = point_stream_seed(seed, i);
            const geo64::V3 pos = geo64::v3(model_xyz[3 * (size_t)i], model_xyz[3 * (size_t)i + 1],
                                            model_xyz[3 * (size_t)i + 2]);
            if (!geo64::Orbit::make(schwarz_r, pos, geo64::v3(-pos.y, pos.x, 0.), 18. + 2. * wyrand_f64(&s), &orb[i]))
                st = GEO_EINVAL;  // the reference unwraps: a vertex inside the horizon panics
            rng[i] = s;
        }
        if (!st && ((st = dmalloc(&r->orbits, 2 * (size_t)n)) || (st = dmalloc(&r->rng, 2 * (size_t)n)) ||
                    (st = dmalloc(&r->step_respawn, n)) || (st = dmalloc(&r->step_respawn_pos, 3 * (size_t)n))))
            st = GEO_ENOMEM;
        if (!st && (hipMemcpy(r->orbits, orb.data(), sizeof(geo64::Orbit) * n, hipMemcpyHostToDevice) != hipSuccess ||
                    hipMemcpy(r->rng, rng.data(), sizeof(uint64_t) * n, hipMemcpyHostToDevice) != hipSuccess))
            st = GEO_EHIP;
    }
    if (!st && (hipEventCreateWithFlags(&p->updated, hipEventDisableTiming) != hipSuccess ||
                hipEventCreateWithFlags(&p->drawn, hipEventDisableTiming) != hipSuccess))
        st = GEO_EHIP;
    // reset_ray(observer_pos) for every connector (:43, :46)
    if (!st) st = rays_launch(r, observer_xyz[0], observer_xyz[1], observer_xyz[2], nullptr, 0u, 1, -1.0, nullptr, 0);
    if (!st && hipStreamSynchronize(nullptr) != hipSuccess) st = GEO_EHIP;  // the reset above, not the device
    if (st) {
        for (hipEvent_t e : {p->updated, p->drawn})
            if (e) (void)hipEventDestroy(e);
        rays_free(r);
        delete p;
        return st;
    }
    *out = p;
    return GEO_OK;
}

void geo_points_destroy(geo_points* p) {
    if (!p) return;
    DeviceGuard g(p->rays.device);
    for (hipEvent_t e : {p->updated, p->drawn})
        if (e) (void)hipEventDestroy(e);
    rays_free(&p->rays);
    delete p;
}

int geo_points_count(const geo_points* p) { return p ? (int)p->rays.n_points : GEO_EINVAL; }

int geo_points_update(geo_points* p, const float* observer_xyz, double dt, void* stream) {
    if (!p || !finite3(observer_xyz) || !(dt >= 0.0)) return GEO_EINVAL;
    geo_rays* r = &p->rays;
    DeviceGuard g(r->device);
    if (!g.ok) return GEO_EHIP;
    hipStream_t s = (hipStream_t)stream;
    // every draw so far read the vertices (the chained `drawn`); the last
    // update, on whatever stream, wrote the state this one reads
    if (p->drawn_rec && hipStreamWaitEvent(s, p->drawn, 0) != hipSuccess) return GEO_EHIP;
    if (p->updated_rec && hipStreamWaitEvent(s, p->updated, 0) != hipSuccess) return GEO_EHIP;
    // (with orbits: the orbit step and respawns, fused) update_ray(observer_pos, 1) (:143-146)
    const int st = rays_launch(r, observer_xyz[0], observer_xyz[1], observer_xyz[2], nullptr, 1u, 0,
                               p->has_orbits ? dt : -1.0, nullptr, s);
    if (st) return st;
    if (hipEventRecord(p->updated, s) != hipSuccess) return GEO_EHIP;
    p->updated_rec = true;
    return GEO_OK;
}

const float* geo_points_vertices(const geo_points* p, int farside) {
    if (!p) return nullptr;
    const geo_rays* r = &p->rays;
    if (farside && !(r->sides & GEO_RAYS_FAR)) return nullptr;
    return reinterpret_cast<const float*>(r->verts + (farside ? r->n_points : 0));
}

int geo_points_positions(const geo_points* p, float* out_xyz, void* stream) {
    if (!p || !out_xyz) return GEO_EINVAL;
    const geo_rays* r = &p->rays;
    DeviceGuard g(r->device);
    if (!g.ok) return GEO_EHIP;
    std::vector<float> soa(3 * (size_t)r->n_points);
    hipStream_t s = (hipStream_t)stream;
    if (p->updated_rec && hipStreamWaitEvent(s, p->updated, 0) != hipSuccess) return GEO_EHIP;
    if (hipMemcpyAsync(soa.data(), r->pos, soa.size() * sizeof(float), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return GEO_EHIP;
    for (uint32_t i = 0; i < r->n_points; ++i)
        for (int k = 0; k < 3; ++k) out_xyz[3 * (size_t)i + k] = soa[(size_t)k * r->n_points + i];
    return GEO_OK;
}

}  // extern "C"

namespace {
int draw_launch(const geo_frame* frame, const float* vertices, uint32_t n, uint32_t width, uint32_t height,
                uint32_t row0, uint32_t nrows, uint8_t* out_rgba8, int* out_xy, hipStream_t stream) {
    DrawArgs a;
    std::memcpy(&a.frame, frame, sizeof(geo_frame));
    a.verts = reinterpret_cast<const float4*>(vertices);
    a.n = n;
    a.width = width;
    a.height = height;
    a.row0 = row0;
    a.nrows = nrows;
    a.out_rgba = reinterpret_cast<uint32_t*>(out_rgba8);
    a.out_xy = reinterpret_cast<int2*>(out_xy);
    hipLaunchKernelGGL(geo_draw_kernel, dim3((n + kRaysBlock - 1) / kRaysBlock), dim3(kRaysBlock), 0, stream, a);
    return hipGetLastError() == hipSuccess ? GEO_OK : GEO_EHIP;
}

bool draw_args_ok(const geo_frame* frame, uint32_t width, uint32_t height, uint32_t row0, uint32_t nrows,
                  const uint8_t* out_rgba8) {
    return frame && out_rgba8 && width && height && nrows && row0 < height && nrows <= height - row0;
}
}  // namespace

extern "C" {

int geo_draw_points(geo_ctx* ctx, const geo_frame* frame, const float* vertices, uint32_t n, uint32_t width,
                    uint32_t height, uint32_t row0, uint32_t nrows, uint8_t* out_rgba8, int* out_xy, void* stream) {
    if (!ctx || (!vertices && n) || !draw_args_ok(frame, width, height, row0, nrows, out_rgba8)) return GEO_EINVAL;
    if (n == 0) return GEO_OK;
    DeviceGuard g(ctx->device);
    if (!g.ok) return GEO_EHIP;
    return draw_launch(frame, vertices, n, width, height, row0, nrows, out_rgba8, out_xy, (hipStream_t)stream);
}

int geo_points_draw(geo_points* p, const geo_frame* frame, uint32_t width, uint32_t height, uint32_t row0,
                    uint32_t nrows, uint8_t* out_rgba8, int* out_xy, void* stream) {
    if (!p || !draw_args_ok(frame, width, height, row0, nrows, out_rgba8)) return GEO_EINVAL;
    const geo_rays* r = &p->rays;
    DeviceGuard g(r->device);
    if (!g.ok) return GEO_EHIP;
    hipStream_t s = (hipStream_t)stream;
    if (p->updated_rec && hipStreamWaitEvent(s, p->updated, 0) != hipSuccess) return GEO_EHIP;
    // the near-side mesh, then the far-side one (lib.rs:415-418, renderer.rs:256-264),
    // in ONE launch over both: every point writes the same colour with REPLACE
    // blending, so the order of the two meshes cannot show, and the far side's
    // vertices (and xy slots) follow the near side's
    const int sides = (r->sides & GEO_RAYS_FAR) ? 2 : 1;
    const int st = draw_launch(frame, reinterpret_cast<const float*>(r->verts), (uint32_t)sides * r->n_points, width,
                               height, row0, nrows, out_rgba8, out_xy, s);
    if (st) return st;
    if (p->drawn_rec && hipStreamWaitEvent(s, p->drawn, 0) != hipSuccess) return GEO_EHIP;  // chain the draws
    if (hipEventRecord(p->drawn, s) != hipSuccess) return GEO_EHIP;
    p->drawn_rec = true;
    return GEO_OK;
}

}  // extern "C"
