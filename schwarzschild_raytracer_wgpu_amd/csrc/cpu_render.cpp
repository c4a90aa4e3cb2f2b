// cpu_render.cpp — geo_render_cpu (include/geo/geo_cpu.h): the per-pixel path
// of geo_render_kernel (geo_render.hip: camera ray, aberration, geodesic,
// sky UV, bilinear sample, blend) on the host cores, from the same header
// geo_pixel.h, so its f32 sequence is the kernel's.  Built into its own
// library, libgeo_cpu.so (__graft_entry__.build), with g++ -O2
// -ffp-contract=off -mfma -msse4.1: hardware FMA where the header writes
// fmaf, no other contraction.  The CPU baseline of bench.py; never loaded by the
// package.
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/geo/geo_cpu.h"
#include "geo_pixel.h"

namespace {

struct CpuJob {
    const geo_frame* f;
    const geo_scene* s;
    geo::PixelConsts k;
    geo::CameraConsts cam;
    float kt;
    const uint32_t* sky;
    uint32_t sw, sh;
    bool opaque;
    const float* fan;
    uint32_t n_fan;
    uint32_t width, row0, nrows, row_step;
    uint32_t* rgba;
    uint8_t* mask;
    float* uv;
    uint32_t* steps;
};

float geodesic(const CpuJob& j, float st, float ct, float rct, uint32_t* n) {
    const geo::PixelConsts& k = j.k;
    if (j.s->mode == GEO_MODE_FAN) return geo::fan_lerp(j.fan, j.n_fan, st);
    if (j.s->mode == GEO_MODE_ADAPTIVE) {
        switch (geo::geodesic_kind(k)) {
            case geo::kCurvedOut: return geo::kPi2 - geo::geodesic_angle_adaptive<geo::kCurvedOut>(k, st, ct, rct, n);
            case geo::kCurvedIn: return geo::kPi2 - geo::geodesic_angle_adaptive<geo::kCurvedIn>(k, st, ct, rct, n);
            default: return geo::kPi2 - geo::geodesic_angle_adaptive<geo::kFlat>(k, st, ct, rct, n);
        }
    }
    switch (geo::geodesic_kind(k)) {
        case geo::kCurvedOut: return geo::kPi2 - geo::geodesic_angle_v<geo::kCurvedOut>(k, st, ct, rct, n);
        case geo::kCurvedIn: return geo::kPi2 - geo::geodesic_angle_v<geo::kCurvedIn>(k, st, ct, rct, n);
        default: return geo::kPi2 - geo::geodesic_angle_v<geo::kFlat>(k, st, ct, rct, n);
    }
}

// rows tid, tid + nthreads, ... of the job (interleaved: the frame's cost is
// centre-heavy); returns the thread's executed RK4 steps
unsigned long long run_rows(const CpuJob& j, unsigned tid, unsigned nthreads) {
    unsigned long long total = 0;
    const float psi_k = j.f->psi_factor_and_position[0];
    const bool composite = (j.s->flags & GEO_FLAG_COMPOSITE) != 0;
    auto fetch = [sky = j.sky](uint32_t i) { return sky[i]; };
    for (uint32_t ly = tid; ly < j.nrows; ly += nthreads) {
        const uint32_t py = j.row0 + ly * j.row_step;
        for (uint32_t px = 0; px < j.width; ++px) {
            float c2x, c2y, c2z;
            geo::pixel_central_dir(j.cam, j.f->movement_to_central, psi_k, j.kt, px, py, &c2x, &c2y, &c2z);
            const float st = geo::central_sin(c2z);
            const float ct = geo::central_rho(c2x, c2y);
            const float rct = geo::rcpf_(ct);
            uint32_t n = 0;
            const float lam = geodesic(j, st, ct, rct, &n);
            const bool bh = lam < geo::kBlackHoleLambda;
            float U = 0.0f, V = 0.0f;
            if (!bh || j.uv) geo::sky_uv(j.f->central_to_uv, c2x, c2y, ct, rct, lam, &U, &V);
            const size_t o = (size_t)ly * j.width + px;
            if (composite) {
                if (!bh) {
                    const uint32_t sm = geo::sample_sky_raw(fetch, j.sw, j.sh, U, V);
                    j.rgba[o] = j.opaque ? sm : geo::composite_(sm, j.rgba[o]);
                }
            } else {
                j.rgba[o] = bh ? geo::kBlackRGBA : geo::sample_sky(fetch, j.sw, j.sh, j.opaque, U, V);
            }
            if (j.mask) j.mask[o] = bh ? 1 : 0;
            if (j.uv) {
                j.uv[2 * o] = U;
                j.uv[2 * o + 1] = V;
            }
            if (j.steps) j.steps[o] = n;
            total += n;
        }
    }
    return total;
}

}  // namespace

extern "C" int geo_render_cpu(const geo_frame* frame, const geo_scene* scene, const uint8_t* sky_rgba8,
                              uint32_t sky_w, uint32_t sky_h, const float* fan, uint32_t n_fan, uint32_t width,
                              uint32_t height, uint32_t row0, uint32_t nrows, uint32_t row_step, int threads,
                              uint8_t* out_rgba8, uint8_t* out_mask, float* out_uv, uint32_t* out_steps,
                              unsigned long long* steps_total) {
    if (!frame || !scene || !sky_rgba8 || !out_rgba8 || sky_w == 0 || sky_h == 0 || width == 0 || height == 0 ||
        row_step == 0 || width > (1u << 20) || height > (1u << 20))
        return GEO_EINVAL;
    if (nrows == 0) {
        if (steps_total) *steps_total = 0;
        return GEO_OK;
    }
    if ((uint64_t)row0 + (uint64_t)(nrows - 1) * row_step >= height) return GEO_EINVAL;
    if (scene->mode != GEO_MODE_DIRECT && scene->mode != GEO_MODE_FAN && scene->mode != GEO_MODE_ADAPTIVE)
        return GEO_EINVAL;
    if ((scene->flags & ~(GEO_FLAG_DEFER_STEPS | GEO_FLAG_COMPOSITE)) != 0) return GEO_EINVAL;
    if (scene->mode == GEO_MODE_FAN && (!fan || n_fan < 2)) return GEO_EINVAL;
    if (scene->mode != GEO_MODE_FAN &&
        (!(scene->step > 0.0f) || !(scene->r_obs > 0.0f) || !(scene->sphere_r > 0.0f) || !(scene->rs >= 0.0f)))
        return GEO_EINVAL;
    const bool adaptive = scene->mode == GEO_MODE_ADAPTIVE;
    if (adaptive ? !(scene->tol >= 0.0f && scene->tol <= 3.0e38f) : scene->tol != 0.0f) return GEO_EINVAL;
    // the texture as u32 texels (any alignment of the caller's bytes)
    std::vector<uint32_t> sky((size_t)sky_w * sky_h);
    std::memcpy(sky.data(), sky_rgba8, sky.size() * 4u);
    bool opaque = true;
    for (size_t i = 0; i < sky.size() && opaque; ++i) opaque = (sky[i] >> 24) == 255u;
    CpuJob j;
    j.f = frame;
    j.s = scene;
    j.k = geo::make_consts(scene->rs, scene->sphere_r, scene->r_obs, scene->step, scene->max_steps, scene->tol);
    j.cam = geo::camera_consts(frame->display_to_movement, frame->movement_to_central, width, height);
    j.kt = geo::aberration_kt(frame->psi_factor_and_position[0]);
    j.sky = sky.data();
    j.sw = sky_w;
    j.sh = sky_h;
    j.opaque = opaque;
    j.fan = fan;
    j.n_fan = n_fan;
    j.width = width;
    j.row0 = row0;
    j.nrows = nrows;
    j.row_step = row_step;
    j.rgba = reinterpret_cast<uint32_t*>(out_rgba8);
    j.mask = out_mask;
    j.uv = out_uv;
    j.steps = out_steps;
    unsigned n = threads > 0 ? (unsigned)threads : std::thread::hardware_concurrency();
    if (n == 0) n = 1;
    if (n > nrows) n = nrows;
    std::vector<unsigned long long> part(n, 0);
    std::vector<std::thread> pool;
    pool.reserve(n - 1);
    for (unsigned t = 1; t < n; ++t) pool.emplace_back([&j, &part, t, n] { part[t] = run_rows(j, t, n); });
    part[0] = run_rows(j, 0, n);
    for (auto& th : pool) th.join();
    unsigned long long total = 0;
    for (unsigned long long p : part) total += p;
    if (steps_total) *steps_total = total;
    return GEO_OK;
}
