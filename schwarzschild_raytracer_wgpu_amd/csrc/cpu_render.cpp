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
#include "geo_band.h"
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
    // GEO_FLAG_MIPS: the chain's levels (geo::mip_down of level 0)
    bool mips;
    const uint32_t* lvl[geo::kSkyMipLevels];
    uint32_t lw[geo::kSkyMipLevels], lh[geo::kSkyMipLevels];
    // GEO_FLAG_RING_F64 (geo_band.h): the band's f64 constants, when it applies
    bool ring;
    geo::BandConsts band;
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

// One traced pixel of a GEO_FLAG_MIPS frame: lambda', its UV (every pixel's,
// as the kernel's lanes compute it for their quad partners) and its steps.
struct Traced {
    float lam, U, V;
    uint32_t n;
};

Traced trace(const CpuJob& j, uint32_t px, uint32_t py) {
    float c2x, c2y, c2z;
    geo::pixel_central_dir(j.cam, j.f->movement_to_central, j.f->psi_factor_and_position[0], j.kt, px, py, &c2x, &c2y,
                           &c2z);
    const float st = geo::central_sin(c2z);
    const float ct = geo::central_rho(c2x, c2y);
    const float rct = geo::rcpf_(ct);
    Traced t;
    t.n = 0;
    t.lam = geodesic(j, st, ct, rct, &t.n);
    geo::sky_uv(j.f->central_to_uv, c2x, c2y, ct, rct, t.lam, &t.U, &t.V);
    return t;
}

// The kernel's sample_trilinear (geo_render.hip) on the host chain: levels
// floor(lambda) and the next, blended with frac(lambda) in 8 bits.
uint32_t sample_trilinear(const CpuJob& j, float rho2, float U, float V) {
    const uint32_t q = geo::lod_q8(rho2);
    const uint32_t l0 = q >> 8, f = q & 255u;
    const uint32_t l1 = l0 + 1u < (uint32_t)geo::kSkyMipLevels ? l0 + 1u : l0;
    auto fetch0 = [p = j.lvl[l0]](uint32_t i) { return p[i]; };
    auto fetch1 = [p = j.lvl[l1]](uint32_t i) { return p[i]; };
    const uint32_t s0 = geo::sample_sky_raw(fetch0, j.lw[l0], j.lh[l0], U, V);
    const uint32_t s1 = geo::sample_sky_raw(fetch1, j.lw[l1], j.lh[l1], U, V);
    return geo::mip_blend(s0, s1, f);
}

// GEO_FLAG_MIPS rows: each pixel's level of detail comes from its
// frame-aligned 2 x 2 quad (partners x ^ 1 and y ^ 1, traced even where they
// lie outside the frame or the requested rows, like the kernel's helper
// lanes).  A thread takes the requested rows of every nthreads-th quad row
// pair (frame rows 2k, 2k + 1), so a pair is traced once when both of its
// rows are requested.
unsigned long long run_rows_mips(const CpuJob& j, unsigned tid, unsigned nthreads) {
    unsigned long long total = 0;
    const bool composite = (j.s->flags & GEO_FLAG_COMPOSITE) != 0;
    const uint32_t gw = j.width + (j.width & 1u);
    std::vector<Traced> rows[2] = {std::vector<Traced>(gw), std::vector<Traced>(gw)};
    int64_t have[2] = {-1, -1};  // the frame row each buffer holds
    auto row_of = [&](uint32_t py) -> const std::vector<Traced>& {
        for (int b = 0; b < 2; ++b)
            if (have[b] == (int64_t)py) return rows[b];
        const int b = have[0] == (int64_t)(py ^ 1u) ? 1 : 0;  // keep the partner row
        for (uint32_t x = 0; x < gw; ++x) rows[b][x] = trace(j, x, py);
        have[b] = py;
        return rows[b];
    };
    for (uint32_t ly = 0; ly < j.nrows; ++ly) {
        const uint32_t py = j.row0 + ly * j.row_step;
        if ((py >> 1) % nthreads != tid) continue;
        (void)row_of(py);
        const std::vector<Traced>& ry = row_of(py ^ 1u);  // never evicts row py
        const std::vector<Traced>& rr = have[0] == (int64_t)py ? rows[0] : rows[1];
        for (uint32_t px = 0; px < j.width; ++px) {
            const Traced& t = rr[px];
            const Traced& tx = rr[px ^ 1u];
            const Traced& ty = ry[px];
            const float rho2 = geo::mip_rho2(t.U - tx.U, t.V - tx.V, t.U - ty.U, t.V - ty.V, (float)j.sw, (float)j.sh);
            const bool bh = t.lam < geo::kBlackHoleLambda;
            const size_t o = (size_t)ly * j.width + px;
            if (composite) {
                if (!bh) {
                    const uint32_t sm = sample_trilinear(j, rho2, t.U, t.V);
                    j.rgba[o] = j.opaque ? sm : geo::composite_(sm, j.rgba[o]);
                }
            } else {
                j.rgba[o] = bh ? geo::kBlackRGBA : geo::over_clear(sample_trilinear(j, rho2, t.U, t.V), j.opaque);
            }
            if (j.mask) j.mask[o] = bh ? 1 : 0;
            if (j.uv) {
                j.uv[2 * o] = t.U;
                j.uv[2 * o + 1] = t.V;
            }
            if (j.steps) j.steps[o] = t.n;
            total += t.n;
        }
    }
    return total;
}

// rows tid, tid + nthreads, ... of the job (interleaved: the frame's cost is
// centre-heavy); returns the thread's executed RK4 steps
unsigned long long run_rows(const CpuJob& j, unsigned tid, unsigned nthreads) {
    if (j.mips) return run_rows_mips(j, tid, nthreads);
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
            float lam;
            bool bh;
            if (j.ring && geo::in_band(j.band.kx, ct)) {
                const double l = geo::band_lambda(j.band, px, py, &n);
                lam = (float)l;
                bh = l < (double)geo::kBlackHoleLambda;
            } else {
                lam = geodesic(j, st, ct, rct, &n);
                bh = lam < geo::kBlackHoleLambda;
            }
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
    if ((scene->flags & ~(GEO_FLAG_DEFER_STEPS | GEO_FLAG_COMPOSITE | GEO_FLAG_MIPS | GEO_FLAG_RING_F64)) != 0)
        return GEO_EINVAL;
    const bool ring_flag = (scene->flags & GEO_FLAG_RING_F64) != 0;
    if (ring_flag && (scene->mode == GEO_MODE_FAN || (scene->flags & (GEO_FLAG_COMPOSITE | GEO_FLAG_MIPS)) != 0))
        return GEO_EINVAL;
    if (scene->mode == GEO_MODE_FAN && (!fan || n_fan < 2)) return GEO_EINVAL;
    if (scene->mode != GEO_MODE_FAN &&
        (!(scene->step > 0.0f) || !(scene->r_obs > 0.0f) || !(scene->sphere_r > 0.0f) || !(scene->rs >= 0.0f)))
        return GEO_EINVAL;
    const bool adaptive = scene->mode == GEO_MODE_ADAPTIVE;
    if (adaptive ? !(scene->tol >= 0.0f && scene->tol <= 3.0e38f) : scene->tol != 0.0f) return GEO_EINVAL;
    // what geo_render_rows and geo_set_sky reject, rejected alike: the two
    // paths accept the same inputs, so "equal bit for bit" covers them all
    if (scene->max_steps > (1u << 24)) return GEO_EINVAL;  // render_impl: a wave's step sum must fit u32
    if (sky_w > (1u << 20) || sky_h > (1u << 20)) return GEO_EINVAL;
    uint64_t chain_bytes = 0;  // geo_set_sky: the padded mip chain below 2^31 bytes
    for (int l = 0; l < geo::kSkyMipLevels; ++l)
        chain_bytes += ((uint64_t)geo::mip_dim(sky_w, l) + 2u) * ((uint64_t)geo::mip_dim(sky_h, l) + 2u) * 4u;
    if (chain_bytes >= (1ull << 31)) return GEO_EINVAL;
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
    j.ring = ring_flag && scene->rs > 0.0f && scene->r_obs > scene->rs;
    if (j.ring) j.band = geo::band_consts(*frame, *scene, width, height);
    // GEO_FLAG_MIPS: the chain geo_set_sky builds (geo::mip_down, level by level)
    j.mips = (scene->flags & GEO_FLAG_MIPS) != 0;
    std::vector<uint32_t> chain[geo::kSkyMipLevels];
    for (int l = 0; l < geo::kSkyMipLevels; ++l) {
        j.lw[l] = geo::mip_dim(sky_w, l);
        j.lh[l] = geo::mip_dim(sky_h, l);
        if (l == 0) {
            j.lvl[0] = sky.data();
        } else if (j.mips) {
            chain[l].resize((size_t)j.lw[l] * j.lh[l]);
            geo::mip_down(j.lvl[l - 1], j.lw[l - 1], j.lh[l - 1], chain[l].data());
            j.lvl[l] = chain[l].data();
        } else {
            j.lvl[l] = nullptr;
        }
    }
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
