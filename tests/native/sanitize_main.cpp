// Sanitizer run of the product's host-compilable code (race
// detection / sanitizers): the per-pixel header (geo_pixel.h), the point-path
// header (geo_rays.h) and the observer (observer.cpp, geo_orbit.h), built
// with -fsanitize=address,undefined and checked against the oracle (linked
// in) on small frames.  Exit status 0 = clean and bit-identical.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../include/geo/geo.h"
#include "../../oracle/geo_oracle.h"
#include "../../schwarzschild_raytracer_wgpu_amd/csrc/geo_pixel.h"
#include "../../schwarzschild_raytracer_wgpu_amd/csrc/geo_rays.h"

static float angle_for(const geo::PixelConsts& k, uint32_t mode, float st, float ct, uint32_t* n) {
    const float rct = geo::rcpf_(ct);
    switch (geo::geodesic_kind(k)) {
        case geo::kCurvedOut:
            return mode == GEO_MODE_ADAPTIVE ? geo::geodesic_angle_adaptive<geo::kCurvedOut>(k, st, ct, rct, n)
                                             : geo::geodesic_angle_v<geo::kCurvedOut>(k, st, ct, rct, n);
        case geo::kCurvedIn:
            return mode == GEO_MODE_ADAPTIVE ? geo::geodesic_angle_adaptive<geo::kCurvedIn>(k, st, ct, rct, n)
                                             : geo::geodesic_angle_v<geo::kCurvedIn>(k, st, ct, rct, n);
        default:
            return mode == GEO_MODE_ADAPTIVE ? geo::geodesic_angle_adaptive<geo::kFlat>(k, st, ct, rct, n)
                                             : geo::geodesic_angle_v<geo::kFlat>(k, st, ct, rct, n);
    }
}

static int render_check(double px_, double py_, double pz_, float rs, uint32_t mode, uint32_t max_steps) {
    const uint32_t W = 48, H = 27;
    geo_observer* o = nullptr;
    if (geo_observer_create(rs, M_PI / 2, W, H, &o) != GEO_OK) return 1;
    geo_observer_set_position(o, px_, py_, pz_);
    geo_observer_set_camera(o, M_PI + 0.2, 0.1);
    geo_frame f;
    geo_observer_calc_transformation_pipeline(o, &f);
    const float r = (float)geo_observer_radial_position(o);
    geo_observer_destroy(o);
    geo_scene s = {rs, 50.0f, r, (float)(M_PI / 100), max_steps, mode, 0u, 0.0f};
    std::vector<uint8_t> sky(16 * 8 * 4);
    for (size_t i = 0; i < sky.size(); ++i) sky[i] = (uint8_t)(i * 37u + 11u);
    std::vector<uint8_t> rgba(W * H * 4), mask(W * H);
    std::vector<float> uv(W * H * 2);
    std::vector<uint32_t> steps(W * H);
    uint64_t total = 0;
    if (geo_oracle_render_f32(&f, &s, nullptr, 0, sky.data(), 16, 8, W, H, 0, H, 1, 1, rgba.data(), mask.data(),
                              uv.data(), steps.data(), &total) != 0)
        return 1;
    const geo::PixelConsts k = geo::make_consts(s.rs, s.sphere_r, s.r_obs, s.step, s.max_steps, s.tol);
    const uint32_t* skyp = reinterpret_cast<const uint32_t*>(sky.data());
    int bad = 0;
    const geo::CameraConsts cam = geo::camera_consts(f.display_to_movement, f.movement_to_central, W, H);
    for (uint32_t py = 0; py < H; ++py)
        for (uint32_t px = 0; px < W; ++px) {
            float c2x, c2y, c2z;
            geo::pixel_central_dir(cam, f.movement_to_central, f.psi_factor_and_position[0],
                                   geo::aberration_kt(f.psi_factor_and_position[0]), px, py, &c2x, &c2y, &c2z);
            const float st = geo::central_sin(c2z), ct = geo::central_rho(c2x, c2y);
            uint32_t n = 0;
            const float lam = geo::kPi2 - angle_for(k, mode, st, ct, &n);
            float U, V;
            geo::sky_uv(f.central_to_uv, c2x, c2y, ct, geo::rcpf_(ct), lam, &U, &V);
            const bool bh = lam < geo::kBlackHoleLambda;
            const uint32_t c = bh ? geo::kBlackRGBA
                                  : geo::sample_sky([skyp](uint32_t i) { return skyp[i]; }, 16, 8, false, U, V);
            const size_t o = (size_t)py * W + px;
            uint32_t ref;
            std::memcpy(&ref, &rgba[4 * o], 4);
            bad += (c != ref) || (n != steps[o]) || (bh != (mask[o] != 0));
        }
    if (bad) std::printf("render mismatch: %d pixels (r=%.2f mode=%u)\n", bad, (double)r, mode);
    return bad != 0;
}

static int rays_check() {
    const uint32_t n = 40;
    std::vector<float> pos(3 * n), u(2 * n * 48, 1.0f), uo(2 * n * 48, 1.0f), out(8 * n);
    std::vector<uint8_t> needs(2 * n, 1), needso(2 * n, 1);
    for (uint32_t i = 0; i < n; ++i) {
        const double a = 0.37 * i;
        pos[3 * i] = (float)(18 * std::cos(a));
        pos[3 * i + 1] = (float)(18 * std::sin(a));
        pos[3 * i + 2] = 0.3f;
    }
    int bad = 0;
    for (int frame = 0; frame < 6; ++frame) {
        const float obs[3] = {(float)(20 - 3 * frame), (float)(2 * frame), 0.5f};
        geo_oracle_rays_update(1.0f, n, 3u, pos.data(), uo.data(), needso.data(), obs, 0, 1, frame == 0, out.data(), 0);
        for (uint32_t c = 0; c < 2 * n; ++c) {
            const uint32_t p = c % n;
            float nu[48];
            bool nd = needs[c] != 0;
            float* uc = &u[(size_t)c * 48];
            const float ang = geo::ray_connect(1.0f, c < n, pos[3 * p], pos[3 * p + 1], pos[3 * p + 2], obs[0], obs[1],
                                               obs[2], frame == 0, 1u, &nd, [uc](int i) { return uc[i]; }, nu);
            std::memcpy(uc, nu, sizeof(nu));
            needs[c] = nd ? 1 : 0;
            bad += std::memcmp(&ang, &out[4 * c + 3], 4) != 0;
        }
    }
    if (bad) std::printf("ray connector mismatch: %d\n", bad);
    return bad != 0;
}

int main() {
    int fails = 0;
    fails += render_check(2.5, 0.0, 0.1, 1.0f, GEO_MODE_DIRECT, 2048);
    fails += render_check(2.5, 0.0, 0.1, 1.0f, GEO_MODE_ADAPTIVE, 2048);
    fails += render_check(1.2, 0.5, 0.0, 1.0f, GEO_MODE_DIRECT, 300);
    fails += render_check(0.8, 0.0, 0.05, 1.0f, GEO_MODE_ADAPTIVE, 300);
    fails += render_check(2.5, 0.0, 0.1, 0.0f, GEO_MODE_DIRECT, 512);
    fails += rays_check();
    std::printf(fails ? "FAIL\n" : "sanitized host paths: clean and bit-identical\n");
    return fails ? 1 : 0;
}
