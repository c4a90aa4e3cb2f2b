// Host build of the PRODUCT's per-pixel header (geo_pixel.h) for CPU tests:
// checks, without a GPU, that the kernel's exact f32 operation sequence
// equals the oracle's independent restatement bit for bit.  Test-only.
#include <cstdint>
#include <cstring>

#include "../../include/geo/geo.h"
#include "../../schwarzschild_raytracer_wgpu_amd/csrc/geo_pixel.h"

template <int LOOP>
static float geo_v(const geo::PixelConsts& k, float st, float ct, float rct, uint32_t* n) {
    switch (geo::geodesic_kind(k)) {
        case geo::kCurvedOut: return geo::geodesic_angle_v<geo::kCurvedOut, LOOP>(k, st, ct, rct, n);
        case geo::kCurvedIn: return geo::geodesic_angle_v<geo::kCurvedIn, LOOP>(k, st, ct, rct, n);
        default: return geo::geodesic_angle_v<geo::kFlat, LOOP>(k, st, ct, rct, n);
    }
}

static float geo_adaptive(const geo::PixelConsts& k, float st, float ct, float rct, uint32_t* n) {
    switch (geo::geodesic_kind(k)) {
        case geo::kCurvedOut: return geo::geodesic_angle_adaptive<geo::kCurvedOut>(k, st, ct, rct, n);
        case geo::kCurvedIn: return geo::geodesic_angle_adaptive<geo::kCurvedIn>(k, st, ct, rct, n);
        default: return geo::geodesic_angle_adaptive<geo::kFlat>(k, st, ct, rct, n);
    }
}

extern "C" int host_render(const geo_frame* f, const geo_scene* s, const float* fan, uint32_t n_fan,
                           const uint32_t* sky, uint32_t sw, uint32_t sh, uint32_t width, uint32_t height,
                           uint32_t row0, uint32_t nrows, uint32_t* rgba, uint8_t* mask, float* uv,
                           uint32_t* steps, int variant) {
    const geo::PixelConsts k = geo::make_consts(s->rs, s->sphere_r, s->r_obs, s->step, s->max_steps, s->tol);
    bool opaque = true;
    for (size_t i = 0; i < (size_t)sw * sh; ++i) opaque = opaque && (sky[i] >> 24) == 255u;
    const geo::CameraConsts cam = geo::camera_consts(f->display_to_movement, f->movement_to_central, width, height);
    for (uint32_t ly = 0; ly < nrows; ++ly) {
        const uint32_t py = row0 + ly;
        for (uint32_t px = 0; px < width; ++px) {
            float c2x, c2y, c2z;
            geo::pixel_central_dir(cam, f->movement_to_central, f->psi_factor_and_position[0],
                                   geo::aberration_kt(f->psi_factor_and_position[0]), px, py, &c2x, &c2y, &c2z);
            const float st = geo::central_sin(c2z);
            const float ct = geo::central_rho(c2x, c2y);
            const float rct = geo::rcpf_(ct);
            uint32_t n = 0;
            float lam;
            if (s->mode == GEO_MODE_FAN)
                lam = geo::fan_lerp(fan, n_fan, st);
            else if (s->mode == GEO_MODE_ADAPTIVE)
                lam = geo::kPi2 - geo_adaptive(k, st, ct, rct, &n);
            else
                lam = geo::kPi2 - (variant == 1 ? geo_v<1>(k, st, ct, rct, &n) : variant == 2 ? geo_v<2>(k, st, ct, rct, &n) : variant == 3 ? geo_v<3>(k, st, ct, rct, &n) : geo_v<4>(k, st, ct, rct, &n));
            const bool bh = lam < geo::kBlackHoleLambda;
            float U, V;
            geo::sky_uv(f->central_to_uv, c2x, c2y, ct, rct, lam, &U, &V);
            const size_t o = (size_t)ly * width + px;
            auto fetch = [sky](uint32_t i) { return sky[i]; };
            if (s->flags & GEO_FLAG_COMPOSITE) {
                if (!bh) {
                    const uint32_t sm = geo::sample_sky_raw(fetch, sw, sh, U, V);
                    rgba[o] = opaque ? sm : geo::composite_(sm, rgba[o]);
                }
            } else {
                rgba[o] = bh ? geo::kBlackRGBA : geo::sample_sky(fetch, sw, sh, opaque, U, V);
            }
            mask[o] = bh ? 1 : 0;
            uv[2 * o] = U;
            uv[2 * o + 1] = V;
            steps[o] = n;
        }
    }
    return 0;
}

// geo::pad_sky + the padded 2 x 2 block (what the device's PaddedSkyQuad reads)
// against WrapClampQuad on the unpadded texture: the sampled RGBA of n (U, V)
// pairs both ways.
extern "C" int host_sample_padded(const uint32_t* sky, uint32_t sw, uint32_t sh, const float* U, const float* V,
                                  uint32_t n, uint32_t* out_wrap, uint32_t* out_pad, uint32_t* out_pair) {
    uint32_t* pad = new uint32_t[((size_t)sw + 2) * ((size_t)sh + 2)];
    geo::pad_sky(reinterpret_cast<const uint8_t*>(sky), sw, sh, pad);
    const uint32_t pitch = sw + 2u;
    // the row pairs the device reads (geo::pair_sky_rows, PairSkyQuad): the
    // quad at padded (x, y) is the 4 texels from 2 (y pitch + x)
    uint32_t* pairs = new uint32_t[2 * ((size_t)sw + 2) * ((size_t)sh + 1)];
    geo::pair_sky_rows(pad, sw, sh, pairs);
    auto paired = [pairs, pitch](int ix0, int iy0, uint32_t (&t)[4]) {
        const size_t i = 2 * ((size_t)(iy0 + 1) * pitch + (size_t)(ix0 + 1));
        t[0] = pairs[i];
        t[2] = pairs[i + 1];
        t[1] = pairs[i + 2];
        t[3] = pairs[i + 3];
    };
    auto padded = [pad, pitch](int ix0, int iy0, uint32_t (&t)[4]) {
        const size_t i = (size_t)(iy0 + 1) * pitch + (size_t)(ix0 + 1);
        t[0] = pad[i];
        t[1] = pad[i + 1];
        t[2] = pad[i + pitch];
        t[3] = pad[i + pitch + 1];
    };
    auto fetch = [sky](uint32_t i) { return sky[i]; };
    for (uint32_t i = 0; i < n; ++i) {
        out_wrap[i] = geo::sample_sky_raw(fetch, sw, sh, U[i], V[i]);
        out_pad[i] = geo::sample_sky_quad(padded, sw, sh, U[i], V[i]);
        out_pair[i] = geo::sample_sky_quad(paired, sw, sh, U[i], V[i]);
    }
    delete[] pad;
    delete[] pairs;
    return 0;
}

// The header's transcendentals on n inputs (host build of geo_math.h), for
// bit comparisons with the oracle's restatement.
extern "C" void host_math(const float* x, uint32_t n, float* out_sin, float* out_cos, float* out_asin) {
    for (uint32_t i = 0; i < n; ++i) {
        geo::sincosf_(x[i], &out_sin[i], &out_cos[i]);
        out_asin[i] = geo::asinf_(x[i]);
    }
}

// The per-pixel sky-direction forms (sincos_sky_, acos_pi_ of x,
// atan2_turns_(y, x)) on n inputs, for bit comparisons with the oracle.
extern "C" void host_sky_math(const float* x, const float* y, uint32_t n, float* out_sin, float* out_cos,
                              float* out_acos_pi, float* out_turns) {
    for (uint32_t i = 0; i < n; ++i) {
        geo::sincos_sky_(x[i], &out_sin[i], &out_cos[i]);
        out_acos_pi[i] = geo::acos_pi_(x[i]);
        out_turns[i] = geo::atan2_turns_(y[i], x[i]);
    }
}

// GEO_FLAG_MIPS pieces of the header on the host: the mip chain (levels one
// after another) and the level of detail, for comparisons with the oracle.
extern "C" void host_mip_chain(const uint8_t* rgba8, uint32_t w, uint32_t h, uint32_t* out) {
    std::memcpy(out, rgba8, (size_t)w * h * 4);
    uint32_t* src = out;
    for (int l = 1; l < geo::kSkyMipLevels; ++l) {
        uint32_t* dst = src + (size_t)geo::mip_dim(w, l - 1) * geo::mip_dim(h, l - 1);
        geo::mip_down(src, geo::mip_dim(w, l - 1), geo::mip_dim(h, l - 1), dst);
        src = dst;
    }
}

extern "C" void host_lod_q8(const float* rho2, uint32_t n, uint32_t* out) {
    for (uint32_t i = 0; i < n; ++i) out[i] = geo::lod_q8(rho2[i]);
}
