// Host build of the PRODUCT's point-path header (geo_rays.h) for CPU tests:
// the RayConnector and vs_main sequences, compiled with g++ and the same
// no-contraction rules, must equal the oracle's independent restatement
// (oracle/geo_oracle_points.c, kernel-polynomial variant) bit for bit.
#include <cstdint>
#include <cstring>

#include "../../include/geo/geo.h"
#include "../../schwarzschild_raytracer_wgpu_amd/csrc/geo_rays.h"

// geo_rays_update semantics over host arrays: connectors near side first,
// state u[c*48 + i], needs[c]; other: 3 floats or 3 per point.
extern "C" int host_rays_update(float rs, uint32_t n_points, uint32_t sides, const float* pos, float* u,
                                uint8_t* needs, const float* other, int per_point, uint32_t iterations, int reset,
                                float* out) {
    const uint32_t nside = ((sides & 1u) ? 1u : 0u) + ((sides & 2u) ? 1u : 0u);
    for (uint32_t c = 0; c < n_points * nside; ++c) {
        const bool far = sides == GEO_RAYS_FAR ? true : c >= n_points;
        const uint32_t p = c >= n_points ? c - n_points : c;
        const float* o = per_point ? other + 3 * (size_t)p : other;
        float* uc = u + (size_t)c * geo::kRayNodes;
        float nu[geo::kRayNodes];
        bool nd = needs[c] != 0;
        const float a = geo::ray_connect(rs, !far, pos[3 * p], pos[3 * p + 1], pos[3 * p + 2], o[0], o[1], o[2],
                                         reset != 0, iterations, &nd, [uc](int i) { return uc[i]; }, nu);
        std::memcpy(uc, nu, sizeof(nu));
        needs[c] = nd ? 1 : 0;
        out[4 * c] = pos[3 * p];
        out[4 * c + 1] = pos[3 * p + 1];
        out[4 * c + 2] = pos[3 * p + 2];
        out[4 * c + 3] = a;
    }
    return 0;
}

extern "C" int host_project(const geo_frame* f, const float* v, uint32_t n, uint32_t w, uint32_t h, int* xy) {
    for (uint32_t i = 0; i < n; ++i) {
        uint32_t ix = 0, iy = 0;
        const bool vis = geo::project_point(f->display_to_movement, f->movement_to_central, f->central_to_uv,
                                            f->psi_factor_and_position[0], v[4 * i], v[4 * i + 1], v[4 * i + 2],
                                            v[4 * i + 3], w, h, &ix, &iy);
        xy[2 * i] = vis ? (int)ix : -1;
        xy[2 * i + 1] = vis ? (int)iy : -1;
    }
    return 0;
}
