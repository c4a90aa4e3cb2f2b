/* A plain-C client of libgeo (include/geo/geo.h): what a host in the
 * reference's position does per frame, without Python or torch.
 *
 *   observer -> 208-B uniform -> geo_render_rows -> RGBA8 frame -> PPM
 *
 * Build (any C99 compiler; HIP's C runtime API only for device memory):
 *   gcc -std=c99 -O2 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include examples/render_frame.c \
 *       -L schwarzschild_raytracer_wgpu_amd -lgeo -L /opt/rocm/lib -lamdhip64 -lm -o render_frame
 *   ./render_frame out.ppm 384 216
 *
 * Prints the FNV-1a hash of the RGBA8 frame (tests/test_gpu_c_client.py
 * checks it against the oracle).  The sky is a synthetic 512x256 equirect:
 * texel (x, y) = (x * 7 ^ y * 13, x + y, x * y, 255) in the low 8 bits. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <hip/hip_runtime_api.h>

#include "geo/geo.h"

static const double kPi = 3.14159265358979323846;

#define CHECK(call)                                                                        \
    do {                                                                                   \
        int st_ = (call);                                                                  \
        if (st_ != GEO_OK) {                                                               \
            fprintf(stderr, "%s: %s\n", #call, geo_status_str(st_));                      \
            return 1;                                                                      \
        }                                                                                  \
    } while (0)

int main(int argc, char** argv) {
    const char* out = argc > 1 ? argv[1] : "frame.ppm";
    const uint32_t W = argc > 2 ? (uint32_t)atoi(argv[2]) : 384u;
    const uint32_t H = argc > 3 ? (uint32_t)atoi(argv[3]) : 216u;
    const uint32_t SW = 512, SH = 256;
    uint8_t* sky = malloc((size_t)SW * SH * 4);
    uint8_t* rgba = malloc((size_t)W * H * 4);
    if (!sky || !rgba) return 1;
    for (uint32_t y = 0; y < SH; ++y)
        for (uint32_t x = 0; x < SW; ++x) {
            uint8_t* t = sky + 4 * ((size_t)y * SW + x);
            t[0] = (uint8_t)((x * 7u) ^ (y * 13u));
            t[1] = (uint8_t)(x + y);
            t[2] = (uint8_t)(x * y);
            t[3] = 255;
        }

    if (geo_abi_version() != GEO_ABI_VERSION) return 1;
    geo_ctx* ctx = NULL;
    CHECK(geo_ctx_create(0, &ctx));
    CHECK(geo_set_sky(ctx, sky, SW, SH));

    /* Observer::new + the reference's default pose scaled to rs = 1 (lib.rs:72, observer.rs:70-81) */
    geo_observer* obs = NULL;
    CHECK(geo_observer_create(1.0, kPi / 2, W, H, &obs));
    CHECK(geo_observer_set_position(obs, 2.5, 0.0, 0.1));
    CHECK(geo_observer_set_state(obs, GEO_OBSERVER_FROZEN_FALL));
    geo_frame frame;
    CHECK(geo_observer_calc_transformation_pipeline(obs, &frame));
    geo_scene scene = {1.0f, 50.0f, (float)geo_observer_radial_position(obs), (float)(kPi / 100.0), 2048u,
                       GEO_MODE_DIRECT, 0u, 0.0f};

    uint8_t* d_rgba = NULL;
    unsigned long long* d_steps = NULL;
    if (hipMalloc((void**)&d_rgba, (size_t)W * H * 4) != hipSuccess ||
        hipMalloc((void**)&d_steps, sizeof(unsigned long long)) != hipSuccess ||
        hipMemset(d_steps, 0, sizeof(unsigned long long)) != hipSuccess)
        return 1;
    CHECK(geo_render_rows(ctx, &frame, &scene, W, H, 0, H, d_rgba, NULL, NULL, NULL, d_steps, NULL));
    unsigned long long steps = 0;
    if (hipMemcpy(rgba, d_rgba, (size_t)W * H * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&steps, d_steps, sizeof(steps), hipMemcpyDeviceToHost) != hipSuccess)
        return 1;

    uint64_t hash = 1469598103934665603ull;
    for (size_t i = 0; i < (size_t)W * H * 4; ++i) hash = (hash ^ rgba[i]) * 1099511628211ull;
    FILE* f = fopen(out, "wb");
    if (!f) return 1;
    fprintf(f, "P6\n%u %u\n255\n", W, H);
    for (size_t i = 0; i < (size_t)W * H; ++i) fwrite(rgba + 4 * i, 1, 3, f);
    fclose(f);
    printf("frame %ux%u steps %llu fnv1a %016llx\n", W, H, steps, (unsigned long long)hash);

    hipFree(d_rgba);
    hipFree(d_steps);
    geo_observer_destroy(obs);
    geo_ctx_destroy(ctx);
    free(sky);
    free(rgba);
    return 0;
}
