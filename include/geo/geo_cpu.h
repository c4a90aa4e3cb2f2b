/*
 * geo_cpu.h — the CPU baseline path (libgeo_cpu.so), SURVEY.md §8b's
 * geo_render_cpu: the product's per-pixel header (geo_pixel.h, the same f32
 * operation sequence the gfx950 kernel runs) compiled for the host, scalar,
 * over std::thread row blocks ("the same FP32 integrator
 * header, scalar, run over std::thread row blocks").
 *
 * It is the reported-but-not-optimised baseline bench.py times beside the
 * GPU (north_star: "a CPU reference path ... timed in the same run").  It is
 * a separate library: libgeo.so and the Python package never load it, so the
 * product has no CPU fallback (geo_ctx_create fails without a HIP device).
 * Output equals geo_render_rows' bit for bit (tests/test_cpu_baseline.py).
 * GEO_FLAG_MIPS builds the same 4-level chain as geo_set_sky and takes each
 * pixel's level of detail from its frame-aligned 2 x 2 quad, tracing the
 * quad partners outside the frame or the requested rows as the kernel's
 * helper lanes do; any row0 and row_step are accepted.
 */
#ifndef GEO_GEO_CPU_H
#define GEO_GEO_CPU_H

#include <stdint.h>

#include "geo.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Rows row0, row0 + row_step, ... (nrows of them) of a width x height frame,
 * in the layout of geo_render_rows' outputs (row i of the outputs = frame row
 * row0 + i row_step).  sky_rgba8: the sky texture (row-major RGBA8, host);
 * fan/n_fan: the ray fan (GEO_MODE_FAN only).  out_rgba8 is required (read
 * too under GEO_FLAG_COMPOSITE); out_mask, out_uv, out_steps and steps_total
 * may be NULL.  threads <= 0: std::thread::hardware_concurrency().  Returns
 * GEO_OK or GEO_EINVAL.  Scenes and skies geo_render_rows or geo_set_sky
 * reject are rejected here too (max_steps > 2^24, a sky side > 2^20, a
 * padded mip chain of 2^31 bytes or more), so the bit-for-bit equality holds
 * for every scene and sky either path accepts; row0 and row_step are free
 * (the device's GEO_FLAG_MIPS even-row rule does not apply).  Blocking;
 * reentrant. */
int geo_render_cpu(const geo_frame* frame, const geo_scene* scene, const uint8_t* sky_rgba8, uint32_t sky_w,
                   uint32_t sky_h, const float* fan, uint32_t n_fan, uint32_t width, uint32_t height, uint32_t row0,
                   uint32_t nrows, uint32_t row_step, int threads, uint8_t* out_rgba8, uint8_t* out_mask,
                   float* out_uv, uint32_t* out_steps, unsigned long long* steps_total);

#ifdef __cplusplus
}
#endif

#endif /* GEO_GEO_CPU_H */
