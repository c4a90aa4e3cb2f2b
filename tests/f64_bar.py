"""The north_star parity bar against the f64 literal restatement.

The HIP kernel equals the oracle's f32 mirror bit for bit (test_gpu_parity);
this module measures both against the f64 LITERAL restatement of the
reference (oracle geo_oracle_pixel_f64: sphere_ray_tracer.rs:60-193 and
shader.wgsl:57-106 expression by expression), with the bar north_star states:

* hit-classification mask identical pixel for pixel, except inside an
  epsilon-band around the critical impact parameter b_c = 3 sqrt(3)/2 rs,
  where the traveled angle diverges (the capture orbit) and no f32 evaluation
  of the ray's angle can decide the f64 one;
* sky-sphere UV within 1e-4 "relative", defined here against the [0, 1] UV
  range: per pixel err = max(min(|dU|, 1 - |dU|), |dV|) (U wraps at the seam,
  where a per-component relative error is ill-posed: U ~ 0 next to U ~ 1),
  over the pixels both sides draw (mask 0) outside the same band.

The band is |b/b_c - 1| < BAND_EPS with b = r cos(theta)/E the ray's impact
parameter from the f64 per-pixel theta (solve_ray_fan, sphere_ray_tracer.rs:
38-49: rotation = r cos theta, energy = sqrt(1 - rs/r)).  Pixels in it are
counted and reported, not hidden.
"""
from __future__ import annotations

import math

import numpy as np

import oracle as O

UV_BAR = 1e-4    # north_star: sky-sphere UV within 1e-4 (of the [0, 1] range, wrap-aware)
# |b/b_c - 1| below this: the capture-orbit band.  The traveled angle there
# grows like -ln|b - b_c|, so a 1-ulp f32 error in the pixel's direction moves
# lambda' by ~ulp/|b/b_c - 1|; near the sky's poles U magnifies it again by
# 1/sin(colatitude).  Measured: every pixel beyond 1.81e-3 of
# b_c meets the UV bar on full 1080p and 4K frames; 2e-3 is the band.
BAND_EPS = 2e-3


def uv_err(uv_a, uv_b):
    """Per-pixel wrap-aware UV error against the [0, 1] range."""
    a = uv_a.astype(np.float64)
    b = uv_b.astype(np.float64)
    du = np.abs(a[..., 0] - b[..., 0])
    du = np.minimum(du, 1.0 - du)
    dv = np.abs(a[..., 1] - b[..., 1])
    return np.maximum(du, dv)


def f64_rows(frame, scene, width, height, row0, nrows, row_step, fan=None, threads=16):
    """The f64 literal restatement on frame rows row0 + i row_step, i < nrows:
    mask, uv, lam and theta per pixel (arrays of shape (nrows, width))."""
    return O.render_f64(frame, scene, width, height, row0=row0, nrows=nrows, row_step=row_step, fan=fan,
                        threads=threads)


def band_mask(theta, rs, r_obs):
    """Pixels whose ray's impact parameter lies within BAND_EPS of b_c (outside the horizon)."""
    if rs <= 0.0 or r_obs <= rs:
        return np.zeros(theta.shape, dtype=bool)
    e = math.sqrt(1.0 - rs / r_obs)
    b = r_obs * np.cos(theta) / e
    bc = 1.5 * math.sqrt(3.0) * rs
    return np.abs(b / bc - 1.0) < BAND_EPS


def compare(hip_mask, hip_uv, ref, rs, r_obs):
    """The bar's statistics for HIP (or the f32 mirror) rows against f64 rows."""
    band = band_mask(ref["theta"], rs, r_obs)
    flip = hip_mask != ref["mask"]
    sky = (hip_mask == 0) & (ref["mask"] == 0)
    e = uv_err(hip_uv, ref["uv"])
    e_out = e[sky & ~band]
    e_all = e[sky]
    q = (lambda x, p: float(np.quantile(x, p)) if x.size else 0.0)
    return {
        "pixels": int(hip_mask.size),
        "band_pixels": int(band.sum()),
        "mask_flips": int(flip.sum()),
        "mask_flips_outside_band": int((flip & ~band).sum()),
        "sky_pixels_outside_band": int(e_out.size),
        "uv_median": q(e_out, 0.5),
        "uv_p99": q(e_out, 0.99),
        "uv_p9999": q(e_out, 0.9999),
        "uv_max": float(e_out.max()) if e_out.size else 0.0,
        "uv_over_bar_outside_band": int((e_out > UV_BAR).sum()),
        "uv_max_in_band": float(e[sky & band].max()) if (sky & band).any() else 0.0,
        "uv_max_all": float(e_all.max()) if e_all.size else 0.0,
    }
