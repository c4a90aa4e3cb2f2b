"""The north_star parity bar against the f64 literal restatement.

The HIP kernel equals the oracle's f32 mirror bit for bit (test_gpu_parity);
this module measures both against the f64 LITERAL restatement of the
reference (oracle geo_oracle_pixel_f64: sphere_ray_tracer.rs:60-193 and
shader.wgsl:57-106 expression by expression), with the bar north_star states:

* hit-classification mask identical pixel for pixel, except in the capture
  band, where the traveled angle diverges (the capture orbit) and no f32
  evaluation of the ray can decide the f64 one;
* sky-sphere UV within 1e-4 "relative", defined here against the [0, 1] UV
  range: per pixel err = max(min(|dU|, 1 - |dU|), |dV|) (U wraps at the seam,
  where a per-component relative error is ill-posed: U ~ 0 next to U ~ 1),
  over the pixels both sides draw (mask 0), except where the error model
  below predicts more than the bar; there each pixel is held to the model's
  own bound instead.

The bands come from the error model (below), not from the data: the capture
band is where the capture orbit's amplification alone could move V by more
than the bar, |b/b_c - 1| < K u/(pi UV_BAR) ~ 1.5e-3, with b = r cos(theta)/E
the ray's impact parameter from the f64 per-pixel theta (solve_ray_fan,
sphere_ray_tracer.rs:38-49: rotation = r cos theta, energy = sqrt(1 - rs/r));
the UV band adds the sky's poles.  Pixels in the bands are counted and
reported, and checked against the model.
"""
from __future__ import annotations

import math

import numpy as np

import oracle as O

UV_BAR = 1e-4    # north_star: sky-sphere UV within 1e-4 (of the [0, 1] range, wrap-aware)

# ---- the error model -------------------------------------
# An f32 evaluation of a pixel differs from the f64 one by a direction error
# delta (rad) of the sky direction it draws.  The UV bar's error is then at
# most m * delta, m = max(1/pi, 1/(2 pi cos lat)): a great-circle move by
# delta changes the latitude by <= delta (V = 1/2 - lat/pi) and the longitude
# by <= delta/cos lat (U = lon/(2 pi)); lat is the f64 hit latitude.
# delta has two parts, in units of u = 2^-24:
#   * A: the roundings of a well-conditioned ray (the f32 traveled-angle sum
#     `angle += step` over S steps, the sky map's sincos/atan2/asin);
#   * K/|x|, x = b/b_c - 1: near the capture orbit the traveled angle is
#     alpha(b) = -ln(b/b_c - 1) + const (strong-deflection limit, coefficient
#     1 for Schwarzschild), so an error K u in the ray's b/b_c (its initial
#     direction's roundings, and the integration's, which the unstable orbit
#     amplifies as a shift of b) moves alpha by K u/|x|.
# So per pixel  err <= PRED = m u (A + K/|x|).  The form is the physics and
# geometry above.  A priori worst-case roundings give A <= 2 S + 8 and
# K <= ~76 (12 roundings of the initial state, and 2u per step summed
# against the orbit's e^-phi growth: 2u/h = 64u); both are far from tight.
# The constants used are measured on a calibration set that is none of the
# configs (tests/test_f64_bar_cpu.py::test_band_model_calibration: the
# default pose at 480 x 270 under five cameras, f32 specification vs f64
# literal, every pixel): max err |x|/(m u) = 6.7 for |x| < 0.1, max err/(m u)
# = 58 for |x| >= 0.1, each rounded up to a power of two.  The config frames
# (tests/test_gpu_f64_bar.py, HIP) are the validation.
K_AMP = 8.0    # u: the ray's equivalent b/b_c error near the capture orbit
A_DIR = 64.0   # u: the direction error of a well-conditioned ray (rad)
U32 = 2.0 ** -24
# The band: the pixels where PRED exceeds the bar (the capture-orbit band,
# |x| < ~1.5e-3 where m = 1/pi, and the sky's poles, cos lat < ~0.006).
# Outside it every pixel is held to the bar; inside it to PRED itself.


def model(theta, uv_ref, rs, r_obs):
    """(x, m, pred) per pixel from the f64 pixel's theta and UV."""
    lat = math.pi * (0.5 - uv_ref[..., 1].astype(np.float64))
    m = np.maximum(1.0 / math.pi, 1.0 / (2.0 * math.pi * np.maximum(np.cos(lat), 1e-30)))
    if rs <= 0.0 or r_obs <= rs:
        x = np.full(theta.shape, np.inf)  # no capture orbit outside the horizon's reach
    else:
        e = math.sqrt(1.0 - rs / r_obs)
        x = np.abs(r_obs * np.cos(theta) / e / (1.5 * math.sqrt(3.0) * rs) - 1.0)
    with np.errstate(divide="ignore"):
        pred = m * U32 * (A_DIR + K_AMP / x)
    return x, m, pred


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


def capture_band(theta, rs, r_obs):
    """Pixels where the capture orbit's amplification alone (K u/|x|, at the
    smallest m = 1/pi) exceeds the UV bar: where the mask may flip."""
    x, _, _ = model(theta, np.zeros(theta.shape + (2,), np.float32) + 0.5, rs, r_obs)
    with np.errstate(divide="ignore"):
        return U32 * K_AMP / x / math.pi > UV_BAR


def compare(hip_mask, hip_uv, ref, rs, r_obs):
    """The bar's statistics for HIP (or the f32 mirror) rows against f64 rows."""
    x, m, pred = model(ref["theta"], ref["uv"], rs, r_obs)
    flip = hip_mask != ref["mask"]
    sky = (hip_mask == 0) & (ref["mask"] == 0)
    cap = capture_band(ref["theta"], rs, r_obs)
    band = sky & (pred > UV_BAR)  # the UV band: sky pixels the model does not hold to the bar
    e = uv_err(hip_uv, ref["uv"])
    e_out = e[sky & ~band]
    e_all = e[sky]
    e_in, p_in = e[sky & band], pred[sky & band]
    q = (lambda v, p: float(np.quantile(v, p)) if v.size else 0.0)
    return {
        "pixels": int(hip_mask.size),
        "band_pixels": int(cap.sum()),
        "uv_band_pixels": int(band.sum()),
        "uv_band_pole_pixels": int((band & ~cap).sum()),
        "mask_flips": int(flip.sum()),
        "mask_flips_outside_band": int((flip & ~cap).sum()),
        "sky_pixels_outside_band": int(e_out.size),
        "uv_median": q(e_out, 0.5),
        "uv_p99": q(e_out, 0.99),
        "uv_p9999": q(e_out, 0.9999),
        "uv_max": float(e_out.max()) if e_out.size else 0.0,
        "uv_max_over_bar": (float(e_out.max()) if e_out.size else 0.0) / UV_BAR,
        "uv_over_bar_outside_band": int((e_out > UV_BAR).sum()),
        "uv_max_in_band": float(e_in.max()) if e_in.size else 0.0,
        "in_band_over_model": int((e_in > p_in).sum()),
        "max_err_over_model": float((e[sky] / pred[sky]).max()) if sky.any() else 0.0,
        "uv_max_all": float(e_all.max()) if e_all.size else 0.0,
        "model": f"pred = m u ({A_DIR:g} + {K_AMP:g}/|b/b_c - 1|), u = 2^-24",
    }


# ---- fan mode: the reference's display path (shader.wgsl:77-88) ---------
# A fan-mode pixel lerps the f32 fan (R32Float, ray_fan_texture.rs:65-90) at
# t = (pi/2 - lambda)/pi (n - 1) and draws the sky direction that lerp gives.
# Both sides read the same f32 nodes, so they differ only by the pixel's own
# roundings: an error in its angle to the black hole, a few u, amplified by
# the asin's conditioning near lambda = +-pi/2 (1/|cos lambda|) and carried
# into lambda' by the fan's slope there, s = |fan[i+1] - fan[i]| (n - 1)/pi
# (steep only in the interval where the fan falls to NO_VALUE, the black
# hole's edge); plus the sky map's own roundings (A_DIR).  So
#   direction error <= u (A_DIR + C_FAN s q),  q = 1 + 1/|cos lambda|,
# UV error <= m times that (m as above), and the mask may flip only where
# |lambda'_f64 + 7| is within the lambda' part, u C_FAN s q (+ the lerp's own
# rounding, 8 u |lambda'|).  C_FAN is measured on the same calibration set
# as the direct model (tests/test_f64_bar_cpu.py::test_fan_model_calibration:
# 2.62), rounded up to a power of two.
C_FAN = 4.0
BLACK_HOLE_LAMBDA = -7.0  # shader.wgsl:88


def fan_terms(theta, uv_ref, fan):
    """(m, s q) per pixel of an f64 fan-mode frame: the UV factor and the
    fan's slope at the pixel times the asin's conditioning."""
    n = len(fan)
    f = np.asarray(fan, dtype=np.float64)
    t = np.clip((math.pi / 2 - theta) / math.pi, 0.0, 1.0) * (n - 1)
    i = np.minimum(np.floor(t).astype(np.int64), n - 2)
    s = np.abs(f[i + 1] - f[i]) * (n - 1) / math.pi
    q = 1.0 + 1.0 / np.maximum(np.abs(np.cos(theta)), 1e-3)
    lat = math.pi * (0.5 - uv_ref[..., 1].astype(np.float64))
    m = np.maximum(1.0 / math.pi, 1.0 / (2.0 * math.pi * np.maximum(np.cos(lat), 1e-30)))
    return m, s * q


def fan_model(theta, lam, uv_ref, fan):
    """(pred UV error, lambda' error bound) per pixel of an f64 fan-mode frame."""
    m, sq = fan_terms(theta, uv_ref, fan)
    dlam = U32 * (C_FAN * sq + 8.0 * np.abs(lam))
    return m * U32 * (A_DIR + C_FAN * sq), dlam


def compare_fan(hip_mask, hip_uv, ref, fan):
    """The bar's statistics for fan-mode rows against the f64 literal fan-mode rows."""
    pred, dlam = fan_model(ref["theta"], ref["lam"], ref["uv"], fan)
    flip = hip_mask != ref["mask"]
    edge = np.abs(ref["lam"] - BLACK_HOLE_LAMBDA) <= 2.0 * dlam  # where the mask may flip
    sky = (hip_mask == 0) & (ref["mask"] == 0)
    band = sky & (pred > UV_BAR)
    e = uv_err(hip_uv, ref["uv"])
    e_out = e[sky & ~band]
    e_in, p_in = e[sky & band], pred[sky & band]
    return {
        "pixels": int(hip_mask.size),
        "edge_pixels": int(edge.sum()),
        "mask_flips": int(flip.sum()),
        "mask_flips_outside_edge": int((flip & ~edge).sum()),
        "uv_band_pixels": int(band.sum()),
        "sky_pixels_outside_band": int(e_out.size),
        "uv_p99": float(np.quantile(e_out, 0.99)) if e_out.size else 0.0,
        "uv_max": float(e_out.max()) if e_out.size else 0.0,
        "uv_over_bar_outside_band": int((e_out > UV_BAR).sum()),
        "uv_max_in_band": float(e_in.max()) if e_in.size else 0.0,
        "in_band_over_model": int((e_in > p_in).sum()),
        "max_err_over_model": float((e[sky] / pred[sky]).max()) if sky.any() else 0.0,
        "model": f"pred = m u ({A_DIR:g} + {C_FAN:g} s (1 + 1/|cos lambda|)), u = 2^-24",
    }
