"""The f64 bar's error model, measured on the CPU (the oracle's f32 mirror is
the HIP kernel bit for bit, so its errors are the kernel's).

For the sampled pixels of a frame, against the f64 literal restatement:
  x  = b/b_c - 1, b = r cos(theta)/E (theta, E of the f64 pixel),
  m  = max(1/pi, 1/(2 pi cos lat)): UV per radian of a direction error at the
       f64 hit latitude lat (a great-circle move of d changes lat by <= d
       and lon by <= d/cos lat; V = 1/2 - lat/pi, U = lon/(2 pi)),
  err = the bar's wrap-aware UV error,
and the normalised errors err/m (a direction error, rad) and err |x|/m (the
capture-orbit amplification removed), in units of u = 2^-24, by |x| decade.

  python tools/f64_band_model.py cfg3_4k 27 [mode]
  python tools/f64_band_model.py sweep
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import f64_bar as B  # noqa: E402
import oracle as O  # noqa: E402
from helpers import default_frame, default_scene  # noqa: E402
from schwarzschild_raytracer_wgpu_amd import make_scene  # noqa: E402
from schwarzschild_raytracer_wgpu_amd._lib import GEO_MODE_ADAPTIVE, GEO_MODE_DIRECT  # noqa: E402
from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky  # noqa: E402

U = 2.0 ** -24


def measure(frame, scene, literal, w, h, rs, r, row0=0, row_step=1, threads=8):
    nrows = (h - row0 + row_step - 1) // row_step
    p = O.render_f32(frame, scene, make_sky("equirect", (64, 32)), w, h, row0=row0, nrows=nrows,
                     row_step=row_step, threads=threads)
    ref = O.render_f64(frame, literal, w, h, row0=row0, nrows=nrows, row_step=row_step, threads=threads)
    sky = (p["mask"] == 0) & (ref["mask"] == 0)
    e = B.uv_err(p["uv"], ref["uv"])
    E = math.sqrt(1.0 - rs / r)
    x = np.abs(r * np.cos(ref["theta"]) / E / (1.5 * math.sqrt(3.0) * rs) - 1.0)
    lat = math.pi * (0.5 - ref["uv"][..., 1].astype(np.float64))
    m = np.maximum(1.0 / math.pi, 1.0 / (2.0 * math.pi * np.maximum(np.cos(lat), 1e-12)))
    flips = p["mask"] != ref["mask"]
    return dict(sky=sky, err=e, x=x, m=m, flips=flips)


def report(name, d):
    sky, e, x, m = d["sky"], d["err"], d["x"], d["m"]
    print(f"{name}: {sky.sum()} sky pixels, {d['flips'].sum()} mask flips (min |x| of a flip "
          f"{x[d['flips']].min() if d['flips'].any() else float('nan'):.2e}), max err {e[sky].max():.2e}")
    edges = [0, 1e-4, 3e-4, 1e-3, 3e-3, 1e-2, 3e-2, 1e-1, 1e9]
    for lo, hi in zip(edges[:-1], edges[1:]):
        sel = sky & (x >= lo) & (x < hi)
        if not sel.any():
            continue
        dirn = e[sel] / m[sel] / U
        amp = e[sel] * x[sel] / m[sel] / U
        print(f"  |x| in [{lo:.0e}, {hi:.0e}): n={sel.sum():7d}  err max {e[sel].max():.2e}  "
              f"err/m: p99 {np.quantile(dirn, .99):8.1f} max {dirn.max():9.1f} u   "
              f"err|x|/m: p99 {np.quantile(amp, .99):7.2f} max {amp.max():7.2f} u")


def config_case(cfgname, row_step, mode_name=None):
    cfg = CONFIGS[cfgname]
    w, h = cfg.width, cfg.height
    frame = default_frame(w, h, pos=cfg.position, camera=cfg.camera, rs=cfg.rs, fov=cfg.fov, energy=cfg.energy)
    r = math.sqrt(sum(c * c for c in cfg.position))
    mode = GEO_MODE_ADAPTIVE if (mode_name or cfg.mode) == "adaptive" else GEO_MODE_DIRECT
    scene = make_scene(cfg.rs, cfg.sphere_r, r, cfg.step, cfg.max_steps, mode,
                       tol=cfg.tol if mode == GEO_MODE_ADAPTIVE else 0.0)
    literal = make_scene(cfg.rs, cfg.sphere_r, r, cfg.step, cfg.max_steps, GEO_MODE_DIRECT)
    return measure(frame, scene, literal, w, h, cfg.rs, r, row0=row_step // 2, row_step=row_step)


if __name__ == "__main__":
    if sys.argv[1] == "sweep":
        w, h = 480, 270
        for cam in [(math.pi, 0.0), (math.pi + 0.5, 0.4), (math.pi - 1.0, -0.7), (0.3, 0.2), (math.pi, 1.3)]:
            f = default_frame(w, h, camera=cam)
            s = default_scene(2048)
            report(f"sweep {cam}", measure(f, s, s, w, h, 1.0, math.sqrt(2.5 ** 2 + 0.1 ** 2)))
    else:
        report(" ".join(sys.argv[1:]), config_case(sys.argv[1], int(sys.argv[2]), sys.argv[3] if len(sys.argv) > 3
                                                   else None))
