#!/usr/bin/env python3
"""How wide GEO_FLAG_RING_F64's band must be: the f32 path's UV error against
the f64 reference, binned by the band-test quantity x = |kx cos(theta) - 1|
of each pixel's f32 ray (the kernel's in_band, geo_band.h), on every k-th row
of a config frame.  CPU only (the oracle's f32 mirror is the HIP kernel bit
for bit); the reference is the f64 literal (fixed-step configs) or the f64
step/32 RK4 in the adaptive mode (the adaptive configs, as the ring tests).

    python tools/ring_width_margin.py cfg2_1080p cfg3_4k cfg5_8k_adaptive [--row-step 2] [--out F.json]

Per bin: sky pixels (f32 and f64 both sky), the largest UV error, pixels over
the 1e-4 bar and mask flips; the pole rows (|latitude| > 89 deg of the f64
hit, where 1e-4 of U is a 1/(2 pi cos lat) longitude swing) counted apart.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import f64_bar as B  # noqa: E402
import oracle as O  # noqa: E402
import schwarzschild_raytracer_wgpu_amd as g  # noqa: E402
from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky  # noqa: E402

EDGES = [0.0, 1e-3, 2e-3, 3e-3, 4e-3, 5e-3, 6e-3, 8e-3, 1.2e-2, 2e-2, 5e-2, np.inf]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("configs", nargs="*", default=["cfg2_1080p", "cfg3_4k"])
    p.add_argument("--row-step", type=int, default=1)
    p.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    p.add_argument("--chunk", type=int, default=216)
    p.add_argument("--out", default=None)
    a = p.parse_args()
    res = {}
    for name in a.configs:
        cfg = CONFIGS[name]
        w, h = cfg.width, cfg.height
        obs = g.Observer(cfg.rs, cfg.fov, w, h)
        obs.set_position(*cfg.position)
        obs.set_camera(*cfg.camera)
        obs.set_energy(cfg.energy)
        frame = obs.calc_transformation_pipeline()
        r = obs.get_radial_position()
        adaptive = cfg.mode == "adaptive"
        mode = g.GEO_MODE_ADAPTIVE if adaptive else g.GEO_MODE_DIRECT
        scene = g.make_scene(cfg.rs, cfg.sphere_r, r, cfg.step, cfg.max_steps, mode,
                             tol=cfg.tol if adaptive else 0.0)  # the plain f32 path (no flag)
        ring = g.make_scene(cfg.rs, cfg.sphere_r, r, cfg.step, cfg.max_steps, mode, tol=cfg.tol if adaptive else 0.0)
        ring.flags |= g._lib.GEO_FLAG_RING_F64  # only for the band-test quantity
        ref = (g.make_scene(cfg.rs, cfg.sphere_r, r, cfg.step, cfg.max_steps, mode, tol=cfg.tol) if adaptive
               else g.make_scene(cfg.rs, cfg.sphere_r, r, cfg.step, cfg.max_steps, g.GEO_MODE_DIRECT))
        sky = make_sky(cfg.sky, (64, 32))
        k_ = a.row_step
        hs = (h + k_ - 1) // k_
        nb = len(EDGES) - 1
        stats = {"sky": np.zeros(nb, np.int64), "over": np.zeros(nb, np.int64), "flips": np.zeros(nb, np.int64),
                 "max": np.zeros(nb), "pole_over": np.zeros(nb, np.int64), "pixels": np.zeros(nb, np.int64)}
        for i0 in range(0, hs, a.chunk):
            n = min(a.chunk, hs - i0)
            f32 = O.render_f32(frame, scene, sky, w, h, row0=i0 * k_, nrows=n, row_step=k_, threads=a.threads,
                               want_steps=False)
            f64 = O.render_f64(frame, ref, w, h, row0=i0 * k_, nrows=n, row_step=k_, threads=a.threads)
            x = O.ring_x(frame, ring, w, h, i0 * k_, n, k_)
            e = B.uv_err(f32["uv"], f64["uv"])
            lat = np.abs(90.0 - f64["uv"][..., 1].astype(np.float64) * 180.0)  # V = 1/2 - lat/pi
            pole = lat > 89.0
            sky_px = (f32["mask"] == 0) & (f64["mask"] == 0)
            flip = f32["mask"] != f64["mask"]
            b = np.clip(np.searchsorted(EDGES, x, side="right") - 1, 0, nb - 1)
            for j in range(nb):
                m = b == j
                stats["pixels"][j] += int(m.sum())
                s = m & sky_px & ~pole
                stats["sky"][j] += int(s.sum())
                stats["over"][j] += int((s & (e > B.UV_BAR)).sum())
                stats["pole_over"][j] += int((m & sky_px & pole & (e > B.UV_BAR)).sum())
                stats["flips"][j] += int((m & flip).sum())
                if s.any():
                    stats["max"][j] = max(stats["max"][j], float(e[s].max()))
        rows = []
        for j in range(nb):
            rows.append({"x_lo": EDGES[j], "x_hi": None if np.isinf(EDGES[j + 1]) else EDGES[j + 1],
                         "pixels": int(stats["pixels"][j]), "sky_pixels_non_pole": int(stats["sky"][j]),
                         "uv_max": float(stats["max"][j]), "over_bar": int(stats["over"][j]),
                         "over_bar_poles": int(stats["pole_over"][j]), "mask_flips": int(stats["flips"][j])})
            print(f"{name:18s} x in [{EDGES[j]:.0e}, {EDGES[j + 1]:.0e}): px {rows[-1]['pixels']:9d}  "
                  f"uv_max {rows[-1]['uv_max']:.2e}  over {rows[-1]['over_bar']:4d}  poles over "
                  f"{rows[-1]['over_bar_poles']:3d}  flips {rows[-1]['mask_flips']:3d}", flush=True)
        res[name] = {"rows": f"every {k_}th row" if k_ > 1 else "all rows",
                     "reference": "f64 RK4 at step/32" if adaptive else "f64 literal", "bins": rows}
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
