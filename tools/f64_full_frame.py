#!/usr/bin/env python3
"""The north_star bar against the f64 literal on EVERY pixel of a config
frame, on the CPU: the oracle's f32 mirror (which the HIP kernel equals bit
for bit: tests/test_gpu_parity.py, tests/test_gpu_fuzz.py) against the f64
literal restatement, with the statistics of tests/f64_bar.py (its error
model, band and bar).  The GPU tests sample rows of the config frames; this
covers the rows between them, where the pixels closest to the capture orbit
may lie.  Diagnostic, CPU only (reads the oracle, never the product path).

    python tools/f64_full_frame.py cfg2_1080p cfg3_4k [--ring] [--threads 8] [--out FILE.json]

With --ring the f32 side is GEO_FLAG_RING_F64's (the band's pixels drawn in
f64, as the library does on the GPU).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import f64_bar as B  # noqa: E402
import oracle as O  # noqa: E402
import schwarzschild_raytracer_wgpu_amd as g  # noqa: E402
from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("configs", nargs="*", default=["cfg2_1080p", "cfg3_4k"])
    p.add_argument("--threads", type=int, default=os.cpu_count() or 8)
    p.add_argument("--chunk", type=int, default=216, help="rows per oracle call (bounds memory)")
    p.add_argument("--ring", action="store_true", help="GEO_FLAG_RING_F64: the band's pixels in f64 (geo.h)")
    p.add_argument("--fine", action="store_true",
                   help="adaptive configs: against the fine f64 reference (fixed RK4 at step/32, oracle pixel_f64 "
                        "in the adaptive mode) instead of the fixed-step literal")
    p.add_argument("--row-step", type=int, default=1, help="every k-th row (1: all)")
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
        mode = g.GEO_MODE_ADAPTIVE if cfg.mode == "adaptive" else g.GEO_MODE_DIRECT
        scene = g.make_scene(cfg.rs, cfg.sphere_r, r, cfg.step, cfg.max_steps, mode,
                             tol=cfg.tol if cfg.mode == "adaptive" else 0.0)
        if a.ring:
            scene.flags |= g._lib.GEO_FLAG_RING_F64
        literal = g.make_scene(cfg.rs, cfg.sphere_r, r, cfg.step, cfg.max_steps, g.GEO_MODE_DIRECT)
        if a.fine and mode == g.GEO_MODE_ADAPTIVE:
            literal = g.make_scene(cfg.rs, cfg.sphere_r, r, cfg.step, cfg.max_steps, mode, tol=cfg.tol)
        sky = make_sky(cfg.sky, (64, 32))  # the UV and mask do not depend on the sky
        t0 = time.time()
        k_ = a.row_step
        hs = (h + k_ - 1) // k_  # sampled rows 0, k, 2k, ...
        mask = np.empty((hs, w), np.uint8)
        uv = np.empty((hs, w, 2), np.float32)
        ref = {"mask": np.empty((hs, w), np.uint8), "uv": np.empty((hs, w, 2), np.float32),
               "theta": np.empty((hs, w), np.float64)}
        for i0 in range(0, hs, a.chunk):
            n = min(a.chunk, hs - i0)
            f32 = O.render_f32(frame, scene, sky, w, h, row0=i0 * k_, nrows=n, row_step=k_, threads=a.threads,
                               want_steps=False)
            mask[i0:i0 + n], uv[i0:i0 + n] = f32["mask"], f32["uv"]
            f64 = O.render_f64(frame, literal, w, h, row0=i0 * k_, nrows=n, row_step=k_, threads=a.threads)
            for k in ref:
                ref[k][i0:i0 + n] = f64[k]
        st = B.compare(mask, uv, ref, cfg.rs, r)
        x, _, _ = B.model(ref["theta"], ref["uv"], cfg.rs, r)
        e = B.uv_err(uv, ref["uv"])
        sky_px = (mask == 0) & (ref["mask"] == 0)
        over = sky_px & (e > B.UV_BAR)
        band = (O.ring_band(frame, scene, w, h, 0, hs, k_).astype(bool) if a.ring else np.zeros((hs, w), bool))
        fine = a.fine and mode == g.GEO_MODE_ADAPTIVE
        st.update(config=name, rows=f"all {h} rows" if k_ == 1 else f"every {k_}th row ({hs})", ring_f64=a.ring,
                  ring_pixels=int(band.sum()),
                  reference="f64 RK4 at step/32 (the adaptive mode's own check)" if fine else "f64 literal, step pi/100",
                  side="oracle f32 mirror (= HIP bit for bit)", seconds=round(time.time() - t0, 1),
                  pixels_over_bar=int(over.sum()),
                  min_abs_x=float(np.min(x)) if np.isfinite(x).any() else None,
                  over_bar_abs_x_max=float(x[over].max()) if over.any() else None)
        res[name] = st
        print(name, json.dumps(st), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
