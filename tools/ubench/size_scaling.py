#!/usr/bin/env python3
"""Fixed vs per-pixel cost of one render launch: the same scene (the
configs' observer and camera) rendered at 16:9 sizes from 960x540 to
7680x4320, each launch timed by an event pair on its own dispatch
(geo_time_next_render).  A least-squares line kernel_ms = a + b * pixels
separates what a launch costs whatever its size (launch, ramp-up of the
first waves, the tail behind the slowest ones) from the steady per-pixel
cost b.  Mode "fan" (the reference's display path: fan lerp + sky sample)
or "direct" (per-pixel RK4, 2048 steps).  One JSON line.

  python tools/ubench/size_scaling.py [fan|direct] [launches per size]
"""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

import schwarzschild_raytracer_wgpu_amd as g  # noqa: E402
from schwarzschild_raytracer_wgpu_amd.scenes import CONFIGS, make_sky  # noqa: E402
from schwarzschild_raytracer_wgpu_amd.timing import HipEvent  # noqa: E402

mode_name = sys.argv[1] if len(sys.argv) > 1 else "fan"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
mode = {"fan": g.GEO_MODE_FAN, "direct": g.GEO_MODE_DIRECT}[mode_name]
cfg = CONFIGS["cfg3_4k"]
sizes = [(960, 540), (1920, 1080), (2880, 1620), (3840, 2160), (5760, 3240), (7680, 4320)]
ctx = g.Context(0)
ctx.set_sky(make_sky(cfg.sky, cfg.sky_size))
dev = torch.device("cuda:0")
rows = []
for W, H in sizes:
    obs = g.Observer(cfg.rs, cfg.fov, W, H)
    obs.set_position(*cfg.position)
    obs.set_camera(*cfg.camera)
    obs.set_energy(cfg.energy)
    frame = obs.calc_transformation_pipeline()
    r = obs.get_radial_position()
    if mode == g.GEO_MODE_FAN:
        ctx.solve_ray_fan(cfg.sphere_r, cfg.rs, cfg.max_steps, cfg.step, 400, r, host=False)
    scene = g.make_scene(cfg.rs, cfg.sphere_r, r, cfg.step, cfg.max_steps, mode)
    out = torch.empty(W * H * 4, dtype=torch.uint8, device=dev)
    steps = torch.zeros(1, dtype=torch.int64, device=dev)
    ctx.render_rows(frame, scene, W, H, 0, H, out, steps_total=steps)
    torch.cuda.synchronize()
    spin = max(50, int(3e8 / (W * H * (1 if mode == g.GEO_MODE_FAN else 40))))  # ~ >= 50 ms of GPU work
    for _ in range(spin):
        ctx.render_rows(frame, scene, W, H, 0, H, out)
    evs = [(HipEvent(), HipEvent()) for _ in range(n)]
    w0, w1 = HipEvent(), HipEvent()
    w0.record()
    for a, b in evs:
        ctx.time_next_render(a, b)
        ctx.render_rows(frame, scene, W, H, 0, H, out)
    w1.record()
    torch.cuda.synchronize()
    ks = np.array([a.elapsed_time(b) for a, b in evs])
    rows.append({"width": W, "height": H, "pixels": W * H, "kernel_ms_mean": float(ks.mean()),
                 "kernel_ms_median": float(np.median(ks)), "kernel_ms_min": float(ks.min()),
                 "wall_ms_per_launch": w0.elapsed_time(w1) / n, "steps": int(steps.item())})
px = np.array([r["pixels"] for r in rows], dtype=np.float64)
km = np.array([r["kernel_ms_median"] for r in rows])
b, a = np.polyfit(px, km, 1)
fit = {"intercept_ms": float(a), "ms_per_mpixel": float(b * 1e6),
       "residual_max_ms": float(np.max(np.abs(km - (a + b * px))))}
print(json.dumps({"mode": mode_name, "launches_per_size": n, "sizes": rows, "fit_kernel_ms_median": fit}))
