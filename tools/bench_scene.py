#!/usr/bin/env python3
"""The reference's whole frame on one GPU (SR/lib.rs:62-94, 413-419,
renderer.rs:208-264).  The reference builds three spheres -- sky (r 50),
planet (r 1.1) and translucent clouds (r 1.2) -- but draws only the sky:
lib.rs:415 passes `&[&self.first_sphere/*, &self.second_sphere ,
&self.third_sphere*/]`.  --spheres 1 (default) is that frame: the sky's
per-pixel geodesic draw, then the accretion disk (PointCloud::update with f64
orbits and both RayConnector sides, then the near and far point draws).
--spheres 3 adds the commented-out planet and clouds, composited in order.
One JSON line: ms per frame (wall, K frames back to back), frames/s, and
each part's GPU time from event pairs (parts back to back on one stream).
--overlap 1 (default) puts the disk update on a side stream: it is
latency-bound (10 000 lanes of sequential 48-node solves) and hides under the
VALU-bound sky draw; the point draw waits for it (geo_points_draw).

--mode fan draws every sphere the way the reference displays it: each frame
solves the sphere's 400-node f64 ray fan (geo_solve_ray_fan, SphereRayTracer::
solve_ray_fan, lib.rs:292-295) and the sky lerps into it per pixel
(shader.wgsl:77-84); with --overlap 1 the fans go on side streams and
overlap the previous frame's draws.  --mode direct (default) integrates every
pixel.

  python tools/bench_scene.py [--width 3840 --height 2160] [--frames 200] [--points 5000] [--spheres 1|3] [--overlap 1|0] [--mode direct|fan]

Textures are synthetic (the reference's are absent): the benchmark equirect
sky, a 2048x1024 checkerboard planet and a seeded random-alpha cloud layer.
Units: rs = 1 (the reference's rs = 10 scene divided by 10), observer
FrozenFall from (2.5, 0, 0.1), moving with the reference's controls idle.
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--width", type=int, default=3840)
    p.add_argument("--height", type=int, default=2160)
    p.add_argument("--frames", type=int, default=200)
    p.add_argument("--warmup", type=int, default=100)
    p.add_argument("--points", type=int, default=5000)
    p.add_argument("--max-steps", type=int, default=1000, help="per sphere (basic_sphere_buffer.rs:42-51)")
    p.add_argument("--spheres", type=int, default=1, choices=[1, 3],
                   help="1: the sky only, as the reference draws (lib.rs:415); 3: with planet and clouds")
    p.add_argument("--overlap", type=int, default=1, choices=[0, 1],
                   help="1: the disk update on a side stream, overlapping the sphere draws (geo_points_draw "
                        "orders the point draw after it); 0: everything on one stream")
    p.add_argument("--mode", default="direct", choices=["direct", "fan"],
                   help="direct: per-pixel geodesics; fan: the reference's per-frame 400-node fan + per-pixel lerp")
    args = p.parse_args()

    import numpy as np
    import torch

    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky
    from schwarzschild_raytracer_wgpu_amd.timing import HipEvent

    w, h = args.width, args.height
    obs = g.Observer(1.0, math.pi / 2, w, h)
    obs.set_position(2.5, 0.0, 0.1)
    sky = make_sky("equirect", (4096, 2048))
    planet = make_sky("equirect", (2048, 1024), seed=7)
    clouds = np.random.default_rng(11).integers(0, 256, size=(1024, 2048, 4), dtype=np.uint8)
    mode = g.GEO_MODE_FAN if args.mode == "fan" else g.GEO_MODE_DIRECT
    spheres = [g.BasicSphereBuffer(0, 50.0, 1.0, sky, max_iter=args.max_steps, mode=mode),
               g.BasicSphereBuffer(0, 1.1, 1.0, planet, max_iter=args.max_steps, mode=mode),
               g.BasicSphereBuffer(0, 1.2, 1.0, clouds, max_iter=args.max_steps, mode=mode)][:args.spheres]
    disk = g.PointCloud.new_accretion_disk(spheres[0].ctx, 1.0, obs.get_position(), True, n=args.points)
    tgt = g.RenderTarget(w, h, torch.empty(w * h * 4, dtype=torch.uint8, device="cuda:0"))

    parts = ("disk update", "sky", "planet", "clouds")[:2 + len(spheres) - 1] + ("points",)
    side = torch.cuda.Stream() if args.overlap else None

    # fan mode with --overlap 1: the spheres' fans (latency-bound, one lane per
    # node, 7 waves) solved on one side stream each; the context double-buffers
    # its fan and orders solves and draws with events, so frame i's fans
    # overlap frame i-1's draws and the draws still read their own frame's fan
    fan_streams = [torch.cuda.Stream() for _ in spheres] if (args.mode == "fan" and args.overlap) else None

    def frame(evs=None):
        obs.update_position((0.0, 0.0, 0.0), 1 / 60)
        r = obs.get_radial_position()
        for i, s in enumerate(spheres):  # fan mode: the fan on the device; direct: records r
            s.update_ray_fan(r, stream=fan_streams[i] if (fan_streams and not evs) else None)
        f = obs.calc_transformation_pipeline()
        if evs:  # per-part timing: the parts back to back on one stream (fan mode: the fans lie before
            evs[0].record()  # evs[0], in no part's time)
            disk.update(obs.get_position(), 1 / 60)
            evs[1].record()
        else:
            disk.update(obs.get_position(), 1 / 60, stream=side)
        for i, s in enumerate(spheres):
            s.draw(f, tgt, composite=i > 0)
            if evs:
                evs[2 + i].record()
        disk.draw(f, tgt)
        if evs:
            evs[2 + len(spheres)].record()

    for _ in range(args.warmup):
        frame()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.frames):
        frame()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / args.frames
    # per-part GPU time on separate frames with event pairs
    acc = np.zeros(len(parts))
    nev = 20
    for _ in range(nev):
        evs = [HipEvent() for _ in range(len(parts) + 1)]
        frame(evs)
        torch.cuda.synchronize()
        acc += [evs[i].elapsed_time(evs[i + 1]) for i in range(len(parts))]
    acc /= nev
    print(json.dumps({
        "what": ("the reference's frame as drawn (lib.rs:415): the sky's per-pixel geodesic draw + accretion disk "
                 "(orbits, 2 x RayConnector, point draws)" if len(spheres) == 1 else
                 "the reference's frame with its commented-out planet and clouds: 3 composited per-pixel geodesic "
                 "spheres + accretion disk (orbits, 2 x RayConnector, point draws)"),
        "mode": args.mode,
        "spheres": len(spheres),
        "overlap": bool(args.overlap),
        "width": w, "height": h, "frames": args.frames, "points": args.points, "max_steps": args.max_steps,
        "ms_per_frame": wall * 1e3, "frames_per_s": 1.0 / wall,
        "gpu_ms": {k: float(v) for k, v in zip(parts, acc)},
        "data": "synthetic textures (sky 4096x2048, planet 2048x1024, random-alpha clouds 2048x1024)",
    }), flush=True)


if __name__ == "__main__":
    main()
