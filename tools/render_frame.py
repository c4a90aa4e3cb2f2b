#!/usr/bin/env python3
"""Render the reference's scene (SR/lib.rs:62-94: sky sphere, planet sphere,
translucent cloud sphere, accretion disk) on the GPU and save it as PNG/PPM —
the present step of the absent wgpu_renderer loop.

  python tools/render_frame.py out.png [--width 1920 --height 1080]
        [--sky eso0932a.jpg --planet world_8k.png --clouds transparent_clouds.png]
        [--frames 60 --orbit 3.2] [--mipmaps] [--fan]

Without texture files the synthetic equirect sky of the benchmarks is used for
the sky sphere and the planet/cloud spheres are skipped.  Units: rs = 1 (the
reference's rs = 10 scene divided by 10).
"""
from __future__ import annotations

import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("out")
    p.add_argument("--width", type=int, default=1920)
    p.add_argument("--height", type=int, default=1080)
    p.add_argument("--sky")
    p.add_argument("--planet")
    p.add_argument("--clouds")
    p.add_argument("--frames", type=int, default=1, help="frames of motion before the saved one (dt = 1/60 s)")
    p.add_argument("--orbit", type=float, default=0.0, help="start an orbit with this rotation (observer.rs:162)")
    p.add_argument("--no-disk", action="store_true")
    p.add_argument("--mipmaps", action="store_true", help="trilinear mip-mapped textures, as the reference samples them")
    p.add_argument("--fan", action="store_true",
                   help="the reference's display path: per-frame 400-node f64 ray fans and the fan lerp "
                        "(GEO_MODE_FAN) instead of a geodesic per pixel")
    args = p.parse_args()

    import torch

    import schwarzschild_raytracer_wgpu_amd as g
    from schwarzschild_raytracer_wgpu_amd import imageio
    from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

    w, h = args.width, args.height
    obs = g.Observer(1.0, math.pi / 2, w, h)
    obs.set_position(2.5, 0.0, 0.1)
    if args.orbit:
        obs.start_orbit(args.orbit)
    sky = imageio.load_texture(args.sky) if args.sky else make_sky("equirect", (4096, 2048))
    mode = g.GEO_MODE_FAN if args.fan else g.GEO_MODE_DIRECT
    spheres = [g.BasicSphereBuffer(0, 50.0, 1.0, sky, mode=mode, mipmaps=args.mipmaps)]
    if args.planet:
        spheres.append(g.BasicSphereBuffer(0, 1.1, 1.0, imageio.load_texture(args.planet), mode=mode,
                                           mipmaps=args.mipmaps))
    if args.clouds:
        spheres.append(g.BasicSphereBuffer(0, 1.2, 1.0, imageio.load_texture(args.clouds), mode=mode,
                                           mipmaps=args.mipmaps))
    disk = None if args.no_disk else g.PointCloud.new_accretion_disk(spheres[0].ctx, 1.0, obs.get_position(), True)
    tgt = g.RenderTarget(w, h, torch.empty(w * h * 4, dtype=torch.uint8, device="cuda:0"))
    renderer = g.Renderer(obs)
    for _ in range(args.frames):
        obs.update_position((0.0, 0.0, 0.0), 1 / 60)
        r = obs.get_radial_position()
        for s in spheres:
            s.update_ray_fan(r)
        if disk is not None:
            disk.update(obs.get_position(), 1 / 60)
        renderer.render(spheres, tgt, point_clouds=[disk] if disk is not None else [])
    if args.out.endswith(".ppm"):
        imageio.save_ppm(args.out, tgt.rgba, w, h)
    else:
        imageio.save_png(args.out, tgt.rgba, w, h)
    print(f"wrote {args.out} ({w}x{h}, {len(spheres)} sphere(s){', accretion disk' if disk else ''}, "
          f"{'fan lerp' if args.fan else 'per-pixel geodesics'})")


if __name__ == "__main__":
    main()
