#!/usr/bin/env python3
"""Dumps an accretion disk's state after a run of PointCloud updates with
orbits (respawns included: rs = 15 makes every particle fall) and a point
draw, so two builds of libgeo can be compared byte for byte (an A/B of two libraries).

  python tools/points_dump.py OUT.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch

    import schwarzschild_raytracer_wgpu_amd as g
    from helpers import default_frame
    from test_points import accretion_disk

    ctx = g.Context(0)
    out = {}
    # dt per frame: fixed, or changing (every third frame, then in runs), which
    # discards the orbit step run ahead
    for name, rs, n, seed, obs, dts in (("disk", 1.0, 3000, 4, (25.0, 0.0, 1.0), [1 / 60] * 120),
                                        ("falling", 15.0, 1000, 5, (40.0, 0.0, 1.0), [0.5] * 200),
                                        ("dt_changes", 15.0, 1000, 6, (40.0, 0.0, 1.0),
                                         [0.5 if f % 3 else 0.25 for f in range(60)] + [0.4] * 5 + [0.3] * 5),
                                        # a cloud past the fused update's size (geo_points.hip kFusedMaxConnectors)
                                        ("large", 15.0, 70000, 7, (40.0, 0.0, 1.0), [0.5] * 12)):
        pc = g.PointCloud(ctx, accretion_disk(n, seed=seed), rs, obs, True, True, seed=seed + 90)
        for f, dt in enumerate(dts):
            pc.update((obs[0], obs[1] + 0.01 * f, obs[2]), dt)
        w, h = 640, 360
        tgt = g.RenderTarget(w, h, torch.zeros(w * h * 4, dtype=torch.uint8, device="cuda:0"))
        xy = torch.empty((2 * n, 2), dtype=torch.int32, device="cuda:0")
        pc.draw(default_frame(w, h, pos=obs), tgt, out_xy=xy)
        torch.cuda.synchronize()
        out[name + "_near"] = pc.get_vertices(False)
        out[name + "_far"] = pc.get_vertices(True)
        out[name + "_pos"] = pc.positions()
        out[name + "_xy"] = xy.cpu().numpy()
        out[name + "_rgba"] = tgt.rgba.cpu().numpy()
    np.savez(sys.argv[1], **out)


if __name__ == "__main__":
    main()
