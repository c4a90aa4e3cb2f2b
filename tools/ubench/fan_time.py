#!/usr/bin/env python3
"""Time geo_solve_ray_fan (device only, stream-ordered) per fan: the default
scene's sky fan (rs 1, sphere 50, r 2.5), the reference's unscaled scene
(rs 10, sphere 500, r 25) and its planet/clouds spheres (r 1.1, 1.2 rs).
One JSON line; events around 200 back-to-back solves after a 200-solve
spin-up."""
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

import schwarzschild_raytracer_wgpu_amd as g  # noqa: E402
from schwarzschild_raytracer_wgpu_amd.timing import HipEvent  # noqa: E402

ctx = g.Context(0)
cases = {"sky r2.5": (50.0, 1.0, 1000, math.pi / 100, 400, math.sqrt(2.5 ** 2 + 0.01)),
         "ref r25": (500.0, 10.0, 1000, math.pi / 100, 400, 25.0),
         "planet": (1.1, 1.0, 1000, math.pi / 100, 400, math.sqrt(2.5 ** 2 + 0.01)),
         "clouds": (1.2, 1.0, 1000, math.pi / 100, 400, math.sqrt(2.5 ** 2 + 0.01))}
out = {}
for name, a in cases.items():
    for _ in range(200):
        ctx.solve_ray_fan(*a, host=False)
    e0, e1 = HipEvent(), HipEvent()
    e0.record()
    for _ in range(200):
        ctx.solve_ray_fan(*a, host=False)
    e1.record()
    torch.cuda.synchronize()
    out[name] = round(e0.elapsed_time(e1) / 200, 5)
print(json.dumps({"fan_ms": out, "lib": os.environ.get("FAN_LIB", "in-tree")}))
