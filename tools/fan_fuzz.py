"""Fuzz the f64 ray-fan kernel (geo_solve_ray_fan, scaled 14-op RK4 in
groups) against the oracle's literal f64 restatement of solve_ray_fan
(sphere_ray_tracer.rs:35-193) on random scenes: every node within one f32 ulp
(the stated bound), or reports the worst offenders.

    python tools/fan_fuzz.py [N] [SEED0]
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 500
    seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    import oracle as O
    import schwarzschild_raytracer_wgpu_amd as g

    ctx = g.Context(0)
    bad = 0
    worst = []
    for s in range(seed0, seed0 + n):
        rng = np.random.default_rng(s)
        rs = 0.0 if rng.random() < 0.1 else float(rng.uniform(0.2, 20.0))
        sphere_r = float(rng.uniform(1.05, 60.0) * (rs if rs > 0 else 1.0))
        r = float(rng.uniform(0.3, 1.5) * sphere_r) if rng.random() < 0.8 else float(rng.uniform(0.2, 3.0) * max(rs, 1.0))
        step = math.pi / 100 if rng.random() < 0.6 else float(rng.uniform(0.005, 0.1))
        nodes = int(rng.choice([2, 3, 17, 400, 400, 1024, 4096]))
        max_iter = int(rng.choice([1, 5, 100, 1000, 1000, 2000]))
        args = (sphere_r, rs, max_iter, step, nodes, r)
        gpu = ctx.solve_ray_fan(*args).astype(np.float64)
        ref = O.solve_ray_fan(*args)
        d = np.abs(gpu - ref)
        tol = np.spacing(np.abs(ref).astype(np.float32)).astype(np.float64)
        off = np.nonzero(d > tol)[0]
        if off.size:
            bad += 1
            i = int(off[np.argmax(d[off])])
            worst.append((s, args, int(off.size), i, float(gpu[i]), float(ref[i])))
    print(f"{n} fans, {bad} with nodes beyond one f32 ulp")
    for w in worst[:12]:
        print("  seed %d args %s: %d nodes, e.g. node %d gpu %.9g ref %.9g" % w)


if __name__ == "__main__":
    main()
