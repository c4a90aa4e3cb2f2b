"""Fuzz the RayConnector batch kernel (geo_rays_update) against the oracle's
f32 restatement (oracle/geo_oracle_points.c, the kernel's polynomials) on
random point sets, Schwarzschild radii, observer paths and iteration counts:
vertices bit for bit after every update.

    python tools/rays_fuzz.py [N] [SEED0]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    import torch

    import oracle as O
    import schwarzschild_raytracer_wgpu_amd as g

    ctx = g.Context(0)
    bad = []
    for s in range(seed0, seed0 + n):
        rng = np.random.default_rng(s)
        rs = float(rng.choice([0.5, 1.0, 1.0, 10.0]))
        npts = int(rng.choice([1, 7, 64, 1000, 3000]))
        d = rng.normal(size=(npts, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        pos = (d * rng.uniform(1.6, 40.0, size=(npts, 1)) * rs).astype(np.float32)
        sides = int(rng.choice([1, 2, 3]))
        hip = g.RayConnectors(ctx, rs, pos, sides=sides)
        ref = O.Rays(rs, pos, sides=sides, libm=False)
        for f in range(6):
            od = rng.normal(size=3)
            obs = (od / np.linalg.norm(od) * rng.uniform(1.3, 50.0) * rs).astype(np.float32)
            it = int(rng.choice([0, 1, 1, 3, 10]))
            reset = it == 0
            o = (hip.reset_ray(obs) if reset else hip.update_ray(obs, it))
            torch.cuda.synchronize()
            o = o.cpu().numpy()
            e = ref.update(obs, it, reset=reset)
            # bit for bit, except that any NaN equals any NaN (a failed
            # solve: the sign and payload of a NaN are not specified)
            diff = (o.view(np.uint32) != e.view(np.uint32)) & ~(np.isnan(o) & np.isnan(e))
            if diff.any():
                k = np.argwhere(diff)
                bad.append((s, f, rs, npts, sides, it, len(k), k[0].tolist(), o[k[0][0]].tolist(), e[k[0][0]].tolist()))
                break
    print(f"{n} point sets x 6 updates, {len(bad)} differ")
    for b in bad[:10]:
        print("  ", b)


if __name__ == "__main__":
    main()
