"""Generates the committed golden fixtures of tests/golden/ from the oracle.

The reference itself cannot run here (Rust/WGSL, no toolchain), so these
vectors are the oracle's own outputs, committed to pin it against regressions
(the analytic KATs in tests/test_oracle_kat.py pin it against physics).
Re-run only on purpose:  python tests/golden/make_golden.py
"""
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import oracle as O  # noqa: E402
from helpers import default_scene  # noqa: E402
from schwarzschild_raytracer_wgpu_amd import make_scene  # noqa: E402
from schwarzschild_raytracer_wgpu_amd._lib import GEO_MODE_ADAPTIVE, GEO_MODE_FAN  # noqa: E402
from schwarzschild_raytracer_wgpu_amd.scenes import make_sky  # noqa: E402

STEP = math.pi / 100


def oracle_frame(w, h, pos=(2.5, 0.0, 0.1), cam=(math.pi, 0.0), state=1):
    return O.observer_frame(1.0, math.pi / 2, w, h, pos, cam[0], cam[1], state, 1.0)


def main():
    # reference default scene fan (basic_sphere_buffer.rs:42-51, lib.rs:72, renderer.rs:83, observer.rs:70)
    fan_ref = O.solve_ray_fan(500.0, 10.0, 1000, STEP, 400, math.sqrt(25.0 ** 2 + 1.0))
    # reference's own smoke case (tests.rs:8-13): SphereRayTracer::new(100, 10, 100, PI/100, 10).solve_ray_fan(25)
    fan_test = O.solve_ray_fan(100.0, 10.0, 100, STEP, 20, 25.0)
    # per-theta traveled angles and step counts, rs=1 sphere 50 r=2.5
    thetas = np.linspace(-math.pi / 2, math.pi / 2, 257)
    ang = np.empty_like(thetas)
    st = np.empty(thetas.shape, np.uint32)
    for i, t in enumerate(thetas):
        ang[i], st[i] = O.geodesic_at_theta(50.0, 1.0, 2048, STEP, 2.5, float(t))
    # configs' observer radii (rs = 1): configs 1-4 at |(2.5, 0, 0.1)|, config 5 at 1.3 (inside the photon sphere)
    fan_cfg = O.solve_ray_fan(50.0, 1.0, 1000, STEP, 400, math.sqrt(2.5 ** 2 + 0.1 ** 2))
    fan_cfg5 = O.solve_ray_fan(50.0, 1.0, 1000, STEP, 400, 1.3)
    np.savez(os.path.join(HERE, "fans.npz"), fan_ref=fan_ref, fan_test=fan_test, thetas=thetas,
             angles=ang, steps=st, fan_cfg=fan_cfg, fan_cfg5=fan_cfg5)

    w, h = 64, 36
    frame = oracle_frame(w, h)
    sc = default_scene(2048)
    p64 = O.render_f64(frame, sc, w, h, threads=4)
    sky = make_sky("equirect", (64, 32))
    p32 = O.render_f32(frame, sc, sky, w, h, threads=4)
    fan = O.solve_ray_fan(50.0, 1.0, 1000, STEP, 400, math.sqrt(2.5 ** 2 + 0.1 ** 2))
    scf = default_scene(1000, mode=GEO_MODE_FAN)
    f32fan = O.render_f32(frame, scf, sky, w, h, fan=fan, threads=4)
    np.savez(os.path.join(HERE, "pixels_64x36.npz"),
             frame=np.frombuffer(bytes(frame), dtype=np.float32),
             sky=sky,
             f64_mask=p64["mask"], f64_uv=p64["uv"], f64_steps=p64["steps"], f64_lam=p64["lam"],
             f32_rgba=p32["rgba"], f32_mask=p32["mask"], f32_uv=p32["uv"], f32_steps=p32["steps"],
             fan=fan, fan_rgba=f32fan["rgba"], fan_mask=f32fan["mask"], fan_uv=f32fan["uv"])
    adaptive()
    print("wrote", os.listdir(HERE))


def adaptive():
    """Config 5 at 64x36: GEO_MODE_ADAPTIVE (f32 kernel order) and its f64
    check (fixed RK4 at step/32)."""
    w, h = 64, 36
    frame = oracle_frame(w, h, pos=(1.2, 0.5, 0.0), cam=(math.pi + 0.6, 0.3))
    sc = make_scene(1.0, 50.0, 1.3, STEP, 2048, GEO_MODE_ADAPTIVE, tol=1e-6)
    sky = make_sky("equirect", (64, 32))
    p32 = O.render_f32(frame, sc, sky, w, h, threads=4)
    p64 = O.render_f64(frame, sc, w, h, threads=4)
    np.savez(os.path.join(HERE, "adaptive_64x36.npz"),
             frame=np.frombuffer(bytes(frame), dtype=np.float32), sky=sky,
             f32_rgba=p32["rgba"], f32_mask=p32["mask"], f32_uv=p32["uv"], f32_steps=p32["steps"],
             f64_mask=p64["mask"], f64_uv=p64["uv"])


if __name__ == "__main__":
    main()
