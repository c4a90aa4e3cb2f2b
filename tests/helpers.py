"""Shared scene helpers for the tests (default scene of SURVEY.md §8d)."""
import math

import numpy as np

from schwarzschild_raytracer_wgpu_amd import Observer, make_scene
from schwarzschild_raytracer_wgpu_amd._lib import GEO_MODE_DIRECT

POS = (2.5, 0.0, 0.1)
R_OBS = math.sqrt(POS[0] ** 2 + POS[1] ** 2 + POS[2] ** 2)


def default_frame(width, height, pos=POS, camera=(math.pi, 0.0), rs=1.0, fov=math.pi / 2, state=1, energy=1.0):
    o = Observer(rs, fov, width, height)
    o.set_position(*pos)
    o.set_camera(*camera)
    o.set_energy(energy)
    if state == 0:
        o.start_unmoving()
    else:
        o.start_frozen_fall()
    return o.calc_transformation_pipeline()


def default_scene(max_steps=2048, mode=GEO_MODE_DIRECT, rs=1.0, sphere_r=50.0, r_obs=R_OBS, step=math.pi / 100):
    return make_scene(rs, sphere_r, r_obs, step, max_steps, mode)


def wrap_du(a, b):
    d = np.abs(a.astype(np.float64) - b.astype(np.float64))
    return np.minimum(d, 1.0 - d)
