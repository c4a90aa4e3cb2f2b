"""N1: what the per-pixel integrator changes against the reference's display
path (the 400-node ray fan lerped per pixel, shader.wgsl:77-84), measured on
the f32 restatement (= the HIP output bit for bit): the black-hole mask
agrees except at the fan-lerp -7 crossing, and the sky UV differs where the
traveled angle varies faster than the fan resolves (the photon ring).  A
10x finer fan converges toward the per-pixel result.  CPU only."""
import math

import numpy as np

import oracle as O
from helpers import default_frame, default_scene, wrap_du
from schwarzschild_raytracer_wgpu_amd._lib import GEO_MODE_FAN
from schwarzschild_raytracer_wgpu_amd.scenes import make_sky


def _compare(n_fan, w=480, h=270):
    sky = make_sky("equirect", (256, 128))
    frame = default_frame(w, h)
    r = math.sqrt(2.5 ** 2 + 0.01)
    d = O.render_f32(frame, default_scene(2048), sky, w, h, threads=8)
    fan = O.solve_ray_fan(50.0, 1.0, 1000, math.pi / 100, n_fan, r)
    f = O.render_f32(frame, default_scene(1000, mode=GEO_MODE_FAN), sky, w, h, fan=fan, threads=8)
    both = (d["mask"] == 0) & (f["mask"] == 0)
    err = np.maximum(wrap_du(d["uv"][..., 0], f["uv"][..., 0]), np.abs(d["uv"][..., 1] - f["uv"][..., 1]))[both]
    return (d["mask"] == f["mask"]).mean(), err


def test_direct_vs_reference_fan():
    agree, err = _compare(400)
    assert agree > 0.9998
    assert np.median(err) < 1e-5           # most of the sky: the same pixel
    assert np.percentile(err, 99) < 5e-3   # the photon ring: the fan's lerp error
    agree10, err10 = _compare(4000)
    assert agree10 >= agree
    assert np.percentile(err10, 99) < np.percentile(err, 99) / 10
