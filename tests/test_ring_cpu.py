"""GEO_FLAG_RING_F64 in the oracle (CPU): the band is decided on the f32 ray
and its pixels are the f64 literal restatement's; every other pixel is the
plain f32 mirror's.  (The GPU side: tests/test_gpu_ring.py.)"""
import math

import numpy as np

import oracle as O
from helpers import default_frame, default_scene
from schwarzschild_raytracer_wgpu_amd import GeoScene, make_scene
from schwarzschild_raytracer_wgpu_amd._lib import GEO_FLAG_RING_F64, GEO_MODE_DIRECT, GEO_RING_X
from schwarzschild_raytracer_wgpu_amd.scenes import make_sky


def _ring(scene):
    s = GeoScene.from_buffer_copy(bytes(scene))
    s.flags |= GEO_FLAG_RING_F64
    return s


def test_ring_kx_is_the_impact_parameter_ratio():
    s = _ring(default_scene(64))
    sc = O.as_scene(s)
    kx = O.lib.geo_oracle_ring_kx(O._addr(sc))
    r, rs = float(np.float32(s.r_obs)), float(np.float32(s.rs))
    want = r / (math.sqrt(1.0 - rs / r) * 1.5 * math.sqrt(3.0) * rs)
    assert abs(kx - want) <= 1e-6 * want


def test_ring_band_follows_the_orbit_and_only_applies_outside_the_horizon():
    w, h = 240, 135
    frame = default_frame(w, h)
    band = O.ring_band(frame, _ring(default_scene(64)), w, h).astype(bool)
    assert 50 < band.sum() < band.size // 10
    assert O.ring_band(frame, default_scene(64), w, h).sum() == 0  # flag off
    for s in (make_scene(0.0, 50.0, 2.5, math.pi / 100, 64, GEO_MODE_DIRECT),
              make_scene(1.0, 50.0, 0.7, math.pi / 100, 64, GEO_MODE_DIRECT)):
        assert O.ring_band(frame, _ring(s), w, h).sum() == 0
    assert GEO_RING_X == 8e-3


def test_ring_render_is_f32_outside_and_f64_literal_inside():
    w, h = 240, 135
    sky = make_sky("equirect", (256, 128))
    frame = default_frame(w, h, camera=(math.pi + 0.2, 0.1))
    plain_scene = default_scene(2048)
    scene = _ring(plain_scene)
    band = O.ring_band(frame, scene, w, h).astype(bool)
    plain = O.render_f32(frame, plain_scene, sky, w, h, threads=8)
    ring = O.render_f32(frame, scene, sky, w, h, threads=8)
    lit = O.render_f64(frame, plain_scene, w, h, threads=8)
    out = ~band
    for f in ("rgba", "mask", "steps"):
        assert np.array_equal(ring[f][out], plain[f][out])
        assert np.array_equal(ring[f][band], lit[f][band]) if f != "rgba" else True
    assert np.array_equal(ring["uv"][out].view(np.uint32), plain["uv"][out].view(np.uint32))
    assert np.array_equal(ring["uv"][band].view(np.uint32), lit["uv"][band].view(np.uint32))
    assert ring["steps_total"] == plain["steps_total"]  # the f32 draw's count
    # the band is where the f32 draw is off the literal the most
    e = np.abs(plain["uv"].astype(np.float64) - lit["uv"].astype(np.float64)).max(axis=-1)
    sky_px = (plain["mask"] == 0) & (lit["mask"] == 0)
    assert e[sky_px & band].max() > e[sky_px & ~band].max() or e[sky_px & band].max() < 1e-4
