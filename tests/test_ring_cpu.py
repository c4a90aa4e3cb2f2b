"""GEO_FLAG_RING_F64 on the CPU: the band is decided on the f32 ray; its
pixels take lambda' and the mask from the f64 path (geo_band.h; the oracle's
own restatement, band_lambda) and the sky from the f32 ray; every other
pixel is the plain f32 mirror's.  The host build of geo_band.h
(libgeo_cpu.so) equals the oracle bit for bit, and the band matches the f64
literal's mask and steps.  (The GPU side: tests/test_gpu_ring.py.)"""
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
    assert GEO_RING_X == 5e-3


def test_ring_render_is_f32_outside_and_f64_inside():
    w, h = 240, 135
    sky = make_sky("equirect", (256, 128))
    frame = default_frame(w, h, camera=(math.pi + 0.2, 0.1))
    plain_scene = default_scene(2048)
    scene = _ring(plain_scene)
    band = O.ring_band(frame, scene, w, h).astype(bool)
    assert band.sum() > 50
    plain = O.render_f32(frame, plain_scene, sky, w, h, threads=8)
    ring = O.render_f32(frame, scene, sky, w, h, threads=8)
    lit = O.render_f64(frame, plain_scene, w, h, threads=8)
    out = ~band
    for f in ("rgba", "mask", "steps"):
        assert np.array_equal(ring[f][out], plain[f][out])
    assert np.array_equal(ring["uv"][out].view(np.uint32), plain["uv"][out].view(np.uint32))
    # the band: the f64 literal's mask and steps; the UV within the f32 sky map's roundings of it
    assert np.array_equal(ring["mask"][band], lit["mask"][band])
    assert np.array_equal(ring["steps"][band], lit["steps"][band])
    sky_px = (ring["mask"] == 0) & band
    du = np.abs(ring["uv"][sky_px].astype(np.float64) - lit["uv"][sky_px])
    du[:, 0] = np.minimum(du[:, 0], 1.0 - du[:, 0])
    assert du.max() < 2e-6
    # steps_total counts what each pixel reports
    assert ring["steps_total"] == int(ring["steps"].astype(np.int64).sum())
    # the band is where the f32 draw is off the literal the most
    e = np.abs(plain["uv"].astype(np.float64) - lit["uv"].astype(np.float64)).max(axis=-1)
    s_px = (plain["mask"] == 0) & (lit["mask"] == 0)
    assert e[s_px & band].max() > e[s_px & ~band].max() or e[s_px & band].max() < 1e-4


def test_ring_host_header_equals_the_oracle():
    """geo_band.h compiled for the host (libgeo_cpu.so, the CPU baseline) ==
    the oracle's independent restatement, bit for bit, on the default pose
    and fuzz scenes (direct and adaptive modes)."""
    from fuzz_scenes import random_scene
    from test_cpu_baseline import render_cpu, same

    import ctypes
    from test_cpu_baseline import LIB

    lib = ctypes.CDLL(LIB)
    vp, u32 = ctypes.c_void_p, ctypes.c_uint32
    lib.geo_render_cpu.restype = ctypes.c_int
    lib.geo_render_cpu.argtypes = [vp, vp, vp, u32, u32, vp, u32, u32, u32, u32, u32, u32, ctypes.c_int, vp, vp, vp,
                                   vp, vp]
    sky = make_sky("equirect", (256, 128))
    cases = [(default_frame(240, 135, camera=cam), _ring(default_scene(2048)), 240, 135)
             for cam in [(math.pi, 0.0), (math.pi + 0.3, 0.2)]]
    for seed in range(40_000, 40_120):
        frame, scene, _ = random_scene(seed, 96, 54)
        if scene.mode != 1:  # not the fan mode
            cases.append((frame, _ring(scene), 96, 54))
    seen = 0
    for frame, scene, w, h in cases:
        rc, c = render_cpu(lib, frame, scene, sky, w, h, threads=8)
        assert rc == 0
        o = O.render_f32(frame, scene, sky, w, h, threads=8)
        assert same(c, o) and c["total"] == o["steps_total"]
        seen += int(O.ring_band(frame, scene, w, h).any())
    assert seen > 20
