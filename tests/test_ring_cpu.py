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


def _skip_slack(frame, scene, w, h):
    """geo_render.hip ring_fork's tile-skip slack, restated (f64)."""
    f = np.frombuffer(bytes(frame), dtype=np.float32)
    m0 = f[:16]
    W, H = float(w), float(h)
    sx, ox, sy, oy = 2.0 / W, (1.0 - W) / W, -2.0 / H, (H - 1.0) / H
    A, B, C = [], [], []
    for i in range(3):  # geo_pixel.h camera_consts
        p = -float(m0[12]) * float(m0[i])
        q = -float(m0[13]) * float(m0[4 + i])
        r = float(m0[14]) * float(m0[8 + i])
        A.append(float(np.float32(sy * p)))
        B.append(float(np.float32(sx * q)))
        C.append(float(np.float32((oy * p + ox * q) + r)))
    A, B, C = np.array(A), np.array(B), np.array(C)
    n = np.cross(A, B)
    nn = float(np.linalg.norm(n))
    dist = abs(float(n @ C)) / nn if nn > 0 else 0.0
    D = 4.0 * (float(np.linalg.norm(A)) + float(np.linalg.norm(B)))
    k = abs(float(f[48]))
    sc = O.as_scene(scene)  # alive across the call
    kx = float(O.lib.geo_oracle_ring_kx(O._addr(sc)))
    if not (dist > 0 and D < dist and k < 1):
        return math.inf
    return kx * math.sqrt((1 + k) / (1 - k)) * math.asin(D / dist) * 1.01 + 1e-4


def test_ring_tile_skip_never_skips_a_band_pixel():
    """geo_ring_scan skips an 8 x 8 tile when its centre pixel's band test
    exceeds GEO_RING_X by the slack (a Lipschitz bound on the f32 ray's
    direction over 4 pixels).  On fuzz scenes and the default pose: every
    band pixel lies in a tile whose centre passes."""
    from fuzz_scenes import random_scene

    cases = [(default_frame(w, h, camera=cam), _ring(default_scene(64)), w, h)
             for (w, h) in [(240, 136), (480, 272)]
             for cam in [(math.pi, 0.0), (math.pi + 0.4, 0.3), (0.5, -0.2)]]
    for seed in range(60_000, 60_200):
        frame, scene, _ = random_scene(seed, 128, 72)
        cases.append((frame, _ring(scene), 128, 72))
    checked = 0
    for frame, scene, w, h in cases:
        if not (scene.rs > 0 and scene.r_obs > scene.rs):
            continue
        slack = _skip_slack(frame, scene, w, h)
        x = O.ring_x(frame, scene, w, h)
        tiles_x, tiles_y = w // 8, h // 8  # whole tiles (their centres inside the frame)
        xt = x[: tiles_y * 8, : tiles_x * 8].reshape(tiles_y, 8, tiles_x, 8)
        centre = xt[:, 4, :, 4]
        has_band = (xt < GEO_RING_X).any(axis=(1, 3))
        passes = ~(centre >= GEO_RING_X + slack)
        assert not (has_band & ~passes).any(), (w, h, slack)
        checked += int(has_band.sum())
    assert checked > 1000
