"""The kernel's per-pixel header (geo_pixel.h), compiled for the HOST with the
same no-contraction rules, must equal the oracle's independent f32
restatement bit for bit.  CPU only: catches restatement/restructuring bugs
before the GPU parity tests (which run the same sequence on gfx950)."""
import ctypes
import math
import os
import subprocess

import numpy as np
import pytest

import oracle as O
from helpers import default_frame, default_scene
from schwarzschild_raytracer_wgpu_amd._lib import GEO_MODE_FAN
from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "pixel_host.cpp")
SO = os.path.join(HERE, "native", "libpixel_host.so")


@pytest.fixture(scope="module")
def host():
    deps = [SRC] + [os.path.join(HERE, "..", "schwarzschild_raytracer_wgpu_amd", "csrc", h)
                    for h in ("geo_pixel.h", "geo_math.h")]
    if not os.path.exists(SO) or any(os.path.getmtime(d) > os.path.getmtime(SO) for d in deps):
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-mfma", "-msse4.1",
                        "-o", SO, SRC], check=True)
    lib = ctypes.CDLL(SO)
    lib.host_render.restype = ctypes.c_int
    return lib


def run_host(lib, frame, scene, sky, w, h, fan=None, variant=2, target=None):
    fr, sc = O.as_frame(frame), O.as_scene(scene)
    sky = np.ascontiguousarray(sky)
    fan_a = np.ascontiguousarray(fan, np.float32) if fan is not None else None
    rgba = np.zeros((h, w, 4), np.uint8) if target is None else np.array(target, np.uint8)
    mask = np.empty((h, w), np.uint8)
    uv = np.empty((h, w, 2), np.float32)
    steps = np.empty((h, w), np.uint32)
    vp = ctypes.c_void_p
    lib.host_render(ctypes.byref(fr), ctypes.byref(sc), vp(fan_a.ctypes.data if fan_a is not None else 0),
                    ctypes.c_uint32(0 if fan_a is None else fan_a.size), vp(sky.ctypes.data),
                    ctypes.c_uint32(sky.shape[1]), ctypes.c_uint32(sky.shape[0]), ctypes.c_uint32(w),
                    ctypes.c_uint32(h), ctypes.c_uint32(0), ctypes.c_uint32(h), vp(rgba.ctypes.data),
                    vp(mask.ctypes.data), vp(uv.ctypes.data), vp(steps.ctypes.data), ctypes.c_int(variant))
    return dict(rgba=rgba, mask=mask, uv=uv, steps=steps)


CASES = [
    ("default_16x9", 160, 90, {}, dict(max_steps=2048)),
    ("budget_128", 128, 128, {}, dict(max_steps=128)),
    ("budget_odd_37", 96, 54, {}, dict(max_steps=37)),
    ("budget_1", 64, 36, {}, dict(max_steps=1)),
    ("budget_0", 32, 18, {}, dict(max_steps=0)),
    ("unmoving", 96, 54, dict(state=0), dict(max_steps=512)),
    ("inside_photon_sphere", 96, 54, dict(pos=(1.3, 0.2, 0.05), camera=(math.pi + 0.6, 0.3)),
     dict(r_obs=math.sqrt(1.3 ** 2 + 0.2 ** 2 + 0.05 ** 2))),
    ("inside_horizon", 64, 64, dict(pos=(0.8, 0.0, 0.05)), dict(r_obs=math.sqrt(0.64 + 0.0025))),
    ("flat_space", 64, 36, dict(rs=0.0, state=0), dict(rs=0.0)),
    ("outside_sphere", 64, 36, dict(pos=(60.0, 0.0, 1.0)), dict(r_obs=math.sqrt(3601.0))),
    # the one-test-per-group loop (absorbing stop set) right at its limit, SU = 1.5/1.51 < 1,
    # and the per-step loop with the sphere inside the photon sphere (SU = 1.5/1.4 > 1)
    ("sphere_just_beyond_photon_sphere", 96, 54, dict(pos=(1.2, 0.3, 0.05), camera=(math.pi + 0.4, 0.2)),
     dict(sphere_r=1.51, r_obs=math.sqrt(1.44 + 0.09 + 0.0025))),
    ("sphere_1p6_observer_near_it", 96, 54, dict(pos=(1.55, 0.1, 0.0), camera=(0.3, 0.1)),
     dict(sphere_r=1.6, r_obs=math.sqrt(1.55 ** 2 + 0.01))),
    ("sphere_inside_photon_sphere", 96, 54, dict(pos=(1.2, 0.0, 0.05), camera=(math.pi + 1.0, 0.0)),
     dict(sphere_r=1.4, r_obs=math.sqrt(1.44 + 0.0025))),
]


@pytest.mark.parametrize("variant", [1, 2, 3, 4])
@pytest.mark.parametrize("name,w,h,fk,sk", CASES, ids=[c[0] for c in CASES])
def test_host_header_equals_oracle(host, name, w, h, fk, sk, variant):
    """Every RK4 loop structure of geo_pixel.h (G = 1..4 steps per exit test) equals the literal loop."""
    sky = make_sky("equirect", (128, 64))
    frame, scene = default_frame(w, h, **fk), default_scene(**sk)
    a = run_host(host, frame, scene, sky, w, h, variant=variant)
    b = O.render_f32(frame, scene, sky, w, h, threads=4)
    for f in ("mask", "steps", "rgba"):
        assert np.array_equal(a[f], b[f]), (f, np.argwhere(a[f] != b[f])[:5])
    assert np.array_equal(a["uv"].view(np.uint32), b["uv"].view(np.uint32))


def test_host_header_fan_mode(host):
    sky = make_sky("equirect", (128, 64))
    w, h = 96, 54
    fan = O.solve_ray_fan(50.0, 1.0, 1000, math.pi / 100, 400, math.sqrt(2.5 ** 2 + 0.01))
    frame, scene = default_frame(w, h), default_scene(1000, mode=GEO_MODE_FAN)
    a = run_host(host, frame, scene, sky, w, h, fan=fan)
    b = O.render_f32(frame, scene, sky, w, h, fan=fan, threads=4)
    for f in ("mask", "rgba"):
        assert np.array_equal(a[f], b[f])
    assert np.array_equal(a["uv"].view(np.uint32), b["uv"].view(np.uint32))


def test_host_header_translucent_sky(host):
    """Sky with alpha < 255: the alpha blend over the clear colour (rgb*a/255)."""
    rng = np.random.default_rng(7)
    sky = rng.integers(0, 256, size=(64, 128, 4), dtype=np.uint8)
    w, h = 96, 54
    frame, scene = default_frame(w, h), default_scene(512)
    a = run_host(host, frame, scene, sky, w, h)
    b = O.render_f32(frame, scene, sky, w, h, threads=4)
    assert np.array_equal(a["rgba"], b["rgba"])
    assert np.all(b["rgba"][..., 3] == 255)


ADAPTIVE_CASES = [
    ("default", 160, 90, {}, dict(max_steps=2048)),
    ("cfg5_inside_photon_sphere", 160, 90, dict(pos=(1.2, 0.5, 0.0), camera=(math.pi + 0.6, 0.3)),
     dict(r_obs=1.3)),
    ("budget_5", 96, 54, {}, dict(max_steps=5)),
    ("budget_0", 32, 18, {}, dict(max_steps=0)),
    ("tol_1e-9", 96, 54, {}, dict(tol=1e-9)),
    ("tol_1e-3", 96, 54, {}, dict(tol=1e-3)),
    ("inside_horizon", 64, 64, dict(pos=(0.8, 0.0, 0.05)), dict(r_obs=math.sqrt(0.64 + 0.0025))),
    ("flat_space", 64, 36, dict(rs=0.0, state=0), dict(rs=0.0)),
    ("outside_sphere", 64, 36, dict(pos=(60.0, 0.0, 1.0)), dict(r_obs=math.sqrt(3601.0))),
]


@pytest.mark.parametrize("name,w,h,fk,sk", ADAPTIVE_CASES, ids=[c[0] for c in ADAPTIVE_CASES])
def test_host_header_adaptive_equals_oracle(host, name, w, h, fk, sk):
    """GEO_MODE_ADAPTIVE: the header's DP5(4) loop equals the oracle's literal adaptive loop."""
    from schwarzschild_raytracer_wgpu_amd import make_scene
    from schwarzschild_raytracer_wgpu_amd._lib import GEO_MODE_ADAPTIVE

    sky = make_sky("equirect", (128, 64))
    p = dict(rs=1.0, r_obs=math.sqrt(2.5 ** 2 + 0.01), max_steps=2048, tol=0.0)
    p.update(sk)
    frame = default_frame(w, h, **fk)
    scene = make_scene(p["rs"], 50.0, p["r_obs"], math.pi / 100, p["max_steps"], GEO_MODE_ADAPTIVE, tol=p["tol"])
    a = run_host(host, frame, scene, sky, w, h)
    b = O.render_f32(frame, scene, sky, w, h, threads=4)
    for f in ("mask", "steps", "rgba"):
        assert np.array_equal(a[f], b[f]), (f, np.argwhere(a[f] != b[f])[:5])
    assert np.array_equal(a["uv"].view(np.uint32), b["uv"].view(np.uint32))


def three_spheres(w, h):
    """The reference's frame (lib.rs:62-89): sky sphere r = 50 (opaque), a
    planet sphere r = 1.1 (opaque) and a cloud sphere r = 1.2 (translucent),
    drawn in that order with alpha blending (rs = 1 units)."""
    from schwarzschild_raytracer_wgpu_amd import make_scene
    from schwarzschild_raytracer_wgpu_amd._lib import GEO_FLAG_COMPOSITE

    rng = np.random.default_rng(12)
    planet = make_sky("equirect", (96, 48), seed=0x1234)
    clouds = rng.integers(0, 256, size=(40, 80, 4), dtype=np.uint8)
    clouds[..., 3] = (clouds[..., 3] // 2)  # alpha <= 127
    frame = default_frame(w, h, pos=(2.5, 0.0, 0.1))
    r = math.sqrt(2.5 ** 2 + 0.01)
    passes = [(make_scene(1.0, 50.0, r, math.pi / 100, 2048), make_sky("equirect", (128, 64))),
              (make_scene(1.0, 1.1, r, math.pi / 100, 2048, flags=GEO_FLAG_COMPOSITE), planet),
              (make_scene(1.0, 1.2, r, math.pi / 100, 2048, flags=GEO_FLAG_COMPOSITE), clouds)]
    return frame, passes


def test_host_header_composite_three_spheres(host):
    """GEO_FLAG_COMPOSITE: the reference's three-sphere frame; every pass equals the oracle's."""
    w, h = 128, 72
    frame, passes = three_spheres(w, h)
    a = b = None
    for scene, sky in passes:
        a = run_host(host, frame, scene, sky, w, h, target=None if a is None else a["rgba"])
        b = O.render_f32(frame, scene, sky, w, h, threads=4, target=None if b is None else b["rgba"])
        assert np.array_equal(a["rgba"], b["rgba"])
    # the cloud pass changed pixels where the cloud sphere is hit, and only there
    assert 0 < (b["mask"] == 0).sum() < w * h


def test_composite_over_clear_equals_plain_draw():
    """A sphere composited over the cleared target (0,0,0,255) equals the plain draw."""
    from schwarzschild_raytracer_wgpu_amd import make_scene
    from schwarzschild_raytracer_wgpu_amd._lib import GEO_FLAG_COMPOSITE

    w, h = 96, 54
    rng = np.random.default_rng(3)
    sky = rng.integers(0, 256, size=(64, 128, 4), dtype=np.uint8)
    frame = default_frame(w, h)
    r = math.sqrt(2.5 ** 2 + 0.01)
    plain = O.render_f32(frame, make_scene(1.0, 50.0, r, math.pi / 100, 512), sky, w, h)
    clear = np.zeros((h, w, 4), np.uint8)
    clear[..., 3] = 255
    comp = O.render_f32(frame, make_scene(1.0, 50.0, r, math.pi / 100, 512, flags=GEO_FLAG_COMPOSITE), sky, w, h,
                        target=clear)
    assert np.array_equal(plain["rgba"], comp["rgba"])


@pytest.mark.parametrize("sw,sh", [(1, 1), (2, 1), (7, 5), (64, 32), (513, 257)])
def test_padded_sky_quad_equals_wrap_clamp(host, sw, sh):
    """The device's sky sampling reads a padded copy (geo::pad_sky, 2 x 2 block
    at (ix0 + 1, iy0 + 1); level 0 as its row pairs, geo::pair_sky_rows, one
    16-byte quad); it must sample exactly what the wrap/clamp quad on
    the unpadded texture does: random (U, V), the edges and corners, and the
    texel centres next to them."""
    rng = np.random.default_rng(sw * 1000 + sh)
    sky = rng.integers(0, 2**32, size=(sh, sw), dtype=np.uint64).astype(np.uint32)
    edge = np.array([0.0, 1.0, 0.5 / sw, 1 - 0.5 / sw, 1e-7, 1 - 1e-7, 0.5, np.nextafter(1.0, 0.0)], np.float32)
    U = np.concatenate([rng.random(4000, dtype=np.float32), np.repeat(edge, edge.size)]).astype(np.float32)
    V = np.concatenate([rng.random(4000, dtype=np.float32), np.tile(edge, edge.size)]).astype(np.float32)
    a = np.empty(U.size, np.uint32)
    b = np.empty(U.size, np.uint32)
    c = np.empty(U.size, np.uint32)
    vp = ctypes.c_void_p
    host.host_sample_padded(vp(sky.ctypes.data), ctypes.c_uint32(sw), ctypes.c_uint32(sh), vp(U.ctypes.data),
                            vp(V.ctypes.data), ctypes.c_uint32(U.size), vp(a.ctypes.data), vp(b.ctypes.data),
                            vp(c.ctypes.data))
    assert np.array_equal(a, b)
    assert np.array_equal(a, c)  # the row-pair copy the device reads (geo::pair_sky_rows)


def test_host_transcendentals_equal_oracle(host):
    """geo_math.h's sincosf_ (quadrant and rint by the 1.5 * 2^23 shifter) and
    asinf_ (|x| clamped by fminf) host-compiled equal the oracle's
    restatement (rintf, fminf) bit for bit: random and huge arguments,
    x * 2/pi at and next to half-integers (the rounding ties), |x| > 1 and
    NaN for asin (NaN -> +-pi/2 by its sign bit)."""
    rng = np.random.default_rng(7)
    two_over_pi = np.float32(0.636619772367581343076)
    ties = []
    for k in range(-600, 600):
        t = np.float32(k + 0.5)
        # arguments whose rounded product with 2/pi lands on, just below and just above k + 1/2
        x0 = np.float32(t / two_over_pi)
        for x in (x0, np.nextafter(x0, np.float32(np.inf)), np.nextafter(x0, np.float32(-np.inf))):
            ties.append(x)
    xs = np.concatenate([rng.uniform(-10, 10, 20000), rng.uniform(-1.2, 1.2, 20000), rng.uniform(-9000, 9000, 5000),
                         np.array(ties, np.float64), [0.0, -0.0, 1.0, -1.0, 1.5, -1.5, np.nan, -np.nan]]
                        ).astype(np.float32)
    n = xs.size
    s, c, a = (np.empty(n, np.float32) for _ in range(3))
    host.host_math(xs.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(n), s.ctypes.data_as(ctypes.c_void_p),
                   c.ctypes.data_as(ctypes.c_void_p), a.ctypes.data_as(ctypes.c_void_p))
    for i, x in enumerate(xs):
        os_, oc = O.sincosf(float(x))
        oa = O.asinf(float(x))
        if math.isnan(x):
            assert abs(a[i]) == np.float32(math.pi / 2)
            continue
        assert np.float32(os_).view(np.uint32) == s[i].view(np.uint32), (x, os_, s[i])
        assert np.float32(oc).view(np.uint32) == c[i].view(np.uint32), (x, oc, c[i])
        assert np.float32(oa).view(np.uint32) == a[i].view(np.uint32), (x, oa, a[i])
    assert O.asinf(-1.5) == np.float32(-math.pi / 2)
    assert abs(O.asinf(float("nan"))) == np.float32(math.pi / 2)


def test_host_sky_transcendentals_equal_oracle(host):
    """geo_math.h's per-pixel forms sincos_sky_ (rint by the shifter, parity
    bit XOR), acos_pi_ (sqrt floor by fmaxf) and atan2_turns_ host-compiled
    equal the oracle's restatement bit for bit: random and huge arguments,
    x / pi at and next to half-integers (the shifter's ties), |x| > 1, signed
    zeros, the axes and NaN."""
    rng = np.random.default_rng(17)
    inv_pi = np.float32(0.318309886183790671538)
    ties = []
    for k in range(-600, 600):
        x0 = np.float32(np.float32(k + 0.5) / inv_pi)
        ties += [x0, np.nextafter(x0, np.float32(np.inf)), np.nextafter(x0, np.float32(-np.inf))]
    special = [0.0, -0.0, 1.0, -1.0, 1.5, -1.5, np.nan, -np.nan, 1 - 2**-24, -(1 - 2**-24)]
    xs = np.concatenate([rng.uniform(-10, 10, 20000), rng.uniform(-1.2, 1.2, 20000), rng.uniform(-9000, 9000, 5000),
                         np.array(ties, np.float64), special]).astype(np.float32)
    ys = np.concatenate([rng.standard_normal(xs.size - 2 * len(special)), special, special[::-1]]).astype(np.float32)
    n = xs.size
    s, c, a, u = (np.empty(n, np.float32) for _ in range(4))
    vp = ctypes.c_void_p
    host.host_sky_math(vp(xs.ctypes.data), vp(ys.ctypes.data), ctypes.c_uint32(n), vp(s.ctypes.data),
                       vp(c.ctypes.data), vp(a.ctypes.data), vp(u.ctypes.data))
    bits = lambda v: np.float32(v).view(np.uint32)  # noqa: E731
    for i in range(n):
        x, y = float(xs[i]), float(ys[i])
        os_, oc = O.sincos_sky(x)
        assert (bits(os_), bits(oc)) == (s[i].view(np.uint32), c[i].view(np.uint32)) or math.isnan(x), (x, os_, s[i])
        assert bits(O.acos_pi(x)) == a[i].view(np.uint32), (x, O.acos_pi(x), a[i])
        ou = O.atan2_turns(y, x)
        assert bits(ou) == u[i].view(np.uint32) or (math.isnan(ou) and math.isnan(u[i])), (y, x, ou, u[i])
