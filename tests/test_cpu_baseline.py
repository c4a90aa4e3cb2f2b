"""The CPU baseline library (libgeo_cpu.so, include/geo/geo_cpu.h): the
product's per-pixel header on the host cores.  It must compute what the
kernel computes -- the oracle's f32 mirror bit for bit (the GPU suite ties
the kernel to the same mirror) -- on any thread count and row sampling, and
reject what geo_render_rows rejects."""
import ctypes
import math
import os

import numpy as np
import pytest

import oracle as O
from helpers import default_frame, default_scene
from schwarzschild_raytracer_wgpu_amd import make_scene
from schwarzschild_raytracer_wgpu_amd._lib import (GEO_EINVAL, GEO_FLAG_COMPOSITE, GEO_FLAG_MIPS, GEO_MODE_ADAPTIVE,
                                                   GEO_MODE_FAN, GEO_OK)
from schwarzschild_raytracer_wgpu_amd.scenes import make_sky

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "schwarzschild_raytracer_wgpu_amd", "libgeo_cpu.so")


@pytest.fixture(scope="module")
def cpu():
    if not os.path.exists(LIB):
        import __graft_entry__

        __graft_entry__.build()
    lib = ctypes.CDLL(LIB)
    vp, u32 = ctypes.c_void_p, ctypes.c_uint32
    lib.geo_render_cpu.restype = ctypes.c_int
    lib.geo_render_cpu.argtypes = [vp, vp, vp, u32, u32, vp, u32, u32, u32, u32, u32, u32, ctypes.c_int, vp, vp, vp,
                                   vp, vp]
    return lib


def render_cpu(lib, frame, scene, sky, w, h, row0=0, nrows=None, row_step=1, threads=4, fan=None, target=None):
    nrows = (h - row0 + row_step - 1) // row_step if nrows is None else nrows
    sky = np.ascontiguousarray(sky, dtype=np.uint8)
    fan_a = None if fan is None else np.ascontiguousarray(fan, dtype=np.float32)
    rgba = np.zeros((nrows, w, 4), np.uint8) if target is None else np.array(target, np.uint8).reshape(nrows, w, 4)
    mask = np.empty((nrows, w), np.uint8)
    uv = np.empty((nrows, w, 2), np.float32)
    steps = np.empty((nrows, w), np.uint32)
    total = ctypes.c_ulonglong()
    rc = lib.geo_render_cpu(ctypes.addressof(frame), ctypes.addressof(scene), sky.ctypes.data, sky.shape[1],
                            sky.shape[0], None if fan_a is None else fan_a.ctypes.data,
                            0 if fan_a is None else fan_a.size, w, h, row0, nrows, row_step, threads, rgba.ctypes.data,
                            mask.ctypes.data, uv.ctypes.data, steps.ctypes.data, ctypes.addressof(total))
    return rc, dict(rgba=rgba, mask=mask, uv=uv, steps=steps, total=total.value)


def same(a, b):
    return (all(np.array_equal(a[f], b[f]) for f in ("rgba", "mask", "steps"))
            and np.array_equal(a["uv"].view(np.uint32), b["uv"].view(np.uint32)))


CASES = [
    ("default", {}, {}),
    ("offaxis_adaptive", dict(pos=(1.2, 0.5, 0.0), camera=(math.pi + 0.6, 0.3)),
     dict(mode=GEO_MODE_ADAPTIVE, r_obs=1.3)),
    ("inside_horizon", dict(pos=(0.8, 0.0, 0.05)), dict(r_obs=math.sqrt(0.64 + 0.0025), max_steps=512)),
    ("flat", dict(rs=0.0, state=0), dict(rs=0.0, max_steps=512)),
]


@pytest.mark.parametrize("name,fk,sk", CASES, ids=[c[0] for c in CASES])
def test_cpu_baseline_equals_oracle(cpu, name, fk, sk):
    w, h = 96, 54
    sky = make_sky("equirect", (128, 64))
    frame = default_frame(w, h, **fk)
    mode = sk.pop("mode", None)
    base = default_scene(**sk)
    scene = base if mode is None else make_scene(base.rs, base.sphere_r, base.r_obs, base.step, base.max_steps, mode)
    rc, a = render_cpu(cpu, frame, scene, sky, w, h, threads=3)
    assert rc == GEO_OK
    b = O.render_f32(frame, scene, sky, w, h, threads=4)
    assert same(a, b), name
    assert a["total"] == b["steps_total"]


def test_cpu_baseline_threads_rows_fan_composite(cpu):
    w, h = 80, 45
    sky = np.random.default_rng(5).integers(0, 256, size=(64, 128, 4), dtype=np.uint8)  # translucent texels
    frame, scene = default_frame(w, h), default_scene(2048)
    ref = O.render_f32(frame, scene, sky, w, h, row0=3, nrows=14, row_step=3, threads=2)
    for t in (1, 2, 7, 64):
        rc, a = render_cpu(cpu, frame, scene, sky, w, h, row0=3, nrows=14, row_step=3, threads=t)
        assert rc == GEO_OK and same(a, ref) and a["total"] == ref["steps_total"], t
    fan = O.solve_ray_fan(50.0, 1.0, 1000, math.pi / 100, 400, scene.r_obs)
    fs = make_scene(1.0, 50.0, scene.r_obs, scene.step, 1000, GEO_MODE_FAN)
    rc, a = render_cpu(cpu, frame, fs, sky, w, h, fan=fan)
    assert rc == GEO_OK and same(a, O.render_f32(frame, fs, sky, w, h, fan=fan, threads=2))
    tgt = np.random.default_rng(6).integers(0, 256, size=(h, w, 4), dtype=np.uint8)
    cs = make_scene(1.0, 50.0, scene.r_obs, scene.step, 2048, flags=GEO_FLAG_COMPOSITE)
    rc, a = render_cpu(cpu, frame, cs, sky, w, h, target=tgt)
    assert rc == GEO_OK and same(a, O.render_f32(frame, cs, sky, w, h, threads=2, target=tgt))


def test_cpu_baseline_rejects(cpu):
    w, h = 16, 16
    sky = make_sky("flat", (1, 1))
    frame, scene = default_frame(w, h), default_scene(64)
    assert render_cpu(cpu, frame, scene, sky, w, h, row0=10, nrows=4, row_step=2)[0] == GEO_EINVAL  # row 16
    bad = default_scene(64)
    bad.mode = 7
    assert render_cpu(cpu, frame, bad, sky, w, h)[0] == GEO_EINVAL
    fs = default_scene(64)
    fs.mode = GEO_MODE_FAN
    assert render_cpu(cpu, frame, fs, sky, w, h)[0] == GEO_EINVAL  # fan mode without a fan
    neg = default_scene(64, step=-0.1)
    assert render_cpu(cpu, frame, neg, sky, w, h)[0] == GEO_EINVAL
    # what geo_render_rows / geo_set_sky reject: the step budget
    # past 2^24, a sky side past 2^20
    big = default_scene(max_steps=(1 << 24) + 1)
    assert render_cpu(cpu, frame, big, sky, w, h)[0] == GEO_EINVAL
    assert render_cpu(cpu, frame, default_scene(max_steps=1 << 24), sky, w, h, nrows=1)[0] == GEO_OK
    tall = np.zeros(((1 << 20) + 1, 1, 4), np.uint8)
    assert render_cpu(cpu, frame, scene, tall, w, h, nrows=1)[0] == GEO_EINVAL


def test_cpu_baseline_mips(cpu):
    """GEO_FLAG_MIPS: the CPU library equals the oracle's trilinear mirror
    (render_mips_f32) on ragged frames (quad partners past the right and
    bottom edges), in direct, adaptive and fan mode and composited over a
    target; sampled rows (any row0, any row_step) equal the same rows of the
    full frame, their quad partners traced as helpers."""
    sky = np.random.default_rng(11).integers(0, 256, size=(48, 96, 4), dtype=np.uint8)  # translucent texels
    for (w, h) in ((66, 38), (65, 37)):
        frame = default_frame(w, h)
        scene = default_scene(2048)
        scene.flags |= GEO_FLAG_MIPS
        rc, a = render_cpu(cpu, frame, scene, sky, w, h, threads=3)
        ref = O.render_mips_f32(frame, scene, sky, w, h, threads=4)
        assert rc == GEO_OK and same(a, ref) and a["total"] == ref["steps_total"], (w, h)
        for r0, n, rs in ((1, 12, 3), (4, 9, 4), (h - 1, 1, 1)):
            rc, b = render_cpu(cpu, frame, scene, sky, w, h, row0=r0, nrows=n, row_step=rs, threads=2)
            rows = [r0 + i * rs for i in range(n)]
            sub = {f: a[f][rows] for f in ("rgba", "mask", "uv", "steps")}
            assert rc == GEO_OK and same(b, sub), (w, h, r0, rs)
    w, h = 66, 38
    frame = default_frame(w, h, pos=(1.2, 0.5, 0.0), camera=(math.pi + 0.6, 0.3))
    sa = make_scene(1.0, 50.0, 1.3, math.pi / 100, 2048, GEO_MODE_ADAPTIVE, flags=GEO_FLAG_MIPS)
    rc, a = render_cpu(cpu, frame, sa, sky, w, h, threads=4)
    assert rc == GEO_OK and same(a, O.render_mips_f32(frame, sa, sky, w, h, threads=4))
    frame = default_frame(w, h)
    r = math.sqrt(2.5 ** 2 + 0.1 ** 2)
    fan = O.solve_ray_fan(50.0, 1.0, 1000, math.pi / 100, 400, r)
    sf = make_scene(1.0, 50.0, r, math.pi / 100, 1000, GEO_MODE_FAN, flags=GEO_FLAG_MIPS)
    rc, a = render_cpu(cpu, frame, sf, sky, w, h, fan=fan)
    assert rc == GEO_OK and same(a, O.render_mips_f32(frame, sf, sky, w, h, fan=fan, threads=4))
    tgt = np.random.default_rng(12).integers(0, 256, size=(h, w, 4), dtype=np.uint8)
    sc = make_scene(1.0, 50.0, r, math.pi / 100, 2048, flags=GEO_FLAG_COMPOSITE | GEO_FLAG_MIPS)
    rc, a = render_cpu(cpu, frame, sc, sky, w, h, target=tgt)
    assert rc == GEO_OK and same(a, O.render_mips_f32(frame, sc, sky, w, h, threads=4, target=tgt))
