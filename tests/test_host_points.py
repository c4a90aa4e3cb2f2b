"""The product's point-path header (geo_rays.h), compiled for the HOST, equals
the oracle's independent restatement (kernel-polynomial variant) bit for bit:
RayConnector batches over moving observers and vs_main.  CPU only."""
import ctypes
import math
import os
import subprocess

import numpy as np
import pytest

import oracle as O
from helpers import default_frame
from test_points import accretion_disk

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "native", "rays_host.cpp")
SO = os.path.join(HERE, "native", "librays_host.so")


@pytest.fixture(scope="module")
def host():
    deps = [SRC] + [os.path.join(HERE, "..", "schwarzschild_raytracer_wgpu_amd", "csrc", h)
                    for h in ("geo_rays.h", "geo_math.h")]
    if not os.path.exists(SO) or any(os.path.getmtime(d) > os.path.getmtime(SO) for d in deps):
        subprocess.run(["g++", "-O2", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off", "-mfma", "-msse4.1",
                        "-o", SO, SRC], check=True)
    return ctypes.CDLL(SO)


class HostRays:
    def __init__(self, lib, rs, pos, sides):
        self.lib, self.rs, self.pos, self.sides = lib, float(rs), np.ascontiguousarray(pos, np.float32), sides
        self.n = self.pos.shape[0]
        nside = (sides & 1) + ((sides >> 1) & 1)
        self.u = np.ones((self.n * nside, 48), np.float32)
        self.needs = np.ones(self.n * nside, np.uint8)

    def update(self, other, iterations=1, reset=False):
        other = np.ascontiguousarray(other, np.float32)
        out = np.empty((self.u.shape[0], 4), np.float32)
        vp = ctypes.c_void_p
        self.lib.host_rays_update(ctypes.c_float(self.rs), ctypes.c_uint32(self.n), ctypes.c_uint32(self.sides),
                                  vp(self.pos.ctypes.data), vp(self.u.ctypes.data), vp(self.needs.ctypes.data),
                                  vp(other.ctypes.data), ctypes.c_int(int(other.size != 3)),
                                  ctypes.c_uint32(iterations), ctypes.c_int(int(reset)), vp(out.ctypes.data))
        return out


@pytest.mark.parametrize("rs,sides", [(1.0, 3), (0.0, 1), (5.0, 2), (15.0, 3)])
def test_host_rays_equal_oracle(host, rs, sides):
    pos = accretion_disk(600, seed=int(rs) + sides)
    a, b = HostRays(host, rs, pos, sides), O.Rays(rs, pos, sides=sides, libm=False)
    for f in range(10):
        r = 30.0 * (1.1 / 30.0) ** (f / 9)
        obs = np.array([r * math.cos(0.7 * f), r * math.sin(0.7 * f), 0.2 - 0.05 * f], np.float32)
        it = 5 if f % 4 == 3 else 1
        x, y = a.update(obs, it, reset=(f == 6)), b.update(obs, it, reset=(f == 6))
        assert np.array_equal(x.view(np.uint32), y.view(np.uint32)), f
        assert np.array_equal(a.u.view(np.uint32), b.u.view(np.uint32)) and np.array_equal(a.needs, b.needs)
    # per-point other ends
    others = accretion_disk(600, seed=99) * np.float32(0.3)
    x, y = a.update(others, 2), b.update(others, 2)
    assert np.array_equal(x.view(np.uint32), y.view(np.uint32))


def test_host_projection_equals_oracle(host):
    w, h = 400, 225
    frame = default_frame(w, h, pos=(25.0, 0.0, 1.0))
    verts = O.Rays(1.0, accretion_disk(2000, seed=6), sides=3, libm=False).update(
        np.array([25.0, 0.0, 1.0], np.float32), reset=True)
    xy = np.empty((verts.shape[0], 2), np.int32)
    fr = O.as_frame(frame)
    host.host_project(ctypes.byref(fr), ctypes.c_void_p(verts.ctypes.data), ctypes.c_uint32(verts.shape[0]),
                      ctypes.c_uint32(w), ctypes.c_uint32(h), ctypes.c_void_p(xy.ctypes.data))
    _, ref = O.draw_points(frame, verts, w, h)
    assert np.array_equal(xy, ref)
    assert (xy[:, 0] >= 0).sum() > 500
