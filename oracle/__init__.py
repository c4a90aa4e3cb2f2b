"""ORACLE loader — test infrastructure only.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package, and only as the checker / the timed CPU baseline; the
product (schwarzschild_raytracer_wgpu_amd, libgeo.so) never does.

PARITY UNPINNED against reference outputs: the Rust/WGSL reference cannot be
built or run here, and its only hot-path test asserts nothing
(SR/simulation/tests.rs:8-13).  Pinned by analytic KATs and committed goldens
(tests/golden/).  See geo_oracle.h.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")


class GeoFrameC(ctypes.Structure):
    _fields_ = [
        ("display_to_movement", ctypes.c_float * 16),
        ("movement_to_central", ctypes.c_float * 16),
        ("central_to_uv", ctypes.c_float * 16),
        ("psi_factor_and_position", ctypes.c_float * 4),
    ]


class GeoSceneC(ctypes.Structure):
    _fields_ = [
        ("rs", ctypes.c_float),
        ("sphere_r", ctypes.c_float),
        ("r_obs", ctypes.c_float),
        ("step", ctypes.c_float),
        ("max_steps", ctypes.c_uint32),
        ("mode", ctypes.c_uint32),
        ("flags", ctypes.c_uint32),
        ("tol", ctypes.c_float),
    ]


class OraclePx(ctypes.Structure):
    _fields_ = [
        ("lam", ctypes.c_double),
        ("u", ctypes.c_double),
        ("v", ctypes.c_double),
        ("theta", ctypes.c_double),
        ("steps", ctypes.c_uint32),
        ("bh", ctypes.c_int),
    ]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def _load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        build()
    lib = ctypes.CDLL(LIB_PATH)
    vp, u32, f64, i = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_double, ctypes.c_int
    sig = {
        "geo_oracle_solve_geodesic_f64": (f64, [f64, f64, u32, f64, f64, f64, f64, i, vp]),
        "geo_oracle_solve_ray_fan_f64": (None, [f64, f64, u32, f64, u32, f64, vp]),
        "geo_oracle_geodesic_at_theta_f64": (f64, [f64, f64, u32, f64, f64, f64, vp]),
        "geo_oracle_pixel_f64": (None, [vp, vp, vp, u32, u32, u32, u32, u32, vp]),
        "geo_oracle_render_f64": (i, [vp, vp, vp, u32, u32, u32, u32, u32, u32, i, vp, vp, vp, vp, vp]),
        "geo_oracle_render_f32": (i, [vp, vp, vp, u32, vp, u32, u32, u32, u32, u32, u32, u32, i, vp, vp, vp,
                                      vp, vp]),
        "geo_oracle_observer_frame": (None, [f64, f64, f64, f64, vp, f64, f64, i, f64, vp]),
        "geo_oracle_geodesic_f32": (ctypes.c_float, [vp, ctypes.c_float, ctypes.c_float, vp]),
        "geo_oracle_rays_update": (i, [ctypes.c_float, u32, u32, vp, vp, vp, vp, i, i, i, vp, i]),
        "geo_oracle_points_run": (i, [ctypes.c_float, vp, u32, i, i, ctypes.c_uint64, u32, vp, vp, vp, vp, vp, i]),
        "geo_oracle_project_point": (i, [vp, vp, u32, u32, vp, vp]),
        "geo_oracle_draw_points": (i, [vp, vp, u32, u32, u32, u32, u32, vp, vp]),
        "geo_oracle_acosf": (ctypes.c_float, [ctypes.c_float]),
        "geo_oracle_orbit_frames": (i, [f64, f64, f64, f64, vp, f64, f64, f64, u32, f64, vp, vp]),
        "geo_oracle_asinf": (ctypes.c_float, [ctypes.c_float]),
        "geo_oracle_atan2f": (ctypes.c_float, [ctypes.c_float, ctypes.c_float]),
        "geo_oracle_sincosf": (None, [ctypes.c_float, vp, vp]),
        "geo_oracle_sincos_sky": (None, [ctypes.c_float, vp, vp]),
        "geo_oracle_acos_pi": (ctypes.c_float, [ctypes.c_float]),
        "geo_oracle_atan2_turns": (ctypes.c_float, [ctypes.c_float, ctypes.c_float]),
        "geo_oracle_mip_chain_texels": (ctypes.c_uint64, [u32, u32]),
        "geo_oracle_mip_chain": (None, [vp, u32, u32, vp]),
        "geo_oracle_lod_q8_n": (None, [vp, u32, vp]),
        "geo_oracle_render_mips_f32": (i, [vp, vp, vp, u32, vp, u32, u32, u32, u32, u32, u32, i, vp, vp, vp, vp,
                                           vp]),
        "geo_oracle_ring_kx": (ctypes.c_float, [vp]),
        "geo_oracle_ring_band": (i, [vp, vp, u32, u32, u32, u32, u32, vp]),
        "geo_oracle_ring_x": (i, [vp, vp, u32, u32, u32, u32, u32, vp]),
    }
    for n, (r, a) in sig.items():
        fn = getattr(lib, n)
        fn.restype = r
        fn.argtypes = a
    return lib


lib = _load()


def _addr(x):
    return None if x is None else ctypes.cast(ctypes.byref(x), ctypes.c_void_p)


def _np(a):
    return None if a is None else a.ctypes.data


def as_frame(frame) -> GeoFrameC:
    """Copy any 208-byte TransformationPipeline-like ctypes struct."""
    out = GeoFrameC()
    ctypes.memmove(ctypes.byref(out), ctypes.byref(frame), ctypes.sizeof(GeoFrameC))
    return out


def as_scene(scene) -> GeoSceneC:
    out = GeoSceneC()
    ctypes.memmove(ctypes.byref(out), ctypes.byref(scene), ctypes.sizeof(GeoSceneC))
    return out


def solve_geodesic(sphere_r, schwarz_r, max_iter, step, r, energy, rotation, r_falling):
    steps = ctypes.c_uint32()
    a = lib.geo_oracle_solve_geodesic_f64(sphere_r, schwarz_r, max_iter, step, r, energy, rotation,
                                          int(bool(r_falling)), ctypes.byref(steps))
    return a, steps.value


def geodesic_f32(scene, st, ct):
    """Traveled angle (f32 kernel order; scene.mode selects fixed or adaptive) and steps."""
    steps = ctypes.c_uint32()
    sc = as_scene(scene)
    a = lib.geo_oracle_geodesic_f32(_addr(sc), st, ct, ctypes.byref(steps))
    return a, steps.value


def geodesic_at_theta(sphere_r, schwarz_r, max_iter, step, r, theta):
    steps = ctypes.c_uint32()
    a = lib.geo_oracle_geodesic_at_theta_f64(sphere_r, schwarz_r, max_iter, step, r, theta, ctypes.byref(steps))
    return a, steps.value


def solve_ray_fan(sphere_r, schwarz_r, max_iter, step, nr_nodes, r) -> np.ndarray:
    out = np.empty(nr_nodes, dtype=np.float32)
    lib.geo_oracle_solve_ray_fan_f64(sphere_r, schwarz_r, max_iter, step, nr_nodes, r, out.ctypes.data)
    return out


def observer_frame(schwarz_r, fov, width, height, pos, cam_phi, cam_theta, state=1, energy=1.0) -> GeoFrameC:
    f = GeoFrameC()
    p = (ctypes.c_double * 3)(*pos)
    lib.geo_oracle_observer_frame(schwarz_r, fov, width, height, ctypes.cast(p, ctypes.c_void_p), cam_phi,
                                  cam_theta, state, energy, _addr(f))
    return f


def pixel_f64(frame, scene, width, height, px, py, fan=None) -> OraclePx:
    fr, sc = as_frame(frame), as_scene(scene)
    fan_a = None if fan is None else np.ascontiguousarray(fan, dtype=np.float32)
    out = OraclePx()
    lib.geo_oracle_pixel_f64(_addr(fr), _addr(sc), _np(fan_a), 0 if fan_a is None else fan_a.size, width, height,
                             px, py, _addr(out))
    return out


def render_f64(frame, scene, width, height, row0=0, nrows=None, fan=None, threads=8, row_step=1):
    """The f64 literal restatement on rows row0, row0 + row_step, ... (nrows of
    them): mask, uv, steps, lam (traveled-angle result lambda') and theta
    (the pixel's angle to the black hole) per pixel."""
    nrows = (height - row0 + row_step - 1) // row_step if nrows is None else nrows
    fr, sc = as_frame(frame), as_scene(scene)
    fan_a = None if fan is None else np.ascontiguousarray(fan, dtype=np.float32)
    mask = np.empty((nrows, width), np.uint8)
    uv = np.empty((nrows, width, 2), np.float32)
    steps = np.empty((nrows, width), np.uint32)
    lam = np.empty((nrows, width), np.float64)
    theta = np.empty((nrows, width), np.float64)
    rc = lib.geo_oracle_render_f64(_addr(fr), _addr(sc), _np(fan_a), 0 if fan_a is None else fan_a.size, width,
                                   height, row0, nrows, row_step, threads, _np(mask), _np(uv), _np(steps), _np(lam),
                                   _np(theta))
    if rc != 0:
        raise ValueError(f"geo_oracle_render_f64: {rc}")
    return dict(mask=mask, uv=uv, steps=steps, lam=lam, theta=theta)


def ring_band(frame, scene, width, height, row0=0, nrows=None, row_step=1):
    """GEO_FLAG_RING_F64's band (geo.h) on rows row0 + i row_step: 1 where the
    f32 ray's |b/b_c - 1| < GEO_RING_X (all 0 when the flag does not apply)."""
    nrows = (height - row0 + row_step - 1) // row_step if nrows is None else nrows
    band = np.empty((nrows, width), np.uint8)
    fr, sc = as_frame(frame), as_scene(scene)  # alive across the call
    rc = lib.geo_oracle_ring_band(_addr(fr), _addr(sc), width, height, row0, nrows, row_step, _np(band))
    if rc != 0:
        raise ValueError(f"geo_oracle_ring_band: {rc}")
    return band


def ring_x(frame, scene, width, height, row0=0, nrows=None, row_step=1):
    """|kx cos(theta) - 1| of each pixel's f32 ray (GEO_FLAG_RING_F64's band
    test quantity) on rows row0 + i row_step."""
    nrows = (height - row0 + row_step - 1) // row_step if nrows is None else nrows
    x = np.empty((nrows, width), np.float32)
    fr, sc = as_frame(frame), as_scene(scene)
    rc = lib.geo_oracle_ring_x(_addr(fr), _addr(sc), width, height, row0, nrows, row_step, _np(x))
    if rc != 0:
        raise ValueError(f"geo_oracle_ring_x: {rc}")
    return x


def render_f32(frame, scene, sky, width, height, row0=0, nrows=None, row_step=1, fan=None, threads=8,
               want_uv=True, want_steps=True, target=None):
    """target: the (nrows, width, 4) image a GEO_FLAG_COMPOSITE scene draws over (copied)."""
    nrows = height - row0 if nrows is None else nrows
    fr, sc = as_frame(frame), as_scene(scene)
    sky_a = np.ascontiguousarray(sky, dtype=np.uint8)
    fan_a = None if fan is None else np.ascontiguousarray(fan, dtype=np.float32)
    rgba = np.zeros((nrows, width, 4), np.uint8) if target is None else np.array(target, np.uint8).reshape(
        nrows, width, 4)
    mask = np.empty((nrows, width), np.uint8)
    uv = np.empty((nrows, width, 2), np.float32) if want_uv else None
    steps = np.empty((nrows, width), np.uint32) if want_steps else None
    total = ctypes.c_uint64()
    rc = lib.geo_oracle_render_f32(_addr(fr), _addr(sc), _np(fan_a), 0 if fan_a is None else fan_a.size,
                                   _np(sky_a), sky_a.shape[1], sky_a.shape[0], width, height, row0, nrows, row_step,
                                   threads, _np(rgba), _np(mask), _np(uv), _np(steps), _addr(total))
    if rc != 0:
        raise ValueError(f"geo_oracle_render_f32: {rc}")
    return dict(rgba=rgba, mask=mask, uv=uv, steps=steps, steps_total=total.value)


def mip_chain(sky) -> list:
    """The GEO_FLAG_MIPS mip chain of an (h, w, 4) RGBA8 texture: 4 levels
    (geo_pixel.h mip_down, box filter), each an (h_l, w_l, 4) array."""
    sky_a = np.ascontiguousarray(sky, dtype=np.uint8)
    h, w = sky_a.shape[:2]
    out = np.empty(int(lib.geo_oracle_mip_chain_texels(w, h)), np.uint32)
    lib.geo_oracle_mip_chain(_np(sky_a), w, h, _np(out))
    levels, o = [], 0
    for lvl in range(4):
        lw, lh = max(1, w >> lvl), max(1, h >> lvl)
        levels.append(out[o:o + lw * lh].view(np.uint8).reshape(lh, lw, 4))
        o += lw * lh
    return levels


def render_mips_f32(frame, scene, sky, width, height, row0=0, nrows=None, fan=None, threads=8, target=None):
    """The GEO_FLAG_MIPS mirror: rows [row0, row0 + nrows) (row0 even) sampled
    trilinearly through the sky's mip chain; target as in render_f32."""
    nrows = height - row0 if nrows is None else nrows
    fr, sc = as_frame(frame), as_scene(scene)
    sky_a = np.ascontiguousarray(sky, dtype=np.uint8)
    fan_a = None if fan is None else np.ascontiguousarray(fan, dtype=np.float32)
    rgba = np.zeros((nrows, width, 4), np.uint8) if target is None else np.array(target, np.uint8).reshape(
        nrows, width, 4)
    mask = np.empty((nrows, width), np.uint8)
    uv = np.empty((nrows, width, 2), np.float32)
    steps = np.empty((nrows, width), np.uint32)
    total = ctypes.c_uint64()
    rc = lib.geo_oracle_render_mips_f32(_addr(fr), _addr(sc), _np(fan_a), 0 if fan_a is None else fan_a.size,
                                        _np(sky_a), sky_a.shape[1], sky_a.shape[0], width, height, row0, nrows,
                                        threads, _np(rgba), _np(mask), _np(uv), _np(steps), _addr(total))
    if rc != 0:
        raise ValueError(f"geo_oracle_render_mips_f32: {rc}")
    return dict(rgba=rgba, mask=mask, uv=uv, steps=steps, steps_total=total.value)


def asinf(x: float) -> float:
    return lib.geo_oracle_asinf(x)


def atan2f(y: float, x: float) -> float:
    return lib.geo_oracle_atan2f(y, x)


def sincosf(x: float):
    s, c = ctypes.c_float(), ctypes.c_float()
    lib.geo_oracle_sincosf(x, _addr(s), _addr(c))
    return s.value, c.value


def sincos_sky(x: float):
    """the per-pixel form (geo_math.h sincos_sky_)"""
    s, c = ctypes.c_float(), ctypes.c_float()
    lib.geo_oracle_sincos_sky(x, _addr(s), _addr(c))
    return s.value, c.value


def acos_pi(x: float) -> float:
    """acos(x) / pi (geo_math.h acos_pi_)"""
    return lib.geo_oracle_acos_pi(x)


def atan2_turns(y: float, x: float) -> float:
    """atan2(y, x) / 2pi taken into [0, 1] (geo_math.h atan2_turns_)"""
    return lib.geo_oracle_atan2_turns(y, x)


# ---- accretion-disk points (geo_oracle_points.c) ----------------------------

NR_NODES = 48


class Rays:
    """Host mirror of a geo_rays batch (ray_connector.rs): n points x sides
    connectors (near side first), state u[c, 48] and needs_reset[c]."""

    def __init__(self, rs, pos, sides=1, libm=True):
        self.rs = float(rs)
        self.pos = np.ascontiguousarray(pos, dtype=np.float32).reshape(-1, 3)
        self.n = self.pos.shape[0]
        self.sides = sides
        nside = (sides & 1) + ((sides >> 1) & 1)
        self.u = np.ones((self.n * nside, NR_NODES), np.float32)   # RayConnector::new: u_ray = 1
        self.needs = np.ones(self.n * nside, np.uint8)             # needs_reset = true
        self.libm = int(bool(libm))

    def update(self, other, iterations=1, reset=False):
        other = np.ascontiguousarray(other, dtype=np.float32)
        per_point = int(other.size != 3)
        out = np.empty((self.u.shape[0], 4), np.float32)
        lib.geo_oracle_rays_update(self.rs, self.n, self.sides, _np(self.pos), _np(self.u), _np(self.needs),
                                   _np(other), per_point, int(iterations), int(bool(reset)), _np(out), self.libm)
        return out


def points_run(rs, model, observers, dts, farside=True, orbits=True, seed=0, libm=False):
    """PointCloud::new(model, observers[0]) then len(dts) updates; returns
    (near (n,4), far (n,4) or None, positions (n,3))."""
    model = np.ascontiguousarray(model, dtype=np.float32).reshape(-1, 3)
    n = model.shape[0]
    obs = np.ascontiguousarray(observers, dtype=np.float32).reshape(-1, 3)
    dts = np.ascontiguousarray(dts, dtype=np.float64)
    assert obs.shape[0] == dts.size + 1
    near = np.empty((n, 4), np.float32)
    far = np.empty((n, 4), np.float32) if farside else None
    pos = np.empty((n, 3), np.float32)
    r = lib.geo_oracle_points_run(float(rs), _np(model), n, int(farside), int(orbits), ctypes.c_uint64(seed),
                                  dts.size, _np(obs), _np(dts), _np(near), _np(far), _np(pos), int(bool(libm)))
    if r != 0:
        raise RuntimeError(f"geo_oracle_points_run: {r}")
    return near, far, pos


def draw_points(frame, verts, width, height, rgba=None, row0=0, nrows=None):
    """vs_main + PointList raster over an RGBA frame (rows [row0, row0+nrows));
    returns (rgba, xy (n, 2) int32, -1 when clipped)."""
    verts = np.ascontiguousarray(verts, dtype=np.float32).reshape(-1, 4)
    nrows = height - row0 if nrows is None else nrows
    if rgba is None:
        rgba = np.zeros((nrows, width, 4), np.uint8)
    xy = np.empty((verts.shape[0], 2), np.int32)
    fr = as_frame(frame)
    lib.geo_oracle_draw_points(_addr(fr), _np(verts), verts.shape[0], width, height, row0, nrows, _np(rgba), _np(xy))
    return rgba, xy


def orbit_frames(rs, fov, width, height, pos, camera, rotation, nframes, dt):
    """Orbiting observer replay: (frames: list of GeoFrameC, positions (n, 3)) or None."""
    frames = (GeoFrameC * nframes)()
    positions = np.empty((nframes, 3), np.float64)
    p = (ctypes.c_double * 3)(*pos)
    r = lib.geo_oracle_orbit_frames(rs, fov, width, height, ctypes.cast(p, ctypes.c_void_p), camera[0], camera[1],
                                    rotation, nframes, dt, ctypes.cast(frames, ctypes.c_void_p), _np(positions))
    if r != 0:
        return None
    return list(frames), positions
