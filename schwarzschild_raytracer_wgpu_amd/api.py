"""Python mirror of the reference's host interface for the sky-sphere path,
over the libgeo C-ABI.  Names and argument meaning follow the Rust sources:

  Observer            SR/simulation/observer.rs:42-297
  SphereRayTracer     SR/simulation/sphere_ray_tracer.rs:12-56
  BasicSphereBuffer   SR/schwarzschild_sphere_shader/sphere_buffer/basic_sphere_buffer.rs:12-101
  Renderer.render     SR/renderer/renderer.rs:208-283 (sphere pass only)

Device buffers are torch tensors (PyTorch is plumbing here: device memory and
streams); every compute call goes to the HIP kernels in libgeo.so.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import GeoFrame, GeoScene, check, lib

FRAC_PI_2 = math.pi / 2


def _stream_handle(stream) -> int | None:
    if stream is None:
        import torch

        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def _ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


class Observer:
    """Observer (observer.rs).  Observer.new(schwarz_r, fov, width, height)."""

    def __init__(self, schwarz_r: float, fov: float, width: float, height: float):
        h = ctypes.c_void_p()
        check("geo_observer_create", lib.geo_observer_create(schwarz_r, fov, width, height, ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.geo_observer_destroy(h)
            self._h = None

    def set_position(self, x: float, y: float, z: float) -> None:
        check("geo_observer_set_position", lib.geo_observer_set_position(self._h, x, y, z))

    def get_position(self) -> tuple[float, float, float]:
        out = (ctypes.c_double * 3)()
        check("geo_observer_get_position", lib.geo_observer_get_position(self._h, out))
        return (out[0], out[1], out[2])

    def set_camera(self, phi: float, theta: float) -> None:
        check("geo_observer_set_camera", lib.geo_observer_set_camera(self._h, phi, theta))

    def set_energy(self, energy: float) -> None:
        check("geo_observer_set_energy", lib.geo_observer_set_energy(self._h, energy))

    def start_unmoving(self) -> None:
        check("geo_observer_set_state", lib.geo_observer_set_state(self._h, _lib.GEO_OBSERVER_UNMOVING))

    def start_frozen_fall(self) -> None:
        check("geo_observer_set_state", lib.geo_observer_set_state(self._h, _lib.GEO_OBSERVER_FROZEN_FALL))

    def start_orbit(self, rotation: float) -> bool:
        st = lib.geo_observer_start_orbit(self._h, rotation)
        if st == _lib.GEO_ESTATE:
            return False
        check("geo_observer_start_orbit", st)
        return True

    @property
    def state(self) -> int:
        return lib.geo_observer_get_state(self._h)

    def get_radial_position(self) -> float:
        return lib.geo_observer_radial_position(self._h)

    def update_position(self, desired_direction, dt: float) -> None:
        f, l, u = desired_direction
        check("geo_observer_update_position", lib.geo_observer_update_position(self._h, f, l, u, dt))

    def move_camera(self, horizontal_pixels: float, vertical_pixels: float) -> None:
        check("geo_observer_move_camera", lib.geo_observer_move_camera(self._h, horizontal_pixels, vertical_pixels))

    def update_screen_format(self, width: float, height: float) -> None:
        check("geo_observer_update_screen_format", lib.geo_observer_update_screen_format(self._h, width, height))

    def is_singular(self) -> bool:
        return bool(lib.geo_observer_is_singular(self._h))

    def calc_transformation_pipeline(self) -> GeoFrame:
        fr = GeoFrame()
        check("geo_observer_calc_transformation_pipeline",
              lib.geo_observer_calc_transformation_pipeline(self._h, ctypes.byref(fr)))
        return fr


class Context:
    """One libgeo device context (sky texture + ray fan + step counters)."""

    def __init__(self, device: int = 0):
        h = ctypes.c_void_p()
        check("geo_ctx_create", lib.geo_ctx_create(device, ctypes.byref(h)))
        self._h = h
        self.device = device

    def close(self) -> None:
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.geo_ctx_destroy(h)
        self._h = None

    def __del__(self):
        self.close()

    def set_sky(self, rgba8: np.ndarray) -> None:
        a = np.ascontiguousarray(rgba8, dtype=np.uint8)
        if a.ndim != 3 or a.shape[2] != 4:
            raise ValueError("sky must be an (h, w, 4) uint8 array")
        check("geo_set_sky", lib.geo_set_sky(self._h, a.ctypes.data, a.shape[1], a.shape[0]))

    def set_fan(self, fan: np.ndarray) -> None:
        a = np.ascontiguousarray(fan, dtype=np.float32)
        check("geo_set_fan", lib.geo_set_fan(self._h, a.ctypes.data, a.size))

    def solve_ray_fan(self, sphere_r: float, schwarz_r: float, max_iter: int, step: float, nr_nodes: int,
                      r: float, stream=None) -> np.ndarray:
        out = np.empty(nr_nodes, dtype=np.float32)
        check("geo_solve_ray_fan", lib.geo_solve_ray_fan(self._h, sphere_r, schwarz_r, max_iter, step, nr_nodes, r,
                                                         out.ctypes.data, _stream_handle(stream)))
        return out

    def steps_flush(self, steps_total, stream=None) -> None:
        """geo_steps_flush: add the GEO_FLAG_DEFER_STEPS accumulator to steps_total (device u64)."""
        check("geo_steps_flush", lib.geo_steps_flush(self._h, _ptr(steps_total), _stream_handle(stream)))

    def render_rows(self, frame: GeoFrame, scene: GeoScene, width: int, height: int, row0: int, nrows: int,
                    out_rgba, out_mask=None, out_uv=None, out_steps=None, steps_total=None, stream=None) -> None:
        """geo_render_rows; outputs are device tensors (rgba: nrows*width*4 u8)."""
        for t, n in ((out_rgba, nrows * width * 4), (out_mask, nrows * width), (out_uv, nrows * width * 2),
                     (out_steps, nrows * width), (steps_total, 1)):
            if t is not None and (not t.is_cuda or not t.is_contiguous() or t.numel() < n):
                raise ValueError("outputs must be contiguous device tensors of sufficient size")
        check("geo_render_rows", lib.geo_render_rows(
            self._h, ctypes.byref(frame), ctypes.byref(scene), width, height, row0, nrows,
            _ptr(out_rgba), _ptr(out_mask), _ptr(out_uv), _ptr(out_steps), _ptr(steps_total),
            _stream_handle(stream)))


    def render_bands(self, frame: GeoFrame, scene: GeoScene, width: int, height: int, band_rows: int, band0: int,
                     band_step: int, nbands: int, out_rgba, out_mask=None, out_uv=None, out_steps=None,
                     steps_total=None, stream=None) -> None:
        """geo_render_bands; outputs packed band after band (nbands*band_rows rows)."""
        nrows = nbands * band_rows
        for t, n in ((out_rgba, nrows * width * 4), (out_mask, nrows * width), (out_uv, nrows * width * 2),
                     (out_steps, nrows * width), (steps_total, 1)):
            if t is not None and (not t.is_cuda or not t.is_contiguous() or t.numel() < n):
                raise ValueError("outputs must be contiguous device tensors of sufficient size")
        check("geo_render_bands", lib.geo_render_bands(
            self._h, ctypes.byref(frame), ctypes.byref(scene), width, height, band_rows, band0, band_step, nbands,
            _ptr(out_rgba), _ptr(out_mask), _ptr(out_uv), _ptr(out_steps), _ptr(steps_total),
            _stream_handle(stream)))


def make_scene(rs: float, sphere_r: float, r_obs: float, step: float = math.pi / 100.0, max_steps: int = 1000,
               mode: int = _lib.GEO_MODE_DIRECT, flags: int = 0, tol: float = 0.0) -> GeoScene:
    """geo_scene; tol = GEO_MODE_ADAPTIVE's error tolerance in u (0 = 1e-6, must be 0 in other modes)."""
    return GeoScene(rs, sphere_r, r_obs, step, max_steps, mode, flags, tol)


class SphereRayTracer:
    """SphereRayTracer::new(sphere_r, schwarz_r, max_iter, default_step, nr_nodes_half)
    (sphere_ray_tracer.rs:24-33); solve_ray_fan runs the f64 GPU kernel."""

    NO_VALUE = _lib.NO_VALUE

    def __init__(self, sphere_r: float, schwarz_r: float, max_iter: int, default_step: float, nr_nodes_half: int,
                 ctx: Context | None = None):
        self.sphere_r = sphere_r
        self.schwarz_r = schwarz_r
        self.max_iter = max_iter
        self.default_step = default_step
        self.nr_nodes = 2 * nr_nodes_half
        self.ctx = ctx if ctx is not None else Context(0)
        self.interpolation_grid = np.full(self.nr_nodes, self.NO_VALUE, dtype=np.float32)

    def solve_ray_fan(self, r: float) -> np.ndarray:
        self.interpolation_grid = self.ctx.solve_ray_fan(self.sphere_r, self.schwarz_r, self.max_iter,
                                                         self.default_step, self.nr_nodes, r)
        return self.interpolation_grid


@dataclass
class RenderTarget:
    """The colour target of one sphere pass (plus optional diagnostics)."""

    width: int
    height: int
    rgba: object  # torch uint8 tensor (height*width*4) on the device
    mask: object = None
    uv: object = None
    steps: object = None
    steps_total: object = None


class BasicSphereBuffer:
    """BasicSphereBuffer::new(..., sphere_radius, schwarz_radius, texture_image)
    (basic_sphere_buffer.rs:21-60): N = 400 fan nodes, max_iter 1000, step PI/100."""

    NR_NODES_HALF = 200
    MAX_ITER = 1000
    STEP = math.pi / 100.0

    def __init__(self, ctx: Context, sphere_radius: float, schwarz_radius: float, texture_rgba: np.ndarray,
                 max_iter: int = MAX_ITER, step: float = STEP, mode: int = _lib.GEO_MODE_DIRECT):
        self.ctx = ctx
        self.sphere_radius = sphere_radius
        self.schwarz_radius = schwarz_radius
        self.max_iter = max_iter
        self.step = step
        self.mode = mode
        ctx.set_sky(texture_rgba)
        self.ray_tracer = SphereRayTracer(sphere_radius, schwarz_radius, max_iter, step, self.NR_NODES_HALF, ctx)
        self.radial_position = None

    def update_ray_fan(self, radial_position: float) -> None:
        """basic_sphere_buffer.rs:85-88.  The fan is only consumed in fan mode;
        direct mode integrates per pixel, so it just records r."""
        self.radial_position = radial_position
        if self.mode == _lib.GEO_MODE_FAN:
            self.ray_tracer.solve_ray_fan(radial_position)

    def scene(self) -> GeoScene:
        if self.radial_position is None:
            raise RuntimeError("update_ray_fan must be called before draw")
        return make_scene(self.schwarz_radius, self.sphere_radius, self.radial_position, self.step, self.max_iter,
                          self.mode)

    def draw(self, frame: GeoFrame, target: RenderTarget, row0: int = 0, nrows: int | None = None,
             stream=None) -> None:
        """SchwarzschildSphereShaderDraw::draw + fs_main over rows [row0, row0+nrows)."""
        nrows = target.height - row0 if nrows is None else nrows
        self.ctx.render_rows(frame, self.scene(), target.width, target.height, row0, nrows, target.rgba,
                             target.mask, target.uv, target.steps, target.steps_total, stream)


class Renderer:
    """The sphere pass of Renderer::render (renderer.rs:208-258): clear to
    (0,0,0,1), then draw each sphere over the whole target."""

    def __init__(self, observer: Observer):
        self.observer = observer

    def render(self, spheres, target: RenderTarget, stream=None) -> GeoFrame:
        frame = self.observer.calc_transformation_pipeline()
        for s in spheres:
            s.draw(frame, target, stream=stream)
        return frame
