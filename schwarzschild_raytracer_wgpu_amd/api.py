"""Python mirror of the reference's host interface for the sky-sphere path,
over the libgeo C-ABI.  Names and argument meaning follow the Rust sources:

  Observer            SR/simulation/observer.rs:42-297
  SphereRayTracer     SR/simulation/sphere_ray_tracer.rs:12-56
  BasicSphereBuffer   SR/schwarzschild_sphere_shader/sphere_buffer/basic_sphere_buffer.rs:12-101
  RayConnectors       SR/simulation/ray_connector.rs:6-157 (a device batch)
  PointCloud          SR/schwarzschild_point_shader/point_cloud.rs:7-156
  Renderer.render     SR/renderer/renderer.rs:208-283 (sphere pass + point pass)

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
                      r: float, stream=None, host: bool = True) -> np.ndarray | None:
        """geo_solve_ray_fan: the context's fan, solved on the device.  host=True also
        returns it (synchronises `stream`); host=False leaves it stream-ordered on the
        device only, for the fan-mode draws that follow on `stream`."""
        out = np.empty(nr_nodes, dtype=np.float32) if host else None
        check("geo_solve_ray_fan", lib.geo_solve_ray_fan(self._h, sphere_r, schwarz_r, max_iter, step, nr_nodes, r,
                                                         out.ctypes.data if host else None, _stream_handle(stream)))
        return out

    def time_next_render(self, start, stop) -> None:
        """geo_time_next_render: the next render's kernel dispatch carries these
        two HipEvents (timing.HipEvent): its execution time, no marker packets."""
        check("geo_time_next_render", lib.geo_time_next_render(self._h, start.h, stop.h))

    def set_dispatch(self, mode: int, period: int = 16) -> None:
        """geo_set_dispatch: GEO_DISPATCH_LONGEST_FIRST (default; the order is
        re-learned on the device every `period` renders of a grid) or
        GEO_DISPATCH_ROW_MAJOR."""
        check("geo_set_dispatch", lib.geo_set_dispatch(self._h, mode, period))

    def dispatch_stats(self) -> tuple[int, int]:
        """geo_dispatch_stats: (renders that recorded tile costs, rebuilt orders adopted)."""
        rec, adopted = ctypes.c_ulonglong(), ctypes.c_ulonglong()
        check("geo_dispatch_stats", lib.geo_dispatch_stats(self._h, ctypes.byref(rec), ctypes.byref(adopted)))
        return rec.value, adopted.value

    def set_tile_order(self, tiles_x: int, tiles_y: int, order=None) -> None:
        """geo_set_tile_order: workgroup dispatch order (packed y << 16 | x per
        tile, a permutation of the grid) for renders of a tiles_x x tiles_y grid;
        order=None restores row-major."""
        if order is None:
            check("geo_set_tile_order", lib.geo_set_tile_order(self._h, 0, 0, None))
            return
        o = np.ascontiguousarray(order, dtype=np.uint32)
        if o.size != tiles_x * tiles_y:
            raise ValueError("order must hold tiles_x * tiles_y tiles")
        check("geo_set_tile_order", lib.geo_set_tile_order(self._h, tiles_x, tiles_y, o.ctypes.data))

    def steps_flush(self, steps_total, stream=None) -> None:
        """geo_steps_flush: add the GEO_FLAG_DEFER_STEPS accumulator to steps_total (device u64)."""
        check("geo_steps_flush", lib.geo_steps_flush(self._h, _ptr(steps_total), _stream_handle(stream)))

    def assemble_bands(self, src, rank_stride: int, frame_stride: int, world: int, band_rows: int, width: int,
                       height: int, nframes: int, dst, src_bpp: int = 4, stream=None) -> None:
        """geo_assemble_bands: rank-packed bands (device, RGBA8 or RGB24) -> nframes RGBA8 frames (device)."""
        check("geo_assemble_bands", lib.geo_assemble_bands(self._h, _ptr(src), rank_stride, frame_stride, world,
                                                           band_rows, width, height, nframes, src_bpp, _ptr(dst),
                                                           _stream_handle(stream)))

    def assemble_lead(self, lead_src, lead_frame_stride: int, lead: int, src, rank_stride: int, frame_stride: int,
                      world: int, band_rows: int, width: int, height: int, nframes: int, dst, src_bpp: int = 4,
                      stream=None) -> None:
        """geo_assemble_lead: rank 0's own packed RGBA8 bands (lead*band_rows rows per cycle) plus the gathered
        peer blocks (RGBA8 or RGB24; block 0 unread) -> nframes RGBA8 frames (device)."""
        check("geo_assemble_lead", lib.geo_assemble_lead(
            self._h, _ptr(lead_src), lead_frame_stride, lead, _ptr(src), rank_stride, frame_stride, world, band_rows,
            width, height, nframes, src_bpp, _ptr(dst), _stream_handle(stream)))

    def assemble_shares(self, lead_src, lead_frame_stride: int, lead_rows: int, src, rank_stride: int,
                        frame_stride: int, world: int, band_rows: int, width: int, height: int, nframes: int, dst,
                        src_bpp: int = 4, stream=None) -> None:
        """geo_assemble_shares: geo_assemble_lead with rank 0's rows per cycle (lead_rows) given directly."""
        check("geo_assemble_shares", lib.geo_assemble_shares(
            self._h, _ptr(lead_src), lead_frame_stride, lead_rows, _ptr(src), rank_stride, frame_stride, world,
            band_rows, width, height, nframes, src_bpp, _ptr(dst), _stream_handle(stream)))

    def pack_rgb(self, rgba, npixels: int, rgb, stream=None) -> None:
        """geo_pack_rgb: RGBA8 -> RGB24 on the device (npixels % 4 == 0)."""
        check("geo_pack_rgb", lib.geo_pack_rgb(self._h, _ptr(rgba), npixels, _ptr(rgb), _stream_handle(stream)))

    def render_rows(self, frame: GeoFrame, scene: GeoScene, width: int, height: int, row0: int, nrows: int,
                    out_rgba, out_mask=None, out_uv=None, out_steps=None, steps_total=None, stream=None) -> None:
        """geo_render_rows; outputs are device tensors (rgba: nrows*width*4 u8)."""
        _check_outputs(nrows, width, out_rgba, out_mask, out_uv, out_steps, steps_total)
        check("geo_render_rows", lib.geo_render_rows(
            self._h, ctypes.byref(frame), ctypes.byref(scene), width, height, row0, nrows,
            _ptr(out_rgba), _ptr(out_mask), _ptr(out_uv), _ptr(out_steps), _ptr(steps_total),
            _stream_handle(stream)))


    def render_band_set_frames(self, frames, scene: GeoScene, width: int, height: int, band_rows: int, row0: int,
                               row_stride: int, nbands: int, out_rgba, frame_stride: int | None = None,
                               steps_total=None, stream=None) -> None:
        """geo_render_band_set_frames: len(frames) (1 .. GEO_MAX_BATCH_FRAMES) frames of one scene in one
        launch; frame f's packed bands at byte f*frame_stride of out_rgba (default: packed back to back).
        Colour only."""
        n = len(frames)
        if not 1 <= n <= _lib.GEO_MAX_BATCH_FRAMES:
            raise ValueError(f"1 .. {_lib.GEO_MAX_BATCH_FRAMES} frames per batch")
        fbytes = nbands * band_rows * width * 4
        frame_stride = fbytes if frame_stride is None else frame_stride
        import torch

        _check_buffer("out_rgba", out_rgba, (n - 1) * frame_stride + fbytes)
        _check_buffer("steps_total", steps_total, 8, (torch.int64, torch.uint64))
        arr = (GeoFrame * n)(*frames)
        check("geo_render_band_set_frames", lib.geo_render_band_set_frames(
            self._h, arr, n, ctypes.byref(scene), width, height, band_rows, row0, row_stride, nbands,
            _ptr(out_rgba), frame_stride, _ptr(steps_total), _stream_handle(stream)))

    def render_bands(self, frame: GeoFrame, scene: GeoScene, width: int, height: int, band_rows: int, band0: int,
                     band_step: int, nbands: int, out_rgba, out_mask=None, out_uv=None, out_steps=None,
                     steps_total=None, stream=None) -> None:
        """geo_render_bands; outputs packed band after band (nbands*band_rows rows)."""
        nrows = nbands * band_rows
        _check_outputs(nrows, width, out_rgba, out_mask, out_uv, out_steps, steps_total)
        check("geo_render_bands", lib.geo_render_bands(
            self._h, ctypes.byref(frame), ctypes.byref(scene), width, height, band_rows, band0, band_step, nbands,
            _ptr(out_rgba), _ptr(out_mask), _ptr(out_uv), _ptr(out_steps), _ptr(steps_total),
            _stream_handle(stream)))

    def render_band_set(self, frame: GeoFrame, scene: GeoScene, width: int, height: int, band_rows: int, row0: int,
                        row_stride: int, nbands: int, out_rgba, out_mask=None, out_uv=None, out_steps=None,
                        steps_total=None, stream=None) -> None:
        """geo_render_band_set: bands at rows row0 + j*row_stride (j < nbands), band_rows tall, packed."""
        nrows = nbands * band_rows
        _check_outputs(nrows, width, out_rgba, out_mask, out_uv, out_steps, steps_total)
        check("geo_render_band_set", lib.geo_render_band_set(
            self._h, ctypes.byref(frame), ctypes.byref(scene), width, height, band_rows, row0, row_stride, nbands,
            _ptr(out_rgba), _ptr(out_mask), _ptr(out_uv), _ptr(out_steps), _ptr(steps_total),
            _stream_handle(stream)))


def _check_outputs(nrows: int, width: int, rgba, mask, uv, steps, steps_total) -> None:
    """The kernel writes 4 B of RGBA8, 1 B of mask, 2 f32 of UV and one u32 of
    steps per pixel, and adds into one u64 total: every output must be a
    contiguous device tensor holding at least that many BYTES (a tensor of
    the right element count but a narrower dtype would be overrun), and the
    typed ones must carry their type (f32 UV, 4-byte steps, 64-bit total)."""
    import torch

    n = nrows * width
    for name, t, nbytes, dtypes in (("out_rgba", rgba, 4 * n, None), ("out_mask", mask, n, None),
                                    ("out_uv", uv, 8 * n, (torch.float32,)),
                                    ("out_steps", steps, 4 * n, (torch.int32, torch.uint32)),
                                    ("steps_total", steps_total, 8, (torch.int64, torch.uint64))):
        _check_buffer(name, t, nbytes, dtypes)


def _check_buffer(name: str, t, nbytes: int, dtypes=None) -> None:
    """t (optional) is a contiguous device tensor of >= nbytes bytes and, if
    dtypes is given, one of those dtypes."""
    if t is None:
        return
    if not t.is_cuda or not t.is_contiguous():
        raise ValueError(f"{name} must be a contiguous device tensor")
    if dtypes is not None and t.dtype not in dtypes:
        raise ValueError(f"{name} must be one of {dtypes}, got {t.dtype}")
    if t.numel() * t.element_size() < nbytes:
        raise ValueError(f"{name} holds {t.numel() * t.element_size()} bytes, the rows need {nbytes}")


def _check_point_outputs(target: "RenderTarget", row0: int, nrows: int, out_xy, n_xy: int) -> None:
    """The point draws write RGBA8 pixels of rows [row0, row0 + nrows) of the
    target (laid out from row0, as geo_render_rows' output) and 2 int32 per
    vertex into out_xy."""
    import torch

    _check_buffer("target.rgba", target.rgba, 4 * nrows * target.width)
    _check_buffer("out_xy", out_xy, 8 * n_xy, (torch.int32,))


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

    def update_device_fan(self, r: float, stream=None) -> None:
        """The fan for observer radius r into the context only (stream-ordered, no
        host copy): what a fan-mode draw reads.  interpolation_grid is not updated."""
        self.ctx.solve_ray_fan(self.sphere_r, self.schwarz_r, self.max_iter, self.default_step, self.nr_nodes, r,
                               stream=stream, host=False)


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
    (basic_sphere_buffer.rs:21-60): N = 400 fan nodes, max_iter 1000, step PI/100.
    A sphere owns its Context (its texture and ray fan live there, as the
    reference's per-sphere bind groups do): pass a device index, or a Context
    no other sphere uses."""

    NR_NODES_HALF = 200
    MAX_ITER = 1000
    STEP = math.pi / 100.0

    def __init__(self, ctx: Context | int, sphere_radius: float, schwarz_radius: float, texture_rgba: np.ndarray,
                 max_iter: int = MAX_ITER, step: float = STEP, mode: int = _lib.GEO_MODE_DIRECT,
                 mipmaps: bool = False, ring_f64: bool = False):
        """mipmaps: sample the texture's 4-level mip chain trilinearly, as the
        reference's textureSample does (Texture::new_with_mipmaps(..., 4),
        GEO_FLAG_MIPS); off, the level-0 bilinear sample the benchmark measures.
        ring_f64: the capture band's lanes integrate in f64 (GEO_FLAG_RING_F64:
        direct or adaptive mode, the level-0 sampler, not as a composited sphere)."""
        ctx = Context(ctx) if isinstance(ctx, int) else ctx
        self.ctx = ctx
        self.mipmaps = mipmaps
        self.ring_f64 = ring_f64
        self.sphere_radius = sphere_radius
        self.schwarz_radius = schwarz_radius
        self.max_iter = max_iter
        self.step = step
        self.mode = mode
        ctx.set_sky(texture_rgba)
        self.ray_tracer = SphereRayTracer(sphere_radius, schwarz_radius, max_iter, step, self.NR_NODES_HALF, ctx)
        self.radial_position = None

    def update_ray_fan(self, radial_position: float, stream=None) -> None:
        """basic_sphere_buffer.rs:85-88.  The fan is only consumed in fan mode,
        where it is solved into the sphere's context on `stream` (the reference
        writes it into the sphere's fan texture; no host copy, so a frame loop
        does not synchronise); direct mode integrates per pixel, so it just
        records r."""
        self.radial_position = radial_position
        if self.mode == _lib.GEO_MODE_FAN:
            self.ray_tracer.update_device_fan(radial_position, stream=stream)

    def scene(self) -> GeoScene:
        if self.radial_position is None:
            raise RuntimeError("update_ray_fan must be called before draw")
        return make_scene(self.schwarz_radius, self.sphere_radius, self.radial_position, self.step, self.max_iter,
                          self.mode, flags=(_lib.GEO_FLAG_MIPS if self.mipmaps else 0) |
                          (_lib.GEO_FLAG_RING_F64 if self.ring_f64 else 0))

    def draw(self, frame: GeoFrame, target: RenderTarget, row0: int = 0, nrows: int | None = None,
             stream=None, composite: bool = False) -> None:
        """SchwarzschildSphereShaderDraw::draw + fs_main over rows [row0, row0+nrows);
        composite: alpha-blend over the target's contents (a 2nd/3rd sphere)."""
        nrows = target.height - row0 if nrows is None else nrows
        scene = self.scene()
        if composite:
            scene.flags |= _lib.GEO_FLAG_COMPOSITE
        self.ctx.render_rows(frame, scene, target.width, target.height, row0, nrows, target.rgba,
                             target.mask, target.uv, target.steps, target.steps_total, stream)


def _hip():
    """The HIP runtime torch loaded (the libamdhip64.so.7 soname), for raw
    device copies of library-owned buffers."""
    global _HIP
    if _HIP is None:
        import torch  # noqa: F401

        h = ctypes.CDLL("libamdhip64.so.7")
        h.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _HIP = h
    return _HIP


_HIP = None


def _f32x3(v) -> ctypes.Array:
    a = np.ascontiguousarray(v, dtype=np.float32).reshape(-1)
    if a.size != 3:
        raise ValueError("expected 3 floats")
    return (ctypes.c_float * 3)(*a.tolist())


class RayConnectors:
    """A device batch of RayConnector (ray_connector.rs:6-157) on n points: a
    near-side connector (less_than_180 = true) per point and/or a far-side
    one.  RayConnector::new(schwarz_r, pos, less_than_180) for every
    (point, side); `update_ray` / `reset_ray` run the HIP kernel over all
    connectors (near side first) into `self.vertices` (device, (count, 4):
    [x, y, z, incoming angle])."""

    def __init__(self, ctx: Context, schwarz_r: float, positions, sides: int = _lib.GEO_RAYS_NEAR):
        import torch

        pos = np.ascontiguousarray(positions, dtype=np.float32).reshape(-1, 3)
        self.ctx, self.n_points = ctx, pos.shape[0]
        h = ctypes.c_void_p()
        check("geo_rays_create", lib.geo_rays_create(ctx._h, schwarz_r, self.n_points, sides, pos.ctypes.data,
                                                     ctypes.byref(h)))
        self._h = h
        self.count = lib.geo_rays_count(h)
        self.vertices = torch.empty((self.count, 4), dtype=torch.float32, device=f"cuda:{ctx.device}")

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.geo_rays_destroy(h)
            self._h = None

    def set_positions(self, positions) -> None:
        pos = np.ascontiguousarray(positions, dtype=np.float32).reshape(-1, 3)
        if pos.shape[0] != self.n_points:
            raise ValueError(f"positions: {self.n_points} points expected, got {pos.shape[0]}")
        check("geo_rays_set_positions", lib.geo_rays_set_positions(self._h, pos.ctypes.data))

    def _call(self, other, iterations: int, reset: bool, stream):
        o = np.ascontiguousarray(other, dtype=np.float32).reshape(-1)
        per_point = o.size != 3
        if per_point and o.size != 3 * self.n_points:
            raise ValueError("other: 3 floats or 3 per point")
        check("geo_rays_update", lib.geo_rays_update(self._h, o.ctypes.data, int(per_point), iterations,
                                                     int(reset), _ptr(self.vertices), _stream_handle(stream)))
        return self.vertices

    def update_ray(self, other_position, iterations: int = 1, stream=None):
        """update_ray(other, iterations) for every connector (one other end for
        all, or one per point)."""
        return self._call(other_position, iterations, False, stream)

    def reset_ray(self, other_position, stream=None):
        return self._call(other_position, 0, True, stream)


class PointCloud:
    """PointCloud (point_cloud.rs:7-156) on the device: RayConnectors for the
    near (and far) side of every model vertex, optionally driven by f64
    orbits with respawn.  Randomness: per-point wyrand streams from `seed`."""

    def __init__(self, ctx: Context, model_vertices, schwarz_r: float, observer_pos, activate_farside: bool,
                 activate_orbits: bool, seed: int = 0):
        model = np.ascontiguousarray(model_vertices, dtype=np.float32).reshape(-1, 3)
        self.ctx, self.n = ctx, model.shape[0]
        self.has_farside = bool(activate_farside)
        h = ctypes.c_void_p()
        check("geo_points_create", lib.geo_points_create(ctx._h, schwarz_r, model.ctypes.data, self.n,
                                                         _f32x3(observer_pos), int(activate_farside),
                                                         int(activate_orbits), seed, ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            lib.geo_points_destroy(h)
            self._h = None

    # model generators (point_cloud.rs:67-115)
    @classmethod
    def new_spiral(cls, ctx: Context, schwarz_r: float, observer_pos, activate_farside: bool) -> "PointCloud":
        n = 10000
        t = np.arange(n, dtype=np.float32) / np.float32(n) * np.float32(2 * math.pi + 0.05)
        r = np.float32(16) + np.float32(2) * t
        pts = np.stack([-r * np.cos(np.float32(10) * t), -r * np.sin(np.float32(10) * t),
                        np.full(n, 0.001, np.float32)], 1)
        return cls(ctx, pts, schwarz_r, observer_pos, activate_farside, False)

    @classmethod
    def new_accretion_disk(cls, ctx: Context, schwarz_r: float, observer_pos, activate_farside: bool,
                           seed: int = 0, n: int = 5000) -> "PointCloud":
        rng = np.random.default_rng(seed)
        r = 16.0 + 10.0 * rng.random(n)
        phi = rng.random(n) * 2 * math.pi
        theta = 0.2 * (rng.random(n) - 0.5)
        pts = np.stack([r * np.cos(phi) * np.cos(theta), r * np.sin(phi) * np.cos(theta), r * np.sin(theta)], 1)
        return cls(ctx, pts.astype(np.float32), schwarz_r, observer_pos, activate_farside, True, seed)

    @classmethod
    def new_heart(cls, ctx: Context, schwarz_r: float, observer_pos, activate_farside: bool) -> "PointCloud":
        n = 4000
        t = np.arange(n, dtype=np.float32) / np.float32(n) * np.float32(2 * math.pi)
        pts = np.stack([np.full(n, 11.0, np.float32), np.float32(16) * np.sin(t) ** 3,
                        np.float32(13) * np.cos(t) - np.float32(5) * np.cos(2 * t) - np.float32(2) * np.cos(3 * t)
                        - np.cos(4 * t)], 1)
        return cls(ctx, pts.astype(np.float32), schwarz_r, observer_pos, activate_farside, False)

    def update(self, observer_pos, dt: float, stream=None) -> None:
        """PointCloud::update (:117-148): orbits step + respawn, update_ray(observer, 1)."""
        check("geo_points_update", lib.geo_points_update(self._h, _f32x3(observer_pos), dt,
                                                         _stream_handle(stream)))

    def vertices_ptr(self, farside: bool = False) -> int:
        p = lib.geo_points_vertices(self._h, int(farside))
        if not p:
            raise ValueError("no far side")
        return p

    def get_vertices(self, farside: bool = False) -> np.ndarray:
        """Host copy of get_vertices / get_vertices_farside ((n, 4) f32); synchronises."""
        import torch

        torch.cuda.synchronize()
        out = np.empty((self.n, 4), np.float32)
        if _hip().hipMemcpy(out.ctypes.data, self.vertices_ptr(farside), out.nbytes, 2) != 0:  # DeviceToHost
            raise RuntimeError("hipMemcpy")
        return out

    def positions(self, stream=None) -> np.ndarray:
        out = np.empty((self.n, 3), np.float32)
        check("geo_points_positions", lib.geo_points_positions(self._h, out.ctypes.data, _stream_handle(stream)))
        return out

    def draw(self, frame: GeoFrame, target: "RenderTarget", out_xy=None, stream=None) -> None:
        """The point pipeline over the target, near then far vertex buffer
        (geo_points_draw).  It waits for the last update() on whatever stream
        that ran, and the next update() waits for it, so update() may run on
        a side stream, overlapping the sphere draws.  out_xy (device, int32):
        2 per connector, near side first."""
        _check_point_outputs(target, 0, target.height, out_xy, self.n * (2 if self.has_farside else 1))
        check("geo_points_draw", lib.geo_points_draw(self._h, ctypes.byref(frame), target.width, target.height, 0,
                                                     target.height, _ptr(target.rgba), _ptr(out_xy),
                                                     _stream_handle(stream)))


def draw_points(ctx: Context, frame: GeoFrame, vertices, n: int, target: "RenderTarget", row0: int = 0,
                nrows: int | None = None, out_xy=None, stream=None) -> None:
    """geo_draw_points: vs_main + PointList raster (shader.wgsl:36-74) of n
    vertices (device pointer or tensor, 4 floats each) over target rows."""
    nrows = target.height - row0 if nrows is None else nrows
    _check_point_outputs(target, row0, nrows, out_xy, n)
    if not isinstance(vertices, int):
        _check_buffer("vertices", vertices, 16 * n)
    vp = vertices if isinstance(vertices, int) else _ptr(vertices)
    check("geo_draw_points", lib.geo_draw_points(ctx._h, ctypes.byref(frame), vp, n, target.width, target.height,
                                                 row0, nrows, _ptr(target.rgba), _ptr(out_xy),
                                                 _stream_handle(stream)))


class Renderer:
    """Renderer::render (renderer.rs:208-258): clear to (0,0,0,1), the spheres
    in order with alpha blending (the first over the cleared target, the rest
    GEO_FLAG_COMPOSITE over the previous ones), then the point meshes (near and
    far vertex buffers of each PointCloud) over the target."""

    def __init__(self, observer: Observer):
        self.observer = observer

    def render(self, spheres, target: RenderTarget, point_clouds=(), stream=None) -> GeoFrame:
        frame = self.observer.calc_transformation_pipeline()
        for i, s in enumerate(spheres):
            s.draw(frame, target, stream=stream, composite=i > 0)
        for pc in point_clouds:
            pc.draw(frame, target, stream=stream)
        return frame
