"""ctypes binding of libgeo.so (include/geo/geo.h).

The product path is the HIP library only: if libgeo.so is missing this module
raises at import — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgeo.so")

GEO_OK = 0
GEO_EINVAL = -1
GEO_EHIP = -2
GEO_ENOMEM = -3
GEO_ENODEV = -4
GEO_ESTATE = -5

GEO_MODE_DIRECT = 0
GEO_MODE_FAN = 1
GEO_MODE_ADAPTIVE = 2
GEO_ADAPTIVE_DEFAULT_TOL = 1e-6
GEO_DISPATCH_ROW_MAJOR = 0
GEO_DISPATCH_LONGEST_FIRST = 1
GEO_DISPATCH_EXPLICIT = 2
GEO_ADAPTIVE_MAX_GROWTH = 16
GEO_FLAG_DEFER_STEPS = 1
GEO_FLAG_COMPOSITE = 2
GEO_FLAG_MIPS = 4
GEO_FLAG_RING_F64 = 8
GEO_RING_X = 5e-3
GEO_MAX_BATCH_FRAMES = 8

GEO_RAYS_NEAR = 1
GEO_RAYS_FAR = 2

GEO_OBSERVER_UNMOVING = 0
GEO_OBSERVER_FROZEN_FALL = 1
GEO_OBSERVER_ORBITING = 2

NO_VALUE = 15.0


class GeoFrame(ctypes.Structure):
    """TransformationPipeline (SR/simulation/observer.rs:21-28), 208 bytes."""

    _fields_ = [
        ("display_to_movement", ctypes.c_float * 16),
        ("movement_to_central", ctypes.c_float * 16),
        ("central_to_uv", ctypes.c_float * 16),
        ("psi_factor_and_position", ctypes.c_float * 4),
    ]


class GeoScene(ctypes.Structure):
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


assert ctypes.sizeof(GeoFrame) == 208
assert ctypes.sizeof(GeoScene) == 32

_vp = ctypes.c_void_p
_u32 = ctypes.c_uint32
_f64 = ctypes.c_double
_int = ctypes.c_int

# name -> (restype, argtypes); mirrors include/geo/geo.h one-for-one.
SIGNATURES = {
    "geo_abi_version": (_int, []),
    "geo_status_str": (ctypes.c_char_p, [_int]),
    "geo_ctx_create": (_int, [_int, ctypes.POINTER(_vp)]),
    "geo_ctx_destroy": (None, [_vp]),
    "geo_set_sky": (_int, [_vp, _vp, _u32, _u32]),
    "geo_set_fan": (_int, [_vp, _vp, _u32]),
    "geo_solve_ray_fan": (_int, [_vp, _f64, _f64, _u32, _f64, _u32, _f64, _vp, _vp]),
    "geo_render_rows": (
        _int,
        [_vp, ctypes.POINTER(GeoFrame), ctypes.POINTER(GeoScene), _u32, _u32, _u32, _u32, _vp, _vp,
         _vp, _vp, _vp, _vp],
    ),
    "geo_render_bands": (
        _int,
        [_vp, ctypes.POINTER(GeoFrame), ctypes.POINTER(GeoScene), _u32, _u32, _u32, _u32, _u32, _u32, _vp,
         _vp, _vp, _vp, _vp, _vp],
    ),
    "geo_render_band_set": (
        _int,
        [_vp, ctypes.POINTER(GeoFrame), ctypes.POINTER(GeoScene), _u32, _u32, _u32, _u32, _u32, _u32, _vp,
         _vp, _vp, _vp, _vp, _vp],
    ),
    "geo_render_band_set_frames": (
        _int,
        [_vp, ctypes.POINTER(GeoFrame), _u32, ctypes.POINTER(GeoScene), _u32, _u32, _u32, _u32, _u32, _u32, _vp,
         ctypes.c_size_t, _vp, _vp],
    ),
    "geo_render_band_set_batch": (
        _int,
        [_vp, ctypes.POINTER(GeoFrame), ctypes.POINTER(GeoScene), _u32, _u32, _u32, _u32, _u32, _u32, _u32, _vp,
         ctypes.c_size_t, _vp, _vp],
    ),
    "geo_steps_flush": (_int, [_vp, _vp, _vp]),
    "geo_set_tile_order": (_int, [_vp, _u32, _u32, _vp]),
    "geo_set_dispatch": (_int, [_vp, _int, _u32]),
    "geo_dispatch_stats": (_int, [_vp, _vp, _vp]),
    "geo_time_next_render": (_int, [_vp, _vp, _vp]),
    "geo_assemble_bands": (_int, [_vp, _vp, ctypes.c_size_t, ctypes.c_size_t, _u32, _u32, _u32, _u32, _u32, _u32,
                                  _vp, _vp]),
    "geo_assemble_lead": (_int, [_vp, _vp, ctypes.c_size_t, _u32, _vp, ctypes.c_size_t, ctypes.c_size_t, _u32, _u32,
                                 _u32, _u32, _u32, _u32, _vp, _vp]),
    "geo_assemble_shares": (_int, [_vp, _vp, ctypes.c_size_t, _u32, _vp, ctypes.c_size_t, ctypes.c_size_t, _u32,
                                   _u32, _u32, _u32, _u32, _u32, _vp, _vp]),
    "geo_pack_rgb": (_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp]),
    "geo_rays_create": (_int, [_vp, ctypes.c_float, _u32, _u32, _vp, ctypes.POINTER(_vp)]),
    "geo_rays_destroy": (None, [_vp]),
    "geo_rays_count": (_int, [_vp]),
    "geo_rays_set_positions": (_int, [_vp, _vp]),
    "geo_rays_update": (_int, [_vp, _vp, _int, _u32, _int, _vp, _vp]),
    "geo_rays_vertices": (_vp, [_vp]),
    "geo_points_create": (_int, [_vp, ctypes.c_float, _vp, _u32, _vp, _int, _int, ctypes.c_ulonglong,
                                 ctypes.POINTER(_vp)]),
    "geo_points_destroy": (None, [_vp]),
    "geo_points_count": (_int, [_vp]),
    "geo_points_update": (_int, [_vp, _vp, _f64, _vp]),
    "geo_points_vertices": (_vp, [_vp, _int]),
    "geo_points_positions": (_int, [_vp, _vp, _vp]),
    "geo_draw_points": (_int, [_vp, ctypes.POINTER(GeoFrame), _vp, _u32, _u32, _u32, _u32, _u32, _vp, _vp, _vp]),
    "geo_points_draw": (_int, [_vp, ctypes.POINTER(GeoFrame), _u32, _u32, _u32, _u32, _vp, _vp, _vp]),
    "geo_observer_create": (_int, [_f64, _f64, _f64, _f64, ctypes.POINTER(_vp)]),
    "geo_observer_destroy": (None, [_vp]),
    "geo_observer_set_position": (_int, [_vp, _f64, _f64, _f64]),
    "geo_observer_get_position": (_int, [_vp, ctypes.POINTER(_f64)]),
    "geo_observer_set_camera": (_int, [_vp, _f64, _f64]),
    "geo_observer_set_energy": (_int, [_vp, _f64]),
    "geo_observer_set_state": (_int, [_vp, _int]),
    "geo_observer_start_orbit": (_int, [_vp, _f64]),
    "geo_observer_get_state": (_int, [_vp]),
    "geo_observer_radial_position": (_f64, [_vp]),
    "geo_observer_update_position": (_int, [_vp, _f64, _f64, _f64, _f64]),
    "geo_observer_move_camera": (_int, [_vp, _f64, _f64]),
    "geo_observer_update_screen_format": (_int, [_vp, _f64, _f64]),
    "geo_observer_is_singular": (_int, [_vp]),
    "geo_observer_calc_transformation_pipeline": (_int, [_vp, ctypes.POINTER(GeoFrame)]),
}


class GeoError(RuntimeError):
    def __init__(self, fn: str, status: int):
        self.status = status
        super().__init__(f"{fn} failed: {status} ({status_str(status)})")


def _load() -> ctypes.CDLL:
    # One HIP runtime per process: torch's libtorch_hip NEEDs "libamdhip64.so"
    # while libgeo NEEDs the soname "libamdhip64.so.7".  Loading torch first
    # makes libgeo bind to torch's already-loaded runtime (soname match), so
    # torch tensors' device pointers are valid in libgeo.  Without torch in the
    # process (a plain C/Rust host) libgeo uses /opt/rocm's runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libgeo.so not found at {LIB_PATH}; build it with `python -c 'import __graft_entry__ as g; g.build()'`"
        )
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def status_str(status: int) -> str:
    return lib.geo_status_str(status).decode()


def check(fn: str, status: int) -> int:
    if status < 0:
        raise GeoError(fn, status)
    return status
