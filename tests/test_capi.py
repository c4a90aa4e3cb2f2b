"""libgeo.so loads, exports every symbol include/geo/geo.h declares, and its host
(observer) half agrees with the oracle.  No device compute here."""
import ctypes
import math
import os
import re

import numpy as np
import pytest

import oracle as O
import schwarzschild_raytracer_wgpu_amd as g
from schwarzschild_raytracer_wgpu_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "geo", "geo.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(geo_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_api():
    syms = declared_symbols()
    for s in ("geo_render_rows", "geo_ctx_create", "geo_set_sky", "geo_set_fan", "geo_solve_ray_fan",
              "geo_observer_calc_transformation_pipeline"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    assert set(declared_symbols()) == set(_lib.SIGNATURES), "ctypes table out of sync with geo.h"


def test_abi_and_status():
    assert _lib.lib.geo_abi_version() == 8
    assert _lib.status_str(0) == "ok"
    assert "invalid" in _lib.status_str(-1)


def test_struct_layout():
    assert ctypes.sizeof(g.GeoFrame) == 208  # TransformationPipeline, observer.rs:21-28
    assert ctypes.sizeof(g.GeoScene) == 32


def test_null_args_rejected():
    lib = _lib.lib
    assert lib.geo_ctx_create(0, None) == _lib.GEO_EINVAL
    assert lib.geo_render_rows(None, None, None, 1, 1, 0, 1, None, None, None, None, None, None) == _lib.GEO_EINVAL
    assert lib.geo_set_sky(None, None, 1, 1) == _lib.GEO_EINVAL
    fr = (g.GeoFrame * 9)()
    sc = g.GeoScene()
    buf = ctypes.create_string_buffer(64)
    for n in (0, _lib.GEO_MAX_BATCH_FRAMES + 1):  # batch sizes out of range, before any device work
        assert lib.geo_render_band_set_frames(None, fr, n, ctypes.byref(sc), 8, 8, 8, 0, 8, 1, buf, 256, None,
                                              None) == _lib.GEO_EINVAL


def test_ctx_without_gpu_fails_loudly():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(g.GeoError) as e:
        g.Context(0)
    assert e.value.status == _lib.GEO_ENODEV


@pytest.mark.parametrize("pos,cam,state,wh", [
    ((2.5, 0.0, 0.1), (math.pi, 0.0), 1, (256, 256)),
    ((25.0, 0.0, 1.0), (math.pi, 0.0), 1, (1920, 1080)),
    ((2.5, 0.0, 0.1), (math.pi + 0.6, 0.3), 0, (3840, 2160)),
    ((-3.0, 4.0, 2.0), (0.3, -0.4), 1, (640, 480)),
])
def test_observer_matches_oracle(pos, cam, state, wh):
    rs = 1.0 if pos[0] != 25.0 else 10.0
    o = g.Observer(rs, math.pi / 2, *wh)
    o.set_position(*pos)
    o.set_camera(*cam)
    if state == 0:
        o.start_unmoving()
    f = np.frombuffer(bytes(o.calc_transformation_pipeline()), np.float32)
    ref = np.frombuffer(bytes(O.observer_frame(rs, math.pi / 2, wh[0], wh[1], pos, cam[0], cam[1], state, 1.0)),
                        np.float32)
    np.testing.assert_allclose(f, ref, rtol=0, atol=2e-7)


def test_observer_reference_semantics():
    o = g.Observer(10.0, math.pi / 2, 1920, 1080)  # Observer::new defaults (observer.rs:68-87)
    assert o.get_position() == (25.0, 0.0, 1.0)
    f = o.calc_transformation_pipeline()
    d = np.frombuffer(bytes(f), np.float32)
    # FOV scale in column w (observer.rs:253-254)
    np.testing.assert_allclose(d[12:16], [1.0, 1920 / 1080, 1.0, 1.0], rtol=1e-6)
    # FrozenFall E = 1: psi = 1/h, factor sqrt((psi-1)/psi) = sqrt(rs/r)
    r = math.sqrt(626.0)
    assert abs(f.psi_factor_and_position[0] - math.sqrt(10.0 / r)) < 1e-6
    o.start_unmoving()
    assert o.calc_transformation_pipeline().psi_factor_and_position[0] == 0.0
    # move_camera clamps theta at +-(PI/2 - 1e-4) (observer.rs:274-286)
    o.move_camera(0, 1e9)
    o.update_position((1.0, 0.0, 0.0), 0.016)  # forward along camera phi = PI: x decreases by 0.051
    x, y, z = o.get_position()
    assert abs(x - (25.0 - 0.051)) < 1e-12 and abs(y) < 1e-12


def test_observer_orbit_api():
    o = g.Observer(1.0, math.pi / 2, 256, 256)
    o.set_position(0.5, 0.0, 0.0)
    assert not o.start_orbit(3.0)  # inside the horizon: Orbit::new returns None (orbit.rs:33-35)
    o.set_position(6.0, 0.0, 0.0)
    assert o.start_orbit(3.0)
    assert o.state == _lib.GEO_OBSERVER_ORBITING
    p0 = o.get_position()
    for _ in range(10):
        o.update_position((0.0, 0.0, 0.0), 0.1)
    p1 = o.get_position()
    assert p0 != p1 and abs(math.hypot(p1[0], p1[1]) - 6.0) < 0.5
    d = np.frombuffer(bytes(o.calc_transformation_pipeline()), np.float32)
    assert np.all(np.isfinite(d))
