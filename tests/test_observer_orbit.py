"""N2: observer motion states + orbit (SR/simulation/observer.rs:104-124,
162-169, 197-262; orbit.rs).  The library's host observer (observer.cpp +
geo_orbit.h) replays an orbit frame by frame against the oracle's independent
restatement (oracle/geo_oracle_points.c): f64 positions within 1e-12
relative (both use glibc, but the compilers may pair sin/cos into sincos), the
208-byte f32 frame within one f32 ulp (in practice identical).  CPU only."""
import math

import numpy as np
import pytest

import oracle as O
import schwarzschild_raytracer_wgpu_amd as g

W, H = 640, 360


@pytest.mark.parametrize("rotation", [2.0, 3.2, 4.0, 6.0])
def test_orbit_replay_frames_bitexact(rotation):
    obs = g.Observer(1.0, math.pi / 2, W, H)
    obs.set_position(2.5, 0.0, 0.1)
    obs.set_camera(math.pi + 0.3, 0.1)
    started = obs.start_orbit(rotation)
    ref = O.orbit_frames(1.0, math.pi / 2, W, H, (2.5, 0.0, 0.1), (math.pi + 0.3, 0.1), rotation, 240, 1 / 60)
    assert started == (ref is not None)
    frames, pos = ref
    assert obs.state == 2  # GEO_OBSERVER_ORBITING
    for f in range(240):
        obs.update_position((0.0, 0.0, 0.0), 1 / 60)
        np.testing.assert_allclose(np.array(obs.get_position()), pos[f], rtol=1e-12, atol=1e-14)
        a = np.frombuffer(bytes(obs.calc_transformation_pipeline()), np.float32)
        b = np.frombuffer(bytes(frames[f]), np.float32)
        ulp = np.abs(a.view(np.int32).astype(np.int64) - b.view(np.int32).astype(np.int64))
        assert ulp.max() <= 1, (f, ulp.max())


def test_orbit_cannot_start_inside_horizon():
    obs = g.Observer(1.0, math.pi / 2, W, H)
    obs.set_position(0.5, 0.0, 0.0)
    assert not obs.start_orbit(3.0)
    assert obs.state == 1  # stays FrozenFall (observer.rs:164-168)
    assert O.orbit_frames(1.0, math.pi / 2, W, H, (0.5, 0.0, 0.0), (math.pi, 0.0), 3.0, 1, 1 / 60) is None


def test_orbit_moves_and_is_bound():
    """rotation 3.2 at r = 2.5: a bound, precessing orbit outside the photon
    sphere; the aberration factor stays in (0, 1)."""
    obs = g.Observer(1.0, math.pi / 2, W, H)
    obs.set_position(2.5, 0.0, 0.1)
    obs.start_orbit(3.2)
    rs_, ks = [], []
    for _ in range(600):
        obs.update_position((0.0, 0.0, 0.0), 1 / 60)
        rs_.append(obs.get_radial_position())
        ks.append(obs.calc_transformation_pipeline().psi_factor_and_position[0])
    assert 1.5 < min(rs_) and max(rs_) < 10.0 and max(rs_) - min(rs_) > 0.5
    assert 0.0 < min(ks) and max(ks) < 1.0
