"""The accretion-disk point path on the CPU oracle
(oracle/geo_oracle_points.c): the reference's own RayConnector tests
(SR/simulation/tests.rs:15-79, 5e-4 rad — "one pixel on a 4k display"), run
literally on both transcendental variants, plus orbit/point-cloud and
point-projection properties.  The HIP kernels are tied to the `libm=False`
variant bit for bit by tests/test_gpu_points.py."""
import math

import numpy as np
import pytest

import oracle as O

TOL = np.float32(5e-4)  # tests.rs:26, 59-60


def glam_acos_approx(v):
    v = np.float32(v)
    x = np.float32(abs(v))
    omx = max(np.float32(1) - x, np.float32(0))
    root = np.float32(math.sqrt(omx))
    c = [np.float32(k) for k in (-0.0012624911, 0.0066700901, -0.0170881256, 0.0308918810, -0.0501743046,
                                 0.0889789874, -0.2145988016, 1.5707963050)]
    r = c[0]
    for k in c[1:]:
        r = np.float32(r * x + k)
    r = np.float32(r * root)
    return r if v >= 0 else np.float32(np.float32(math.pi) - r)


def glam_angle_between(a, b):
    a, b = a.astype(np.float32), b.astype(np.float32)
    dot = np.float32(np.float32(a[0] * b[0] + a[1] * b[1]) + a[2] * b[2])
    la = np.float32(np.float32(a[0] * a[0] + a[1] * a[1]) + a[2] * a[2])
    lb = np.float32(np.float32(b[0] * b[0] + b[1] * b[1]) + b[2] * b[2])
    return glam_acos_approx(np.float32(dot / np.float32(math.sqrt(np.float32(la * lb)))))


@pytest.mark.parametrize("libm", [True, False], ids=["libm", "kernel_poly"])
def test_ray_connector_euclidian(libm):
    """tests.rs:15-38: rs = 0, connector at (20, 0, 0.1), observer on the
    r = 19 circle at 100 angles in [0, pi): reset_ray's incoming angle equals
    the Euclidean angle between (pos - obs) and -obs within 5e-4."""
    pos = np.array([20.0, 0.0, 0.1], np.float32)
    fails = []
    for i in range(100):
        angle = np.float32(np.float32(i) / np.float32(100) * np.float32(math.pi))
        obs = np.array([np.float32(19) * np.cos(angle), np.float32(19) * np.sin(angle), 0.0], np.float32)
        rc = O.Rays(0.0, pos, sides=1, libm=libm)
        out = rc.update(obs, reset=True)
        euclid = glam_angle_between(pos - obs, -obs)
        err = abs(euclid - out[0, 3])
        if not err < TOL:
            fails.append((i, float(err)))
    assert not fails, fails


@pytest.mark.parametrize("libm", [True, False], ids=["libm", "kernel_poly"])
def test_ray_connector_euclidian_tracing(libm):
    """tests.rs:42-79: rs = 5, observer flying once around the black hole on
    the r = 7 circle in 60 frames; 1-iteration updates track 5-iteration
    updates within 5e-4, near and far side."""
    pos = np.array([20.0, 0.0, 0.1], np.float32)
    rc = O.Rays(5.0, pos, sides=3, libm=libm)       # near + far, 1 iteration
    control = O.Rays(5.0, pos, sides=3, libm=libm)  # near + far, 5 iterations
    fails = []
    for i in range(60):
        angle = np.float32(np.float32(i) / np.float32(60) * np.float32(2 * math.pi))
        obs = np.array([np.float32(7) * np.cos(angle), np.float32(7) * np.sin(angle), 0.0], np.float32)
        out = rc.update(obs, iterations=1)
        out2 = control.update(obs, iterations=5)
        err = np.abs(out2[:, 3] - out[:, 3])
        if not np.all(err < TOL):
            fails.append((i, err.tolist()))
    assert not fails, fails


def test_kernel_transcendentals_track_libm():
    """The kernel's acos/atan polynomials change the RayConnector's answer by
    at most a few f32 ulps of the angle."""
    rng = np.random.default_rng(5)
    pos = rng.uniform(-25, 25, size=(300, 3)).astype(np.float32)
    pos[:, 2] *= 0.1
    obs = np.array([2.5, 0.0, 0.1], np.float32)
    a = O.Rays(1.0, pos, sides=3, libm=True).update(obs, reset=True)
    b = O.Rays(1.0, pos, sides=3, libm=False).update(obs, reset=True)
    assert np.max(np.abs(a[:, 3] - b[:, 3])) < 2e-6


def test_connector_state_machine():
    """needs_reset: set by new and by a nearly-straight ray (< 0.05 rad), which
    also skips the solve; a jump of the other end by > 0.5 forces a reset
    (5 iterations), so the result equals a fresh reset_ray."""
    pos = np.array([20.0, 0.0, 0.1], np.float32)
    rc = O.Rays(1.0, pos)
    assert rc.needs[0] == 1
    rc.update(np.array([-3.0, 1.0, 0.0], np.float32))
    assert rc.needs[0] == 0
    rc.update(np.array([10.0, 0.0, 0.05], np.float32))  # nearly on the line to pos
    assert rc.needs[0] == 1
    jumped = np.array([-5.0, 0.5, 0.2], np.float32)
    rc.update(np.array([-3.0, 1.0, 0.0], np.float32))
    a = rc.update(jumped)  # |r| jumps 3.16 -> 5.03
    fresh = O.Rays(1.0, pos).update(jumped, reset=True)
    assert a[0, 3] == fresh[0, 3]


def test_farside_angle_sign_and_symmetry():
    """Far-side rays (the long way round) report negative angles
    (calc_ray_angle, ray_connector.rs:155)."""
    rng = np.random.default_rng(9)
    pos = rng.uniform(12, 25, size=(64, 3)).astype(np.float32) * np.array([1, 1, 0.05], np.float32)
    out = O.Rays(1.0, pos, sides=3).update(np.array([-6.0, 0.3, 0.1], np.float32), reset=True)
    near, far = out[:64, 3], out[64:, 3]
    assert np.all(near > 0) and np.all(far < 0)


def accretion_disk(n, seed=1):
    """new_accretion_disk's distribution (point_cloud.rs:84-99): r in [16, 26),
    phi in [0, 2 pi), theta in [-0.1, 0.1)."""
    rng = np.random.default_rng(seed)
    r = 16 + 10 * rng.random(n)
    phi = rng.random(n) * 2 * math.pi
    th = 0.2 * (rng.random(n) - 0.5)
    return np.stack([r * np.cos(phi) * np.cos(th), r * np.sin(phi) * np.cos(th), r * np.sin(th)], 1).astype(np.float32)


def test_point_cloud_orbits_and_respawn():
    """PointCloud::new + 120 updates at dt = 1/60 s: deterministic, every point
    stays on a bound orbit or respawns into the disk (r in [16, 26] +- the
    orbit's excursion), angles finite, rs = 1."""
    model = accretion_disk(200)
    obs = np.tile(np.array([25.0, 0.0, 1.0], np.float32), (121, 1))
    dts = np.full(120, 1 / 60)
    near, far, pos = O.points_run(1.0, model, obs, dts, seed=42)
    near2, far2, pos2 = O.points_run(1.0, model, obs, dts, seed=42)
    assert np.array_equal(near, near2) and np.array_equal(far, far2)
    r = np.linalg.norm(pos, axis=1)
    assert np.all(r > 1.0) and np.all(r < 40.0)
    assert np.all(np.isfinite(near)) and np.all(np.isfinite(far))
    assert np.array_equal(near[:, :3], pos) and np.array_equal(far[:, :3], pos)
    # rotation 18..20 at r 16..26 is a bound, precessing orbit: particles move
    assert np.mean(np.linalg.norm(pos - model, axis=1)) > 0.05


def test_point_cloud_respawn_path():
    """rs = 15: every particle with rotation < sqrt(3) rs = 26 falls in; the
    respawn (reset at the new position, then update at the old one —
    point_cloud.rs:123-143) keeps the cloud populated with finite vertices."""
    model = accretion_disk(64, seed=3)
    obs = np.tile(np.array([40.0, 0.0, 1.0], np.float32), (401, 1))
    near, far, pos = O.points_run(15.0, model, obs, np.full(400, 0.5), seed=7)
    assert np.all(np.isfinite(near[:, 3])) and np.all(np.isfinite(far[:, 3]))
    assert np.all(np.linalg.norm(pos, axis=1) > 0)


def test_projection_straight_ahead_hits_frame_centre():
    """vs_main inverts fs_main's camera: in flat space for an unmoving observer
    (no aberration) a point straight ahead of the camera lands on the centre
    pixel, and points mirrored across the view axis land on mirrored pixels."""
    from helpers import default_frame

    w, h = 321, 181
    o = np.array([2.5, 0.0, 0.1], np.float32)
    frame = default_frame(w, h, pos=tuple(o), camera=(math.pi, 0.0), rs=0.0, state=0)
    fwd = np.array([-1.0, 0.0, 0.0], np.float32)  # polar2_to_carthesic(pi, 0)
    pts = np.stack([o + 10 * fwd, o + 10 * fwd + np.array([0, 2, 0], np.float32),
                    o + 10 * fwd + np.array([0, -2, 0], np.float32)]).astype(np.float32)
    rays = O.Rays(0.0, pts, sides=1)
    verts = rays.update(o, reset=True)
    _, xy = O.draw_points(frame, verts, w, h)
    assert tuple(xy[0]) == (w // 2, h // 2)
    assert xy[1, 1] == xy[2, 1] == h // 2
    assert xy[1, 0] + xy[2, 0] == w - 1 and xy[1, 0] != xy[2, 0]
    behind = O.Rays(0.0, (o - 10 * fwd)[None], sides=1).update(o, reset=True)
    _, xy = O.draw_points(frame, behind, w, h)
    assert tuple(xy[0]) == (-1, -1)  # clipped
