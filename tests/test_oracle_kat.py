"""Pins the f64 oracle (restatement of SR/simulation/sphere_ray_tracer.rs:35-193)
against analytic known answers and its committed golden vectors.  CPU only.

The reference's own hot-path test (SR/simulation/tests.rs:8-13,
sphere_geodesics_test) asserts nothing; these KATs are the pins.
"""
import math
import os

import numpy as np
import pytest

import oracle as O

STEP = math.pi / 100
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_reference_smoke_case_runs():
    # tests.rs:8-13: SphereRayTracer::new(100., 10., 100, PI/100., 10).solve_ray_fan(25.)
    fan = O.solve_ray_fan(100.0, 10.0, 100, STEP, 20, 25.0)
    assert fan.shape == (20,)
    assert np.all(np.isfinite(fan))
    gold = np.load(os.path.join(GOLD, "fans.npz"))["fan_test"]
    np.testing.assert_array_equal(fan, gold)


@pytest.mark.parametrize("r,R", [(25.0, 100.0), (25.0, 500.0), (2.5, 50.0), (40.0, 41.0)])
def test_kat1_flat_space_matches_triangle(r, R):
    """rs = 0: straight lines.  Traveled angle = PI - alpha - asin(r sin(alpha)/R),
    alpha = PI/2 - theta (angle between the view ray and the inward radial)."""
    errs = []
    for theta in np.linspace(-math.pi / 2 + 1e-3, math.pi / 2 - 1e-3, 201):
        a, _ = O.geodesic_at_theta(R, 0.0, 1000, STEP, r, float(theta))
        alpha = math.pi / 2 - theta
        exact = math.pi - alpha - math.asin(r * math.sin(alpha) / R)
        errs.append(abs(a - exact))
    assert max(errs) < 1e-7, max(errs)


@pytest.mark.parametrize("r", [2.5, 5.0, 25.0])
def test_kat2_capture_threshold(r):
    """Falling rays (theta > 0) from r > 1.5 rs are captured iff b < 3*sqrt(3)/2 rs."""
    rs, R = 1.0, 50.0
    bc = 1.5 * math.sqrt(3.0) * rs
    e = math.sqrt(1.0 - rs / r)
    checked = 0
    for theta in np.linspace(1e-3, math.pi / 2 - 1e-3, 400):
        b = r * math.cos(theta) / e
        if abs(b - bc) < 1e-3 * bc:
            continue
        a, _ = O.geodesic_at_theta(R, rs, 100000, STEP, r, float(theta))
        captured = a == 15.0
        assert captured == (b < bc), (theta, b, a)
        checked += 1
    assert checked > 300


def test_kat2_outgoing_rays_always_hit():
    rs, R, r = 1.0, 50.0, 2.5
    for theta in np.linspace(-math.pi / 2 + 1e-3, -1e-3, 200):
        a, _ = O.geodesic_at_theta(R, rs, 100000, STEP, r, float(theta))
        assert a != 15.0 and 0.0 <= a < math.pi


def test_kat3_scale_invariance():
    """The step is an angle: (500, 10, r=25) and (50, 1, r=2.5) give the same geodesics."""
    # theta = 0 exactly is excluded: there u'_0 = sqrt(1/b^2 - h/r^2) has a
    # radicand that is 0 in exact arithmetic and +-1 ulp of noise in f64, so the
    # two scalings start from different u'_0 ~ 1e-8 (sphere_ray_tracer.rs:123).
    for theta in np.linspace(-math.pi / 2, math.pi / 2, 256):
        a1, s1 = O.geodesic_at_theta(500.0, 10.0, 1000, STEP, 25.0, float(theta))
        a2, s2 = O.geodesic_at_theta(50.0, 1.0, 1000, STEP, 2.5, float(theta))
        assert abs(a1 - a2) <= 1e-12 and s1 == s2
    f1 = O.solve_ray_fan(500.0, 10.0, 1000, STEP, 400, 25.0)
    f2 = O.solve_ray_fan(50.0, 1.0, 1000, STEP, 400, 2.5)
    assert np.abs(f1.astype(np.float64) - f2).max() <= 1e-6


def test_kat4_radial_nodes():
    fan = O.solve_ray_fan(500.0, 10.0, 1000, STEP, 400, 25.0)
    assert fan[0] == np.float32(math.pi / 2 - 15.0)  # looking into the hole: NO_VALUE
    assert fan[-1] == np.float32(math.pi / 2)  # looking straight out: angle 0
    # flat space radial inward ray passes the centre: PI
    a, _ = O.solve_geodesic(100.0, 0.0, 1000, STEP, 25.0, 1.0, 0.0, True)
    assert a == math.pi


def test_reference_default_fan_golden_and_shape():
    """The fan the reference computes every frame (lib.rs:292-295) at its default
    pose: 119 nodes below -7 (118 captured + the radial node 0), 281 hits."""
    gold = np.load(os.path.join(GOLD, "fans.npz"))
    fan = O.solve_ray_fan(500.0, 10.0, 1000, STEP, 400, math.sqrt(25.0 ** 2 + 1.0))
    np.testing.assert_array_equal(fan, gold["fan_ref"])
    f25 = O.solve_ray_fan(500.0, 10.0, 1000, STEP, 400, 25.0)
    assert int((f25 < -7).sum()) == 119 and int((f25 >= -7).sum()) == 281
    np.testing.assert_allclose(f25[395:], [1.5321684, 1.5418259, 1.5514829, 1.5611397, 1.5707964], atol=1e-6)


def test_theta_sweep_golden():
    gold = np.load(os.path.join(GOLD, "fans.npz"))
    for t, a, s in zip(gold["thetas"], gold["angles"], gold["steps"]):
        a2, s2 = O.geodesic_at_theta(50.0, 1.0, 2048, STEP, 2.5, float(t))
        assert a2 == a and s2 == s


def test_config_radii_fan_goldens():
    """400-node fans at the configs' observer radii (rs = 1): configs 1-4 at
    |(2.5, 0, 0.1)| and config 5 at 1.3 rs.  Inside the photon sphere every
    falling ray (theta > 0: nodes 0..199) is captured by the pre-filter
    (sphere_ray_tracer.rs:116)."""
    gold = np.load(os.path.join(GOLD, "fans.npz"))
    np.testing.assert_array_equal(O.solve_ray_fan(50.0, 1.0, 1000, STEP, 400, math.sqrt(2.5 ** 2 + 0.01)),
                                  gold["fan_cfg"])
    f5 = O.solve_ray_fan(50.0, 1.0, 1000, STEP, 400, 1.3)
    np.testing.assert_array_equal(f5, gold["fan_cfg5"])
    assert np.all(f5[:200] < -7)
    assert np.all(f5[-20:] > -7)  # outgoing rays near radial escape to the sphere
