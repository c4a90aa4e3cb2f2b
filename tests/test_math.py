"""Accuracy of the fixed-order f32 transcendentals (geo_math.h, mirrored by the
oracle's geo_oracle_{asinf,atan2f,sincosf} and, for the per-pixel sky
direction, geo_oracle_{sincos_sky,acos_pi,atan2_turns}) against libm in f64.
CPU only; the GPU tests check the kernel's bits equal the oracle's."""
import math

import numpy as np

import oracle as O


def ulp(x):
    return np.spacing(np.float32(abs(x)))


def test_asinf_accuracy():
    xs = np.concatenate([np.linspace(-1, 1, 20001), [0.5, -0.5, 0.49999997, 0.50000006, 1.0, -1.0, 0.0]])
    worst = 0.0
    for x in xs.astype(np.float32):
        got = O.asinf(float(x))
        ref = math.asin(float(x))
        worst = max(worst, abs(got - ref))
        assert abs(got - ref) <= 3 * ulp(ref) + 1e-12, (x, got, ref)
    assert O.asinf(1.5) == np.float32(math.pi / 2)  # clamped


def test_atan2f_accuracy():
    rng = np.random.default_rng(1)
    pts = rng.standard_normal((20000, 2)).astype(np.float32)
    for y, x in pts:
        got = O.atan2f(float(y), float(x))
        ref = math.atan2(float(y), float(x))
        assert abs(got - ref) <= 4 * ulp(ref) + 1e-9, (y, x, got, ref)
    assert O.atan2f(0.0, 0.0) == 0.0
    assert abs(O.atan2f(0.0, -1.0) - math.pi) < 1e-6
    assert abs(O.atan2f(1.0, 0.0) - math.pi / 2) < 1e-6
    assert abs(O.atan2f(-1.0, 0.0) + math.pi / 2) < 1e-6


def test_sincosf_accuracy():
    for x in np.linspace(-70, 70, 50001).astype(np.float32):
        s, c = O.sincosf(float(x))
        assert abs(s - math.sin(float(x))) <= 2e-7 and abs(c - math.cos(float(x))) <= 2e-7, x


# ---- the per-pixel sky-direction forms (round 6): absolute error <= 2e-7 ----


def test_sincos_sky_accuracy():
    """sin and cos by the reduction modulo pi (the deflected angle lambda' of
    every pixel lies in [-8, 2]; a discarded black-hole lane's may be
    anything, so the range checked is wider)."""
    xs = np.concatenate([np.linspace(-70, 70, 100001), np.linspace(-8, 2, 20001),
                         [k * math.pi / 2 for k in range(-40, 41)]]).astype(np.float32)
    worst = 0.0
    for x in xs:
        s, c = O.sincos_sky(float(x))
        worst = max(worst, abs(s - math.sin(float(x))), abs(c - math.cos(float(x))))
    assert worst <= 2e-7, worst  # cos near r = +-pi/2: 1 + z C(z) cancels to ~0
    s, c = O.sincos_sky(0.0)
    assert s == 0.0 and c == 1.0


def test_acos_pi_accuracy():
    """acos(x) / pi on [-1, 1] (the sky's V = 1/2 - asin(z)/pi and the fan
    index's (pi/2 - asin(st))/pi): within 1.5e-7, in [0, 1] for every input
    including |x| > 1 and NaN."""
    xs = np.concatenate([np.linspace(-1, 1, 200001), [0.5, -0.5, 1.0, -1.0, 0.0, -0.0, 1 - 2**-24, -1 + 2**-24,
                                                      2**-30, -2**-30]]).astype(np.float32)
    worst = 0.0
    for x in xs:
        got = O.acos_pi(float(x))
        worst = max(worst, abs(got - math.acos(float(x)) / math.pi))
        assert 0.0 <= got <= 1.0
    assert worst <= 1.5e-7, worst
    assert O.acos_pi(1.5) < 1e-14 and O.acos_pi(-1.5) == 1.0  # |x| clamped to 1 (sqrt floor 2^-48)
    assert 0.0 <= O.acos_pi(float("nan")) < 1e-14


def test_atan2_turns_accuracy():
    """atan2(y, x) / 2pi taken into [0, 1]: within 1e-7 (the U wrap at the
    seam measured as a distance on the circle), the axes and signed zeros."""
    rng = np.random.default_rng(11)
    pts = np.concatenate([rng.standard_normal((60000, 2)), rng.uniform(-1, 1, (20000, 2)) * 1e-3]).astype(np.float32)
    worst = 0.0
    for y, x in pts:
        got = O.atan2_turns(float(y), float(x))
        assert 0.0 <= got <= 1.0
        ref = (math.atan2(float(y), float(x)) / (2 * math.pi)) % 1.0
        d = abs(got - ref)
        worst = max(worst, min(d, 1.0 - d))
    assert worst <= 1e-7, worst
    assert O.atan2_turns(0.0, 0.0) == 0.0 and O.atan2_turns(-0.0, 0.0) == 0.0
    assert O.atan2_turns(0.0, -1.0) == 0.5 and O.atan2_turns(-0.0, -1.0) == 0.5
    assert O.atan2_turns(1.0, 0.0) == 0.25 and O.atan2_turns(-1.0, 0.0) == 0.75
    assert math.copysign(1.0, O.atan2_turns(0.0, 1.0)) == 1.0  # never -0
