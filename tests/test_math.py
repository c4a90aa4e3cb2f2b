"""Accuracy of the fixed-order f32 transcendentals (geo_math.h, mirrored by the
oracle's geo_oracle_{asinf,atan2f,sincosf}) against libm in f64.  CPU only;
the GPU tests check the kernel's bits equal the oracle's."""
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
