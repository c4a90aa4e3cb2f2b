#!/usr/bin/env python3
"""Fits the fixed polynomials of the sky-direction transcendentals (round 6,
geo_math.h `sincos_sky_`, `acos_pi_`, `atan2_turns_`): near-minimax
absolute-error fits (Lawson's iteratively reweighted least squares on a dense
grid), coefficients rounded to f32, and the f32 evaluation's error against
numpy's f64 functions measured with each fma emulated in f64 (the product of
two f32 is exact in f64).  Prints the coefficients as C literals.

    python tools/fit_sky_polys.py

The forms:
  sin r = r + r z S(z),  cos r = 1 + z C(z),  z = r^2, |r| <= pi/2 (S, C cubic)
  acos(a) / pi = sqrt(1 - a) P(a),  0 <= a <= 1                     (P degree 6)
  atan(t) / (2 pi) = t A(t^2),  |t| <= tan(pi/8)                    (A cubic)
"""
from __future__ import annotations

import numpy as np

f32 = np.float32


def lawson(X, f, its=200):
    w = np.ones_like(f)
    for _ in range(its):
        sw = np.sqrt(w)
        c, *_ = np.linalg.lstsq(X * sw[:, None], f * sw, rcond=None)
        e = np.abs(X @ c - f)
        w = np.maximum(w * e / (w * e).sum() * len(f), 1e-15)
    return c


def fma(a, b, c):
    return f32(np.float64(a) * np.float64(b) + np.float64(c))


def horner(cs, z):
    p = f32(cs[-1]) * np.ones_like(z, dtype=f32)
    for c in cs[-2::-1]:
        p = fma(p, z, f32(c))
    return p


def lit(c):
    return "%.9ef" % f32(c)


def main():
    # sin/cos on [-pi/2, pi/2]
    r = np.linspace(0, np.pi / 2, 400001)
    z = r * r
    S = lawson((r * z)[:, None] * np.vander(z, 4, increasing=True), np.sin(r) - r)
    Cc = lawson(z[:, None] * np.vander(z, 4, increasing=True), np.cos(r) - 1)
    S32, C32 = [f32(c) for c in S], [f32(c) for c in Cc]
    r32 = r.astype(f32)
    z32 = (r32 * r32).astype(f32)
    sn = fma(f32(1) * (r32 * z32).astype(f32), horner(S32, z32), r32)
    cs = fma(z32, horner(C32, z32), f32(1))
    print("sin S:", ", ".join(map(lit, S32)), " max abs err %.2e" % np.abs(sn - np.sin(r32.astype(np.float64))).max())
    print("cos C:", ", ".join(map(lit, C32)), " max abs err %.2e" % np.abs(cs - np.cos(r32.astype(np.float64))).max())

    # acos / pi
    a = np.linspace(0, 1, 400001)
    s = np.sqrt(1 - a)
    P = lawson(np.vander(a, 7, increasing=True) * s[:, None], np.arccos(a) / np.pi)
    P32 = [f32(c) for c in P]
    a32 = a.astype(f32)
    s32 = np.sqrt((f32(1) - a32).astype(f32)).astype(f32)  # correctly rounded
    v = (s32 * horner(P32, a32)).astype(f32)
    print("acos/pi P:", ", ".join(map(lit, P32)),
          " max abs err %.2e" % np.abs(v - np.arccos(a32.astype(np.float64)) / np.pi).max())

    # atan / 2pi on [0, tan(pi/8)]
    t = np.linspace(0, np.tan(np.pi / 8), 400001)
    A = lawson(t[:, None] * np.vander(t * t, 4, increasing=True), np.arctan(t) / (2 * np.pi))
    A32 = [f32(c) for c in A]
    t32 = t.astype(f32)
    z32 = (t32 * t32).astype(f32)
    u = fma(t32, horner(A32, z32), f32(0))
    print("atan/2pi A:", ", ".join(map(lit, A32)),
          " max abs err %.2e" % np.abs(u - np.arctan(t32.astype(np.float64)) / (2 * np.pi)).max())


if __name__ == "__main__":
    main()
