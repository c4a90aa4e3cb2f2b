#!/usr/bin/env python3
"""Coefficients of the Dormand-Prince RK5(4) pair in Nystrom form for the
adaptive mode (GEO_MODE_ADAPTIVE): the autonomous system (U, V)' = (V, F(U))
gives U_i = U + c_i h V + h^2 sum_j (A^2)_ij G_j with G_j = F(U_j), so the
stage U values need no V_i.  Exact rationals, each rounded once (nearest-even)
to f32; printed as C hex-float literals for csrc/geo_pixel.h and
oracle/geo_oracle.c (both carry the same table).

Dormand & Prince, "A family of embedded Runge-Kutta formulae",
J. Comput. Appl. Math. 6 (1980) 19-26, Table 2 (RK5(4)7M).
"""
from fractions import Fraction as Fr
import math
import struct

A = [[Fr(0)] * 7 for _ in range(7)]
A[1][0] = Fr(1, 5)
A[2][:2] = [Fr(3, 40), Fr(9, 40)]
A[3][:3] = [Fr(44, 45), Fr(-56, 15), Fr(32, 9)]
A[4][:4] = [Fr(19372, 6561), Fr(-25360, 2187), Fr(64448, 6561), Fr(-212, 729)]
A[5][:5] = [Fr(9017, 3168), Fr(-355, 33), Fr(46732, 5247), Fr(49, 176), Fr(-5103, 18656)]
A[6][:6] = [Fr(35, 384), Fr(0), Fr(500, 1113), Fr(125, 192), Fr(-2187, 6784), Fr(11, 84)]
B5 = A[6][:6] + [Fr(0)]
B4 = [Fr(5179, 57600), Fr(0), Fr(7571, 16695), Fr(393, 640), Fr(-92097, 339200), Fr(187, 2100), Fr(1, 40)]
C = [sum(row) for row in A]
E = [b5 - b4 for b5, b4 in zip(B5, B4)]


def f32(q: Fr) -> float:
    """Exact rational -> nearest-even binary32."""
    if q == 0:
        return 0.0
    s = -1 if q < 0 else 1
    q = abs(q)
    e = math.floor(math.log2(q.numerator) - math.log2(q.denominator))
    while Fr(2) ** e > q:
        e -= 1
    while Fr(2) ** (e + 1) <= q:
        e += 1
    m = q / Fr(2) ** (e - 23)  # in [2^23, 2^24)
    n = m.numerator // m.denominator
    rem = m - n
    if rem > Fr(1, 2) or (rem == Fr(1, 2) and n % 2 == 1):
        n += 1
    v = s * n * 2.0 ** (e - 23)
    assert struct.unpack("f", struct.pack("f", v))[0] == v
    return v


def A2(i, j):
    return sum(A[i][m] * A[m][j] for m in range(7))


def table():
    rows = {}
    rows["c"] = [C[i] for i in range(1, 6)]  # c2..c6
    rows["a2"] = {i: [A2(i, j) for j in range(i - 1)] for i in range(2, 6)}  # stages 3..6: j < i-1
    rows["bA"] = [sum(B5[i] * A[i][j] for i in range(7)) for j in range(6)]
    rows["b"] = B5[:6]
    rows["eA"] = [sum(E[i] * A[i][j] for i in range(7)) for j in range(6)]
    assert rows["bA"][5] == 0 and sum(rows["bA"]) == Fr(1, 2) and sum(E) == 0
    assert all(A2(i, i - 1) == 0 for i in range(1, 7))
    return rows


def hexf(q):
    return float.hex(f32(q)) + "f"


if __name__ == "__main__":
    t = table()
    print("// c2..c6")
    print(", ".join(hexf(q) for q in t["c"]))
    for i, r in t["a2"].items():
        print(f"// (A^2) row {i + 1}, j = 1..{i - 1}")
        print(", ".join(hexf(q) for q in r))
    print("// bA, j = 1..5 (j = 6 is 0)")
    print(", ".join(hexf(q) for q in t["bA"][:5]))
    print("// b, j = 1..6 (b2 = 0)")
    print(", ".join(hexf(q) for q in t["b"]))
    print("// eA = (b5 - b4) A, j = 1..6")
    print(", ".join(hexf(q) for q in t["eA"]))
