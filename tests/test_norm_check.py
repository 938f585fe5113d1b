"""CPU check of the RMSNorm certainty test's arithmetic (csrc/device_util.h rms_mean_certain, DESIGN.md
§3): whenever the integer test on q = fl64(T/n) passes, no float32 rounding boundary lies in
q·[1 − ρ, 1 + ρ], ρ = n·2^−51 + 2^−48 — checked exactly with rationals on random q, on q placed just
inside / outside the margin around a boundary, and at binade edges.  Restates the device function
bit for bit (test infrastructure, not the product)."""
import random
import struct
from fractions import Fraction

import numpy as np


def certain(q, n):
    """rms_mean_certain(q, n) of csrc/device_util.h on a Python float."""
    b = struct.unpack("<Q", struct.pack("<d", q))[0]
    ex = (b >> 52) & 0x7FF
    low = b & 0x1FFFFFFF
    dist = low - 0x10000000 if low >= 0x10000000 else 0x10000000 - low
    special = b == 0 or ex == 0x7FF
    normal = (1023 - 126) <= ex <= (1023 + 127) and n <= (1 << 22)
    return special or (normal and dist > 4 * n + 40)


def boundaries(q):
    """the float32 rounding boundaries (midpoints) next to fl32(q), exact"""
    f = np.float32(q)
    lo, hi = np.nextafter(f, np.float32(0)), np.nextafter(f, np.float32(np.inf))
    return (Fraction(float(f)) + Fraction(float(lo))) / 2, (Fraction(float(f)) + Fraction(float(hi))) / 2


def sound(q, n):
    rho = Fraction(n, 2 ** 51) + Fraction(1, 2 ** 48)
    m_lo, m_hi = boundaries(q)
    Q = Fraction(q)
    return Q * (1 - rho) > m_lo and Q * (1 + rho) < m_hi


def test_certain_implies_no_boundary():
    rng = random.Random(5)
    hits = 0
    for n in (512, 2048, 3072, 16384):
        for _ in range(3000):
            q = rng.uniform(0.5, 2.0) * 2.0 ** rng.randint(-60, 60)
            if certain(q, n):
                hits += 1
                assert sound(q, n), (q, n)
        # q at a boundary offset by d units of its last place: certain only past the margin
        for _ in range(300):
            f = np.float32(rng.uniform(1.0, 2.0) * 2.0 ** rng.randint(-30, 30))
            mid = (float(f) + float(np.nextafter(f, np.float32(np.inf)))) / 2  # exact in double
            for d in (0, 1, 4 * n + 32, 4 * n + 40, 4 * n + 41, 4 * n + 200, -(4 * n + 41), -(4 * n + 200)):
                q = float(np.nextafter(mid, np.inf if d > 0 else -np.inf)) if d == 1 else mid
                if abs(d) > 1:
                    b = struct.unpack("<Q", struct.pack("<d", mid))[0] + d
                    q = struct.unpack("<d", struct.pack("<Q", b))[0]
                c = certain(q, n)
                assert c == (abs(d) > 4 * n + 40), (d, n)
                if c:
                    assert sound(q, n)
    assert hits > 10000


def test_binade_edges_and_specials():
    for n in (2048, 3072):
        for k in (-100, -1, 0, 1, 60):
            p = 2.0 ** k
            for q in (p, float(np.nextafter(p, 0)), float(np.nextafter(p, np.inf))):
                if certain(q, n):
                    assert sound(q, n)
        assert certain(0.0, n) and certain(float("inf"), n) and certain(float("nan"), n)
        assert not certain(2.0 ** -130, n)  # a float32-subnormal mean: sequential fallback
        assert not certain(2.0 ** 129, n)
