"""The f64 score-term formula of the device (koordinator_amd/csrc/ks_device.h term_least / term_most) is
exact: trunc(max(fma(100(h-p), fl(1/c), 2^-44), 0)) == floor(100(h-p)/c) (Go's int64 leastRequestedScore,
load_aware.go:388-397 / least_allocated.go:45-54) and the MostAllocated counterpart, for every capacity
c < 2^43 and request below 2^46.  The fma is replayed with exact rational arithmetic (Fraction -> float is
correctly rounded), so this checks the IEEE result the hardware computes, on the cases the error bound is
tight for: quotients that are exact integers, and quotients one unit (1/c) below an integer."""
from fractions import Fraction

import numpy as np

BIAS = 2.0 ** -44
BIG_CAP = 1 << 43
BIG_REQ = 1 << 46


def fma(a: float, b: float, c: float) -> float:
    return float(Fraction(a) * Fraction(b) + Fraction(c))


def least_f64(c: int, h: int, p: int) -> int:
    hd = float(h) * 100.0 if c else 0.0
    r = 1.0 / float(c) if c else 0.0
    x = max(fma(hd - float(p) * 100.0, r, BIAS), 0.0)
    return int(x)  # trunc (v_cvt_i32_f64)


def most_f64(c: int, h: int, p: int) -> int:
    hd = float(h) * 100.0 if c else 0.0
    r = 1.0 / float(c) if c else 0.0
    y = min(fma(float(p) * 100.0 - hd, r, 100.0 + BIAS), 100.0)
    return int(y) if r != 0.0 else 0


def least_go(c: int, h: int, p: int) -> int:
    requested = c - h + p
    if c == 0 or requested > c:
        return 0
    return (c - requested) * 100 // c


def most_go(c: int, h: int, p: int) -> int:
    if c == 0:
        return 0
    requested = min(c - h + p, c)
    return requested * 100 // c


def _caps(rng):
    caps = [1, 2, 3, 7, 100, 101, 999, 1000, 32000, 96000, 2 ** 20, 3 * 2 ** 30, 128 * 2 ** 30, 512 * 2 ** 30,
            2 ** 40, 2 ** 42 + 1, BIG_CAP - 1, BIG_CAP - 3, 1024 * 2 ** 30 + 17]
    caps += [int(v) for v in rng.integers(1, BIG_CAP, 40)]
    caps += [int(v) for v in np.exp(rng.uniform(0, np.log(BIG_CAP - 1), 40)).astype(np.int64) + 1]
    return caps


def test_least_and_most_exact_on_integer_boundaries():
    rng = np.random.default_rng(7)
    n = 0
    for c in _caps(rng):
        for k in list(range(0, 101, 7)) + [1, 99, 100]:
            # d = h - p with 100 d / c at or just below / above the integer k
            t = k * c
            ds = {t // 100, (t + 99) // 100, t // 100 - 1, (t + 99) // 100 + 1}
            for d in ds:
                if d < -c or d > c:
                    continue
                for p in (0, 1, min(c, BIG_REQ - 1), int(rng.integers(0, BIG_REQ))):
                    h = d + p
                    if h > c:
                        continue
                    assert least_f64(c, h, p) == least_go(c, h, p), (c, h, p)
                    assert most_f64(c, h, p) == most_go(c, h, p), (c, h, p)
                    n += 1
    assert n > 5000


def test_least_and_most_exact_random():
    rng = np.random.default_rng(11)
    for _ in range(4000):
        c = int(rng.integers(1, BIG_CAP))
        p = int(rng.integers(0, BIG_REQ)) if rng.random() < 0.3 else int(rng.integers(0, c + 1))
        h = int(rng.integers(-c, c + 1))
        assert least_f64(c, h, p) == least_go(c, h, p), (c, h, p)
        assert most_f64(c, h, p) == most_go(c, h, p), (c, h, p)


def test_zero_capacity_scores_zero():
    for p in (0, 1, 10 ** 9):
        assert least_f64(0, 0, p) == 0 and most_f64(0, 0, p) == 0
