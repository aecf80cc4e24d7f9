"""The multiply-high division of shot_group / group_step (kernels.h
fast_div_init, lane.h fast_div): the same integer steps in Python, exact
against // for divisors and dividends across the 32-bit range, the edges
included (d = 1, powers of two, 2^32 - 1; n = 0, 2^32 - 1)."""

import random


def magic(d):
    l = 0
    while l < 32 and (1 << l) < d:
        l += 1
    return ((1 << 32) * ((1 << l) - d)) // d + 1, min(l, 1), max(l - 1, 0)


def fast_div(n, d):
    m, s1, s2 = magic(d)
    assert 0 < m < (1 << 32)
    t = (m * n) >> 32
    return (t + ((n - t) >> s1)) >> s2


def test_fast_div_exact():
    rng = random.Random(7)
    ds = [1, 2, 3, 5, 7, 10, 100, 255, 256, 257, 65535, 65536, 65537, 2 ** 31 - 1, 2 ** 31, 2 ** 31 + 1,
          2 ** 32 - 2, 2 ** 32 - 1] + [rng.randrange(1, 2 ** 32) for _ in range(1500)]
    ns = [0, 1, 2, 2 ** 31 - 1, 2 ** 31, 2 ** 32 - 2, 2 ** 32 - 1] + [rng.randrange(0, 2 ** 32) for _ in range(100)]
    for d in ds:
        for n in ns + [d - 1, d, d + 1, 2 * d - 1, 2 * d, 3 * d + 1]:
            if 0 <= n < 2 ** 32:
                assert fast_div(n, d) == n // d, (n, d)
