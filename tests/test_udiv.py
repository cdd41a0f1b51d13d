"""slot_setup's division by host-computed multipliers (wgt_device.h udiv_by, round 6): q = mulhi(x, m)
with m = (2^32 - 1) / d is x / d or up to two less, and two correction steps make it exact.  The
arithmetic restated in numpy uint64 and checked against x // d on random, extreme and near-multiple
dividends for every divisor shape the launch produces (8x8 blocks per tile row and per tile)."""
import numpy as np


def udiv_by(x, d):
    x = x.astype(np.uint64)
    d = np.uint64(d)
    m = np.uint64(0xFFFFFFFF) // d
    q = (x * m) >> np.uint64(32)
    r = x - q * d
    fix = r >= d
    q = q + fix
    r = np.where(fix, r - d, r)
    q = q + (r >= d)
    return q


def test_udiv_by_exact():
    rng = np.random.default_rng(3)
    divisors = [1, 2, 3, 4, 7, 8, 15, 16, 240, 135, 240 * 135, 255, 4096, 8191, 65535, 1 << 20,
                (1 << 26) - 1, 0x7FFFFFFF, 0xFFFFFFFF]
    divisors += list(rng.integers(1, 1 << 32, 40, dtype=np.uint64))
    for d in divisors:
        d = int(d)
        xs = np.concatenate([rng.integers(0, 1 << 32, 20000, dtype=np.uint64),
                             np.array([0, 1, d - 1, d, d + 1, 0xFFFFFFFF, 0xFFFFFFFE, 0x7FFFFFFF], np.uint64) % (1 << 32),
                             (np.arange(1, 2000, dtype=np.uint64) * np.uint64(d)) % np.uint64(1 << 32),
                             (np.arange(1, 2000, dtype=np.uint64) * np.uint64(d) - np.uint64(1)) % np.uint64(1 << 32)])
        assert np.array_equal(udiv_by(xs, d), xs // np.uint64(d)), d
