"""CPU: the modulo the hash partitioners use on the device (sux_p1.h mod_pos, PartDev::rmagic from
sux_internal.h part_magic) equals Spark's pmod / nonNegativeMod for every 32-bit hash and every
partition count.  The GPU partition tests check the kernels against oracle.c; this pins the
arithmetic itself, restated here in numpy uint64 (the device's 64 x 64 -> high-64 multiply
split into 32-bit halves)."""
import numpy as np
import pytest

U64 = (1 << 64) - 1


def part_magic(n: int) -> int:
    return (U64 // n + 1) & U64


def mod_pos(a: np.ndarray, n: int) -> np.ndarray:
    """a: int32 array -> a mod n in [0, n), as the device computes it."""
    m = np.uint64(part_magic(n))
    u = np.where(a < 0, -(a.astype(np.int64)), a.astype(np.int64)).astype(np.uint64)
    with np.errstate(over="ignore"):
        low = m * u  # mod 2^64
    lo32, hi32 = low & np.uint64(0xFFFFFFFF), low >> np.uint64(32)
    nn = np.uint64(n)
    r = (hi32 * nn + ((lo32 * nn) >> np.uint64(32))) >> np.uint64(32)  # (low * n) >> 64
    r = r.astype(np.int64)
    return np.where((a < 0) & (r != 0), n - r, r)


def spark_pmod(a: np.ndarray, n: int) -> np.ndarray:
    """Spark's Pmod for a positive modulus (Java's truncated % then the sign fix)."""
    a = a.astype(np.int64)
    r = np.fmod(a, n)
    return np.where(r < 0, np.fmod(r + n, n), r)


EDGE = np.array([0, 1, -1, 2, -2, 12345, -12345, 2**31 - 1, -(2**31), -(2**31) + 1],
                dtype=np.int32)


@pytest.mark.parametrize("n", [1, 2, 3, 7, 10, 199, 200, 208, 1000, 1024, 1025, 4096, 4097, 8193,
                               10000, 16384, 65535, 65536, 1000003, 2**31 - 1])
def test_mod_pos_matches_pmod(n):
    rng = np.random.default_rng(n)
    a = np.concatenate([EDGE, rng.integers(-(2**31), 2**31, 200_000, dtype=np.int64).astype(np.int32),
                        np.arange(-5000, 5000, dtype=np.int32)])
    assert np.array_equal(mod_pos(a, n), spark_pmod(a, n))


def test_mod_pos_random_moduli():
    rng = np.random.default_rng(7)
    for n in rng.integers(1, 2**31, 200, dtype=np.int64):
        a = np.concatenate([EDGE, rng.integers(-(2**31), 2**31, 5_000, dtype=np.int64).astype(np.int32)])
        assert np.array_equal(mod_pos(a, int(n)), spark_pmod(a, int(n))), n
