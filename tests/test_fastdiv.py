"""Host check of the invariant-divisor division the convolution gathers use (csrc/conv.hip FastDiv,
Granlund & Montgomery 1994): (umulhi(n, m) + n) >> l == n // d for n < 2^31, with the 32-bit sum
never overflowing.  The kernels' results are covered by the conv parity tests (tests/test_conv_gpu.py,
tests/test_lowprec_gpu.py)."""
import numpy as np
import pytest


def fastdiv(d):
    l = 0
    while (1 << l) < d:
        l += 1
    return ((1 << 32) * ((1 << l) - d)) // d + 1, l


@pytest.mark.parametrize("d", [1, 2, 3, 4, 5, 7, 10, 15, 16, 40, 49, 51, 64, 80, 98, 120, 321, 498, 1000, 4000,
                               16000, 65535, (1 << 20) + 1, (1 << 31) - 1])
def test_fastdiv_matches_floor_division(d):
    m, l = fastdiv(d)
    assert 0 < m < (1 << 32)
    rng = np.random.default_rng(d)
    n = np.concatenate([np.arange(0, 50000, dtype=np.uint64), rng.integers(0, 1 << 31, 200000, dtype=np.uint64),
                        np.array([(1 << 31) - 1, (1 << 31) - 2, max(d - 1, 0), d, d + 1, 2 * d - 1], dtype=np.uint64)])
    n = n[n < (1 << 31)]
    s = ((n * np.uint64(m)) >> np.uint64(32)) + n
    assert (s < (1 << 32)).all()
    assert np.array_equal(s >> np.uint64(l), n // np.uint64(d))
