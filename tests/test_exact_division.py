"""CPU: the view-count division of the HIP variance (common.h div_views) is correctly rounded.

costvolume.py:12 and :14 divide by ``n_views``; torch CPU divides (``x / V``, IEEE), and the HIP
kernels must give the same fp32 bits.  They form q = x * r (r = RN(1 / V)), the exact remainder
x - q V by one fma, and q + remainder * r by a second fma.  This file checks that sequence against
the correctly rounded quotient for EVERY fp32 significand (one whole binade: scaling x by 2^k scales
every step exactly while nothing is subnormal), for V = 2..16, and for every subnormal x plus the
four lowest normal binades (where the remainder or the quotient is subnormal), also for every V =
2..16 (MVS_MAX_VIEWS: the kernels take any of them).  The
GPU side is covered end to end: the HIP cost volume equals the oracle bit for bit given the
same sampling matrices (tests/test_gpu_parity.py::test_cost_volume_bit_exact_vs_oracle_given_matrices).

The emulation is exact: x * r (48 bits) and x - q V (< 30 bits) are exact in float64, so one cast
to fp32 is the fma's single rounding; the last fma is rounded by comparing the exact float64 product
e * r with half an ulp of q.  The reference quotient x / V in float64 cast to fp32 cannot double-
round: x / V is never within 2^-53 of an fp32 midpoint for these V.
"""
import numpy as np
import pytest

f32 = np.float32


def div_views_emulated(x, V):
    """(div_views(x, V), x * RN(1/V)) in exact emulation: the multiply-fma-fma sequence, and for
    V = 6, 10, 12, 14 (even, not a power of two) the IEEE quotient where |x| < 2^-120 (common.h)."""
    x = np.asarray(x, np.float32)
    x64 = x.astype(np.float64)
    r = f32(1.0 / V)
    q1 = (x64 * np.float64(r)).astype(np.float32)
    e = (x64 - q1.astype(np.float64) * V).astype(np.float32)
    t = e.astype(np.float64) * np.float64(r)            # exact: 24 x 24 bits
    # RN(q1 + t): the fp32 candidate c nearest to q1 + t, |t| < 2 ulp; c - q1 and (c - q1) - t are
    # exact in float64, ties to the even significand
    cands = [q1]
    for step in (np.inf, -np.inf):
        c = q1
        for _ in range(2):
            c = np.nextafter(c, f32(step))
            cands.append(c)
    best, bdist = q1, np.abs(t)
    for c in cands[1:]:
        d = np.abs((c.astype(np.float64) - q1.astype(np.float64)) - t)
        even = (c.view(np.int32) & 1) == 0
        take = (d < bdist) | ((d == bdist) & even)
        best = np.where(take, c, best)
        bdist = np.where(take, d, bdist)
    top = np.nextafter(np.nextafter(q1, f32(np.inf)), f32(np.inf)).astype(np.float64) - q1.astype(np.float64)
    assert np.all(np.abs(t) < top), "remainder correction beyond two ulps"
    best = best.astype(np.float32)
    if V % 2 == 0 and V & (V - 1):
        tiny = np.abs(x) < f32(2.0 ** -120)
        best = np.where(tiny, (x64 / V).astype(np.float32), best)   # the IEEE division: correctly rounded
    return best, q1


def test_fma_sequence_alone_misrounds_subnormal_ties():
    """Why the IEEE fallback exists: for V = 6 (even, not a power of two) the multiply-fma-fma sequence
    alone rounds exact subnormal ties the wrong way (x = 9 * 2^-149: x / 6 = 1.5 * 2^-149)."""
    x = np.array([9], dtype=np.uint32).view(np.float32)
    r = f32(1.0 / 6)
    q1 = (x.astype(np.float64) * np.float64(r)).astype(np.float32)
    e = (x.astype(np.float64) - q1.astype(np.float64) * 6).astype(np.float32)
    seq = (q1.astype(np.float64) + e.astype(np.float64) * np.float64(r)).astype(np.float32)
    want = (x.astype(np.float64) / 6).astype(np.float32)
    assert seq[0] != want[0] and div_views_emulated(x, 6)[0][0] == want[0]


def _binade(lo_bits, hi_bits):
    return np.arange(lo_bits, hi_bits, dtype=np.uint32).view(np.float32)


@pytest.mark.parametrize("V", list(range(2, 17)))
def test_div_views_correctly_rounded_one_binade(V):
    x = _binade(0x3F800000, 0x40000000)          # [1, 2): every significand
    q, q_mul = div_views_emulated(x, V)
    want = (x.astype(np.float64) / V).astype(np.float32)
    assert np.array_equal(q, want)
    assert np.array_equal(-div_views_emulated(-x, V)[0], want)   # sign symmetric
    if V & (V - 1):   # not a power of two: multiplying by RN(1/V) alone is wrong on many inputs
        assert np.count_nonzero(q_mul != want) > 0


@pytest.mark.parametrize("V", list(range(2, 17)))
def test_div_views_correctly_rounded_subnormal_range(V):
    for lo, hi in ((0x00000000, 0x00800000), (0x00800000, 0x02800000)):   # subnormals, 4 normal binades
        x = _binade(lo, hi)
        q, _ = div_views_emulated(x, V)
        want = (x.astype(np.float64) / V).astype(np.float32)
        assert np.array_equal(q, want), (V, hex(lo))
