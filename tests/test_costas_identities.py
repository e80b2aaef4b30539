"""Bit-level identities the Costas wave of the loop kernel relies on
(qpsk_loop.hip, round 5), checked on the host in IEEE double arithmetic.
The GPU parity tests pin the kernel itself; these pin the algebra.

- The +-2pi wrap (CostasLoopQpsk.cs:89-91): the kernel runs the reference's
  tn - copysign(2pi, tn).  fma(copysign(1, tn), -2pi, tn) is the same bit for
  bit (the product is exact, so it is one rounding of tn -+ 2pi, ties to zero
  included).  The one-op-shorter sign(tn) * (|tn| - 2pi) is NOT: at tn = -2pi
  it gives -0 where the reference gives +0.  This test found that in a build
  that used it; the kernel went back to the reference's form.
- eq * mi with eq = +-1 equals the sign select (eq > 0 ? mi : -mi) bit for
  bit, signed zeros included, so fma(ei, mq, -(eq * mi)) is unchanged.
"""
import numpy as np

TWO_PI = 2.0 * 3.14159265358979311600
PI = 3.14159265358979311600
SIGN = np.uint64(0x8000000000000000)


def _bits(x):
    return np.asarray(x, dtype=np.float64).view(np.uint64)


def _wrap_ref(tn):
    return tn - np.copysign(TWO_PI, tn)


def _wrap_fma(tn):
    # fma(s, -2pi, tn) with s = +-1: s * -2pi is exact, so the fma is the one
    # rounding of this add
    s = np.copysign(1.0, tn)
    return tn + s * -TWO_PI


def _wrap_signed_magnitude(tn):
    u = np.abs(tn) - TWO_PI
    return (_bits(u) ^ (_bits(tn) & SIGN)).view(np.float64)


def _cases(rng):
    parts = [
        rng.uniform(-20.0, 20.0, 400_000),
        rng.uniform(-4.0 * PI, 4.0 * PI, 400_000),
        np.ldexp(rng.uniform(0.5, 1.0, 100_000), rng.integers(-4, 60, 100_000)) * rng.choice([-1.0, 1.0], 100_000),
    ]
    # neighbourhoods of the wrap threshold and of the values where tn -+ 2pi
    # cancels or changes sign
    for c in (PI, 2 * PI, 3 * PI, TWO_PI, 1.5 * TWO_PI):
        near = (np.float64(c).view(np.int64) + np.arange(-2000, 2001, dtype=np.int64)).view(np.float64)
        parts += [near, -near]
    tn = np.concatenate(parts)
    return tn[np.abs(tn) > PI]


def test_wrap_fma_form_equals_reference():
    tn = _cases(np.random.default_rng(2025))
    assert np.array_equal(_bits(_wrap_ref(tn)), _bits(_wrap_fma(tn)))


def test_wrap_signed_magnitude_form_differs_only_at_minus_two_pi():
    tn = _cases(np.random.default_rng(2025))
    bad = _bits(_wrap_ref(tn)) != _bits(_wrap_signed_magnitude(tn))
    assert np.all(tn[bad] == -TWO_PI) and bad.any()
    assert _bits(_wrap_ref(np.array([-TWO_PI])))[0] == 0            # +0
    assert _bits(_wrap_signed_magnitude(np.array([-TWO_PI])))[0] == SIGN   # -0


def test_sign_select_equals_product_by_unit():
    rng = np.random.default_rng(7)
    mi = np.concatenate([rng.normal(size=200_000), rng.normal(size=1000) * 1e-300,
                         np.array([0.0, -0.0, 5e-324, -5e-324, np.inf, -np.inf])])
    for pos in (True, False):
        eq = 1.0 if pos else -1.0
        assert np.array_equal(_bits(eq * mi), _bits(mi if pos else -mi))
    # the phase error built on it: fma(ei, mq, -(eq*mi)) with ei = +-1 is one
    # rounding of an exact sum, here the add of the exact product
    mq = rng.normal(size=mi.size)
    for ei in (1.0, -1.0):
        for pos in (True, False):
            eq = 1.0 if pos else -1.0
            assert np.array_equal(_bits(ei * mq + (-(eq * mi))), _bits(ei * mq + (-(mi if pos else -mi))))
