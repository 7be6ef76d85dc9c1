"""The kernel's range tests as unsigned compares of float bits (render.hip unit_pair, in_interval)
decide exactly as the IEEE comparisons they replace (Quad::Hit's interior test and interval check,
Quad.cpp:19-43), over special values (signed zeros, denormals, infinities, NaNs, the bounds' neighbours)
and random floats of every exponent."""
import numpy as np

F32 = np.float32


def _bits(x):
    return np.asarray(x, dtype=F32).view(np.uint32)


def _specials():
    vals = [0.0, -0.0, 1.0, -1.0, np.inf, -np.inf, np.nan, -np.nan, 1e-45, -1e-45, 1.17549435e-38,
            -1.17549435e-38, 3.4028235e38, -3.4028235e38, 0.001, 0.5, 2.0]
    v = np.array(vals, dtype=F32)
    one = F32(1.0)
    near = np.array([np.nextafter(one, F32(2)), np.nextafter(one, F32(0)), np.nextafter(F32(0), F32(1)),
                     np.nextafter(F32(0), F32(-1)), np.nextafter(F32(0.001), F32(1)),
                     np.nextafter(F32(0.001), F32(0))], dtype=F32)
    return np.concatenate([v, near])


def _randoms(n, rng):
    u = rng.integers(0, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    return u.view(F32)


def unit_pair(a, b):
    """render.hip unit_pair: max(bits(a + 0), bits(b + 0)) <= bits(1.0f)."""
    with np.errstate(invalid="ignore"):
        ka = _bits(a + F32(0.0))
        kb = _bits(b + F32(0.0))
    return np.maximum(ka, kb) <= np.uint32(0x3F800000)


def in_interval(t, lo, hi):
    """render.hip in_interval: bits(t) - bits(lo) <= bits(hi) - bits(lo), unsigned, wrapping."""
    return (_bits(t) - _bits(lo)) <= (_bits(hi) - _bits(lo))


def test_unit_pair_matches_ieee_compares():
    rng = np.random.default_rng(7)
    sp = _specials()
    a = np.concatenate([np.repeat(sp, sp.size), _randoms(200000, rng), rng.random(100000).astype(F32)])
    b = np.concatenate([np.tile(sp, sp.size), _randoms(200000, rng), rng.random(100000).astype(F32)])
    with np.errstate(invalid="ignore"):
        ref = (F32(0) <= a) & (a <= F32(1)) & (F32(0) <= b) & (b <= F32(1))
    assert np.array_equal(unit_pair(a, b), ref)


def test_in_interval_matches_ieee_compares():
    rng = np.random.default_rng(11)
    lo = F32(0.001)  # trace_linear's tmin
    sp = _specials()
    his = np.concatenate([np.array([3.4028235e38, 0.001, 1.0, 555.0], dtype=F32),
                          np.abs(_randoms(64, rng)), rng.random(64).astype(F32) * F32(1000)])
    his = his[np.isfinite(his) & (his >= lo)]  # 0 < lo <= hi <= FLT_MAX, as the kernel's tmax
    t = np.concatenate([sp, _randoms(100000, rng), (rng.random(50000) * 2000 - 1000).astype(F32)])
    for hi in his:
        with np.errstate(invalid="ignore"):
            ref = (lo <= t) & (t <= hi)
        assert np.array_equal(in_interval(t, lo, np.full_like(t, hi)), ref), hi
