"""The selects' squared-domain threshold (common.hpp sq_threshold): the largest float32 T with
sqrt_rn(T) <= thr, in the closed form the kernels use (midpoint of thr and next_up(thr), squared
exactly in float64, rounded down, one step down more on a tie that rounds up), checked against the
definition by search (step t = thr*thr down/up until sqrt_rn flips) on random thresholds over the
whole exponent range and on the edge cases. numpy's float32 sqrt is IEEE correctly rounded, as is
the GPU's default sqrt (-fhip-fp32-correctly-rounded-divide-sqrt). CPU only: the device code is
covered by the GPU tests' bit-exact thresholds and masks."""
import numpy as np

F = np.float32


def closed_form(thr):
    thr = np.asarray(thr, F)
    up = np.nextafter(thr, F(np.inf))
    m = (thr.astype(np.float64) + up.astype(np.float64)) * 0.5
    m2 = m * m
    t = m2.astype(F)
    t = np.where(t.astype(np.float64) > m2, np.nextafter(t, F(0)), t)
    odd = (thr.view(np.uint32) & 1) == 1
    t = np.where((t.astype(np.float64) == m2) & odd, np.nextafter(t, F(0)), t)
    return t


def by_search(thr):
    thr = np.asarray(thr, F)
    t = (thr * thr).astype(F)
    for _ in range(16):
        down = (t > 0) & (np.sqrt(t) > thr)
        t = np.where(down, np.nextafter(t, F(0)), t)
    for _ in range(16):
        nxt = np.nextafter(t, F(np.inf))
        upm = np.sqrt(nxt) <= thr
        t = np.where(upm, nxt, t)
    return t


def test_closed_form_matches_search():
    rng = np.random.Generator(np.random.PCG64(5))
    bits = rng.integers(0, 0x7F000000, size=2_000_000, dtype=np.uint32)  # every exponent up to ~1.7e38
    thr = bits.view(F)
    edge = np.array([0.0, np.float32(1.4e-45), 1e-30, 1e-20, 0.5, 1.0, 2.0, 3.0, 1e10, 1.5e19],
                    F)
    thr = np.concatenate([thr, edge, np.nextafter(edge, F(np.inf)), np.nextafter(edge, F(0))])
    thr = thr[np.isfinite(thr) & (thr >= 0) & (thr < 1.8e19)]  # thr^2 stays finite
    a, b = closed_form(thr), by_search(thr)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    # and it is the largest: sqrt_rn(T) <= thr < sqrt_rn(next_up(T))
    assert np.all(np.sqrt(a) <= thr)
    assert np.all(np.sqrt(np.nextafter(a, F(np.inf))) > thr)
