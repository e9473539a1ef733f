"""custom_src_time in the oracle (src/meep.hpp:1059-1092): a custom current
source whose function is the Gaussian source's current reproduces the
GaussianSource run (to rounding: Python's complex arithmetic is not the C++
one), and the start/end window is honoured."""
import cmath
import math

import numpy as np

from scenarios import make_oracle, vol


def _run(add):
    o = vol(make_oracle, 2, [3.0, 3.0], 10, center_origin=True)
    o.add_pml(0.5)
    add(o)
    o.step(120)
    return o.get_array(2)


def test_custom_equals_gaussian_current():
    f, w, st, et = 0.4, 2.0, 0.0, 20.0
    peak, cutoff = 0.5 * (st + et), float(np.float32((et - st) * 0.5))
    dt = 0.05

    def dip(t):
        tt = t - peak
        if float(np.float32(abs(tt))) > cutoff:
            return 0j
        return cmath.exp(-tt * tt / (2 * w * w)) * cmath.rect(1.0, -2 * math.pi * f * tt) / complex(
            0, -2 * math.pi * f)

    def cur(t):
        return (dip(t + dt) - dip(t)) / dt
    a = _run(lambda o: o.add_gaussian_source(2, f, w, st, et, (0.13, -0.07), 1.0))
    b = _run(lambda o: o.add_custom_source(2, cur, -1e20, 1e20, (0.13, -0.07), 1.0))
    assert np.abs(a).max() > 0
    np.testing.assert_allclose(b, a, rtol=0, atol=1e-12 * np.abs(a).max())


def test_custom_window():
    a = _run(lambda o: o.add_custom_source(2, lambda t: 1.0, 10.0, 20.0, (0.1, 0.1), 1.0))
    assert np.abs(a).max() == 0.0  # 120 steps = t 6 < start 10
    b = _run(lambda o: o.add_custom_source(2, lambda t: 1.0, 2.0, 3.0, (0.1, 0.1), 1.0))
    assert np.abs(b).max() > 0
