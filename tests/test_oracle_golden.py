"""Pin the CPU oracle against the reference's own golden values.

known_results: tests/known_results.cpp:155-169 (rel 1e-5, compare() at :43-49).
survey_*: outputs of the compiled reference recorded in SURVEY.md section 8(c);
the oracle is required to reproduce them bit for bit (same IEEE operation
order, see oracle/mnl_oracle.cpp header).
"""
import math

import numpy as np
import pytest

from oracle.oracle import Bx, Ex, Ez, meep_vol

AMP = complex(0, -2 * math.pi * 0.2)


def _legacy_run(o, comp, ttot):
    # tests/known_results.cpp:60-66: add_point_source(c, 0.2, 3.0, 0.0, 2.0, center, amp)
    o.legacy_point_source(comp, 0.2, 3.0, 0.0, 2.0, o.center(), AMP)
    while o.round_time() < ttot:
        o.step()
    return o.get_field(comp, o.center())


def _rel(a, b):
    return abs(a - b) / abs(b)


def test_known_metallic_2d(golden):
    kr = golden["known_results"]
    v = _legacy_run(meep_vol(2, [1, 1], 10), Ez, 10.0)
    assert _rel(v, kr["metallic_2d_tm_ez"]) < kr["rel_tol"]


def test_known_metallic_3d(golden):
    kr = golden["known_results"]
    v = _legacy_run(meep_vol(3, [1, 1, 1], 10), Ez, 10.0)
    assert _rel(v, kr["metallic_3d_ez"]) < kr["rel_tol"]


def test_known_pml_2d(golden):
    kr = golden["known_results"]
    o = meep_vol(2, [3, 3], 10)
    o.add_pml(1.0)
    v = _legacy_run(o, Ez, 30.0)
    assert _rel(v, kr["pml_2d_tm_ez"]) < kr["rel_tol"]


def test_known_polariton_1d(golden):
    kr = golden["known_results"]
    o = meep_vol(1, [1], 10)
    o.add_lorentzian(0.3, 0.1, [np.full(o.shape(), 7.63), None, None])
    v = _legacy_run(o, Ex, 10.0)
    assert _rel(v, kr["polariton_1d_ex"]) < kr["rel_tol"]


def test_survey_cfg1_bitwise(golden):
    g = golden["survey_cfg1"]
    o = meep_vol(2, [20, 20], 10, center_origin=True)
    o.add_gaussian_source(Ez, 0.15, 10.0, 0.0, 100.0, (0, 0), 1.0, is_integrated=False)
    o.step(500)
    ss = 0.0
    for ix in range(-95, 96, 5):
        for iy in range(-95, 96, 5):
            v = o.get_field(Ez, (ix * 0.1, iy * 0.1))
            ss += v * v
    assert o.get_field(Ez, (0.5, 0.3)) == g["ez_0p5_0p3"]
    assert o.get_field(Ez, (0.0, 0.0)) == g["ez_0_0"]
    assert ss == g["sumsq_39x39"]


def _chi3_run(nl, dim):
    o = meep_vol(1, [20.0], 20) if dim == 1 else meep_vol(2, [4.0, 4.0], 20)
    o.add_pml(1.0)
    c = Ex if dim == 1 else Ez
    if nl:
        for cc in ((Ex,) if dim == 1 else (0, 1, 2)):
            o.set_chi3(cc, np.full(o.shape(), 1e-2))
    o.legacy_point_source(c, 1 / 3.0, 1 / 60.0, 0.0, 4.0, o.center(), 10.0)
    while o.time() < 30.0:
        o.step()
    cen = o.center()
    p = [0, 0, cen[2] + 1.3] if dim == 1 else [cen[0] + 0.7, cen[1] + 0.4]
    return o.get_field(c, p)


@pytest.mark.parametrize("dim,key", [(1, "ex_1d"), (2, "ez_2d")])
def test_survey_chi3_inert_bitwise(golden, dim, key):
    g = golden["survey_chi3"]
    assert _chi3_run(False, dim) == g[key]
    assert _chi3_run(True, dim) == g[key]


def _nr_run(c2):
    o = meep_vol(3, [1, 1, 1], 10)
    for c in (0, 1, 2):
        for d in range(3):
            o.set_chi1inv(c, d, np.full(o.shape(), 0.25 if d == c else 1e-3))
        if c2:
            o.set_chi2(c, np.full(o.shape(), c2))
    cen = o.center()
    o.legacy_point_source(Ez, 0.5, 0.5, 0.0, 3.0, [cen[0] + 0.05, cen[1] + 0.05, cen[2] + 0.05], 5.0)
    o.step(40)
    return o.get_field(Ex, [cen[0] + 0.21, cen[1] + 0.13, cen[2] + 0.07]), o.nr_random_fallbacks()


def test_survey_nr_bitwise(golden):
    g = golden["survey_nr"]
    v0, r0 = _nr_run(0.0)
    v1, r1 = _nr_run(0.5)
    assert v0 == g["ex_chi2_0"]
    assert v1 == g["ex_chi2_0p5"]
    assert r0 == 0 and r1 == 0  # the non-deterministic random fallback is never reached


def test_magnetic_b_not_allocated_in_2d_te():
    # 2-D TM source allocates only TM components (src/fields.cpp:473-491, 566-586)
    o = meep_vol(2, [2, 2], 10)
    o.add_gaussian_source(Ez, 0.5, 1.0, 0, 10, (1.0, 1.0))
    o.step(3)
    assert np.all(o.get_array(Ex) == 0)
    assert np.any(o.get_array(Bx) != 0)
