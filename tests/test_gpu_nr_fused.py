"""chi(2) Newton-Raphson in the fused mode: the fused kernels store
D everywhere and E / P outside the chi2 box grown by one point; nr_fused_e updates that
box (NR kernel + update_P).  Bitwise against the oracle's step_update_EDHB NR branch
(src/step_generic.cpp:730-816) on the C4-NR config at 96^3 (the chi2 box clear of the
PML) and at full size, and across fused <-> unfused transitions."""
import numpy as np
import pytest

from scenarios import ProductSim, make_oracle, sc_c4_nr

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]


def _same(p, o):
    assert p.nr_random_fallbacks() == o.nr_random_fallbacks()
    for c in range(12):
        a, b = p.get_array(c), o.get_array(c)
        assert a.tobytes() == b.tobytes(), (c, float(np.max(np.abs(a - b))))


@pytest.fixture(scope="module")
def oracle96():
    return sc_c4_nr(make_oracle, steps=40, n=96)


def test_nr_fused_active_and_bitwise(oracle96):
    p = sc_c4_nr(ProductSim, steps=0, n=96)
    p.step(40)
    assert p._fields().fused_active()
    _same(p, oracle96)


def test_nr_unfused_bitwise(oracle96):
    p = sc_c4_nr(ProductSim, steps=0, n=96)
    p._fields().set_fused(False)
    p.step(40)
    assert not p._fields().fused_active()
    _same(p, oracle96)


def test_nr_fused_transitions(oracle96):
    p = sc_c4_nr(ProductSim, steps=0, n=96)
    f = p._fields()
    for on in (True, False, True, False, True):
        f.set_fused(on)
        p.step(8)
        assert f.fused_active() == on
    _same(p, oracle96)


def test_nr_fused_full_size():
    p = sc_c4_nr(ProductSim, steps=0)
    p.step(30)
    assert p._fields().fused_active()
    o = sc_c4_nr(make_oracle, steps=30)
    assert o.nr_random_fallbacks() > 0
    _same(p, o)


def test_nr_box_in_pml_stays_unfused():
    """A chi2 box reaching the PML (C4-NR at 64^3: |x| <= 3 crosses the 1.0-thick PML of a
    6.4-wide cell) cannot leave its E to the NR box kernel (the PML E update is the W form):
    the run stays unfused and bitwise."""
    p = sc_c4_nr(ProductSim, steps=0, n=64)
    p.step(30)
    assert not p._fields().fused_active()
    _same(p, sc_c4_nr(make_oracle, steps=30, n=64))
