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


@pytest.mark.parametrize("early", ["1", "0"])
def test_nr_fused_beside_tile_kernel(oracle96, monkeypatch, early):
    """With the polarization chunks' general kernel on a CU split beside the tile kernel
    (MNL_TILE_GEN_CUS), the NR box's E phase runs on the general kernel's stream right after
    it (MNL_NR_EARLY=1, the default) or after both kernels (0): bitwise the oracle either way."""
    monkeypatch.setenv("MNL_TILE_GEN_CUS", "64")
    monkeypatch.setenv("MNL_NR_EARLY", early)
    p = sc_c4_nr(ProductSim, steps=0, n=96)
    p.step(40)
    assert p._fields().fused_active() and p._fields().fused_concurrent()
    _same(p, oracle96)


def test_nr_source_in_box_with_split(monkeypatch):
    """A D source inside the chi2 box (inside the polarization box, so the run leaves the fused
    mode: E would need recomputing after the source; nr_early_ok checks the same case again)
    with the CU split requested: bitwise the oracle."""
    monkeypatch.setenv("MNL_TILE_GEN_CUS", "64")

    def run(make):
        o = sc_c4_nr(make, steps=0, n=96)
        o.add_gaussian_source(1, 0.3, 5.0, 0.0, 50.0, (0.15, -0.25, 0.35), 20.0)
        o.step(30)
        return o

    p = run(ProductSim)
    assert not p._fields().fused_active()
    _same(p, run(make_oracle))
