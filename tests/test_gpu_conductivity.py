"""Conductivity on the GPU (step_curl's cnd branches, src/step_generic.cpp:89-229;
cndinv-scaled current sources, src/step.cpp:300-309): bitwise against the
oracle on one GPU and on 2 / 3 slabs, and the reference's own PML-with-
conductivity check (tests/pml.cpp:323 -> check_pml1d, 75-114) on the product."""
import pytest

from scenarios import (GroupSim, GroupSim3, ProductSim, check_pml1d, compare_all, make_oracle,
                       pml1d_ft, sc_conductive_2d, sc_conductive_3d)

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _bitwise(a, b, comps=tuple(range(12))):
    d = {c: v for c, v in compare_all(a, b, comps).items() if v != 0.0}
    assert not d, d


@pytest.mark.parametrize("G", [ProductSim, GroupSim, GroupSim3])
def test_conductive_3d_bitwise(G):
    p = sc_conductive_3d(G)
    o = sc_conductive_3d(make_oracle)
    _bitwise(p, o)
    assert not p._fields().fused_active() if G is ProductSim else True


@pytest.mark.parametrize("G", [ProductSim, GroupSim3])
def test_conductive_2d_bitwise(G):
    _bitwise(sc_conductive_2d(G), sc_conductive_2d(make_oracle))


def test_pml1d_conductivity_bitwise():
    """Both structures of check_pml1d at res 20, through do_ft: identical step
    counts and Fourier sums (every sampled Ex bit for bit)."""
    for sz, dpml in ((3.0, 1.0), (5.0, 2.0)):
        fp, np_ = pml1d_ft(ProductSim, 20.0, sz, dpml, 10.0)
        fo, no = pml1d_ft(make_oracle, 20.0, sz, dpml, 10.0)
        assert np_ == no and fp == fo


def test_check_pml1d_reference():
    """tests/pml.cpp:323: 'not a pml in 1d + conductivity' must not fire."""
    refl, ok = check_pml1d(ProductSim)
    assert ok, refl
