"""Parity at BASELINE.json's full sizes (every single-GPU config), bit for bit
against the CPU oracle on all twelve component arrays.

  C2  256^3 vacuum + PML(1.0), Ez Gaussian at (0.05,0.05,0.05): 20 steps from
      zero fields, and 20 steps from seeded random D / B everywhere
  C4  256^3 Kerr chi3 + Lorentzian slab |z| < 2 (eps 2.25), PML(1.0), Ex
      Gaussian at z = -3, amp 50: 20 steps from random D / B
  C3  512^3 eps = 12 waveguide + PML(1.0): 2 steps from random D / B (host RAM
      holds the oracle's ~20 GB of chunk arrays plus both sides' copies)

Random initial fields (initialize_field, src/initialize.cpp:135-161) put data
into every tile, z chunk and PML region of the benched grids from step one, so
the kernels' tile / chunk boundaries at the benched sizes are all checked."""
import numpy as np
import pytest

from scenarios import ALL_COMPS, ProductSim, make_oracle, sc_random_fields, sc_vacuum_pml_3d

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]


def _bitwise_free(p, o):
    """Compare component by component, releasing each array pair."""
    bad = {}
    for c in ALL_COMPS:
        a, b = p.get_array(c), o.get_array(c)
        d = float(np.max(np.abs(a - b))) if a.size else 0.0
        if d != 0.0:
            bad[c] = d
        del a, b
    assert not bad, f"max|diff| per component: {bad}"


def test_c2_256_from_zero():
    kw = dict(L=25.6, steps=20)
    p = sc_vacuum_pml_3d(ProductSim, **kw)
    assert p._fields().fused_active()
    _bitwise_free(p, sc_vacuum_pml_3d(make_oracle, **kw))


def test_c2_256_random():
    kw = dict(sizes=(25.6, 25.6, 25.6), steps=20)
    p = sc_random_fields(ProductSim, **kw)
    assert p._fields().fused_active()
    _bitwise_free(p, sc_random_fields(make_oracle, **kw))


def test_c4_256_random():
    kw = dict(sizes=(25.6, 25.6, 25.6), steps=20, kerr_lorentz=True)
    _bitwise_free(sc_random_fields(ProductSim, **kw), sc_random_fields(make_oracle, **kw))


def test_c3_512_random():
    kw = dict(sizes=(51.2, 51.2, 51.2), steps=3, eps=12.0)  # steps 2-3: one pair
    p = sc_random_fields(ProductSim, **kw)
    assert p._fields().fused_active()
    o = sc_random_fields(make_oracle, **kw)
    _bitwise_free(p, o)
