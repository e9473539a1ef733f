"""Multi-GPU decomposition on one GPU: 2 and 3 z-slabs (y-slabs in 2-D) of one
grid with the ghost-plane exchange (E low ghost before curl B, B/H high ghost
before curl D, D and P before the Newton-Raphson E update) must reproduce the
oracle bit for bit -- the reference's chunk-invariance property
(tests/three_d.cpp:35-39 requires 1e-9; we require 0)."""
import pytest

from scenarios import (GroupSim, GroupSim3, compare_all, make_oracle, sc_cfg1, sc_kerr_lorentz_3d,
                       sc_multi_source_3d, sc_nr_pml_dispersive, sc_polariton_1d,
                       sc_te_magnetic_2d, sc_vacuum_pml_3d)

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _bitwise(a, b, comps=tuple(range(12))):
    d = {c: v for c, v in compare_all(a, b, comps).items() if v != 0.0}
    assert not d, d


@pytest.mark.parametrize("G", [GroupSim, GroupSim3])
def test_slabs_vacuum_pml(G):
    _bitwise(sc_vacuum_pml_3d(G), sc_vacuum_pml_3d(make_oracle))


@pytest.mark.parametrize("G", [GroupSim, GroupSim3])
def test_slabs_kerr_lorentz(G):
    _bitwise(sc_kerr_lorentz_3d(G), sc_kerr_lorentz_3d(make_oracle))


def test_slabs_nr_dispersive():
    _bitwise(sc_nr_pml_dispersive(GroupSim3), sc_nr_pml_dispersive(make_oracle))


@pytest.mark.parametrize("G", [GroupSim, GroupSim3])
def test_slabs_nr_integrated_seams(G):
    """Integrated sources on a reference chunk seam AND (2 slabs) next to the slab
    seam at z = 0: ghost copies of the dipole points follow the owner-chunk rule."""
    from scenarios import sc_nr_isrc_seam
    _bitwise(sc_nr_isrc_seam(G), sc_nr_isrc_seam(make_oracle))
    _bitwise(sc_nr_pml_dispersive(G), sc_nr_pml_dispersive(make_oracle))


def test_slabs_multi_source():
    _bitwise(sc_multi_source_3d(GroupSim3), sc_multi_source_3d(make_oracle))


def test_slabs_2d():
    _bitwise(sc_cfg1(GroupSim, steps=120), sc_cfg1(make_oracle, steps=120), comps=(2, 3, 4, 8, 9, 10))
    _bitwise(sc_te_magnetic_2d(GroupSim3), sc_te_magnetic_2d(make_oracle), comps=(0, 1, 5, 6, 7, 11))


def test_slabs_1d():
    _bitwise(sc_polariton_1d(GroupSim), sc_polariton_1d(make_oracle), comps=(0, 4, 6, 10))


@pytest.mark.parametrize("G", [GroupSim, GroupSim3])
def test_slabs_fused_big_box(G):
    """Fused stepping across slabs: lean, wide and 16-column general tiles on every
    rank, chunk 0 on the side stream, the top plane after the B/H exchange, and the
    E exchange at the end of each step (DESIGN.md "Multi-GPU")."""
    from scenarios import sc_big_box_3d
    _bitwise(sc_big_box_3d(G, steps=16), sc_big_box_3d(make_oracle, steps=16))


def test_slabs_fused_toggle():
    """A magnetic source added mid-run switches every slab out of fused mode
    (implicit E and the W aux fields are materialised) and stepping continues."""
    from scenarios import sc_big_box_3d

    def add_h(o):
        o.add_gaussian_source(4, 0.3, 3.0, 0.0, 30.0, (1.0, 0.3, -1.1), 0.8)
    _bitwise(sc_big_box_3d(GroupSim3, steps=12, extra=add_h),
             sc_big_box_3d(make_oracle, steps=12, extra=add_h))


def test_slabs_waveguide():
    from scenarios import sc_waveguide_3d
    _bitwise(sc_waveguide_3d(GroupSim3), sc_waveguide_3d(make_oracle))


def test_slabs_fused_lorentz():
    from scenarios import sc_big_lorentz_3d
    _bitwise(sc_big_lorentz_3d(GroupSim3, steps=16), sc_big_lorentz_3d(make_oracle, steps=16))
