"""Array slices on the product (mnl_fields_array_slice; fields::get_array_slice,
src/array_slice.cpp:251-704) bitwise against the oracle restatement: whole
cells, lines and points with interpolated empty dimensions, 3-D planes and
boxes crossing PML chunk boundaries, E, H and D components; and
Simulation.get_array on top of it."""
import numpy as np
import pytest

from scenarios import (GroupSim, GroupSim3, ProductSim, make_oracle, sc_cfg1, sc_te_magnetic_2d,
                       sc_vacuum_pml_3d)

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]

VOL2 = [([-10, -10, 0], [10, 10, 0]), ([-10, 0.33, 0], [10, 0.33, 0]),
        ([0.5, 0.3, 0], [0.5, 0.3, 0]), ([0.57, 0.31, 0], [0.57, 0.31, 0]),
        ([-3.04, -2.0, 0], [2.61, 7.7, 0])]
VOL3 = [([-1.6, -1.6, 0.12], [1.6, 1.6, 0.12]), ([-1.2, -0.65, -1.0], [0.9, 0.45, 0.3]),
        ([0.05, 0.05, 0.05], [0.05, 0.05, 0.05]), ([-1.6, 0.61, -0.63], [1.6, 0.61, -0.63]),
        ([-0.9, -1.6, -1.6], [-0.9, 1.6, 1.6])]
# whole cell, and planes on / between the 3-slab seams (global z = 11, 22)
VOL3_SEAM = [([-1.6, -1.6, -1.6], [1.6, 1.6, 1.6]), ([-1.6, -1.6, -0.5], [1.6, 1.6, -0.5]),
             ([-1.6, -1.6, -0.45], [1.6, 1.6, -0.45]), ([-1.3, -0.2, 0.6], [0.4, 1.1, 0.6]),
             ([-0.3, 0.2, -0.55], [0.3, 0.2, 0.62])]


def _same(p, o, comps, vols):
    for c in comps:
        for lo, hi in vols:
            for snap in (False, True):
                a, b = p.get_array_slice(c, lo, hi, snap), o.get_array_slice(c, lo, hi, snap)
                assert np.shape(a) == np.shape(b), (c, lo, hi, snap)
                assert np.array_equal(a, b), (c, lo, hi, snap,
                                              float(np.max(np.abs(np.asarray(a) - b))))


def test_slices_2d():
    _same(sc_cfg1(ProductSim, steps=120), sc_cfg1(make_oracle, steps=120), (2, 3, 4, 8), VOL2)
    te = [([0, 0, 0], [2.3, 1.9, 0]), ([0.4, 0.77, 0], [2.0, 0.77, 0])]
    _same(sc_te_magnetic_2d(ProductSim), sc_te_magnetic_2d(make_oracle), (0, 1, 5), te)


@pytest.mark.parametrize("G", [ProductSim, GroupSim, GroupSim3])
def test_slices_3d(G):
    """GroupSim / GroupSim3: distributed fields (2 / 3 z-slabs), the four Yee values
    of each point gathered exactly over the slabs."""
    _same(sc_vacuum_pml_3d(G, steps=40), sc_vacuum_pml_3d(make_oracle, steps=40),
          (0, 2, 3, 5, 7), VOL3)


@pytest.mark.parametrize("G", [ProductSim, GroupSim, GroupSim3])
def test_slices_3d_seams(G):
    """Whole-cell and seam-plane slices over slabs: each rank reads only its own
    box of values plus the next rank's first plane (no whole-cell buffers)."""
    _same(sc_vacuum_pml_3d(G, steps=30), sc_vacuum_pml_3d(make_oracle, steps=30),
          (0, 1, 2, 4, 5, 6, 8, 9, 11), VOL3_SEAM)


def test_slices_2d_slabs():
    _same(sc_cfg1(GroupSim3, steps=120), sc_cfg1(make_oracle, steps=120), (2, 3, 4, 8), VOL2)


def test_simulation_get_array():
    import meep_nl_amd as mp
    sim = mp.Simulation(cell_size=mp.Vector3(4, 3), resolution=10,
                        sources=[mp.Source(mp.GaussianSource(0.4, fwidth=0.3), mp.Ez,
                                           center=mp.Vector3(0.12, -0.3))])
    sim.run(until=5)
    a = sim.get_array(mp.Ez)
    assert a.shape == (40, 30)
    line = sim.get_array(mp.Ez, center=mp.Vector3(0, 0.33), size=mp.Vector3(4, 0))
    assert line.shape == (40,)
    v = sim.get_array(mp.Ez, vol=mp.Volume(center=mp.Vector3(0.12, -0.3), size=mp.Vector3()))
    assert np.ndim(v) == 0 and v != 0
