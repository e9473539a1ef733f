"""GPU parity of DFT field monitors (fields::add_dft_fields, src/dft.cpp:889-903;
fields::get_dft_array / process_dft_component / collapse_array, src/dft.cpp:908-1280,
src/array_slice.cpp:525-601) against the CPU oracle.

Tolerance: BITWISE.  The per-point DFT values are accumulated by the flux objects'
kernels (bitwise the oracle, tests/test_gpu_dft.py) and get_dft_array is formed on
the host with the reference's expressions; across slabs every entry has one owning
rank, so the sum over ranks is exact as well.
"""
import numpy as np
import pytest

from scenarios import (DFTF_FREQS, GroupSim3, ProductSim, make_oracle, sc_dft_fields_2d,
                       sc_dft_fields_3d)

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _same(p, o, objs):
    for h, comps in objs:
        for c in comps:
            for i in range(len(DFTF_FREQS)):
                a, b = p.dft_array(h, c, i), o.dft_array(h, c, i)
                assert a.shape == b.shape and a.size > 0, (h, c, a.shape, b.shape)
                np.testing.assert_array_equal(a, b, err_msg=f"object {h} comp {c} freq {i}")
        assert p.dft_decimation(h) == o.dft_decimation(h)


def test_dft_fields_3d_fused():
    p, objs = sc_dft_fields_3d(ProductSim)
    assert p._fields().fused_active()
    o, _ = sc_dft_fields_3d(make_oracle)
    _same(p, o, objs)
    a = p.dft_array(objs[2][0], 1, 0)
    assert a.ndim == 2 and np.any(a != 0)  # thin plane collapsed to 2-D
    assert p.dft_array(objs[3][0], 0, 0).ndim == 1  # line: two empty dimensions


def test_dft_fields_3d_unfused_lorentz(monkeypatch):
    monkeypatch.setenv("MNL_NO_FUSED", "1")
    p, objs = sc_dft_fields_3d(ProductSim, lorentz=True)
    assert not p._fields().fused_active()
    o, _ = sc_dft_fields_3d(make_oracle, lorentz=True)
    _same(p, o, objs)


def test_dft_fields_3d_slabs():
    p, objs = sc_dft_fields_3d(GroupSim3, steps=40)
    o, _ = sc_dft_fields_3d(make_oracle, steps=40)
    _same(p, o, objs)


def test_dft_fields_2d():
    p, objs = sc_dft_fields_2d(ProductSim)
    o, _ = sc_dft_fields_2d(make_oracle)
    _same(p, o, objs)
    with pytest.raises(RuntimeError, match="outside the range"):
        p.dft_array(objs[0][0], 2, 5)


def _ring_sim(mp):
    """python/tests/test_dft_fields.py::init (ring resonator, PML 2, res 10)."""
    n, w, r, pad, dpml = 3.4, 1.0, 1.0, 4, 2
    sxy = 2.0 * (r + w + pad + dpml)
    geometry = [mp.Cylinder(r + w, material=mp.Medium(epsilon=n ** 2)),
                mp.Cylinder(r, material=mp.vacuum)]
    src = mp.GaussianSource(0.118, fwidth=0.1)
    sim = mp.Simulation(cell_size=mp.Vector3(sxy, sxy), resolution=10, geometry=geometry,
                        sources=[mp.Source(src=src, component=mp.Ez, center=mp.Vector3(r + 0.1))],
                        boundary_layers=[mp.PML(dpml)])
    return sim, sxy


def test_simulation_dft_fields_properties():
    """python/tests/test_dft_fields.py test_get_dft_array / test_decimated...: thin
    volumes collapse to 1-D arrays; the whole-cell flux object's Ez array equals the
    dft_fields object's (HDF5 is absent here, so the two arrays are compared with each
    other); decimation 4 agrees with 1 to 1e-3."""
    import warnings
    import meep_nl_amd as mp
    warnings.simplefilter("ignore", RuntimeWarning)
    sim, sxy = _ring_sim(mp)
    sim.init_sim()
    fcen = 0.118
    dft_fields = sim.add_dft_fields([mp.Ez], fcen, 0, 1)
    dec1 = sim.add_dft_fields([mp.Ez], fcen, 0, 1, decimation_factor=1)
    dec4 = sim.add_dft_fields([mp.Ez], fcen, 0, 1, decimation_factor=4)
    yee = sim.add_dft_fields([mp.Ez], fcen, 0, 1, yee_grid=True)
    flux = sim.add_flux(fcen, 0, 1, mp.FluxRegion(mp.Vector3(), size=mp.Vector3(sxy, sxy),
                                                  direction=mp.X))
    thin_x = sim.add_dft_fields([mp.Ez], fcen, 0, 1, where=mp.Volume(
        center=mp.Vector3(0.35 * sxy), size=mp.Vector3(y=0.8 * sxy)))
    thin_y = sim.add_flux(fcen, 0, 1, mp.FluxRegion(mp.Vector3(y=0.25 * sxy),
                                                    size=mp.Vector3(x=sxy)))
    sim.run(until_after_sources=100)
    assert sim.get_dft_array(thin_x, mp.Ez, 0).ndim == 1
    assert sim.get_dft_array(thin_y, mp.Ez, 0).ndim == 1
    fa, xa = sim.get_dft_array(dft_fields, mp.Ez, 0), sim.get_dft_array(flux, mp.Ez, 0)
    assert fa.shape == xa.shape == (160, 160)
    np.testing.assert_allclose(fa, xa, rtol=0, atol=1e-12 * np.max(np.abs(fa)))
    a1, a4 = sim.get_dft_array(dec1, mp.Ez, 0), sim.get_dft_array(dec4, mp.Ez, 0)
    assert np.linalg.norm(a1 - a4) <= 1e-3 * np.linalg.norm(a1)
    assert sim.get_dft_array(yee, mp.Ez, 0).shape == (160, 160)
