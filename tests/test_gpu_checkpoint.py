"""Checkpoint / resume (fields::dump / fields::load, src/fields_dump.cpp:108-145,
232-270): run N1 steps, dump, run N2 more; a fresh run built the same way that
loads the dump and runs N2 steps must end bit for bit where the first one did
(fused, dispersive, conductive and Newton-Raphson configurations; 1 GPU and 3
slabs; DFT accumulators included; the Simulation-level dump / load)."""
import os

import numpy as np
import pytest

from scenarios import (ALL_COMPS, GroupSim3, ProductSim, compare_all, sc_conductive_3d,
                       sc_flux_3d, sc_kerr_lorentz_3d, sc_nr_pml_dispersive, sc_waveguide_3d)

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]

SCEN = {"waveguide_fused": sc_waveguide_3d, "kerr_lorentz": sc_kerr_lorentz_3d,
        "conductive": sc_conductive_3d, "nr_dispersive": sc_nr_pml_dispersive}


def _resume(make, scen, tmp, n1=17, n2=13):
    a = scen(make, steps=0)
    a.step(n1)
    path = os.path.join(tmp, "fields.mnl")
    a.dump(path)
    a.step(n2)
    b = scen(make, steps=0)
    b.load(path)
    assert b.t == n1
    b.step(n2)
    assert a.t == b.t
    d = {c: v for c, v in compare_all(a, b, ALL_COMPS).items() if v != 0.0}
    assert not d, d
    return a, b


@pytest.mark.parametrize("name", sorted(SCEN))
def test_resume_bitwise(name, tmp_path):
    _resume(ProductSim, SCEN[name], str(tmp_path))


@pytest.mark.parametrize("name", ["waveguide_fused", "conductive"])
def test_resume_bitwise_slabs(name, tmp_path):
    _resume(GroupSim3, SCEN[name], str(tmp_path))


def test_resume_with_flux(tmp_path):
    """The DFT accumulators travel with the fields: the flux after resuming equals
    the uninterrupted one bit for bit."""
    a, hs = sc_flux_3d(ProductSim, steps=0)
    a.step(21)
    path = str(tmp_path / "f.mnl")
    a.dump(path)
    a.step(19)
    b, hb = sc_flux_3d(ProductSim, steps=0)
    b.load(path)
    b.step(19)
    for h, g in zip(hs, hb):
        fa, fb = a.flux(h), b.flux(g)
        assert np.any(np.asarray(fa) != 0)
        assert np.array_equal(fa, fb)


def test_load_mismatch_fails(tmp_path):
    a = sc_waveguide_3d(ProductSim, steps=3)
    path = str(tmp_path / "f.mnl")
    a.dump(path)
    b = sc_kerr_lorentz_3d(ProductSim, steps=0)  # polarizations: different arrays
    with pytest.raises(RuntimeError, match="does not match"):
        b.load(path)


def test_simulation_dump_load(tmp_path):
    import meep_nl_amd as mp

    def make():
        return mp.Simulation(
            cell_size=mp.Vector3(3.2, 3.2, 3.2), resolution=10,
            boundary_layers=[mp.PML(0.8)],
            geometry=[mp.Block(mp.Vector3(mp.inf, 1, 1),
                               material=mp.Medium(epsilon=4.0, D_conductivity=0.2))],
            sources=[mp.Source(mp.GaussianSource(0.3, fwidth=0.2), mp.Ez,
                               center=mp.Vector3(0.05, 0.05, 0.05))])
    s1 = make()
    s1.run(until=2.0)
    s1.dump(str(tmp_path / "ck"))
    s1.run(until=1.5)
    s2 = make()
    s2.load(str(tmp_path / "ck"))
    s2.run(until=1.5)
    assert s1.round_time() == s2.round_time()
    for c in (mp.Ex, mp.Ez, mp.Hy):
        assert np.array_equal(s1.get_component_array(c), s2.get_component_array(c))
