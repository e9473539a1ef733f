"""Simulation-level calls ordinary scripts use: Dielectric / Permeability slices
(Simulation.get_epsilon / get_mu -> get_array(Dielectric), src/array_slice.cpp:385-408)
bitwise against the oracle's chunk-literal restatement; change_sources
(fields::remove_sources + add_source), restart_fields (fields::zero_fields, t = 0) and
the energy-in-box calls."""
import numpy as np
import pytest

from scenarios import GroupSim3, ProductSim, make_oracle, sc_mu_2d, sc_mu_3d

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]

VOLS3 = [([-1.6, -1.5, -1.7], [1.6, 1.5, 1.7]), ([-1.3, -0.2, 0.55], [0.4, 1.1, 0.55]),
         ([-0.3, 0.2, -0.55], [0.3, 0.2, 0.62]), ([0.05, 0.05, 0.05], [0.05, 0.05, 0.05])]


@pytest.mark.parametrize("G", [ProductSim, GroupSim3])
def test_dielectric_permeability_slices_3d(G):
    p, o = sc_mu_3d(G, steps=2), sc_mu_3d(make_oracle, steps=2)
    for c in (12, 13):
        for lo, hi in VOLS3:
            for snap in (False, True):
                a, b = p.get_array_slice(c, lo, hi, snap), o.get_array_slice(c, lo, hi, snap)
                assert np.array_equal(a, b), (c, lo, hi, snap)


def test_dielectric_permeability_slices_2d():
    p, o = sc_mu_2d(ProductSim, steps=2), sc_mu_2d(make_oracle, steps=2)
    for c in (12, 13):
        for lo, hi in [([0, 0, 0], [3.1, 2.7, 0]), ([0.4, 0.77, 0], [2.0, 0.77, 0])]:
            assert np.array_equal(p.get_array_slice(c, lo, hi), o.get_array_slice(c, lo, hi))


def test_simulation_get_epsilon_mu():
    import meep_nl_amd as mp
    geom = [mp.Block(center=mp.Vector3(0.3, -0.2), size=mp.Vector3(1.0, 0.6),
                     material=mp.Medium(epsilon=4.0, mu=2.0))]
    sim = mp.Simulation(cell_size=mp.Vector3(3.0, 2.0), resolution=10, geometry=geom,
                        eps_averaging=False)
    eps, mu = sim.get_epsilon(), sim.get_mu()
    assert eps.shape == (30, 20) and mu.shape == (30, 20)
    assert eps.max() == 4.0 and eps.min() == 1.0 and mu.max() == 2.0 and mu.min() == 1.0
    # a Centered point inside the block: all Yee neighbours inside
    assert eps[18, 8] == 4.0 and mu[18, 8] == 2.0


def _sim(mp, src_pos):
    return mp.Simulation(cell_size=mp.Vector3(3.0, 2.6), resolution=10,
                         boundary_layers=[mp.PML(0.5)],
                         sources=[mp.Source(mp.GaussianSource(0.3, fwidth=0.2), mp.Ez,
                                            center=src_pos)])


def test_change_sources_and_restart_fields():
    import meep_nl_amd as mp
    a = _sim(mp, mp.Vector3(0.1, 0.2))
    a.run(until=2.0)
    a.change_sources([mp.Source(mp.GaussianSource(0.35, fwidth=0.25), mp.Ez,
                                center=mp.Vector3(-0.3, 0.1))])
    a.restart_fields()
    assert a.timestep == 0
    assert not np.any(a.get_component_array(mp.Ez))
    a.run(until=3.0)
    b = mp.Simulation(cell_size=mp.Vector3(3.0, 2.6), resolution=10,
                      boundary_layers=[mp.PML(0.5)],
                      sources=[mp.Source(mp.GaussianSource(0.35, fwidth=0.25), mp.Ez,
                                         center=mp.Vector3(-0.3, 0.1))])
    b.run(until=3.0)
    for c in (mp.Ez, mp.Hx, mp.Hy, mp.Dz, mp.Bx):
        assert np.array_equal(a.get_component_array(c), b.get_component_array(c)), c
    e = a.electric_energy_in_box(center=mp.Vector3(), size=mp.Vector3(1, 1))
    m = a.magnetic_energy_in_box(center=mp.Vector3(), size=mp.Vector3(1, 1))
    t = a.field_energy_in_box(center=mp.Vector3(), size=mp.Vector3(1, 1))
    assert e > 0 and m > 0 and t > 0
