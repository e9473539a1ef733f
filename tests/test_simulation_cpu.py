"""Simulation-level host logic that needs no GPU: Medium permeability parsing and
Simulation.has_mu (python/tests/test_simulation.py::test_has_mu's cases; its
material-function case needs libctl material functions, absent here)."""
import pytest

import meep_nl_amd as mp


@pytest.mark.parametrize("med,default,expected", [
    (mp.Medium(mu_diag=mp.Vector3(2, 1, 1)), mp.Medium(), True),
    (mp.Medium(mu_offdiag=mp.Vector3(0.1, 0.2, 0.3)), mp.Medium(), True),
    (mp.Medium(), mp.Medium(mu_diag=mp.Vector3(1, 1, 1.1)), True),
    (mp.Medium(), mp.Medium(), False),
    (mp.Medium(mu=3.0), mp.Medium(), True),
])
def test_has_mu(med, default, expected):
    sim = mp.Simulation(cell_size=mp.Vector3(5, 5), resolution=10,
                        geometry=[mp.Block(center=mp.Vector3(), size=mp.Vector3(1, 1),
                                           material=med)],
                        default_material=default)
    assert sim.has_mu() is expected


def test_magnetic_susceptibility_offdiag_refused():
    with pytest.raises(NotImplementedError):
        mp.Medium(H_susceptibilities=[mp.LorentzianSusceptibility(
            frequency=1.0, gamma=0.1, sigma_offdiag=mp.Vector3(0.1, 0, 0))])
