"""Upstream-Meep nonlinear mode on the GPU ("upstream
physics behind a flag"): chi2/chi3 through the Pade approximant
calc_nonlinear_u (src/step_generic.cpp:546-553) on every E point, as the
branches the fork comments out in step_update_EDHB.

Pinning: the reference's own golden harmonics of python/tests/test_3rd_harm_1d.py
(tolerance 1e-7, as that test) through the meep.Simulation-style API
(add_flux + run(until_after_sources=stop_when_fields_decayed(...))), and the
fluxes bitwise equal to the oracle's after the same steps; 3-D arrays bitwise
equal to the oracle on one GPU and across 2 / 3 slabs.
"""
import numpy as np
import pytest

from scenarios import (ALL_COMPS, GroupSim, GroupSim3, ProductSim, compare_all, make_oracle,
                       sc_upstream_nl_3d, third_harmonic_1d)

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def test_third_harmonic_golden_simulation_api(golden):
    """python/tests/test_3rd_harm_1d.py, line for line, on meep_nl_amd."""
    import meep_nl_amd as mp
    g = golden["upstream_third_harmonic_1d"]
    sz, fcen, dpml, k, amp = 100, 1 / 3.0, 1.0, 1e-2, 1.0
    df = fcen / 20.0
    sim = mp.Simulation(cell_size=mp.Vector3(0, 0, sz), geometry=[],
                        sources=[mp.Source(mp.GaussianSource(fcen, fwidth=df), component=mp.Ex,
                                           center=mp.Vector3(0, 0, (-0.5 * sz) + dpml),
                                           amplitude=amp)],
                        boundary_layers=[mp.PML(dpml)],
                        default_material=mp.Medium(index=1, chi3=k), resolution=20,
                        dimensions=1, nonlinear_mode="upstream")
    fr = mp.FluxRegion(mp.Vector3(0, 0, (0.5 * sz) - dpml - 0.5))
    nfreq, fmin, fmax = 400, fcen / 2.0, fcen * 4
    trans = sim.add_flux(0.5 * (fmin + fmax), fmax - fmin, nfreq, fr, decimation_factor=1)
    trans1 = sim.add_flux(fcen, 0, 1, fr, decimation_factor=1)
    trans3 = sim.add_flux(3 * fcen, 0, 1, fr, decimation_factor=1)
    sim.run(until_after_sources=mp.stop_when_fields_decayed(
        50, mp.Ex, mp.Vector3(0, 0, (0.5 * sz) - dpml - 0.5), 1e-6))
    h1, h3 = mp.get_fluxes(trans1)[0], mp.get_fluxes(trans3)[0]
    assert abs(h1 - g["flux_fcen"]) <= g["rel_tol"] * abs(g["flux_fcen"])
    assert abs(h3 - g["flux_3fcen"]) <= g["rel_tol"] * abs(g["flux_3fcen"])
    assert len(mp.get_fluxes(trans)) == nfreq
    # the same run on the oracle: bitwise equal fluxes
    o, f1, f3 = third_harmonic_1d(make_oracle)
    assert o.t == sim.timestep
    assert (h1, h3) == (f1, f3)


def test_third_harmonic_scenario_bitwise():
    p, p1, p3 = third_harmonic_1d(ProductSim, decay=1e-3)
    o, o1, o3 = third_harmonic_1d(make_oracle, decay=1e-3)
    assert p.t == o.t and (p1, p3) == (o1, o3)
    np.testing.assert_array_equal(p.get_array(0), o.get_array(0))


def _bitwise(a, b):
    d = {c: v for c, v in compare_all(a, b, ALL_COMPS).items() if v != 0.0}
    assert not d, d


def test_upstream_3d_bitwise():
    p = sc_upstream_nl_3d(ProductSim)
    assert not p._fields().fused_active()
    _bitwise(p, sc_upstream_nl_3d(make_oracle))


@pytest.mark.parametrize("G", [GroupSim, GroupSim3])
def test_upstream_3d_slabs(G):
    _bitwise(sc_upstream_nl_3d(G), sc_upstream_nl_3d(make_oracle))


def test_harmonics_cpp_golden_and_scaling(golden):
    """tests/harmonics.cpp on the GPU: the known 2nd/3rd harmonic ratios (rel 1e-5),
    bitwise equal to the oracle, and the test's scaling checks (doubling chi2 and
    chi3 -> 4x both ratios; doubling J -> 4x / 16x; within 1 %)."""
    from scenarios import harmonics_cpp
    g = golden["upstream_harmonics_cpp"]
    p, a2, a3 = harmonics_cpp(ProductSim, 0.27e-4, 1e-4, 1.0)
    assert abs(a2 - g["A2"]) <= g["rel_tol"] * g["A2"]
    assert abs(a3 - g["A3"]) <= g["rel_tol"] * g["A3"]
    o, b2, b3 = harmonics_cpp(make_oracle, 0.27e-4, 1e-4, 1.0)
    assert (a2, a3) == (b2, b3) and p.t == o.t
    _, c2, c3 = harmonics_cpp(ProductSim, 0.54e-4, 2e-4, 1.0)
    assert abs(c2 / a2 - 4.0) <= 0.04 and abs(c3 / a3 - 4.0) <= 0.04
    _, j2, j3 = harmonics_cpp(ProductSim, 0.27e-4, 1e-4, 2.0)
    assert abs(j2 / a2 - 4.0) <= 0.04 and abs(j3 / a3 - 16.0) <= 0.16


@pytest.mark.parametrize("chi2,chi3", [(True, True), (False, False), (True, False)])
def test_upstream_offdiag_bitwise(chi2, chi3):
    """Off-diagonal chi1inv in upstream mode (OFFDIAG, src/step_generic.cpp:597-598,
    617, 632, 659, 772, 823, 844): reference chunks with both rows, one row (either
    order) and none, with and without the Pade factor, PML and non-PML."""
    kw = dict(offdiag=True, chi2=chi2, chi3=chi3)
    _bitwise(sc_upstream_nl_3d(ProductSim, **kw), sc_upstream_nl_3d(make_oracle, **kw))


def test_upstream_offdiag_slabs():
    kw = dict(offdiag=True)
    _bitwise(sc_upstream_nl_3d(GroupSim3, **kw), sc_upstream_nl_3d(make_oracle, **kw))
