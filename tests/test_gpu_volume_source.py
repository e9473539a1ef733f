"""Volume sources on the GPU (mnl_fields_add_volume_source ->
fields::add_volume_source, src/sources.cpp:455-494) bit for bit against the
oracle: planes crossing PML chunks, off-grid lines with amplitude functions,
boxes, overlapping sources (layered application), 2-D, slabs; the Python
Source(size=...) path; and the reference's own amp_func / amp_data test
(python/tests/test_source.py:160-229)."""
import math

import numpy as np
import pytest

import scenarios as S
from scenarios import GroupSim, GroupSim3, ProductSim, make_oracle

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _bitwise(p, o, comps=tuple(range(12))):
    bad = {c: d for c, d in S.compare_all(p, o, comps).items() if d != 0.0}
    assert not bad, bad


def sc_volume_sources(make, steps=40):
    o = S.vol(make, 3, [3.2, 2.8, 3.0], 10, center_origin=True)
    o.add_pml(0.7)
    for c in range(3):
        x, y, z = o.coords(c)
        o.set_chi1inv(c, c, np.where((np.abs(y) < 0.4) & (np.abs(z) < 0.4), 1 / 6.0, 1.0))
    # plane through the whole cross-section (into every y / z PML chunk), off-grid in x
    o.add_gaussian_volume_source(2, 0.25, 4.0, 0.0, 40.0, (0.213, -1.4, -1.5), (0.213, 1.4, 1.5),
                                 0.6)
    # off-grid line along y with a complex amplitude profile
    o.add_gaussian_volume_source(0, 0.3, 4.0, 0.0, 40.0, (-0.37, -0.83, 0.141), (-0.37, 0.61, 0.141),
                                 complex(0.4, 0.3), amp_func=lambda r: math.cos(2.0 * r[1]) + 0.2j * r[1])
    # a box of H current overlapping another one (merged / layered points)
    o.add_gaussian_volume_source(4, 0.35, 4.0, 0.0, 40.0, (-0.22, -0.3, -0.41), (0.31, 0.24, 0.05), 0.5)
    o.add_gaussian_volume_source(4, 0.35, 4.0, 0.0, 40.0, (-0.05, -0.1, -0.2), (0.4, 0.34, 0.33), 0.3)
    # the same plane again (combinable: amplitudes merge) and a point on it (layers)
    o.add_gaussian_volume_source(2, 0.25, 4.0, 0.0, 40.0, (0.213, -1.4, -1.5), (0.213, 1.4, 1.5),
                                 0.2)
    o.add_gaussian_source(2, 0.25, 4.0, 0.0, 40.0, (0.213, 0.05, 0.05), 1.0)
    o.step(steps)
    return o


@pytest.mark.parametrize("G", [ProductSim, GroupSim, GroupSim3])
def test_volume_sources_bitwise(G):
    _bitwise(sc_volume_sources(G), sc_volume_sources(make_oracle))


def sc_integrated_planes(make, steps=30):
    """Integrated (dipole) volume sources: ~1700 points on two off-grid planes
    crossing PML chunks and slab seams, the same plane twice (one point's entries
    subtracted in list order), a Lorentzian so the dipoles enter D - P."""
    o = S.vol(make, 3, [3.0, 2.6, 2.8], 10, center_origin=True)
    o.add_pml(0.6)
    sig = []
    for c in range(3):
        x, y, z = o.coords(c)
        sig.append(np.where(np.abs(x) < 0.5, 0.3, 0.0))
    o.add_lorentzian(1.2, 0.1, sig)
    o.add_gaussian_volume_source(1, 0.3, 4.0, 0.0, 30.0, (0.117, -1.3, -1.4), (0.117, 1.3, 1.4),
                                 0.7, is_integrated=True)
    o.add_gaussian_volume_source(1, 0.3, 4.0, 0.0, 30.0, (0.117, -1.3, -1.4), (0.117, 1.3, 1.4),
                                 0.25, is_integrated=True)
    o.add_gaussian_volume_source(2, 0.35, 4.0, 0.0, 30.0, (-1.1, -0.43, -1.4), (1.1, -0.43, 1.4),
                                 complex(0.3, 0.2), is_integrated=True)
    o.step(steps)
    return o


@pytest.mark.parametrize("G", [ProductSim, GroupSim3])
def test_integrated_volume_sources_bitwise(G):
    """Beyond the 64 points the E kernel once took from its arguments: sorted
    device arrays, binary search per point."""
    _bitwise(sc_integrated_planes(G), sc_integrated_planes(make_oracle))


def test_volume_source_2d_and_custom():
    def run(make):
        o = S.vol(make, 2, [2.3, 1.9], 10)
        o.add_pml(0.4)
        o.add_gaussian_volume_source(2, 0.4, 3.0, 0.0, 30.0, (0.3, 0.17), (1.9, 0.17), 1.2,
                                     amp_func=lambda r: np.exp(-r[0] ** 2))
        o.add_custom_volume_source(5, lambda t: math.sin(0.9 * t) * math.exp(-0.1 * t), 0.0, 20.0,
                                   (0.77, 0.4), (0.77, 1.45), 0.8)
        o.step(60)
        return o
    _bitwise(run(ProductSim), run(make_oracle), comps=(0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11))


def test_simulation_source_size():
    """Simulation with Source(size=..., amp_func=...) vs the oracle's volume source."""
    import meep_nl_amd as mp
    sim = mp.Simulation(cell_size=mp.Vector3(2.4, 2.0, 2.2), resolution=10,
                        boundary_layers=[mp.PML(0.5)],
                        sources=[mp.Source(mp.GaussianSource(0.3, fwidth=0.2), mp.Ey,
                                           center=mp.Vector3(0.11, 0, 0.07),
                                           size=mp.Vector3(0.9, 0, 0.6), amplitude=0.7,
                                           amp_func=lambda p: 1 + p.x * p.z)])
    sim.run(until=3.0)
    o = make_oracle(3, [24, 20, 22], 10.0, 0.5, [-24, -20, -22])
    o.add_pml(0.5)
    o.add_gaussian_volume_source(1, 0.3, 5.0, 0.0, 50.0, (0.11 - 0.45, 0.0, 0.07 - 0.3),
                                 (0.11 + 0.45, 0.0, 0.07 + 0.3), 0.7,
                                 amp_func=lambda r: 1 + r[0] * r[2])
    o.step(sim.fields.t)
    for c in range(12):
        np.testing.assert_array_equal(sim.fields.get_array(c), o.get_array(c))


def _amp_fun(p):
    return p.x + 2 * p.y


def _amp_run(kind, data=None):
    import meep_nl_amd as mp
    kw = {"amp_func": _amp_fun} if kind == "func" else {"amp_data": data}
    sim = mp.Simulation(cell_size=mp.Vector3(1, 1), resolution=60,
                        sources=[mp.Source(mp.ContinuousSource(0.8, fwidth=0.02), component=mp.Ez,
                                           center=mp.Vector3(0.1, 0.2), size=mp.Vector3(0.3, 0.2),
                                           **kw)])
    sim.run(until=200)
    return sim.get_field_point(mp.Ez, mp.Vector3())


def test_amp_func_vs_amp_data():
    """python/tests/test_source.py:160-229 (TestAmpFileFunc, func vs arr): the
    amplitude function and the same profile sampled on a 100 x 200 array agree
    to 4 places at the origin after 200 time units."""
    import meep_nl_amd as mp
    N, M = 100, 200
    data = np.zeros((N, M, 1), dtype=np.complex128)
    for i in range(N):
        for j in range(M):
            data[i, j] = _amp_fun(mp.Vector3((i / N) * 0.3 - 0.15, (j / M) * 0.2 - 0.1))
    f_func = _amp_run("func")
    f_arr = _amp_run("arr", data)
    assert round(f_arr - f_func, 4) == 0
