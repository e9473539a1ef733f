"""Subpixel averaging on the GPU (mnl_structure_set_epsilon_geometry ->
structure::set_epsilon with anisotropic averaging, src/anisotropic_averaging.cpp:
33-298) bit for bit against the oracle's restatement: every chi1inv row of every
E component in 1-D, 2-D and 3-D for blocks, spheres, cylinders and overlapping
objects, with and without averaging; then fields stepped on the averaged
structure (fork mode, and upstream mode where the off-diagonal rows enter the E
update), on one GPU and on 3 slabs, and the Simulation(eps_averaging=True) path."""
import numpy as np
import pytest

import oracle.oracle as orc
import scenarios as S
from scenarios import OBJS_3D, GroupSim3, ProductSim, make_oracle, sc_averaged

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _product_rows(gv_dim, n, io, objs, default_eps, use_avg=True, tol=1e-4, maxeval=100000):
    from meep_nl_amd import core
    gv = core.GridVolume(gv_dim, n, 10.0, io)
    s = core.Structure(gv)
    s.set_epsilon_geometry(objs, default_eps, use_avg, tol, maxeval)
    comps = (0,) if gv_dim == 1 else (0, 1, 2)
    return {c: [s.get_chi1inv(c, d) for d in range(3)] for c in comps}


def _oracle_rows(dim, n, io, objs, default_eps, use_avg=True, tol=1e-4, maxeval=100000):
    out = {}
    for c in ((0,) if dim == 1 else (0, 1, 2)):
        rows = orc.eps_average(dim, n, io, 10.0, c, objs, default_eps, use_avg, tol, maxeval)
        # the product drops trivial rows (None) like the reference's set_chi1inv
        triv = [r is None or np.all(r == (1.0 if d == c else 0.0)) for d, r in enumerate(rows)]
        out[c] = [None if (r is None or (d != c and triv[d]) or all(triv)) else r
                  for d, r in enumerate(rows)]
    return out


def _same(p, o):
    for c in o:
        for d in range(3):
            a, b = p[c][d], o[c][d]
            assert (a is None) == (b is None), (c, d)
            if a is not None:
                assert a.shape == b.shape
                assert a.tobytes() == b.tobytes(), (c, d, np.max(np.abs(a - b)))


@pytest.mark.parametrize("use_avg,maxeval", [(True, 100000), (True, 5000), (False, 100000)])
def test_rows_3d_bitwise(use_avg, maxeval):
    n, io = [22, 20, 24], [-22, -20, -24]
    p = _product_rows(3, n, io, OBJS_3D, 1.7, use_avg, 1e-4, maxeval)
    o = _oracle_rows(3, n, io, OBJS_3D, 1.7, use_avg, 1e-4, maxeval)
    _same(p, o)
    if use_avg:
        assert any(o[c][d] is not None for c in o for d in range(3) if d != c)


def test_rows_2d_and_1d_bitwise():
    objs2 = [[1, 8.0, 0.07, -0.11, 0.0, 0.63, 0, 0], [0, 3.0, -0.2, 0.3, 0.0, 0.37, 0.55, 0.0]]
    _same(_product_rows(2, [30, 26, 0], [-30, -26, 0], objs2, 1.3),
          _oracle_rows(2, [30, 26, 0], [-30, -26, 0], objs2, 1.3))
    objs1 = [[0, 5.0, 0.0, 0.0, 0.0317, 0.0, 0.0, 0.841], [0, 2.0, 0.0, 0.0, 0.4, 0.0, 0.0, 0.233]]
    _same(_product_rows(1, [0, 0, 40], [0, 0, -40], objs1, 1.0),
          _oracle_rows(1, [0, 0, 40], [0, 0, -40], objs1, 1.0))


@pytest.mark.parametrize("upstream", [False, True])
def test_fields_on_averaged_structure_bitwise(upstream):
    o = sc_averaged(make_oracle, upstream)
    for G in (ProductSim, GroupSim3):
        bad = {c: d for c, d in S.compare_all(sc_averaged(G, upstream), o).items() if d != 0.0}
        assert not bad, (G.__name__, bad)


def test_simulation_eps_averaging():
    import meep_nl_amd as mp
    geom = [mp.Block(size=mp.Vector3(mp.inf, 0.43, 0.37), material=mp.Medium(epsilon=6.0)),
            mp.Sphere(0.52, center=mp.Vector3(0.121, -0.087, 0.053), material=mp.Medium(index=3.0)),
            mp.Cylinder(0.18, height=0.9, axis=mp.Vector3(0, 0, 1),
                        center=mp.Vector3(-0.31, 0.27, 0), material=mp.Medium(epsilon=2.5))]
    sim = mp.Simulation(cell_size=mp.Vector3(2.2, 2.0, 2.4), resolution=10, geometry=geom,
                        boundary_layers=[mp.PML(0.5)], default_material=mp.Medium(epsilon=1.7),
                        sources=[mp.Source(mp.GaussianSource(0.3, fwidth=0.2), mp.Ez,
                                           center=mp.Vector3(0.05, 0.05, 0.05))])
    sim.run(until=2.0)
    n, io = [22, 20, 24], [-22, -20, -24]
    objs = [g.geo_record(g.material.epsilon_diag.x) for g in geom]
    o = _oracle_rows(3, n, io, objs, 1.7)
    p = {c: [sim.structure.get_chi1inv(c, d) for d in range(3)] for c in range(3)}
    _same(p, o)
    # the same structure stepped by the oracle gives the same fields
    orc_sim = S.vol(make_oracle, 3, [2.2, 2.0, 2.4], 10, center_origin=True)
    orc_sim.add_pml(0.5)
    orc_sim.set_epsilon_geometry(objs, 1.7)
    orc_sim.add_gaussian_source(2, 0.3, 5.0, 0.0, 50.0, (0.05, 0.05, 0.05), 1.0)
    orc_sim.step(sim.timestep)
    for c in range(12):
        assert sim.get_component_array(c).tobytes() == orc_sim.get_array(c).tobytes(), c
