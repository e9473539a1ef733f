"""initialize_field (src/initialize.cpp:135-161) and random-field parity.

Seeded random D and B (and E, H) over the whole grid make every tile, z chunk,
PML region, wall and slab seam carry data from the first step, so the HIP path
is compared with the CPU oracle everywhere, bit for bit.  The same scenarios at
BASELINE's full sizes are in tests/test_gpu_fullsize.py."""
import numpy as np
import pytest

from scenarios import (ALL_COMPS, GroupSim, GroupSim3, ProductSim, compare_all, make_oracle,
                       sc_random_fields)

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


def _bitwise(prod, orc, comps=ALL_COMPS):
    bad = {c: d for c, d in compare_all(prod, orc, comps).items() if d != 0.0}
    assert not bad, f"max|diff| per component: {bad}"


def test_initialize_field_no_step():
    """Right after initialize_field(D / B) the fields equal the oracle's: the
    added values, zeroed metal walls, E / H from update_eh (PML W form)."""
    kw = dict(steps=0, eps=12.0)
    _bitwise(sc_random_fields(ProductSim, **kw), sc_random_fields(make_oracle, **kw))


@pytest.mark.parametrize("kw", [dict(), dict(eps=12.0), dict(dpml=0.0),
                                dict(kerr_lorentz=True, sizes=(3.2, 3.2, 6.0))])
def test_random_db(kw):
    _bitwise(sc_random_fields(ProductSim, **kw), sc_random_fields(make_oracle, **kw))


def test_random_all_components():
    """E and H set directly as well (E != chi1inv D for one step: that step runs
    unfused); H before its lazy separation adds to B (H == B until the first
    H update, src/update_eh.cpp:204-209)."""
    kw = dict(comps=ALL_COMPS, eps=12.0)
    _bitwise(sc_random_fields(ProductSim, **kw), sc_random_fields(make_oracle, **kw))


def test_random_fields_after_steps():
    """initialize_field after stepping: H is separate in the PML chunks by then."""
    def run(make):
        o = sc_random_fields(make, steps=5, eps=12.0)
        from scenarios import random_init
        random_init(o, (3, 4, 5, 0, 1, 2), seed=99, scale=0.3)
        o.step(7)
        return o
    _bitwise(run(ProductSim), run(make_oracle))


def test_random_big_box():
    """Many fused tiles (lean, wide and 16-column general) with random data."""
    kw = dict(sizes=(14.0, 4.1, 15.3), dpml=0.7, eps=6.0, steps=10)
    _bitwise(sc_random_fields(ProductSim, **kw), sc_random_fields(make_oracle, **kw))


@pytest.mark.parametrize("G", [GroupSim, GroupSim3])
def test_random_slabs(G):
    kw = dict(comps=ALL_COMPS, eps=12.0, steps=10)
    _bitwise(sc_random_fields(G, **kw), sc_random_fields(make_oracle, **kw))
    kw = dict(kerr_lorentz=True, sizes=(3.2, 3.2, 6.0), steps=10)
    _bitwise(sc_random_fields(G, **kw), sc_random_fields(make_oracle, **kw))


def test_simulation_initialize_field():
    """Simulation.initialize_field(cmpnt, amp_func) (python/simulation.py:2520-2532)
    evaluates amp_func at every point of the component."""
    import meep_nl_amd as mp
    sim = mp.Simulation(cell_size=mp.Vector3(2, 2, 2), resolution=10,
                        boundary_layers=[mp.PML(0.5)])
    sim.initialize_field(mp.Dz, lambda p: np.exp(-(p.x ** 2 + p.y ** 2 + p.z ** 2)))
    sim.run(until=1.0)
    o = make_oracle(3, [20, 20, 20], 10, 0.5, [-20, -20, -20])
    o.add_pml(0.5)
    o.initialize_field(8, lambda x, y, z: np.exp(-(x ** 2 + y ** 2 + z ** 2)))
    o.step(sim.fields.t)
    for c in (2, 8, 3, 9):
        np.testing.assert_array_equal(sim.fields.get_array(c), o.get_array(c))
