"""Custom sources on the GPU (mnl_fields_add_custom_point_source; custom_src_time,
src/meep.hpp:1059-1092): the host calls the Python function per step exactly
as the oracle does, so the fields are bitwise the oracle's -- on one GPU and on
3 slabs (one host thread per slab calling back into Python)."""
import math

import numpy as np
import pytest

from scenarios import GroupSim3, ProductSim, compare_all, make_oracle, sc_custom_source_3d

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


@pytest.mark.parametrize("G", [ProductSim, GroupSim3])
def test_custom_source_bitwise(G):
    d = {c: v for c, v in compare_all(sc_custom_source_3d(G), sc_custom_source_3d(make_oracle)).items()
         if v != 0.0}
    assert not d, d


def test_simulation_custom_source():
    import meep_nl_amd as mp
    sim = mp.Simulation(cell_size=mp.Vector3(3, 3), resolution=10,
                        sources=[mp.Source(mp.CustomSource(lambda t: math.sin(2 * math.pi * 0.3 * t),
                                                           end_time=4.0), mp.Ez,
                                           center=mp.Vector3(0.1, 0.2))])
    sim.run(until_after_sources=2.0)
    assert sim.round_time() >= 6.0 and np.abs(sim.get_array(mp.Ez)).max() > 0
