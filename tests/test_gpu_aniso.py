"""Anisotropic Lorentzian susceptibility on the GPU (update_P 3x3 / 2x2 branches
with OFFDIAG averaging of the neighbouring W, src/susceptibility.cpp:185-250;
WE_stuff ghost exchange, src/step.cpp:111-114): bitwise against the oracle on
one GPU and on 2 / 3 slabs."""
import pytest

from scenarios import GroupSim, GroupSim3, ProductSim, compare_all, make_oracle, sc_aniso_lorentz_3d

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]


@pytest.mark.parametrize("G", [ProductSim, GroupSim, GroupSim3])
@pytest.mark.parametrize("full", [True, False])
def test_aniso_lorentz_bitwise(G, full):
    p = sc_aniso_lorentz_3d(G, full=full)
    o = sc_aniso_lorentz_3d(make_oracle, full=full)
    d = {c: v for c, v in compare_all(p, o).items() if v != 0.0}
    assert not d, d
