"""Volume sources in the CPU oracle (fields::add_volume_source,
src/sources.cpp:455-494; src_vol_chunkloop 243-312).

The loop_in_chunks weights are built so that "the integral of the current is
fixed regardless of resolution" (src/sources.cpp:236-242): for a plane source
of size Ly x Lz (delta function along x) the point amplitudes add up to
amp * Ly * Lz * a^3 whatever the resolution a and wherever the plane's edges
fall.  One step of a unit current (custom source, J = 1) turns D at the source
points into -amp_pt * dt, so sum(D) / (-dt a^3) must equal amp * Ly * Lz."""
import numpy as np
import pytest

import scenarios as S
from scenarios import make_oracle


@pytest.mark.parametrize("a", [10, 20])
def test_plane_source_integral_is_resolution_independent(a):
    o = S.vol(make_oracle, 3, [3.0, 3.0, 3.0], a, center_origin=True)
    ly, lz, amp = 1.37, 0.83, 0.7
    lo, hi = [0.213, -0.61, -0.32], [0.213, -0.61 + ly, -0.32 + lz]
    o.add_custom_volume_source(2, lambda t: 1.0, -1.0, 1e20, lo, hi, amp)
    o.step(1)
    dz = o.get_array(8)
    got = -dz.sum() / (o.dt * a ** 3)
    assert got == pytest.approx(amp * ly * lz, rel=1e-12)


def test_point_equals_zero_size_volume():
    """add_point_source(c, src, p, amp) is add_volume_source(c, src, volume(p, p), amp)
    (src/sources.cpp:215-217)."""
    def run(vol):
        o = S.vol(make_oracle, 3, [2.0, 2.0, 2.0], 10, center_origin=True)
        o.add_pml(0.5)
        p = (0.137, -0.052, 0.249)
        if vol:
            o.add_gaussian_volume_source(2, 0.3, 4.0, 0.0, 40.0, p, p, 0.8)
        else:
            o.add_gaussian_source(2, 0.3, 4.0, 0.0, 40.0, p, 0.8)
        o.step(25)
        return o
    a, b = run(True), run(False)
    for c in range(12):
        np.testing.assert_array_equal(a.get_array(c), b.get_array(c))


def test_source_wider_than_cell():
    """A volume up to one pixel wider than the cell is shrunk to the cell; wider
    aborts (src/sources.cpp:458-466)."""
    o = S.vol(make_oracle, 2, [2.0, 2.0], 10, center_origin=True)
    o.add_gaussian_volume_source(2, 0.3, 4.0, 0.0, 40.0, (-1.04, -0.3, 0), (1.04, 0.2, 0), 1.0)
    with pytest.raises(RuntimeError, match="Source width > cell width"):
        o.add_gaussian_volume_source(2, 0.3, 4.0, 0.0, 40.0, (-1.2, 0, 0), (1.2, 0, 0), 1.0)
