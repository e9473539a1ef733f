"""z-chunk tuning (mnl_fields_tune_zchunk): the tuner steps every
candidate chunk length for real, so a run that tunes first must equal plain stepping
bit for bit, and both must equal the CPU oracle (one GPU and two in-process slabs)."""
import numpy as np
import pytest

from scenarios import ALL_COMPS, GroupSim, ProductSim, make_oracle, sc_random_fields

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]

SIZES = (6.4, 5.2, 9.6)  # 64 x 52 x 96 cells at resolution 10: several z chunks per length
TOTAL = 30


def _tuned(G, kerr):
    p = sc_random_fields(G, sizes=SIZES, steps=0, kerr_lorentz=kerr)
    if G is ProductSim:
        chosen = [p._fields().tune_zchunk(reps=1)]
    else:
        p._all()
        chosen = p._par(lambda f: f.tune_zchunk(reps=1))
    t = p.t
    assert 1 + 6 * 2 <= t <= 2 + 6 * 2, t  # every candidate stepped: the tile mode was on
    p.step(TOTAL - t)
    return p, chosen


@pytest.mark.parametrize("G", [ProductSim, GroupSim])
@pytest.mark.parametrize("kerr", [False, True])
def test_tune_then_step_is_plain_stepping(G, kerr):
    p, chosen = _tuned(G, kerr)
    assert all(c in (0, 16, 20, 24, 32, 48) for c in chosen), chosen  # -1: not tuned
    q = sc_random_fields(G, sizes=SIZES, steps=TOTAL, kerr_lorentz=kerr)
    o = sc_random_fields(make_oracle, sizes=SIZES, steps=TOTAL, kerr_lorentz=kerr)
    for c in ALL_COMPS:
        a, b, r = p.get_array(c), q.get_array(c), o.get_array(c)
        assert np.array_equal(a, b), c
        assert np.array_equal(a, r), (c, float(np.max(np.abs(a - r))))
