"""Tuning of the fused step (mnl_fields_tune): the tuner steps every
candidate (z-chunk length; on one rank with polarization chunks, the CUs of their general
kernel beside the tile kernel) for real, so a run that tunes first must equal plain
stepping bit for bit, and both must equal the CPU oracle (one GPU and two in-process
slabs)."""
import numpy as np
import pytest

from scenarios import ALL_COMPS, GroupSim, ProductSim, make_oracle, sc_random_fields

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]

SIZES = (6.4, 5.2, 9.6)  # 64 x 52 x 96 cells at resolution 10: several z chunks per length
TOTAL = 240  # tune(reps=1) steps at most 2 + 55 * (2 + 2) = 222 (z chunks 6, CU split 6, pairs: 19 shapes forward and backward + the best 3 again, one-step twice)
ZCS = (0, 16, 20, 24, 32, 48)


def _tuned(G, kerr):
    p = sc_random_fields(G, sizes=SIZES, steps=0, kerr_lorentz=kerr)
    if G is ProductSim:
        chosen = [p._fields().tune(reps=1)]
    else:
        p._all()
        chosen = p._par(lambda f: f.tune(reps=1))
    t = p.t
    assert 1 + 6 * 4 <= t <= TOTAL, t  # every z-chunk candidate stepped: the tile mode was on
    p.step(TOTAL - t)
    return p, chosen


@pytest.mark.parametrize("G", [ProductSim, GroupSim])
@pytest.mark.parametrize("kerr", [False, True])
def test_tune_then_step_is_plain_stepping(G, kerr):
    p, chosen = _tuned(G, kerr)
    for zc, gc in chosen:
        assert zc in ZCS, chosen
        if G is ProductSim and kerr:  # polarization chunks on one rank: the split was tuned
            assert gc >= 0, chosen
        else:
            assert gc == -1, chosen
    q = sc_random_fields(G, sizes=SIZES, steps=TOTAL, kerr_lorentz=kerr)
    o = sc_random_fields(make_oracle, sizes=SIZES, steps=TOTAL, kerr_lorentz=kerr)
    for c in ALL_COMPS:
        a, b, r = p.get_array(c), q.get_array(c), o.get_array(c)
        assert np.array_equal(a, b), c
        assert np.array_equal(a, r), (c, float(np.max(np.abs(a - r))))


@pytest.mark.parametrize("split", [0, 24, 96, 200])
def test_general_beside_tile_kernel(split, monkeypatch):
    """Polarization chunks' general kernel on `split` CUs of a side stream beside the tile
    kernel (MNL_TILE_GEN_CUS, read every batch): bitwise the oracle at any split."""
    monkeypatch.setenv("MNL_TILE_GEN_CUS", str(split))
    p = sc_random_fields(ProductSim, sizes=SIZES, steps=TOTAL, kerr_lorentz=True)
    o = sc_random_fields(make_oracle, sizes=SIZES, steps=TOTAL, kerr_lorentz=True)
    for c in ALL_COMPS:
        assert np.array_equal(p.get_array(c), o.get_array(c)), c
