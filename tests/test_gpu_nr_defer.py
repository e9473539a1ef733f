"""The chi(2) Newton-Raphson E update with deferred attempts (run_nr's first attempt
in the E kernels, attempts 1-99 for the voxels where it fails in nr_hard_kernel, one
lane per attempt, the lowest successful attempt kept) on the full-size C4-NR config
(tests/scenarios.py sc_c4_nr, whose strong fields make first attempts and, around
step 22, a random-seed fallback fail):
  * bitwise equal to the in-place sequential product path (MNL_NR_DEFER=0) through
    the random-seed fallbacks, with the same fallback count;
  * bitwise equal to the oracle's runNR (src/newton_raphson.cpp:93-359) through the
    random-seed fallbacks: the reference draws those from std::random_device; product
    and oracle share one deterministic stand-in seeded per point and time step
    (nr_voxel_seed), so both solve the same problems from the same
    seeds and count the same fallbacks."""
import numpy as np
import pytest

from scenarios import ProductSim, make_oracle, sc_c4_nr

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]


def test_c4_nr_deferred_equals_sequential(monkeypatch):
    monkeypatch.setenv("MNL_NR_DEFER", "1")
    p = sc_c4_nr(ProductSim, steps=25)
    pf = p.nr_random_fallbacks()
    arr = {c: p.get_array(c) for c in range(12)}
    del p
    monkeypatch.setenv("MNL_NR_DEFER", "0")
    q = sc_c4_nr(ProductSim, steps=25)
    assert pf > 0 and q.nr_random_fallbacks() == pf
    for c in range(12):
        assert arr[c].tobytes() == q.get_array(c).tobytes(), c


@pytest.mark.parametrize("defer", ["1", "0"])
def test_c4_nr_deferred_equals_oracle(monkeypatch, defer):
    monkeypatch.setenv("MNL_NR_DEFER", defer)
    p = sc_c4_nr(ProductSim, steps=30)
    o = sc_c4_nr(make_oracle, steps=30)
    assert o.nr_random_fallbacks() > 0
    assert p.nr_random_fallbacks() == o.nr_random_fallbacks()
    for c in range(12):
        d = float(np.max(np.abs(p.get_array(c) - o.get_array(c))))
        assert d == 0.0, (c, d)
