"""Field energy on the GPU (mnl_fields_energy_in_box) against the oracle, the
reference's energy golden value and PML tests, and the NaN / Inf guard.

Tolerance: the energies are sums over every grid point.  The oracle (as the
reference, src/integrate.cpp:56-128) adds them sequentially in long double;
the device reduces with TwoSum-compensated partial sums, so the two agree to
rel 1e-12 (every per-point term is bitwise the same: the fields are)."""
import math

import numpy as np
import pytest

import scenarios as S
from scenarios import GroupSim, GroupSim3, ProductSim, make_oracle
from test_oracle_energy import pml_energies, polariton_energy

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(300)]
REL = 1e-12


def test_polariton_energy_golden(golden):
    """tests/known_results.cpp:156 through the HIP path (complex fields as the
    real run with A plus the real run with -i*A, see test_oracle_energy)."""
    A = complex(0, -2 * math.pi * 0.2)
    parts = [polariton_energy(ProductSim, a) for a in (A, -1j * A)]
    ref = [polariton_energy(make_oracle, a) for a in (A, -1j * A)]
    for p, r in zip(parts, ref):
        assert p == pytest.approx(r, rel=REL)
    g = golden["known_results"]["polariton_energy_1d"]
    assert abs(sum(parts) - g) <= abs(g) * 1e-5


def test_three_d_pml_energy_decay():
    """tests/three_d.cpp:163-194 (test_pml) on the GPU: energies equal the
    oracle's and decay below 4e-3 within every 10 time units."""
    a = pml_energies(ProductSim, 1.0)
    b = pml_energies(ProductSim, -1j)
    np.testing.assert_allclose(a, pml_energies(make_oracle, 1.0), rtol=REL)
    np.testing.assert_allclose(b, pml_energies(make_oracle, -1j), rtol=REL)
    e = [x + y for x, y in zip(a, b)]
    for v in e[1:]:
        assert v <= e[0] * 4e-3


@pytest.mark.parametrize("G", [ProductSim, GroupSim, GroupSim3])
def test_three_d_pml_splitting(G):
    """tests/three_d.cpp:196-224 (test_pml_splitting): the split run's probes
    and field energies at t = 10, 20, 30 equal the unsplit oracle's (probes
    bitwise, energies to rel 1e-12 -- the reference asks 1e-9 / compare)."""
    o, eo, po = S.three_d_test_pml_splitting(make_oracle)
    p, ep, pp = S.three_d_test_pml_splitting(G)
    assert pp == po
    assert [t for t, _ in ep] == [t for t, _ in eo]
    np.testing.assert_allclose([v for _, v in ep], [v for _, v in eo], rtol=REL)


@pytest.mark.parametrize("G", [ProductSim, GroupSim3])
def test_energy_in_boxes_random(G):
    """Random fields, PML, dielectric core: electric / magnetic / field energy
    of the whole cell and of boxes crossing PML chunks (on and off the grid),
    before and after fused steps; fields untouched by the synchronization."""
    kw = dict(sizes=(3.2, 2.6, 3.0), steps=4, eps=12.0)
    p, o = S.sc_random_fields(G, **kw), S.sc_random_fields(make_oracle, **kw)
    boxes = [(None, None), ([-1.2, -0.9, -1.4], [1.3, 0.45, 0.66]),
             ([-0.31, -0.83, -0.5], [0.77, 1.3, 1.5]), ([0.2, -1.3, -1.5], [0.2, 1.3, 1.5])]
    for lo, hi in boxes:
        for name in ("electric_energy_in_box", "magnetic_energy_in_box", "field_energy_in_box"):
            a, b = getattr(p, name)(lo, hi), getattr(o, name)(lo, hi)
            assert a == pytest.approx(b, rel=REL, abs=1e-300), (name, lo, hi)
    p.step(5)
    o.step(5)
    assert p.field_energy() == pytest.approx(o.field_energy(), rel=REL)
    bad = {c: d for c, d in S.compare_all(p, o).items() if d}
    assert not bad, bad


def test_energy_first_step_semantics():
    """field_energy before any step: the synchronizing B step is the first
    step_db / update_eh(H), so f_u and H are created there and NOT restored
    (no backup existed, src/energy_and_flux.cpp:97-134) -- as the oracle."""
    def run(make):
        o = S.vol(make, 3, [2.0, 2.0, 2.0], 10, center_origin=True)
        o.add_pml(0.5)
        S.random_init(o, (9, 10, 11, 6, 7, 8))
        e = o.field_energy()
        o.step(6)
        return o, e
    p, ep = run(ProductSim)
    o, eo = run(make_oracle)
    assert ep == pytest.approx(eo, rel=REL)
    bad = {c: d for c, d in S.compare_all(p, o).items() if d}
    assert not bad, bad


def test_nan_guard():
    """fields::step aborts with "simulation fields are NaN or Inf" when the D
    energy density at the cell centre is not finite (src/step.cpp:138-139); the
    check runs on the device every set_nan_check(k) steps inside a batch (default
    every step), the flag is read every 256 steps and at the end of each call, and
    the error names the first failing step.  The time stays at the state the device
    holds (the steps run past the failing one inside the chunk), so after the error
    t and the arrays agree: they equal a run of t steps without the guard."""
    import re
    from meep_nl_amd import core
    gv = core.GridVolume(3, [20, 20, 20], 10.0, [-20, -20, -20])
    s = core.Structure(gv)
    v = np.zeros(gv.shape())
    v[10, 10, 13] = np.inf  # Dz three cells from the centre

    def bad_step(e):
        m = re.search(r"NaN or Inf \(at time step (\d+); fields left at time step (\d+)\)", str(e))
        assert m, str(e)
        return int(m.group(1)), int(m.group(2))

    f = core.Fields(s)
    f.set_nan_check(1)
    f.initialize_field(8, v)
    with pytest.raises(RuntimeError, match="simulation fields are NaN or Inf") as ei:
        for _ in range(20):
            f.step(1)
    bad, left = bad_step(ei.value)
    assert 1 <= bad <= 8 and f.t == bad == left  # one-step calls stop at the failing step
    f2 = core.Fields(s)
    f2.initialize_field(8, v)
    f2.set_nan_check(2)
    with pytest.raises(RuntimeError, match="simulation fields are NaN or Inf") as ei:
        f2.step(50)  # one call: the guard fires inside the batch, the call raises
    bad2, left2 = bad_step(ei.value)
    assert bad2 in (bad, bad + 1)  # its first check at or after the failing step
    # the flag is read at the end of each part of a call (the unfused first step, the pairs,
    # a one-step leftover) and every 256 steps: the device stopped at the first such point
    assert f2.t == left2 and bad2 <= left2 <= 50
    f3 = core.Fields(s)  # default cadence: every step
    f3.initialize_field(8, v)
    with pytest.raises(RuntimeError, match=r"NaN or Inf \(at time step") as ei:
        f3.step(10)  # one call of a few steps: checked (the old host guard ran every 100)
    bad3, left3 = bad_step(ei.value)
    assert bad3 == bad and f3.t == left3 and bad <= left3 <= 10
    f4 = core.Fields(s)  # a long call: the flag is read every 256 steps, not only at the end
    f4.initialize_field(8, v)
    with pytest.raises(RuntimeError, match="simulation fields are NaN or Inf") as ei:
        f4.step(2000)
    bad4, left4 = bad_step(ei.value)
    assert bad4 == bad and f4.t == left4 and bad <= left4 <= 257  # + the unfused first step
    # t and the arrays agree: the same state as t steps without the guard
    f5 = core.Fields(s)
    f5.initialize_field(8, v)
    f5.set_nan_check(10 ** 9)
    f5.step(f4.t)
    assert f5.t == f4.t
    for c in range(3):
        for comp in (c, 6 + c, 9 + c):  # E, D, B (MNL_EX.., MNL_DX.., MNL_BX..)
            assert f4.get_array(comp).tobytes() == f5.get_array(comp).tobytes(), comp
