"""Oracle restatement of the H-side materials: mu (chi1inv of the H components,
structure::set_mu -> set_chi1inv(H_stuff), per-chunk trivial deletion
src/anisotropic_averaging.cpp:279-296) entering update_eh(H_stuff) (src/update_eh.cpp:
67-283 -> step_update_EDHB, src/step_generic.cpp:576-906) and magnetic Lorentzian
susceptibilities (update_pols(H_stuff) after update_eh(H_stuff), src/step.cpp:75-92).

No reference test runs either (the fork's tests never set mu; python/tests/
test_simulation.py::test_has_mu only queries has_mu), so the restatement is pinned
by exact reductions and by the duality of uniform media: with eps = m, mu = 1 and a
current m * J, and with eps = 1, mu = m and the current J, Maxwell's equations give
the same E and B (D scales by m, H = B / m), so the two runs agree to rounding."""
import numpy as np
import pytest

from oracle import oracle as orc
from scenarios import make_oracle, sc_mu_1d, sc_mu_3d, vol


def test_trivial_mu_equals_no_mu():
    """mu = 1 everywhere: the rows are trivial in every chunk and deleted, H stays
    aliased to B -> bitwise the run without mu."""
    def run(mu):
        o = vol(make_oracle, 3, [2.0, 1.8, 2.2], 10, center_origin=True)
        o.add_pml(0.5)
        if mu:
            o.set_mu_fn(lambda *p: np.ones_like(p[0]))
        o.add_gaussian_source(2, 0.3, 3.0, 0.0, 30.0, (0.05, -0.15, 0.1), 1.0)
        o.add_gaussian_source(4, 0.35, 3.0, 0.0, 30.0, (-0.3, 0.2, -0.4), 0.5)
        o.step(30)
        return o
    a, b = run(False), run(True)
    for c in range(12):
        assert np.array_equal(a.get_array(c), b.get_array(c)), c


def test_zero_magnetic_sigma_equals_none():
    """A magnetic susceptibility whose sigma is 0 everywhere needs no P (global
    trivial flags, susceptibility::needs_P) -> bitwise the run without it."""
    def run(add):
        o = vol(make_oracle, 1, [8.0], 10, center_origin=True)
        o.add_pml(1.0)
        if add:
            z = o.coords(orc.Hy)[-1]
            o.add_magnetic_lorentzian(1.1, 0.05, [None, np.zeros_like(z), None])
        o.add_gaussian_source(0, 0.3, 3.0, 0.0, 30.0, (0, 0, -1.0), 1.0)
        o.step(200)
        return o
    a, b = run(False), run(True)
    for c in (orc.Ex, orc.Hy, orc.Dx, orc.By):
        assert np.array_equal(a.get_array(c), b.get_array(c))


@pytest.mark.parametrize("dim", [1, 3])
def test_uniform_duality(dim):
    """eps = m, mu = 1, current m*J  vs  eps = 1, mu = m, current J: same E and B
    (metallic walls, uniform medium) to rounding; H = B / m and D scales by m."""
    m = 2.5

    def run(eps_side):
        if dim == 1:
            o = vol(make_oracle, 1, [6.0], 10, center_origin=True)
            pos, ec, hc = (0, 0, 0.33), orc.Ex, orc.Hy
        else:
            o = vol(make_oracle, 3, [1.6, 1.4, 1.8], 10, center_origin=True)
            pos, ec, hc = (0.05, -0.15, 0.1), orc.Ez, orc.Hx
        one = lambda *p: np.full_like(p[0], m)  # noqa: E731
        if eps_side:
            o.set_epsilon_fn(one)
        else:
            o.set_mu_fn(one)
        o.add_gaussian_source(ec, 0.3, 3.0, 0.0, 30.0, pos, m if eps_side else 1.0)
        o.step(150 if dim == 1 else 40)
        return o, ec, hc
    (a, ec, hc), (b, _, _) = run(True), run(False)
    ea, eb = a.get_array(ec), b.get_array(ec)
    ba, bb = a.get_array(hc + 6), b.get_array(hc + 6)
    scale = max(np.abs(ea).max(), 1e-300)
    assert np.abs(ea).max() > 0
    assert np.abs(ea - eb).max() <= 1e-11 * scale
    assert np.abs(ba - bb).max() <= 1e-11 * max(np.abs(ba).max(), 1e-300)
    hb = b.get_array(hc)
    assert np.abs(hb * m - bb).max() <= 1e-11 * max(np.abs(bb).max(), 1e-300)


def test_mu_slab_slows_the_pulse():
    """A mu = 3 slab (n = sqrt(3)) delays the transmitted pulse: the arrival of the
    field behind the slab is later than in vacuum."""
    def arrival(mu):
        o = vol(make_oracle, 1, [12.0], 10, center_origin=True)
        o.add_pml(1.0)
        if mu:
            o.set_mu_fn(lambda *p: np.where(np.abs(p[0]) < 2.0, 3.0, 1.0))
        o.add_gaussian_source(0, 0.5, 5.0, 0.0, 10.0, (0, 0, -3.0), 1.0)
        t_peak, best = 0, 0.0
        for k in range(250):
            o.step(1)
            v = abs(o.get_field(orc.Ex, (0, 0, 3.0)))
            if v > best:
                best, t_peak = v, k
        return t_peak
    assert arrival(True) > arrival(False) + 20


def test_magnetic_lorentzian_changes_fields_and_stays_finite():
    a = sc_mu_1d(make_oracle, steps=300)
    b = sc_mu_1d(make_oracle, steps=300, lorentz=True)
    ea, eb = a.get_array(orc.Ex), b.get_array(orc.Ex)
    assert np.all(np.isfinite(eb))
    assert np.abs(ea - eb).max() > 1e-6 * np.abs(ea).max()


def test_mu_3d_runs():
    o = sc_mu_3d(make_oracle, steps=20, lorentz=True, offdiag=True)
    for c in range(12):
        assert np.all(np.isfinite(o.get_array(c)))
